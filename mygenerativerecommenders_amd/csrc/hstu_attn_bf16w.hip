// Jagged causal HSTU attention backward, bf16 MFMA operands, WIDE heads (128 < d <= 256,
// dqk == dv) — gfx950, v_mfma_f32_32x32x16_bf16.  The opt-in bf16 compute mode at ml-20m
// width (d = 256, N = 2059); narrower heads keep hstu_attn_bf16.hip.
//
// Same math as hstu_attn_bwd.hip (reference sequential_encoders/hstu.py:134-205 and the
// bias of hstu.py:96-128): S = Q K^T + bias, P = silu(S) / N, dP = dO V^T,
// dS = dP silu'(S) / N, dV = P^T dO, dK = dS^T Q, dQ = dS K, dbias = sum dS.
//
// Layout of the work (one wave per SIMD, 512 registers: the 32 x d f32 accumulators of a
// wave's 32 keys sit beside the keys' K / V fragments):
//   * key-major pass, two workgroup kinds in one launch, 4 waves x 32 keys each:
//       kind V: S (A = Q rows from LDS, B = K^T fragments in registers), P, dV += P^T dO;
//       kind K: S, dP, dS, dK += dS^T Q, the relative-bias gradients, and the bf16 dS
//               blocks for the query-major pass.
//     S / dP are 32 x 32 f32 tiles with the key on the lane and the queries in registers,
//     so P and dS convert in place to the A operand of the next product (X^T B: no LDS
//     round trip); its B operand (dO / Q rows, k = queries) comes from the row-major LDS
//     tile through ds_read_b64_tr_b16 (hardware transpose), in the permuted k order the
//     register operand implies.
//   * query-major pass (dQ = dS K), 4 waves x 32 queries: A = the stored dS block, read
//     back transposed; B = the K tile, transposed reads.  Nothing is recomputed.
// Relative-bias gradients stay fp32 and deterministic: dpos_w per wave as plain stores of
// each diagonal bin (a chunk's wrapped diagonals are carried into the next chunk, whose
// main diagonals are the same bins), dts_w per lane as running (bucket, sum) flushed to
// per-wave LDS histograms; one slab per wave, reduced in a fixed order.
#include "attn_common.h"

#ifndef W_ABL
#define W_ABL 0  // ablation builds only (scripts/attn_micro.py against vlib/ variants)
#endif

#include "../../include/gr_hstu.h"

namespace gr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 f16_zero() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// C += A B over k = 16: a = A[row lane%32][k 8(lane/32) .. +7], b = B[k ..][col lane%32];
// C[row (reg & 3) + 8 (reg >> 2) + 4 (lane / 32)][col lane % 32]
__device__ __forceinline__ f32x16 mfma32(u32x4_t a, u32x4_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
// ds_read_b64_tr_b16: per 16-lane group, lane 4q + p gives the address of row q, columns
// 4p .. 4p + 3 of a 4 x 16 block of bf16; lane i receives column i of the 4 rows.
__device__ __forceinline__ u32x2_t tr16(const __bf16* p) {
  const s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(p));
  return __builtin_bit_cast(u32x2_t, v);
}
// B operand (8 bf16) for k-step s of a product whose A operand is a 32 x 32 accumulator in
// registers: element j of lane half h is k = 16 s + 8 (j >> 2) + 4 h + (j & 3), column =
// c0 + lane % 32, from a row-major [k][col] LDS tile with row stride rs (bf16 units).
__device__ __forceinline__ u32x4_t trB_acc(const __bf16* tile, int rs, int s, int c0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const __bf16* base = tile + (16 * s + 4 * h + q) * rs + c0 + 16 * (g & 1) + 4 * p;
  const u32x2_t lo = tr16(base), hi = tr16(base + 8 * rs);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
// The same in natural k order: element j of lane half h is k = 16 s + 8 h + j.
__device__ __forceinline__ u32x4_t trB_nat(const __bf16* tile, int rs, int s, int c0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const __bf16* base = tile + (16 * s + 8 * h + q) * rs + c0 + 16 * (g & 1) + 4 * p;
  const u32x2_t lo = tr16(base), hi = tr16(base + 4 * rs);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
// The accumulator's registers 8s .. 8s+7 as a bf16 A / B fragment (k-step s)
__device__ __forceinline__ u32x4_t acc_frag(const float (&x)[16], int s) {
  return u32x4_t{pack_bf16(x[8 * s], x[8 * s + 1]), pack_bf16(x[8 * s + 2], x[8 * s + 3]),
                 pack_bf16(x[8 * s + 4], x[8 * s + 5]), pack_bf16(x[8 * s + 6], x[8 * s + 7])};
}

struct AttnBwdArgsW {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const float* dout;
  int64_t ld_dout;
  const int64_t* offsets;
  int B, N, H, d;
  const uint8_t* map_kq;  // key-major bucket map (null: no bias)
  const float* pos_w;
  const float* ts_w;
  int nb;
  const float* hq;
  const float* hk;
  const float* hv;
  int64_t ld_h;
  float* dq;
  float* dk;
  float* dvv;
  int64_t ld_d;
  float* slabs;    // [grid_k][4 waves][2N-1 + nb+1]
  __bf16* ds;      // dS blocks: [bh][tri(qb, kb)][32 keys][32 queries]
  int nbt;         // dS blocks per (sequence, head): NB (NB + 1) / 2, NB = ceil(N / 32)
  float inv_n;
  int n_kt;        // 128-key tiles
  int n_qt;        // 128-query tiles
};

constexpr int WK = 128;  // keys (queries) per workgroup: 4 waves x 32
constexpr int kDtsCopies = 4;  // dts histogram copies per wave (lane % copies)
__host__ __device__ constexpr int w_dts_stride(int nb1) { return ((nb1 + 30) / 32) * 32 + 1; }

// fp32 rows -> bf16 LDS tile, 32 rows x DP columns: thread t owns the column pair
// 2 (t % 128) of rows t / 128 + 2 i (one voffset per thread, the row step in soffset);
// rows past the sequence read 0 (descriptor range), columns >= ncols read 0 (offset)
template <int DP>
struct StageW {
  static constexpr int PER = 16;
  float2 v[PER];
  int voff;
  __device__ __forceinline__ void init(int64_t ld, int ncols) {
    const int c = 2 * (threadIdx.x & 127), rr = threadIdx.x >> 7;
    voff = c < ncols ? (rr * (int)ld + c) * 4 : 0x40000000;
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int64_t ld, int r0) {
    typedef unsigned int u2_ __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const u2_ x = __builtin_amdgcn_raw_buffer_load_b64(r, voff, (r0 + 2 * i) * (int)ld * 4, 0);
      v[i] = make_float2(__uint_as_float(x.x), __uint_as_float(x.y));
    }
  }
  __device__ __forceinline__ void store(__bf16* lds, int rs) const {
    const int c = 2 * (threadIdx.x & 127), rr = threadIdx.x >> 7;
    if (DP == 256 || c < DP) {
#pragma unroll
      for (int i = 0; i < PER; ++i)
        *reinterpret_cast<uint32_t*>(lds + (rr + 2 * i) * rs + c) = pack_bf16(v[i].x, v[i].y);
    }
  }
};

// ------------------------------------------------------------------ key-major pass
// KIND_K = false: dV += P^T dO;  true: dK += dS^T Q, bias gradients, dS blocks.
template <int D32, bool HB, bool KIND_K>
__device__ __forceinline__ void kv_body(const AttnBwdArgsW& a, char* smem, int rank) {
  constexpr int DP = 32 * D32;   // padded head dim
  constexpr int KS = DP / 16;    // k-steps of the S / dP products
  constexpr int RS = DP + 8;     // LDS row stride (bf16): 16-byte aligned rows
  constexpr bool BIAS = HB && KIND_K;
  __bf16* tiles = reinterpret_cast<__bf16*>(smem);  // [2 buffers][Q, dO][32][RS]
  float* tsw = reinterpret_cast<float*>(tiles + 4 * 32 * RS);
  const int npos = 2 * a.N - 1;
  float* posw = tsw + (a.nb + 1);
  const int tss = w_dts_stride(a.nb + 1);
  float* hts = posw + npos;  // [4 waves][kDtsCopies][tss]

  const int BH = a.B * a.H;
  const int kt = rank / BH;  // heaviest (first) key tiles first
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * WK;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int nbins = npos + a.nb + 1;
  float* slab = BIAS ? a.slabs + ((int64_t)rank * 4 + w) * nbins : nullptr;
  if (k0 >= L) {
    if (BIAS)
      for (int i = lane; i < nbins; i += 64) slab[i] = 0.f;
    return;
  }
  if (HB) {
    for (int i = tid; i <= a.nb; i += 256) tsw[i] = a.ts_w[i];
    for (int i = tid; i < npos; i += 256) posw[i] = a.pos_w[i];
  }
  if (BIAS)
    for (int i = tid; i < 4 * kDtsCopies * tss; i += 256) hts[i] = 0.f;
  const int k0w = k0 + 32 * w;   // this wave's first key
  const int kj = k0w + lr;       // this lane's key (column of S / dP)
  const bool k_ok = kj < L;
  // K^T / V^T fragments of the wave's keys: element j of k-step ks = dim 16 ks + 8 lh + j
  // (keys >= L read 0 through the descriptor range; dims >= d are masked)
  u32x4_t kf[KS], vf[KS];
  {
    auto frag = [&](__amdgpu_buffer_rsrc_t r, int64_t ld, int ks) {
      const int c0 = 16 * ks + 8 * lh;
      const int off = (kj * (int)ld + c0) * 4;
      const u32x4_t lo = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      const u32x4_t hi = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
      float x[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = c0 + j < a.d ? __uint_as_float(lo[j]) : 0.f;
        x[4 + j] = c0 + 4 + j < a.d ? __uint_as_float(hi[j]) : 0.f;
      }
      return u32x4_t{pack_bf16(x[0], x[1]), pack_bf16(x[2], x[3]), pack_bf16(x[4], x[5]), pack_bf16(x[6], x[7])};
    };
    const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.d, L, a.d);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = frag(rk, a.ld_qk, ks);
    if (KIND_K) {
      const __amdgpu_buffer_rsrc_t rv = seq_rsrc(a.v, a.ld_v, s0, h * a.d, L, a.d);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) vf[ks] = frag(rv, a.ld_v, ks);
    }
  }
  // output accumulators: tile t = columns 32 t .. 32 t + 31, rows = the wave's keys
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();

  const __amdgpu_buffer_rsrc_t rq = seq_rsrc(a.q, a.ld_qk, s0, h * a.d, L, a.d);
  const __amdgpu_buffer_rsrc_t rdo = seq_rsrc(a.dout, a.ld_dout, s0, h * a.d, L, a.d);
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_kq, b, attn_tiles_per_seq(a.N));
  // dts: running (bucket, sum) of this lane, flushed into per-wave LDS histogram copies
  // when the bucket changes
  float* wts = hts + (w * kDtsCopies + (lr % kDtsCopies)) * tss;
  int run_b = -1;
  float run_s = 0.f;
  // dpos: each bin of the wave's slab is written once: main diagonals of a chunk plus the
  // wrapped diagonals of the previous chunk (carry), see the file header
  float carry = 0.f;

  StageW<DP> stq, std_;
  stq.init(a.ld_qk, a.d);
  std_.init(a.ld_dout, a.d);
  const int n_chunks = (L - k0 + 31) / 32;  // the workgroup's chunks: queries k0, k0 + 32, ...
  const bool w_on = k0w < L;
  const int map_w = (kj & 63) * 16;
  // bucket words of chunk qc: key kj, queries qc + 8m + 4lh .. +3 (key-major 64 x 64 tiles);
  // loaded one chunk ahead
  auto map_words = [&](int qc, uint32_t (&mw)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int qq = qc + 8 * m + 4 * lh;
      mw[m] = buf_ld_u32(rmap, (attn_tile_id(qq >> 6, k0w >> 6) * 1024 + map_w + ((qq & 63) >> 2)) * 4, 0);
    }
  };
  uint32_t mw_next[4] = {0u, 0u, 0u, 0u};
  if (HB && w_on) map_words(k0w, mw_next);
  stq.load(rq, a.ld_qk, k0);
  std_.load(rdo, a.ld_dout, k0);
  stq.store(tiles, RS);
  std_.store(tiles + 32 * RS, RS);
  __syncthreads();
  for (int ci = 0; ci < n_chunks; ++ci) {
    const int qc0 = k0 + 32 * ci;
    const __bf16* Qs = tiles + (ci & 1) * 64 * RS;
    const __bf16* Ds = Qs + 32 * RS;
    __bf16* Qn = tiles + ((ci + 1) & 1) * 64 * RS;
    const bool more = ci + 1 < n_chunks;
    // the next chunk's rows: loaded now, written to the other buffer after this chunk
    if (W_ABL != 2 && more) {
      stq.load(rq, a.ld_qk, qc0 + 32);
      std_.load(rdo, a.ld_dout, qc0 + 32);
    }
    const bool act = w_on && qc0 >= k0w;  // wave-uniform: the chunk reaches the wave's keys
    if (act) {
      uint32_t mw[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) mw[m] = mw_next[m];
      if (HB && more) map_words(qc0 + 32, mw_next);
      // two independent chains per kind (S, dP or the even / odd k-steps of S)
      f32x16 S = f16_zero(), dP = f16_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4_t qa = *reinterpret_cast<const u32x4_t*>(Qs + lr * RS + 16 * ks + 8 * lh);
        if (KIND_K) {
          S = mfma32(qa, kf[ks], S);
          dP = mfma32(*reinterpret_cast<const u32x4_t*>(Ds + lr * RS + 16 * ks + 8 * lh), vf[ks], dP);
        } else if (ks & 1) {
          dP = mfma32(qa, kf[ks], dP);
        } else {
          S = mfma32(qa, kf[ks], S);
        }
      }
      if (!KIND_K) S += dP;
      // element rr: query qc0 + (rr & 3) + 8 (rr >> 2) + 4 lh, key kj
      float x16[16];
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int qi = qc0 + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
        const bool ok = k_ok && qi < L && kj <= qi;
        float x = S[rr];
        int bk = 0;
        if (HB) {
          bk = (mw[rr >> 2] >> (8 * (rr & 3))) & 0xFF;
          int pi = a.N - 1 + kj - qi;
          pi = pi < 0 ? 0 : (pi > npos - 1 ? npos - 1 : pi);
          x = x + (posw[pi] + tsw[bk]);
        }
        const float sg = W_ABL == 1 ? x : sigmoidf_(x);
        const uint32_t msk = ok ? 0xffffffffu : 0u;
        if (!KIND_K) {
          x16[rr] = __uint_as_float(__float_as_uint(x * sg * a.inv_n) & msk);
        } else {
          const float dsv = __uint_as_float(
              __float_as_uint(dP[rr] * (sg * (1.0f + x * (1.0f - sg))) * a.inv_n) & msk);
          x16[rr] = dsv;
        }
      }
      const u32x4_t f0 = acc_frag(x16, 0), f1 = acc_frag(x16, 1);
      // acc += X^T B, B = dO (dV) or Q (dK) rows of the chunk, transposed reads
      const __bf16* Bt = KIND_K ? Qs : Ds;
#pragma unroll
      for (int t = 0; t < (W_ABL == 3 ? 1 : D32); ++t) acc[t] = mfma32(f0, trB_acc(Bt, RS, 0, 32 * t, lane), acc[t]);
#pragma unroll
      for (int t = 0; t < (W_ABL == 3 ? 1 : D32); ++t) acc[t] = mfma32(f1, trB_acc(Bt, RS, 1, 32 * t, lane), acc[t]);
      if (KIND_K) {
        // dS block for the query-major pass: [key][query] image, registers 4g .. 4g+3 =
        // queries 8g + 4lh + 0..3 (8-byte stores)
        const int qb = qc0 >> 5, kb = k0w >> 5;
        __bf16* blk = a.ds + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2 + kb) * 1024;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const u32x2_t v2 = u32x2_t{pack_bf16(x16[4 * g], x16[4 * g + 1]),
                                     pack_bf16(x16[4 * g + 2], x16[4 * g + 3])};
          *reinterpret_cast<u32x2_t*>(blk + lr * 32 + 8 * g + 4 * lh) = v2;
        }
      }
      if (BIAS && W_ABL != 4 && W_ABL != 6) {
        // dts run (a lane's queries ascend with rr), after the math so that the branches
        // do not split its schedule; the accumulator MFMAs above run meanwhile
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int qi = qc0 + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
          const bool ok = k_ok && qi < L && kj <= qi;
          const int bk = (mw[rr >> 2] >> (8 * (rr & 3))) & 0xFF;
          if (ok && bk != run_b) {
            if (run_b >= 0) atomicAdd(&wts[run_b], run_s);
            run_b = bk;
            run_s = 0.f;
          }
          run_s += x16[rr];  // 0 where !ok
        }
      }
      if (BIAS && W_ABL != 5 && W_ABL != 6) {
        // dpos: rotate register rr (row R = (rr & 3) + 8 (rr >> 2) + 4 lh) left by R in
        // the 32-lane half: lane c then holds diagonal c (main) or c - 32 (wrapped)
        float dmain = 0.f, dwrap = 0.f;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int R = (rr & 3) + 8 * (rr >> 2) + 4 * lh;
          const float v = __shfl(x16[rr], (lh << 5) | ((lr + R) & 31), 64);
          const bool mn = lr + R < 32;
          dmain += mn ? v : 0.f;
          dwrap += mn ? 0.f : v;
        }
        auto sm = __builtin_amdgcn_permlane32_swap(__float_as_uint(dmain), __float_as_uint(dmain), false, false);
        auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dwrap), __float_as_uint(dwrap), false, false);
        dmain = __uint_as_float(sm[0]) + __uint_as_float(sm[1]);
        dwrap = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
        const int bin = a.N - 1 + (k0w - qc0) + lr;  // diagonal kj - qi = k0w - qc0 + c - R
        if (lh == 0 && bin >= 0 && bin < npos) slab[bin] = dmain + carry;
        carry = dwrap;
      }
    }
    if (more) {
      if (W_ABL != 2) {
        stq.store(Qn, RS);
        std_.store(Qn + 32 * RS, RS);
      }
      __syncthreads();
    }
  }
  // ---- epilogue: acc[t][rr] = (dV or dK)[key k0w + (rr & 3) + 8 (rr >> 2) + 4 lh][32 t + lr]
  float* outp = KIND_K ? a.dk : a.dvv;
  const float* hp = KIND_K ? a.hk : a.hv;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int key = k0w + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
    const int64_t row = s0 + (key < L ? key : 0);
#pragma unroll
    for (int t = 0; t < D32; ++t) {
      const int c = 32 * t + lr;
      float g = acc[t][rr];
      if (key < L && c < a.d) {
        if (hp) g *= silu_grad_(as_global(hp)[row * a.ld_h + h * a.d + c]);
        outp[row * a.ld_d + h * a.d + c] = g;
      }
    }
  }
  if (BIAS) {
    // the last chunk's wrapped diagonals; zero every bin this wave never wrote: written
    // bins N-1 + d0 + [-32, 31] over d0 = k0w - qc0, qc0 = k0w .. last chunk
    int lo = npos, hi = -1;
    if (w_on) {
      const int d0_last = k0w - (k0 + 32 * (n_chunks - 1));
      const int bin = a.N - 1 + d0_last - 32 + lr;
      if (lh == 0 && bin >= 0 && bin < npos) slab[bin] = carry;
      lo = a.N - 1 + d0_last - 32;
      hi = a.N - 1 + 31;
    }
    for (int i = lane; i < npos; i += 64)
      if (i < lo || i > hi) slab[i] = 0.f;
    if (run_b >= 0) atomicAdd(&wts[run_b], run_s);
    __syncthreads();
    for (int i = lane; i <= a.nb; i += 64) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < kDtsCopies; ++c) s += hts[(w * kDtsCopies + c) * tss + i];
      slab[npos + i] = s;
    }
  }
}

// even workgroups: dK (+ bias, dS), odd: dV; pairs in heaviest-first order
template <int D32, bool HB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void attn_bwd_bf16w_kv_kernel(AttnBwdArgsW a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((blockIdx.x & 1) == 0) kv_body<D32, HB, true>(a, smem, blockIdx.x >> 1);
  else kv_body<D32, HB, false>(a, smem, blockIdx.x >> 1);
}

// ------------------------------------------------------------------ query-major pass
// dQ[q][:] = sum over key blocks of dS block (A: transposed reads of the [key][query] image,
// natural k order) times the K tile (B: transposed reads of the row-major bf16 tile).
template <int D32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void attn_bwd_bf16w_dq_kernel(AttnBwdArgsW a) {
  constexpr int DP = 32 * D32;
  constexpr int RS = DP + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* kt_l = reinterpret_cast<__bf16*>(smem);  // [2][32][RS]
  __bf16* dsl = kt_l + 2 * 32 * RS;                // [4 waves][2][32 x 32]
  const int BH = a.B * a.H;
  const int qt = a.n_qt - 1 - (int)blockIdx.x / BH;  // heaviest tiles first
  const int bh = blockIdx.x % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * WK;
  if (q0 >= L) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31;
  const int q0w = q0 + 32 * w;
  const int qb = q0w >> 5;
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.d, L, a.d);
  StageW<DP> stk;
  stk.init(a.ld_qk, a.d);
  const int n_kb = (min(q0 + WK, L) + 31) / 32;  // key blocks the workgroup needs
  __bf16* mydl = dsl + w * 2 * 1024;
  const bool w_on = q0w < L;
  auto load_ds = [&](int kb, u32x4_t (&v)[2]) {
    // the wave's 2 KB block (qb, kb): 64 lanes x 2 x 16 B
    const __bf16* src = a.ds + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2 + kb) * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      v[i] = (w_on && kb <= qb) ? *reinterpret_cast<const u32x4_t*>(src + 8 * (lane + 64 * i))
                                : u32x4_t{0u, 0u, 0u, 0u};
  };
  u32x4_t dsv[2];
  stk.load(rk, a.ld_qk, 0);
  load_ds(0, dsv);
  stk.store(kt_l, RS);
#pragma unroll
  for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4_t*>(mydl + 8 * (lane + 64 * i)) = dsv[i];
  __syncthreads();
  for (int kb = 0; kb < n_kb; ++kb) {
    const __bf16* Kl = kt_l + (kb & 1) * 32 * RS;
    const __bf16* Dl = mydl + (kb & 1) * 1024;
    const bool more = kb + 1 < n_kb;
    if (more) {
      stk.load(rk, a.ld_qk, 32 * (kb + 1));
      load_ds(kb + 1, dsv);
    }
    if (w_on && kb <= qb) {  // wave-uniform causal skip
      // A: dS[q = lane % 32][keys 16 s + 8 lh + 0..7] from the [key][query] image
      const u32x4_t a0 = trB_nat(Dl, 32, 0, 0, lane), a1 = trB_nat(Dl, 32, 1, 0, lane);
#pragma unroll
      for (int t = 0; t < D32; ++t) {
        acc[t] = mfma32(a0, trB_nat(Kl, RS, 0, 32 * t, lane), acc[t]);
        acc[t] = mfma32(a1, trB_nat(Kl, RS, 1, 32 * t, lane), acc[t]);
      }
    }
    if (more) {
      stk.store(kt_l + ((kb + 1) & 1) * 32 * RS, RS);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<u32x4_t*>(mydl + ((kb + 1) & 1) * 1024 + 8 * (lane + 64 * i)) = dsv[i];
      __syncthreads();
    }
  }
  if (!w_on) return;
  const int lh = lane >> 5;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int qo = q0w + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
    if (qo >= L) continue;
    const int64_t row = s0 + qo;
#pragma unroll
    for (int t = 0; t < D32; ++t) {
      const int c = 32 * t + lr;
      if (c >= a.d) continue;
      float g = acc[t][rr];
      if (a.hq) g *= silu_grad_(as_global(a.hq)[row * a.ld_h + h * a.d + c]);
      a.dq[row * a.ld_d + h * a.d + c] = g;
    }
  }
}

// slabs: [n][2N-1 + nb+1]; fixed-order reduce in two coalesced stages: stage 1 sums slabs
// 64 g .. 64 g + 63 of each bin in order into slab 64 g (each thread reads its own bins
// before overwriting them); stage 2 adds the groups in g order
constexpr int kRedGroup = 64;
__global__ __launch_bounds__(256) void attn_bf16w_bias_reduce1(float* slabs, int n_slabs, int nbins) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nbins) return;
  const int j0 = blockIdx.y * kRedGroup, j1 = min(j0 + kRedGroup, n_slabs);
  float acc = 0.f;
  for (int j = j0; j < j1; ++j) acc += slabs[(int64_t)j * nbins + i];
  slabs[(int64_t)j0 * nbins + i] = acc;
}
__global__ __launch_bounds__(256) void attn_bf16w_bias_reduce2(const float* slabs, int n_slabs,
                                                               int n_pos, int n_ts, float* dpos_w,
                                                               float* dts_w) {
  const int nbins = n_pos + n_ts;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nbins) return;
  float acc = 0.f;
  for (int j = 0; j < n_slabs; j += kRedGroup) acc += slabs[(int64_t)j * nbins + i];
  if (i < n_pos) dpos_w[i] = acc;
  else dts_w[i - n_pos] = acc;
}

static size_t bf16w_slab_bytes(int B, int N, int max_len, int H, int nb) {
  return sizeof(float) * 4 * (size_t)ceil_div(max_len, WK) * B * H * (size_t)(2 * N - 1 + nb + 1);
}
static size_t bf16w_ds_bytes(int B, int N, int H) {
  const size_t nb32 = (size_t)ceil_div(N, 32);
  return 2048 * (nb32 * (nb32 + 1) / 2) * (size_t)B * H;
}

template <int D32>
static int launch_bwd_bf16w(AttnBwdArgsW a, float* dpos_w, float* dts_w, hipStream_t st) {
  constexpr int DP = 32 * D32, RS = DP + 8;
  const size_t npos = 2 * a.N - 1;
  const int tss = w_dts_stride(a.nb + 1);
  const size_t lds_kv = 2 * 4 * 32 * RS + sizeof(float) * ((a.nb + 1) + npos + 4 * kDtsCopies * tss);
  const size_t lds_q = 2 * (2 * 32 * RS + 4 * 2 * 1024);
  GR_REQUIRE(lds_kv <= 160 * 1024, "hstu_attn_bwd_bf16: LDS %zu B exceeds 160 KiB (N=%d)", lds_kv, a.N);
  const int grid = a.n_kt * a.B * a.H;
  auto kkv = a.map_kq ? attn_bwd_bf16w_kv_kernel<D32, true> : attn_bwd_bf16w_kv_kernel<D32, false>;
  GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kkv, dim3(2 * grid), dim3(256), lds_kv, st, a));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide dkv)");
  const int grid_q = a.n_qt * a.B * a.H;
  GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL(attn_bwd_bf16w_dq_kernel<D32>, dim3(grid_q), dim3(256), lds_q, st, a));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide dq)");
  if (a.map_kq) {
    const int nbins = (int)npos + a.nb + 1;
    const int n_slabs = 4 * grid;
    GR_TIMED("attn_bias_reduce", st, hipLaunchKernelGGL(attn_bf16w_bias_reduce1, dim3(ceil_div(nbins, 256), ceil_div(n_slabs, kRedGroup)),
                                                        dim3(256), 0, st, a.slabs, n_slabs, nbins));
    GR_TIMED("attn_bias_reduce", st, hipLaunchKernelGGL(attn_bf16w_bias_reduce2, dim3(ceil_div(nbins, 256)), dim3(256), 0, st,
                                                        a.slabs, n_slabs, (int)npos, a.nb + 1, dpos_w, dts_w));
    GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide bias reduce)");
  }
  return 0;
}

}  // namespace gr

// Wide-head entry (called by hstu_attn_bwd_bf16 for 128 < d <= 256, dqk == dv).
size_t gr_attn_bwd_bf16w_workspace(int B, int N, int max_len, int H, int num_buckets) {
  return ((gr::bf16w_slab_bytes(B, N, max_len, H, num_buckets) + 255) & ~(size_t)255) +
         gr::bf16w_ds_bytes(B, N, H);
}

int gr_attn_bwd_bf16w(const float* q, const float* k, const float* v, int64_t ld_qk, int64_t ld_v,
                      const float* dout, int64_t ld_dout, const int64_t* offsets, int B, int N,
                      int max_len, int H, int d, const uint8_t* map_kq, const float* pos_w,
                      const float* ts_w, int num_buckets, const float* hq, const float* hk,
                      const float* hv, int64_t ld_h, float* dq, float* dk, float* dvv, int64_t ld_d,
                      float* dpos_w, float* dts_w, void* workspace, hipStream_t st) {
  using namespace gr;
  const size_t slab_b = (bf16w_slab_bytes(B, N, max_len, H, num_buckets) + 255) & ~(size_t)255;
  AttnBwdArgsW a{};
  a.q = q; a.k = k; a.v = v; a.ld_qk = ld_qk; a.ld_v = ld_v; a.dout = dout; a.ld_dout = ld_dout;
  a.offsets = offsets; a.B = B; a.N = N; a.H = H; a.d = d;
  a.map_kq = map_kq; a.pos_w = pos_w; a.ts_w = ts_w; a.nb = map_kq ? num_buckets : 0;
  a.hq = hq; a.hk = hk; a.hv = hv; a.ld_h = ld_h;
  a.dq = dq; a.dk = dk; a.dvv = dvv; a.ld_d = ld_d;
  a.slabs = (float*)workspace;
  a.ds = (__bf16*)((char*)workspace + slab_b);
  const int nb32 = ceil_div(N, 32);
  a.nbt = nb32 * (nb32 + 1) / 2;
  a.inv_n = 1.0f / (float)N;
  a.n_kt = ceil_div(max_len, WK);
  a.n_qt = ceil_div(max_len, WK);
  const int D32 = ceil_div(d, 32);
  if (D32 <= 5) return launch_bwd_bf16w<5>(a, dpos_w, dts_w, st);
  if (D32 == 6) return launch_bwd_bf16w<6>(a, dpos_w, dts_w, st);
  if (D32 == 7) return launch_bwd_bf16w<7>(a, dpos_w, dts_w, st);
  return launch_bwd_bf16w<8>(a, dpos_w, dts_w, st);
}
