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
//   * key-major dK pass, 4 waves x 32 keys each: S (A = Q rows from LDS, B = K^T
//     fragments in registers), dP, dS, dK += dS^T Q, the relative-bias gradients, the bf16
//     dS blocks for the query-major pass and the bf16 P blocks for the dV pass;
//   * key-major dV pass: dV += P^T dO with P read back as the dK wave's A-fragment image
//     (S and the sigmoid run once per element; a dV workgroup beside each dK workgroup
//     used to recompute them);
//     S / dP are 32 x 32 f32 tiles with the key on the lane and the queries in registers,
//     so P and dS convert in place to the A operand of the next product (X^T B: no LDS
//     round trip); its B operand (dO / Q rows, k = queries) comes from the row-major LDS
//     tile through ds_read_b64_tr_b16 (hardware transpose), in the permuted k order the
//     register operand implies.
//   * query-major pass (dQ = dS K), 4 waves x 32 queries: A = the stored dS block, read
//     back transposed; B = the K tile, transposed reads.  Nothing is recomputed.
// Operands reach LDS as bf16 through LDS-DMA (global_load_lds_dwordx4, no registers):
// a conversion pass first writes bf16 copies of Q, K, V and dO, [row][head][32 D32] with
// zero padding; LDS tiles are chunk-major, [16-byte column chunk][row][8 bf16], so that
// the DMA's lane-linear image is the tile and both the A-fragment reads (ds_read_b128,
// lanes = consecutive rows) and the transposed B reads need no per-lane address math.
// Relative-bias gradients stay fp32 and deterministic: dpos_w per wave as plain stores of
// each diagonal bin, summed through a per-wave LDS skew image (element (row R, key c) at
// row 31 - c + R: a lane sums one diagonal with no shuffles; a chunk's wrapped diagonals
// are carried into the next chunk, whose main diagonals are the same bins), dts_w per
// lane as running (bucket, sum) flushed to per-wave LDS histograms (a chunk that extends
// every lane's open run skips the per-element loop); one slab per wave, reduced in a
// fixed order.
#include "attn_common.h"
#include <type_traits>
#include "mfma32.h"


#include "../../include/gr_hstu.h"

namespace gr {

#ifdef GR_STAMP
// Diagnostic build only (-DGR_STAMP): per-wave phase cycle sums of the key-major kernel,
// [workgroup][wave][12]: prologue, S/dP, elementwise, dV/dK, dS store + dts, barrier, dpos,
// total, kind
__device__ unsigned long long gr_stamp_bw_buf[1 << 16];
#define BW_ST(i, dep)                                            \
  do {                                                           \
    asm volatile("" ::"v"(dep));                                 \
    __builtin_amdgcn_sched_barrier(0);                           \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                           \
    st_[i] += t1_ - st_t0;                                       \
    st_t0 = t1_;                                                 \
  } while (0)
#else
#define BW_ST(i, dep) do { } while (0)
#endif

// Chunk-major tiles: element (row r, column c) at byte ((c >> 3) * 32 + r) * 16 + (c & 7) * 2.
// trB_acc / trB_nat on such a tile (rows = k): k-step s, columns 32 t .. 32 t + 31.
__device__ __forceinline__ u32x4_t trB_acc_cm(const char* tile, int s, int t, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const char* base = tile + ((4 * t + 2 * (g & 1) + (p >> 1)) * 32 + 16 * s + 4 * h + q) * 16 + 8 * (p & 1);
  const u32x2_t lo = tr16(reinterpret_cast<const __bf16*>(base)),
                hi = tr16(reinterpret_cast<const __bf16*>(base + 8 * 16));
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
// The query-major pass's K tile is swizzled: row r of chunk k sits in slot r ^ 4 (k & 3).
// A chunk is 512 B, so unswizzled the same row of chunks k .. k + 3 shares its LDS banks
// and each transposed read below (lanes over 4 chunks x 4 rows) was a 4-way bank
// conflict; swizzled, those 16 (chunk, row) pairs cover the 64 banks once (dQ 125 -> 118
// us per C3 layer).  The key-major and forward tiles stay unswizzled: their readers'
// extra address VALU cost more than their conflicts did (measured).
__device__ __forceinline__ int swz_row(int r, int k) { return r ^ ((k & 3) << 2); }
__device__ __forceinline__ u32x4_t trB_nat_cm_swz(const char* tile, int s, int t, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int k = 2 * (g & 1) + (p >> 1);  // chunk 4 t + k
  const char* base = tile + ((4 * t + k) * 32 + 16 * s + swz_row(8 * h + q, k)) * 16 + 8 * (p & 1);
  const int d2 = (p >> 1) ? -4 : 4;      // rows + 4 flip bit 2, which the XOR sets for p >> 1
  const u32x2_t lo = tr16(reinterpret_cast<const __bf16*>(base)),
                hi = tr16(reinterpret_cast<const __bf16*>(base + d2 * 16));
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
// A fragment (row lane % 32, k-step ks) of a chunk-major tile: 16 bytes
__device__ __forceinline__ u32x4_t frag_cm(const char* tile, int ks, int lane) {
  return *reinterpret_cast<const u32x4_t*>(tile + ((2 * ks + (lane >> 5)) * 32 + (lane & 31)) * 16);
}
// One 32-row tile of a bf16 copy into chunk-major LDS by LDS-DMA: DMA instruction i moves
// chunks 2i, 2i + 1 (lane l: LDS byte 1024 i + 16 l = chunk 2i + l / 32, slot l % 32); the
// workgroup's 4 waves take i = w, w + 4, ...; rows >= L read the zero row.  SWZ: slot l % 32
// holds row swz_row(l % 32, chunk) (i has the parity of w: one source row per lane).
template <int D32, bool SWZ = false>
__device__ __forceinline__ void dma_tile(char* tile, const __bf16* rows, int64_t rsb, int r0, int L,
                                         const __bf16* zrow, int w, int lane) {
  const int r = r0 + (SWZ ? swz_row(lane & 31, 2 * (w & 1) + (lane >> 5)) : (lane & 31));
  const __bf16* src = (r < L ? rows + (int64_t)r * rsb : zrow) + 8 * (lane >> 5);
#pragma unroll
  for (int i = 0; i < 2 * D32; i += 4)
    if (i + w < 2 * D32)
      __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (i + w)),
                                       (__attribute__((address_space(3))) void*)(tile + 1024 * (i + w)), 16, 0, 0);
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
  __bf16* pb;      // P blocks, same index: the key-major dK wave's A-fragment image of P
                   // (lane l: bytes 16 l and 1024 + 16 l), read back by the dV pass
  __bf16* qb;      // bf16 copies [row][head][32 D32] of Q, K, V, dO
  __bf16* kb;
  __bf16* vb;
  __bf16* ob;
  __bf16* zrow;    // 32 D32 zeros
  int64_t total_rows;  // B N (upper bound of offsets[B])
  int nbt;         // dS blocks per (sequence, head): NB (NB + 1) / 2, NB = ceil(N / 32)
  float inv_n;
  int n_kt;        // 128-key tiles
  int n_qt;        // 128-query tiles
  int64_t rsb_qkv; // bf16 elements between rows of qb / kb / vb (H 32 D32 for the copies,
                   // n_out for the bf16 uvqk of hstu_attn_bwd_a16); ob keeps H 32 D32
  int a16;         // 1: hq / hk / hv are bf16 h_pre and dq / dk / dvv bf16 d_uvqk (the
                   // pointers above reinterpreted), 0: fp32
};

// Epilogue store of 8 accumulator rows: d = acc * silu'(h) in the fp32 or the bf16 layout
template <int D32, typename V, typename RowF, typename ColF>
__device__ __forceinline__ void store_dh(const AttnBwdArgsW& a, const V& val, int L, int64_t s0,
                                         float* out, const float* hp, int h, RowF row_of,
                                         ColF col_of) {
  if (a.a16)
    store_scaled<8, D32>(val, L, a.d, s0, reinterpret_cast<__bf16*>(out), a.ld_d,
                         reinterpret_cast<const __bf16*>(hp), a.ld_h, h * a.d, row_of, col_of);
  else
    store_scaled<8, D32>(val, L, a.d, s0, out, a.ld_d, hp, a.ld_h, h * a.d, row_of, col_of);
}

constexpr int WK = 128;  // keys (queries) per workgroup: 4 waves x 32
constexpr int kDtsCopies = 4;  // dts histogram copies per wave (lane % copies)
constexpr int kSkew = 33;      // dpos skew image row stride (floats; odd: no bank conflicts)
__host__ __device__ constexpr int w_dts_stride(int nb1) { return ((nb1 + 30) / 32) * 32 + 1; }

// fp32 -> bf16 copies [row][head][32 D32] (blockIdx.y = tensor of the set), zero padding
// past d; one thread per 16-byte chunk; block (0, 0) also writes the zero row.
struct ConvSet {
  const float* src[4];
  int64_t ld[4];
  __bf16* dst[4];
  __bf16* zrow;
  const int64_t* offsets;
  int B, H, d, nch;
  int vec4;  // set by launch_convert
};
__global__ __launch_bounds__(256) void attn_bf16w_convert(ConvSet cs) {
  const int y = blockIdx.y;
  const float* src = y == 0 ? cs.src[0] : y == 1 ? cs.src[1] : y == 2 ? cs.src[2] : cs.src[3];
  const int64_t ld = y == 0 ? cs.ld[0] : y == 1 ? cs.ld[1] : y == 2 ? cs.ld[2] : cs.ld[3];
  __bf16* dst = y == 0 ? cs.dst[0] : y == 1 ? cs.dst[1] : y == 2 ? cs.dst[2] : cs.dst[3];
  if (cs.zrow && blockIdx.x == 0 && y == 0 && (int)threadIdx.x < cs.nch)
    *reinterpret_cast<u32x4_t*>(cs.zrow + 8 * threadIdx.x) = u32x4_t{0u, 0u, 0u, 0u};
  // 32-bit index math (the launcher checks rows * H * nch < 2^31): the 64-bit divisions
  // cost more issue slots than the 48 bytes a thread moves
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t nch = (uint32_t)cs.nch, H = (uint32_t)cs.H;
  const uint32_t rh = idx / nch, c = idx - rh * nch;
  const uint32_t row32 = rh / H, h = rh - row32 * H;
  const int64_t row = row32;
  if (row >= cs.offsets[cs.B]) return;
  const float* p = src + row * ld + h * cs.d + 8 * c;
  float x[8];
  if (cs.vec4) {  // d == 8 nch, 16-byte aligned rows: two float4 loads, no guards
    const f4 lo = *reinterpret_cast<const f4*>(p), hi = *reinterpret_cast<const f4*>(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = lo[j];
      x[j + 4] = hi[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float2 v = make_float2(0.f, 0.f);
      if (8 * (int)c + j < cs.d) v = *reinterpret_cast<const float2*>(p + j);  // d, ld even
      x[j] = v.x;
      x[j + 1] = v.y;
    }
  }
  *reinterpret_cast<u32x4_t*>(dst + (row * cs.H + h) * (8 * cs.nch) + 8 * c) =
      u32x4_t{pack_bf16(x[0], x[1]), pack_bf16(x[2], x[3]), pack_bf16(x[4], x[5]), pack_bf16(x[6], x[7])};
}
static int launch_convert(ConvSet cs, int n, int64_t total_rows, hipStream_t st) {
  if (n == 0) return 0;
  const int64_t threads = total_rows * cs.H * cs.nch;
  GR_REQUIRE(threads + 256 < 0x7fffffffLL, "hstu_attn_bf16 copies: %lld rows x heads too many",
             (long long)(total_rows * cs.H));
  cs.vec4 = cs.d == 8 * cs.nch;  // no padding chunk (d % 32 == 0)
  for (int i = 0; i < n; ++i)
    if ((uintptr_t)cs.src[i] % 16 != 0 || cs.ld[i] % 4 != 0) cs.vec4 = 0;
  GR_TIMED("attn_bf16_copies", st, hipLaunchKernelGGL(attn_bf16w_convert, dim3((unsigned)((threads + 255) / 256), n), dim3(256), 0, st, cs));
  GR_LAUNCH_CHECK("hstu_attn_bf16 copies");
  return 0;
}

// ------------------------------------------------------------------ forward
// out = P V, P = silu(S + bias) / N: 4 waves x 32 queries per workgroup.  Per 32-key
// chunk a wave computes S^T = K Q^T (A = K rows from the chunk-major LDS tile, B = its
// queries' Q^T fragments in registers), so the accumulator holds keys in registers and
// queries on lanes -- as an A operand that is P [query][key] -- and out += P V takes B
// from the V tile by transposed reads.  K / V tiles arrive by LDS-DMA one chunk ahead.
struct AttnFwdArgsW {
  const __bf16* qb;
  const __bf16* kb;
  const __bf16* vb;
  const __bf16* zrow;
  const int64_t* offsets;
  int B, N, H, d;
  const uint8_t* map_qk;  // query-major bucket map (null: no bias)
  const float* pos_w;
  const float* ts_w;
  int nb;
  float* out;
  int64_t ld_out;
  float inv_n;
  int n_qt;
  int64_t rsb_qkv;  // bf16 elements between rows of qb / kb / vb: H 32 D32 for the copies,
                    // n_out for the bf16 uvqk itself (hstu_attn_fwd_a16)
};

template <int D32, bool HB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void attn_fwd_bf16w_kernel(AttnFwdArgsW a) {
  constexpr int DP = 32 * D32, KS = 2 * D32, TB = 64 * DP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tiles = smem;  // [2 buffers][K, V][TB]
  float* tsw = reinterpret_cast<float*>(smem + 4 * TB);
  const int npos = 2 * a.N - 1;
  float* posw = tsw + (a.nb + 1);
  // XCD-aware order (x = i % 8 takes the sequence-heads x, x + 8, ...), query-tile-major:
  // every XCD dispatches its heaviest query tiles (the last: most keys) first
  const int x = blockIdx.x & 7, sl = blockIdx.x >> 3;
  const int nbh8 = (a.B * a.H + 7) >> 3;
  const int bh = (sl % nbh8) * 8 + x;
  if (bh >= a.B * a.H) return;
  const int qt = a.n_qt - 1 - sl / nbh8;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * WK;
  if (q0 >= L) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  if (HB) {
    for (int i = tid; i <= a.nb; i += 256) tsw[i] = a.ts_w[i];
    for (int i = tid; i < npos; i += 256) posw[i] = a.pos_w[i];
  }
  const int q0w = q0 + 32 * w;
  const int qi = q0w + lr;  // this lane's query (column of S^T)
  const bool q_ok = qi < L;
  const int64_t rsb = a.rsb_qkv;
  const int64_t hoff = s0 * rsb + (int64_t)h * DP;
  // Q^T fragments of the wave's queries: element j of k-step ks = dim 16 ks + 8 lh + j
  u32x4_t qf[KS];
  {
    const __bf16* qrow = q_ok ? a.qb + hoff + (int64_t)qi * rsb : a.zrow;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const u32x4_t*>(qrow + 16 * ks + 8 * lh);
  }
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_qk, b, attn_tiles_per_seq(a.N));
  const int map_w = (qi & 63) * 16;
  // bucket words of chunk kc: query qi, keys kc + 8m + 4lh .. +3 (query-major 64 x 64 tiles)
  auto map_words = [&](int kc, uint32_t (&mw)[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int kk = kc + 8 * m + 4 * lh;
      mw[m] = buf_ld_u32(rmap, (attn_tile_id(q0w >> 6, kk >> 6) * 1024 + map_w + ((kk & 63) >> 2)) * 4, 0);
    }
  };
  const int n_chunks = (min(q0 + WK, L) + 31) / 32;  // key chunks 0, 32, ... the tile needs
  const bool w_on = q0w < L;
  auto dma = [&](int buf, int r0) {
    dma_tile<D32>(tiles + buf * 2 * TB, a.kb + hoff, rsb, r0, L, a.zrow, w, lane);
    dma_tile<D32>(tiles + buf * 2 * TB + TB, a.vb + hoff, rsb, r0, L, a.zrow, w, lane);
  };
  uint32_t mw_next[4] = {0u, 0u, 0u, 0u};
  if (HB && w_on) map_words(0, mw_next);
  dma(0, 0);
  __syncthreads();
  for (int ci = 0; ci < n_chunks; ++ci) {
    const int kc0 = 32 * ci;
    const char* Ks = tiles + (ci & 1) * 2 * TB;
    const char* Vs = Ks + TB;
    const bool more = ci + 1 < n_chunks;
    if (more) dma((ci + 1) & 1, kc0 + 32);
    const bool act = w_on && kc0 <= q0w + 31;  // wave-uniform causal skip
    if (act) {
      uint32_t mw[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) mw[m] = mw_next[m];
      if (HB && more && kc0 + 32 <= q0w + 31) map_words(kc0 + 32, mw_next);
      // bias of element rr = key kc0 + (rr & 3) + 8 (rr >> 2) + 4 lh, query qi
      float bias_p[16], bias_t[16];
      if (HB) {
        const float* pw = posw + (a.N - 1 + kc0 + 4 * lh - qi);  // plus the key row
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int bk = (mw[rr >> 2] >> (8 * (rr & 3))) & 0xFF;
          bias_p[rr] = pw[(rr & 3) + 8 * (rr >> 2)];
          bias_t[rr] = tsw[bk];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // S^T: A = K rows (k-step ks), B = qf[ks]; two chains (even / odd k-steps)
      constexpr int PF = 4;
      u32x4_t ka[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) ka[i] = frag_cm(Ks, i, lane);
      f32x16 S0 = f16_zero(), S1 = f16_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4_t a0 = ka[ks % PF];
        if (ks + PF < KS) ka[ks % PF] = frag_cm(Ks, ks + PF, lane);
        if (ks & 1) S1 = mfma32(a0, qf[ks], S1);
        else S0 = mfma32(a0, qf[ks], S0);
      }
#pragma unroll
      for (int i = 0; i < PF; ++i) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (ks + PF < KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      S0 += S1;
      float x16[16];
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int kj = kc0 + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
        const bool ok = q_ok && kj <= qi;
        float xv = S0[rr];
        if (HB) {
          float bp = bias_p[rr], bt = bias_t[rr];
          asm volatile("" : "+v"(bp), "+v"(bt));  // keep the add here, after the products
          xv = xv + (bp + bt);
        }
        const float sg = sigmoidf_(xv);
        x16[rr] = __uint_as_float(__float_as_uint(xv * sg * a.inv_n) & (ok ? 0xffffffffu : 0u));
      }
      const u32x4_t f0 = acc_frag(x16, 0), f1 = acc_frag(x16, 1);
      __builtin_amdgcn_sched_barrier(0);
      // out += P V: B = V rows of the chunk (k = keys), transposed reads 4 ahead
      constexpr int NU = 2 * D32, PB = 4;
      u32x4_t bq[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) bq[u] = trB_acc_cm(Vs, u / D32, u % D32, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4_t b0 = bq[u % PB];
        if (u + PB < NU) bq[u % PB] = trB_acc_cm(Vs, (u + PB) / D32, (u + PB) % D32, lane);
        acc[u % D32] = mfma32(u < D32 ? f0 : f1, b0, acc[u % D32]);
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      }
    }
    if (more) __syncthreads();
  }
  if (!w_on) return;
  // acc[t][rr] = out[query q0w + (rr & 3) + 8 (rr >> 2) + 4 lh][32 t + lr]
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int qo = q0w + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
    if (qo >= L) continue;
    float* orow = a.out + (s0 + qo) * a.ld_out + h * a.d;
#pragma unroll
    for (int t = 0; t < D32; ++t) {
      const int c = 32 * t + lr;
      if (c < a.d) orow[c] = acc[t][rr];
    }
  }
}

// ------------------------------------------------------------------ key-major pass
// KIND_K = false: dV += P^T dO;  true: dK += dS^T Q, bias gradients, dS blocks.
template <int D32, bool HB, bool KIND_K, bool PST = false>
__device__ __forceinline__ void kv_body(const AttnBwdArgsW& a, char* smem, int kt, int bh) {
  constexpr int DP = 32 * D32;   // padded head dim
  constexpr int KS = DP / 16;    // k-steps of the S / dP products
  constexpr int TB = 64 * DP;    // bytes of one chunk-major 32-row tile
  constexpr bool BIAS = HB && KIND_K;
  char* tiles = smem;  // [2 buffers][Q, dO][TB]
  float* tsw = reinterpret_cast<float*>(tiles + 4 * TB);
  const int npos = 2 * a.N - 1;
  float* posw = tsw + (a.nb + 1);
  const int tss = w_dts_stride(a.nb + 1);
  float* hts = posw + npos;  // [4 waves][kDtsCopies][tss]
  // dpos skew image per wave: element (query row R, key lane lr) at row e = 31 - lr + R,
  // column R ([64 rows][kSkew]); cells no element maps to stay 0
  float* skw = hts + 4 * kDtsCopies * tss + wave_id() * 64 * kSkew;

  const int BH = a.B * a.H;
  const int rank = kt * BH + bh;  // slab index
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * WK;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int nbins = npos + a.nb + 1;
  float* slab = BIAS ? a.slabs + ((int64_t)rank * 4 + w) * nbins : nullptr;
#ifdef GR_STAMP
  unsigned long long st_[12] = {0, 0, 0, 0, 0, 0, 0, 0, KIND_K ? 1ull : 0ull, 0, 0, 0};
  const unsigned long long st_start = __builtin_amdgcn_s_memtime();
  unsigned long long st_t0 = st_start;
#endif
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
    for (int i = tid; i < 4 * kDtsCopies * tss + 4 * 64 * kSkew; i += 256) hts[i] = 0.f;
  const int k0w = k0 + 32 * w;   // this wave's first key
  const int kj = k0w + lr;       // this lane's key (column of S / dP)
  const bool k_ok = kj < L;
  // bf16 Q / K / V of this (sequence, head): row r at rows + r * rsb; dO copy: rsb_o
  const int64_t rsb = a.rsb_qkv;
  const int64_t hoff = s0 * rsb + (int64_t)h * DP;
  const int64_t rsb_o = (int64_t)a.H * DP;
  const int64_t hoff_o = s0 * rsb_o + (int64_t)h * DP;
  // K^T / V^T fragments of the wave's keys: element j of k-step ks = dim 16 ks + 8 lh + j
  u32x4_t kf[KS], vf[KS];
  {
    const __bf16* krow = k_ok ? a.kb + hoff + (int64_t)kj * rsb : a.zrow;
    const __bf16* vrow = k_ok ? a.vb + hoff + (int64_t)kj * rsb : a.zrow;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = *reinterpret_cast<const u32x4_t*>(krow + 16 * ks + 8 * lh);
    if (KIND_K) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) vf[ks] = *reinterpret_cast<const u32x4_t*>(vrow + 16 * ks + 8 * lh);
    }
  }
  // output accumulators: tile t = columns 32 t .. 32 t + 31, rows = the wave's keys
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();

  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_kq, b, attn_tiles_per_seq(a.N));
  // dts: running (bucket, sum) of this lane, flushed into per-wave LDS histogram copies
  // when the bucket changes
  float* wts = hts + (w * kDtsCopies + (lr % kDtsCopies)) * tss;
  int run_b = -1;
  float run_s = 0.f;
  // dpos: each bin of the wave's slab is written once: main diagonals of a chunk plus the
  // wrapped diagonals of the previous chunk (carry), see the file header
  float carry = 0.f;
  int pend_bin = -1;  // dpos bin held back one chunk
  float pend_v = 0.f;

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
  // the chunk's Q and dO rows by LDS-DMA, one chunk ahead (drained by the chunk's barrier)
  auto dma = [&](int buf, int r0) {
    dma_tile<D32>(tiles + buf * 2 * TB, a.qb + hoff, rsb, r0, L, a.zrow, w, lane);
    dma_tile<D32>(tiles + buf * 2 * TB + TB, a.ob + hoff_o, rsb_o, r0, L, a.zrow, w, lane);
  };
  dma(0, k0);
  __syncthreads();
  BW_ST(0, kf[0].x);
  for (int ci = 0; ci < n_chunks; ++ci) {
    const int qc0 = k0 + 32 * ci;
    const char* Qs = tiles + (ci & 1) * 2 * TB;
    const char* Ds = Qs + TB;
    const bool more = ci + 1 < n_chunks;
    if (more) dma((ci + 1) & 1, qc0 + 32);
    const bool act = w_on && qc0 >= k0w;  // wave-uniform: the chunk reaches the wave's keys
    if (act) {
      uint32_t mw[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) mw[m] = mw_next[m];
      if (HB && more) map_words(qc0 + 32, mw_next);
      // relative bias of the chunk's elements, looked up before the products so the LDS
      // latency hides under them: element rr = query qc0 + (rr & 3) + 8 (rr >> 2) + 4 lh
      float bias_p[16], bias_t[16];
      if (HB) {
        const float* pw = posw + (a.N - 1 + kj - qc0 - 4 * lh);  // minus the row (rr & 3) + 8 (rr >> 2)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int bk = (mw[rr >> 2] >> (8 * (rr & 3))) & 0xFF;
          bias_p[rr] = pw[-((rr & 3) + 8 * (rr >> 2))];
          bias_t[rr] = tsw[bk];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      BW_ST(9, HB ? bias_t[15] + bias_p[15] : 0.f);
      // S (and dP) with the A fragments read PF k-steps ahead; two independent chains per
      // kind (S, dP or the even / odd k-steps of S)
      constexpr int PF = 4;
      u32x4_t qa[PF], da[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        qa[i] = frag_cm(Qs, i, lane);
        if (KIND_K) da[i] = frag_cm(Ds, i, lane);
      }
      f32x16 S = f16_zero(), dP = f16_zero();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u32x4_t a0 = qa[ks % PF];
        u32x4_t a1 = da[ks % PF];
        if (ks + PF < KS) {
          qa[ks % PF] = frag_cm(Qs, ks + PF, lane);
          if (KIND_K) da[ks % PF] = frag_cm(Ds, ks + PF, lane);
        }
        if (KIND_K) {
          S = mfma32(a0, kf[ks], S);
          dP = mfma32(a1, vf[ks], dP);
        } else if (ks & 1) {
          dP = mfma32(a0, kf[ks], dP);
        } else {
          S = mfma32(a0, kf[ks], S);
        }
      }
      // schedule: the PF reads first, then one MFMA (S, dP) per read group, so PF groups
      // of A-fragment reads stay in flight under the products
      constexpr int GR = KIND_K ? 2 : 1;
#pragma unroll
      for (int i = 0; i < PF; ++i) __builtin_amdgcn_sched_group_barrier(0x100, GR, 0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        __builtin_amdgcn_sched_group_barrier(0x008, GR, 0);
        if (ks + PF < KS) __builtin_amdgcn_sched_group_barrier(0x100, GR, 0);
      }
      BW_ST(1, S[0]);
      BW_ST(1, dP[0]);
      if (!KIND_K) S += dP;
      float x16[16];
      // interior chunks (every query after every key of the wave, all rows in range) need
      // no causal / length mask: a mask-free instance of the elementwise pass
      const bool full = qc0 >= k0w + 32 && qc0 + 32 <= L && k0w + 32 <= L;
      float p16[PST ? 16 : 1];
      auto elementwise = [&](auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          float x = S[rr];
          if (HB) {
            float bp = bias_p[rr], bt = bias_t[rr];
            asm volatile("" : "+v"(bp), "+v"(bt));  // keep the add here, after the products
            x = x + (bp + bt);
          }
          const float sg = sigmoidf_(x);
          const float v = KIND_K ? dP[rr] * (sg * (1.0f + x * (1.0f - sg))) * a.inv_n
                                 : x * sg * a.inv_n;
          if constexpr (FULL) {
            x16[rr] = v;
            if constexpr (PST) p16[rr] = x * sg * a.inv_n;
          } else {
            const int qi = qc0 + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
            const bool ok = k_ok && qi < L && kj <= qi;
            const uint32_t msk = ok ? 0xffffffffu : 0u;
            x16[rr] = __uint_as_float(__float_as_uint(v) & msk);
            if constexpr (PST) p16[rr] = __uint_as_float(__float_as_uint(x * sg * a.inv_n) & msk);
          }
        }
      };
      if (full) elementwise(std::true_type{});
      else elementwise(std::false_type{});
      const u32x4_t f0 = acc_frag(x16, 0), f1 = acc_frag(x16, 1);
      BW_ST(2, f1.x);
      __builtin_amdgcn_sched_barrier(0);
      // acc += X^T B, B = dO (dV) or Q (dK) rows of the chunk, transposed reads
      const char* Bt = KIND_K ? Qs : Ds;
      // 2 D32 products (k-step s = u / D32, tile t = u % D32), B fragments read PB ahead
      constexpr int NU = 2 * D32, PB = 4;
      u32x4_t bq[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) bq[u] = trB_acc_cm(Bt, u / D32, u % D32, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4_t b0 = bq[u % PB];
        if (u + PB < NU) bq[u % PB] = trB_acc_cm(Bt, (u + PB) / D32, (u + PB) % D32, lane);
        const int t = u % D32;
        acc[t] = mfma32(u < D32 ? f0 : f1, b0, acc[t]);
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      }
      BW_ST(3, acc[D32 - 1][0]);
      if (KIND_K) {
        // dS block for the query-major pass: [key][query] image, registers 4g .. 4g+3 =
        // queries 8g + 4lh + 0..3 (8-byte stores of the A fragments' packed pairs)
        const int qb = qc0 >> 5, kb = k0w >> 5;
        __bf16* blk = a.ds + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2 + kb) * 1024;
        const u32x4_t fr[2] = {f0, f1};
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<u32x2_t*>(blk + lr * 32 + 8 * g + 4 * lh) =
              u32x2_t{fr[g >> 1][2 * (g & 1)], fr[g >> 1][2 * (g & 1) + 1]};
        if constexpr (PST) {
          // P of the same block as the dV pass's A fragments, 1 KB per store
          char* pblk = reinterpret_cast<char*>(a.pb + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2 + kb) * 1024);
          *reinterpret_cast<u32x4_t*>(pblk + 16 * lane) = acc_frag(p16, 0);
          *reinterpret_cast<u32x4_t*>(pblk + 1024 + 16 * lane) = acc_frag(p16, 1);
        }
      }
      if (BIAS) {
        // dts run (a lane's queries ascend with rr), after the math so that the branches
        // do not split its schedule; the accumulator MFMAs above run meanwhile.  A chunk
        // whose 16 buckets equal every lane's open run (the common case: the lanes' time
        // gaps share their log bucket across 32 queries) only extends the runs, in the
        // same order as the general loop.
        const uint32_t rb4 = (uint32_t)run_b * 0x01010101u;
        const bool same = full && run_b >= 0 && mw[0] == rb4 && mw[1] == rb4 && mw[2] == rb4 &&
                          mw[3] == rb4;
        if (__builtin_amdgcn_ballot_w64(!same) == 0) {
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) run_s += x16[rr];
        } else {
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) {
            const int qi = qc0 + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
            const bool ok = full || (k_ok && qi < L && kj <= qi);
            const int bk = (mw[rr >> 2] >> (8 * (rr & 3))) & 0xFF;
            if (ok && bk != run_b) {
              if (run_b >= 0) atomicAdd(&wts[run_b], run_s);
              run_b = bk;
              run_s = 0.f;
            }
            run_s += x16[rr];  // 0 where !ok
          }
        }
      }
      BW_ST(4, run_s);
      if (BIAS) {
        // dpos: element rr (row R = (rr & 3) + 8 (rr >> 2) + 4 lh, key lane lr) lies on the
        // diagonal c = lr - R of the chunk.  Written to the wave's skew image at row
        // e = 31 - c, column R (immediate offsets per rr), lane e then sums its row: lane
        // 31 - c holds diagonal c >= 0 (main), lane 63 - c diagonal c - 32 (wrapped, the
        // same bins as the next chunk's main diagonals: carried).  The wave's LDS
        // operations complete in order, so the reads see the writes.
        float* wr = skw + (31 - lr) * kSkew + (kSkew + 1) * 4 * lh;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) wr[(kSkew + 1) * ((rr & 3) + 8 * (rr >> 2))] = x16[rr];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float* rd = skw + lane * kSkew;
        float rv[32];
#pragma unroll
        for (int R = 0; R < 32; ++R) rv[R] = rd[R];
        float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int R = 0; R < 32; ++R) ps[R & 3] += rv[R];
        const float dsum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
        auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dsum), __float_as_uint(dsum), false, false);
        // lanes < 32: sw[0] = own (main, c = 31 - lane), sw[1] = lane + 32 (wrapped)
        // the bin is stored at the next chunk (or the epilogue): a store issued here would
        // hold the chunk's barrier until it completes
        if (pend_bin >= 0) slab[pend_bin] = pend_v;
        const int bin = a.N - 1 + (k0w - qc0) + (31 - lane);
        pend_bin = lh == 0 && bin >= 0 && bin < npos ? bin : -1;
        pend_v = __uint_as_float(sw[0]) + carry;
        carry = __uint_as_float(sw[1]);
      }
      BW_ST(6, carry);
    }
    if (more) __syncthreads();
    BW_ST(5, lane);
  }
  // ---- epilogue: acc[t][rr] = (dV or dK)[key k0w + (rr & 3) + 8 (rr >> 2) + 4 lh][32 t + lr]
  float* outp = KIND_K ? a.dk : a.dvv;
  const float* hp = KIND_K ? a.hk : a.hv;
#pragma unroll
  for (int g = 0; g < 16; g += 8)  // 8 rows (8 D32 silu'(h) loads) in flight at a time
    store_dh<D32>(a, [&](int i, int t) { return acc[t][g + i]; }, L, s0, outp, hp, h,
                         [&](int i) { return k0w + ((g + i) & 3) + 8 * ((g + i) >> 2) + 4 * lh; },
                         [&](int t) { return 32 * t + lr; });
  if (BIAS) {
    // the last chunk's wrapped diagonals; zero every bin this wave never wrote: written
    // bins N-1 + d0 + [-32, 31] over d0 = k0w - qc0, qc0 = k0w .. last chunk
    if (pend_bin >= 0) slab[pend_bin] = pend_v;
    int lo = npos, hi = -1;
    if (w_on) {
      const int d0_last = k0w - (k0 + 32 * (n_chunks - 1));
      const int bin = a.N - 1 + d0_last - 32 + (31 - lr);
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
#ifdef GR_STAMP
  st_[7] = __builtin_amdgcn_s_memtime() - st_start;
  if (lane < 12 && blockIdx.x * 48 + 48 <= (1 << 16)) {
    unsigned long long v = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) v = lane == i ? st_[i] : v;
    gr_stamp_bw_buf[(blockIdx.x * 4 + w) * 12 + lane] = v;
  }
#endif
}

// LDS-DMA issued from inline asm (global_load_lds_dwordx4: lane l's 16 bytes land at LDS
// byte lds_off + 16 l).  The builtin makes hipcc wait vmcnt(0) before every later LDS read
// that might alias the destination, which drains a deeper prefetch ring on each chunk;
// hipcc does not see these, so the caller waits (vmcnt) and synchronises itself.  m0 is
// saved and restored around the instruction.
__device__ __forceinline__ void dma16_asm(const void* gaddr, uint32_t lds_off) {
  uint32_t tmp;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
               : "=&s"(tmp)
               : "s"(lds_off), "v"(gaddr)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p);
}

// ------------------------------------------------------------------ dV from the stored P
// dV[key][:] = sum over query chunks of P^T dO: the key-major dK pass stored each 32 x 32
// P block as its wave's A-fragment image, so a wave here loads its two fragments (2 x 16
// B per lane) and streams the dO tiles through LDS: no S product, no bias lookups, no
// sigmoid (it ran once, in the dK pass).  Same block order and MFMA order as the dV
// workgroups of the one-launch form; P comes from the dK wave's S chain (that form summed
// S in two interleaved chains), so dV differs from it at fp32 rounding.
template <int D32>
__device__ __forceinline__ void v_from_p_body(const AttnBwdArgsW& a, char* smem, int kt, int bh) {
  constexpr int DP = 32 * D32;
  constexpr int TB = 64 * DP;
  char* tiles = smem;  // [2 buffers][dO][TB]
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * WK;
  if (k0 >= L) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int k0w = k0 + 32 * w;
  const bool w_on = k0w < L;
  const int64_t rsb = (int64_t)a.H * DP;
  const int64_t hoff = s0 * rsb + (int64_t)h * DP;
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();
  const int n_chunks = (L - k0 + 31) / 32;
  const int kb = k0w >> 5;
  auto pfrag = [&](int qc, u32x4_t& f0, u32x4_t& f1) {
    const int qb = qc >> 5;
    const char* pblk = reinterpret_cast<const char*>(a.pb + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2 + kb) * 1024);
    f0 = *reinterpret_cast<const u32x4_t*>(pblk + 16 * lane);
    f1 = *reinterpret_cast<const u32x4_t*>(pblk + 1024 + 16 * lane);
  };
  u32x4_t n0 = {0u, 0u, 0u, 0u}, n1 = n0;  // the wave's next P block, one chunk ahead
  if (w_on) pfrag(k0w, n0, n1);
  dma_tile<D32>(tiles, a.ob + hoff, rsb, k0, L, a.zrow, w, lane);
  __syncthreads();
  for (int ci = 0; ci < n_chunks; ++ci) {
    const int qc0 = k0 + 32 * ci;
    const char* Ds = tiles + (ci & 1) * TB;
    const bool more = ci + 1 < n_chunks;
    if (more) dma_tile<D32>(tiles + ((ci + 1) & 1) * TB, a.ob + hoff, rsb, qc0 + 32, L, a.zrow, w, lane);
    if (w_on && qc0 >= k0w) {
      const u32x4_t f0 = n0, f1 = n1;
      if (more) pfrag(qc0 + 32, n0, n1);
      constexpr int NU = 2 * D32, PB = 4;
      u32x4_t bq[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) bq[u] = trB_acc_cm(Ds, u / D32, u % D32, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4_t b0 = bq[u % PB];
        if (u + PB < NU) bq[u % PB] = trB_acc_cm(Ds, (u + PB) / D32, (u + PB) % D32, lane);
        acc[u % D32] = mfma32(u < D32 ? f0 : f1, b0, acc[u % D32]);
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      }
    }
    if (more) __syncthreads();
  }
  if (!w_on) return;
#pragma unroll
  for (int g = 0; g < 16; g += 8)
    store_dh<D32>(a, [&](int i, int t) { return acc[t][g + i]; }, L, s0, a.dvv, a.hv, h,
                         [&](int i) { return k0w + ((g + i) & 3) + 8 * ((g + i) >> 2) + 4 * lh; },
                         [&](int t) { return 32 * t + lr; });
}

// dV from P with a 3-deep ring (even D32: every wave issues D32 / 2 dO pieces + 2 P pieces
// per chunk, so one vmcnt count fits all waves).  Chunk ci: wait for chunk ci's DMA
// (vmcnt: chunk ci + 1's 6 or so pieces may stay in flight), barrier (every wave is past
// chunk ci - 1, whose slot the next DMA overwrites), issue chunk ci + 2, compute chunk ci.
// The dO tile and the wave's 2 KB P block both arrive by LDS-DMA, so P costs no
// register-load wait either.
template <int D32>
__device__ __forceinline__ void v_from_p_ring_body(const AttnBwdArgsW& a, char* smem, int kt, int bh) {
  static_assert(D32 % 2 == 0, "uniform DMA pieces per wave");
  constexpr int DP = 32 * D32;
  constexpr int TB = 64 * DP;
  constexpr int NR = 3;             // ring depth
  constexpr int OPS = D32 / 2 + 2;  // asm DMA instructions per wave per chunk
  char* dslot = smem;               // [NR][TB] dO tiles
  char* pslot = smem + NR * TB;     // [NR][4 waves][2 KB] P blocks
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * WK;
  if (k0 >= L) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 31, lh = lane >> 5;
  const int k0w = k0 + 32 * w;
  const bool w_on = k0w < L;
  const int64_t rsb = (int64_t)a.H * DP;
  const int64_t hoff = s0 * rsb + (int64_t)h * DP;
  f32x16 acc[D32];
#pragma unroll
  for (int t = 0; t < D32; ++t) acc[t] = f16_zero();
  const int n_chunks = (L - k0 + 31) / 32;
  const int kb = k0w >> 5;
  auto issue = [&](int c) {  // chunk c's dO tile pieces and this wave's P block
    const int slot = c % NR;
    const int r = k0 + 32 * c + lr;
    const __bf16* src = (r < L ? a.ob + hoff + (int64_t)r * rsb : a.zrow) + 8 * lh;
    const uint32_t dbase = lds_u32(dslot + slot * TB);
#pragma unroll
    for (int i = 0; i < 2 * D32; i += 4) dma16_asm(src + 16 * (i + w), dbase + 1024 * (i + w));
    // the wave's P block (a clamped valid block where the chunk precedes the wave's keys)
    int qb = (k0 + 32 * c) >> 5;
    qb = qb < kb ? kb : qb;
    const int64_t blk = w_on ? (int64_t)qb * (qb + 1) / 2 + kb : 0;  // a wave past L: block 0
    const char* pblk = reinterpret_cast<const char*>(a.pb + ((int64_t)bh * a.nbt + blk) * 1024);
    const uint32_t pbase = lds_u32(pslot + (slot * 4 + w) * 2048);
    dma16_asm(pblk + 16 * lane, pbase);
    dma16_asm(pblk + 1024 + 16 * lane, pbase + 1024);
  };
  issue(0);
  if (n_chunks > 1) issue(1);
  for (int ci = 0; ci < n_chunks; ++ci) {
    const int qc0 = k0 + 32 * ci;
    if (ci + 1 < n_chunks) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ci + 2 < n_chunks) issue(ci + 2);
    const int slot = ci % NR;
    const char* Ds = dslot + slot * TB;
    if (w_on && qc0 >= k0w) {
      const char* pp = pslot + (slot * 4 + w) * 2048;
      const u32x4_t f0 = *reinterpret_cast<const u32x4_t*>(pp + 16 * lane);
      const u32x4_t f1 = *reinterpret_cast<const u32x4_t*>(pp + 1024 + 16 * lane);
      constexpr int NU = 2 * D32, PB = 4;
      u32x4_t bq[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) bq[u] = trB_acc_cm(Ds, u / D32, u % D32, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4_t b0 = bq[u % PB];
        if (u + PB < NU) bq[u % PB] = trB_acc_cm(Ds, (u + PB) / D32, (u + PB) % D32, lane);
        acc[u % D32] = mfma32(u < D32 ? f0 : f1, b0, acc[u % D32]);
      }
#pragma unroll
      for (int u = 0; u < PB + 2; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this chunk's LDS reads done
  }
  if (!w_on) return;
#pragma unroll
  for (int g = 0; g < 16; g += 8)
    store_dh<D32>(a, [&](int i, int t) { return acc[t][g + i]; }, L, s0, a.dvv, a.hv, h,
                         [&](int i) { return k0w + ((g + i) & 3) + 8 * ((g + i) >> 2) + 4 * lh; },
                         [&](int t) { return 32 * t + lr; });
}

// Workgroup i -> (bh, key tile kt), key-tile-major within an XCD (x = i % 8 takes the
// sequence-heads x, x + 8, ...): every XCD dispatches its kt = 0 workgroups first, then
// kt = 1, ..., so the heaviest causal tiles start first and a CU freed early takes the
// next-heaviest (with the sequence-head-major order one CU could draw two heavy tiles)
__device__ __forceinline__ void xcd_slot_kt(const AttnBwdArgsW& a, int& bh, int& kt,
                                            int id = (int)blockIdx.x) {
  const int x = id & 7, sl = id >> 3;
  const int nbh8 = (a.B * a.H + 7) >> 3;
  kt = sl / nbh8;
  bh = (sl % nbh8) * 8 + x;
}

// Two-launch form: dK (+ dS, bias gradients and the P blocks), then dV from P.
template <int D32, bool HB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void attn_bwd_bf16w_k_kernel(AttnBwdArgsW a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int bh, kt;
  xcd_slot_kt(a, bh, kt);
  if (bh >= a.B * a.H) return;
  kv_body<D32, HB, true, true>(a, smem, kt, bh);
}
// The bias-gradient slabs (written by the dK launch) reduced by the first workgroups of
// the dV launch: workgroup r owns bins 16 r .. 16 r + 15; thread (bin, group g) sums
// slabs g, g + 16, ... in order (16 loads in flight), then the 16 groups are added in
// order: a fixed order, no float atomics.
struct BiasRed {
  int n_slabs, npos, nts, nbias;
  float* dpos_w;
  float* dts_w;
};
__device__ __forceinline__ void bias_reduce_wg(const float* slabs, const BiasRed& r, int wg, char* smem) {
  float* part = reinterpret_cast<float*>(smem);  // [16 groups][16 bins]
  const int nbins = r.npos + r.nts;
  const int tid = threadIdx.x, bi = tid & 15, g = tid >> 4;
  const int bin = 16 * wg + bi;
  float acc = 0.f;
  if (bin < nbins) {
    int j = g;
    for (; j + 15 * 16 < r.n_slabs; j += 16 * 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = slabs[(int64_t)(j + 16 * u) * nbins + bin];
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
    for (; j < r.n_slabs; j += 16) acc += slabs[(int64_t)j * nbins + bin];
  }
  part[g * 16 + bi] = acc;
  __syncthreads();
  if (tid < 16 && bin < nbins) {
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += part[u * 16 + bi];
    if (bin < r.npos) r.dpos_w[bin] = s;
    else r.dts_w[bin - r.npos] = s;
  }
}

template <int D32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void attn_bwd_bf16w_vp_kernel(AttnBwdArgsW a, BiasRed r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < r.nbias) {
    bias_reduce_wg(a.slabs, r, blockIdx.x, smem);
    return;
  }
  // r.nbias is a multiple of 8: blockIdx.x - nbias keeps the workgroup's XCD
  int bh, kt;
  xcd_slot_kt(a, bh, kt, (int)blockIdx.x - r.nbias);
  if (bh >= a.B * a.H) return;
  if constexpr (D32 % 2 == 0) v_from_p_ring_body<D32>(a, smem, kt, bh);
  else v_from_p_body<D32>(a, smem, kt, bh);
}

// ------------------------------------------------------------------ query-major pass
// dQ[q][:] = sum over key blocks of dS block (A: transposed reads of the [key][query] image,
// natural k order) times the K tile (B: transposed reads of the chunk-major tile).  K tiles
// and the waves' dS blocks arrive by LDS-DMA one block ahead.
template <int D32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void attn_bwd_bf16w_dq_kernel(AttnBwdArgsW a) {
  constexpr int DP = 32 * D32;
  constexpr int TB = 64 * DP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* kt_l = smem;             // [2][TB]
  char* dsl = smem + 2 * TB;     // [4 waves][2][2048 B]
  int bh, j;
  xcd_slot_kt(a, bh, j);  // tile-major: the heaviest query tiles (the last) first
  if (bh >= a.B * a.H) return;
  const int qt = a.n_qt - 1 - j;
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
  const int64_t rsb = a.rsb_qkv;
  const __bf16* krows = a.kb + s0 * rsb + (int64_t)h * DP;
  const int n_kb = (min(q0 + WK, L) + 31) / 32;  // key blocks the workgroup needs
  char* mydl = dsl + w * 2 * 2048;
  const bool w_on = q0w < L;
  const __bf16* dsrow = a.ds + ((int64_t)bh * a.nbt + qb * (qb + 1) / 2) * 1024;
  auto dma = [&](int kb, int buf) {
    dma_tile<D32, true>(kt_l + buf * TB, krows, rsb, 32 * kb, L, a.zrow, w, lane);
    // the wave's 2 KB dS block (qb, kb): two 1 KB pieces, lane-linear
    const bool ok = w_on && kb <= qb;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const __bf16* src = ok ? dsrow + kb * 1024 + 512 * i + 8 * lane : a.zrow;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(mydl + buf * 2048 + 1024 * i), 16, 0, 0);
    }
  };
  if constexpr (D32 % 2 == 0) {
    // 3-deep ring by inline-asm LDS-DMA (see v_from_p_ring_body): chunk kb waits for its
    // own pieces only, the next key block's stay in flight
    constexpr int NR = 3, OPS = D32 / 2 + 2;
    char* kring = smem;                // [NR][TB] K tiles (swizzled)
    char* dring = smem + NR * TB;      // [NR][4 waves][2 KB] dS blocks
    const int kr_row = swz_row(lr, 2 * (w & 1) + (lane >> 5));
    auto issue = [&](int kb) {
      const int slot = kb % NR;
      const int r = 32 * kb + kr_row;
      const __bf16* src = (r < L ? krows + (int64_t)r * rsb : a.zrow) + 8 * (lane >> 5);
      const uint32_t kbase = lds_u32(kring + slot * TB);
#pragma unroll
      for (int i = 0; i < 2 * D32; i += 4) dma16_asm(src + 16 * (i + w), kbase + 1024 * (i + w));
      const bool ok = w_on && kb <= qb;
      const uint32_t dbase = lds_u32(dring + (slot * 4 + w) * 2048);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dma16_asm(ok ? dsrow + kb * 1024 + 512 * i + 8 * lane : a.zrow, dbase + 1024 * i);
    };
    issue(0);
    if (n_kb > 1) issue(1);
    for (int kb = 0; kb < n_kb; ++kb) {
      if (kb + 1 < n_kb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kb + 2 < n_kb) issue(kb + 2);
      const int slot = kb % NR;
      const char* Kl = kring + slot * TB;
      const __bf16* Dl = reinterpret_cast<const __bf16*>(dring + (slot * 4 + w) * 2048);
      if (w_on && kb <= qb) {
        const u32x4_t a0 = trB_nat(Dl, 32, 0, 0, lane), a1 = trB_nat(Dl, 32, 1, 0, lane);
        constexpr int NU = 2 * D32, PB = 4;
        u32x4_t bq[PB];
#pragma unroll
        for (int u = 0; u < PB; ++u) bq[u] = trB_nat_cm_swz(Kl, u / D32, u % D32, lane);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const u32x4_t b0 = bq[u % PB];
          if (u + PB < NU) bq[u % PB] = trB_nat_cm_swz(Kl, (u + PB) / D32, (u + PB) % D32, lane);
          acc[u % D32] = mfma32(u < D32 ? a0 : a1, b0, acc[u % D32]);
        }
#pragma unroll
        for (int u = 0; u < PB + 2; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this block's LDS reads done
    }
  } else {
  dma(0, 0);
  __syncthreads();
  for (int kb = 0; kb < n_kb; ++kb) {
    const char* Kl = kt_l + (kb & 1) * TB;
    const __bf16* Dl = reinterpret_cast<const __bf16*>(mydl + (kb & 1) * 2048);
    const bool more = kb + 1 < n_kb;
    if (more) dma(kb + 1, (kb + 1) & 1);
    if (w_on && kb <= qb) {  // wave-uniform causal skip
      // A: dS[q = lane % 32][keys 16 s + 8 lh + 0..7] from the [key][query] image
      const u32x4_t a0 = trB_nat(Dl, 32, 0, 0, lane), a1 = trB_nat(Dl, 32, 1, 0, lane);
      constexpr int NU = 2 * D32, PB = 4;
      u32x4_t bq[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) bq[u] = trB_nat_cm_swz(Kl, u / D32, u % D32, lane);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4_t b0 = bq[u % PB];
        if (u + PB < NU) bq[u % PB] = trB_nat_cm_swz(Kl, (u + PB) / D32, (u + PB) % D32, lane);
        acc[u % D32] = mfma32(u < D32 ? a0 : a1, b0, acc[u % D32]);
      }
#pragma unroll
      for (int u = 0; u < PB + 2; ++u) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (u + PB < NU) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
    }
    if (more) __syncthreads();
  }
  }
  if (!w_on) return;
  const int lh = lane >> 5;
#pragma unroll
  for (int g = 0; g < 16; g += 8)
    store_dh<D32>(a, [&](int i, int t) { return acc[t][g + i]; }, L, s0, a.dq, a.hq, h,
                         [&](int i) { return q0w + ((g + i) & 3) + 8 * ((g + i) >> 2) + 4 * lh; },
                         [&](int t) { return 32 * t + lr; });
}

// slabs: [n][2N-1 + nb+1]; fixed-order reduce in two coalesced stages: stage 1 sums slabs
// 64 g .. 64 g + 63 of each bin in order into slab 64 g (each thread reads its own bins
// before overwriting them); stage 2 adds the groups in g order
static size_t bf16w_slab_bytes(int B, int N, int max_len, int H, int nb) {
  return sizeof(float) * 4 * (size_t)ceil_div(max_len, WK) * B * H * (size_t)(2 * N - 1 + nb + 1);
}
static size_t bf16w_ds_bytes(int B, int N, int H) {
  const size_t nb32 = (size_t)ceil_div(N, 32);
  return 2048 * (nb32 * (nb32 + 1) / 2) * (size_t)B * H;
}
static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }
// one bf16 copy [B N rows][H][DPA], DPA = d rounded up to 32
static size_t bf16w_copy_bytes(int B, int N, int H, int d) {
  return al256((size_t)B * N * H * ceil_div(d, 32) * 32 * 2);
}

// Q, K, V copies: [Q][K][V][zero row], each copy al256(B N H DPA 2) bytes
static size_t bf16w_copies_bytes(int B, int N, int H, int d) {
  return 3 * bf16w_copy_bytes(B, N, H, d) + al256(ceil_div(d, 32) * 64);
}
struct CopyPtrs {
  __bf16 *q, *k, *v, *zrow;
};
static CopyPtrs copy_ptrs(const void* copies, int B, int N, int H, int d) {
  const size_t cp_b = bf16w_copy_bytes(B, N, H, d);
  char* c = (char*)copies;
  return {(__bf16*)c, (__bf16*)(c + cp_b), (__bf16*)(c + 2 * cp_b), (__bf16*)(c + 3 * cp_b)};
}

template <int D32>
static int launch_fwd_bf16w(AttnFwdArgsW a, hipStream_t st, int max_len) {
  constexpr int TB = 64 * 32 * D32;
  const size_t lds = 4 * TB + sizeof(float) * ((a.nb + 1) + (2 * a.N - 1));
  GR_REQUIRE(lds <= 160 * 1024, "hstu_attn_fwd_bf16: LDS %zu B exceeds 160 KiB (N=%d)", lds, a.N);
  a.n_qt = ceil_div(max_len, WK);
  const int bh8 = ceil_div(a.B * a.H, 8) * 8;
  auto k = a.map_qk ? attn_fwd_bf16w_kernel<D32, true> : attn_fwd_bf16w_kernel<D32, false>;
  GR_TIMED("attn_fwd", st, hipLaunchKernelGGL(k, dim3(a.n_qt * bh8), dim3(256), lds, st, a));
  GR_LAUNCH_CHECK("hstu_attn_fwd_bf16(wide)");
  return 0;
}

template <int D32>
static int launch_bwd_bf16w(AttnBwdArgsW a, float* dpos_w, float* dts_w, hipStream_t st) {
  constexpr int DP = 32 * D32, TB = 64 * DP;
  const size_t npos = 2 * a.N - 1;
  const int tss = w_dts_stride(a.nb + 1);
  const size_t lds_kv = 4 * TB + sizeof(float) * ((a.nb + 1) + npos + 4 * kDtsCopies * tss + 4 * 64 * kSkew);
  const size_t lds_q = D32 % 2 == 0 ? 3 * TB + 3 * 4 * 2048 : 2 * TB + 4 * 2 * 2048;  // ring / two buffers
  GR_REQUIRE(lds_kv <= 160 * 1024, "hstu_attn_bwd_bf16: LDS %zu B exceeds 160 KiB (N=%d)", lds_kv, a.N);
  const int grid = a.n_kt * a.B * a.H;
  const int bh8 = ceil_div(a.B * a.H, 8) * 8;  // XCD-aware order: see xcd_slot_kt
  // dK (+ dS, the bias gradients and the P blocks), then dV from P: S and the sigmoid are
  // computed once per element (a dV workgroup beside each dK workgroup recomputed them)
  auto kk = a.map_kq ? attn_bwd_bf16w_k_kernel<D32, true> : attn_bwd_bf16w_k_kernel<D32, false>;
  GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kk, dim3(a.n_kt * bh8), dim3(256), lds_kv, st, a));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide dk)");
  // the dV launch also reduces the dK launch's bias slabs (its first workgroups)
  BiasRed red{4 * grid, (int)npos, a.nb + 1, 0, dpos_w, dts_w};
  if (a.map_kq) red.nbias = ceil_div(ceil_div((int)npos + a.nb + 1, 16), 8) * 8;
  const size_t lds_vp = D32 % 2 == 0 ? 3 * TB + 3 * 4 * 2048 : 2 * TB;  // ring / two buffers
  GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(attn_bwd_bf16w_vp_kernel<D32>, dim3(red.nbias + a.n_kt * bh8), dim3(256),
                                                  lds_vp, st, a, red));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide dv)");
  GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL(attn_bwd_bf16w_dq_kernel<D32>, dim3(a.n_qt * bh8), dim3(256), lds_q, st, a));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16(wide dq)");
  return 0;
}

}  // namespace gr

// Wide-head entries (called by hstu_attn_{fwd,bwd}_bf16 for 128 < d <= 256, dqk == dv).
size_t gr_attn_bf16w_copies_bytes(int B, int N, int H, int d) {
  return gr::bf16w_copies_bytes(B, N, H, d);
}

int gr_attn_bf16w_copies(const float* q, const float* k, const float* v, int64_t ld_qk, int64_t ld_v,
                         const int64_t* offsets, int B, int N, int H, int d, void* copies,
                         hipStream_t st) {
  using namespace gr;
  const CopyPtrs c = copy_ptrs(copies, B, N, H, d);
  ConvSet cs{{q, k, v, nullptr}, {ld_qk, ld_qk, ld_v, 0}, {c.q, c.k, c.v, nullptr}, c.zrow,
             offsets, B, H, d, 4 * ceil_div(d, 32)};
  return launch_convert(cs, 3, (int64_t)B * N, st);
}

int gr_attn_fwd_bf16w(const void* copies, const int64_t* offsets, int B, int N, int max_len, int H,
                      int d, const uint8_t* map_qk, const float* pos_w, const float* ts_w,
                      int num_buckets, float* out, int64_t ld_out, hipStream_t st) {
  using namespace gr;
  const CopyPtrs c = copy_ptrs(copies, B, N, H, d);
  AttnFwdArgsW a{};
  a.qb = c.q; a.kb = c.k; a.vb = c.v; a.zrow = c.zrow;
  a.rsb_qkv = (int64_t)H * 32 * ceil_div(d, 32);
  a.offsets = offsets; a.B = B; a.N = N; a.H = H; a.d = d;
  a.map_qk = map_qk; a.pos_w = pos_w; a.ts_w = ts_w; a.nb = map_qk ? num_buckets : 0;
  a.out = out; a.ld_out = ld_out; a.inv_n = 1.0f / (float)N;
  const int D32 = ceil_div(d, 32);
  if (D32 <= 5) return launch_fwd_bf16w<5>(a, st, max_len);
  if (D32 == 6) return launch_fwd_bf16w<6>(a, st, max_len);
  if (D32 == 7) return launch_fwd_bf16w<7>(a, st, max_len);
  return launch_fwd_bf16w<8>(a, st, max_len);
}

// workspace: slabs | dS blocks | P blocks | dO copy + zero row | Q, K, V copies (used when
// the caller passes none)
// own Q/K/V copies sit at the end: a caller passing the forward's copies needs none
size_t gr_attn_bwd_bf16w_workspace(int B, int N, int max_len, int H, int d, int num_buckets,
                                   bool with_copies) {
  using namespace gr;
  return al256(bf16w_slab_bytes(B, N, max_len, H, num_buckets)) + 2 * al256(bf16w_ds_bytes(B, N, H)) +
         bf16w_copy_bytes(B, N, H, d) + al256(ceil_div(d, 32) * 64) +
         (with_copies ? 0 : bf16w_copies_bytes(B, N, H, d));
}

int gr_attn_bwd_bf16w(const float* q, const float* k, const float* v, int64_t ld_qk, int64_t ld_v,
                      const float* dout, int64_t ld_dout, const int64_t* offsets, int B, int N,
                      int max_len, int H, int d, const uint8_t* map_kq, const float* pos_w,
                      const float* ts_w, int num_buckets, const float* hq, const float* hk,
                      const float* hv, int64_t ld_h, float* dq, float* dk, float* dvv, int64_t ld_d,
                      float* dpos_w, float* dts_w, const void* copies, void* workspace, hipStream_t st) {
  using namespace gr;
  const size_t slab_b = al256(bf16w_slab_bytes(B, N, max_len, H, num_buckets));
  const size_t ds_b = al256(bf16w_ds_bytes(B, N, H));
  const size_t cp_b = bf16w_copy_bytes(B, N, H, d);
  const int nch = 4 * ceil_div(d, 32);
  AttnBwdArgsW a{};
  a.q = q; a.k = k; a.v = v; a.ld_qk = ld_qk; a.ld_v = ld_v; a.dout = dout; a.ld_dout = ld_dout;
  a.offsets = offsets; a.B = B; a.N = N; a.H = H; a.d = d;
  a.map_kq = map_kq; a.pos_w = pos_w; a.ts_w = ts_w; a.nb = map_kq ? num_buckets : 0;
  a.hq = hq; a.hk = hk; a.hv = hv; a.ld_h = ld_h;
  a.dq = dq; a.dk = dk; a.dvv = dvv; a.ld_d = ld_d;
  a.slabs = (float*)workspace;
  a.ds = (__bf16*)((char*)workspace + slab_b);
  a.pb = (__bf16*)((char*)workspace + slab_b + ds_b);
  char* cp = (char*)workspace + slab_b + 2 * ds_b;
  a.ob = (__bf16*)cp;
  __bf16* ozrow = (__bf16*)(cp + cp_b);
  char* own = cp + cp_b + al256(nch * 16);
  ConvSet cs{{dout, q, k, v}, {ld_dout, ld_qk, ld_qk, ld_v}, {a.ob, nullptr, nullptr, nullptr}, ozrow,
             offsets, B, H, d, nch};
  int n = 1;
  if (copies) {  // Q, K, V copies from the forward
    const CopyPtrs c = copy_ptrs(copies, B, N, H, d);
    a.qb = c.q; a.kb = c.k; a.vb = c.v;
  } else {
    const CopyPtrs c = copy_ptrs(own, B, N, H, d);
    a.qb = c.q; a.kb = c.k; a.vb = c.v;
    cs.dst[1] = c.q; cs.dst[2] = c.k; cs.dst[3] = c.v;
    n = 4;
  }
  a.zrow = ozrow;
  a.rsb_qkv = (int64_t)H * 32 * ceil_div(d, 32);
  a.a16 = 0;
  a.total_rows = (int64_t)B * N;
  if (launch_convert(cs, n, a.total_rows, st)) return -1;
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

// ------------------------------------------------------------------ bf16 activations (ABI 16)
// autocast_dtype = bfloat16 at wide heads with d % 32 == 0: the projection writes uvqk and
// h_pre as bf16 (hstu_ln_uvqk_fwd_a16), so the attention DMAs its Q / K / V tiles straight
// from the uvqk rows (row stride n_out, no conversion pass), reads silu'(h) from bf16 h_pre
// and writes dQ / dK / dV as bf16 into d_uvqk.  Same kernels, same operands: results are
// the fp32-activation entries' on the bf16-rounded inputs, rounded to bf16 on store.
static bool a16_shape(int d) { return d > 128 && d <= 256 && d % 32 == 0; }
static bool a16_aligned(std::initializer_list<const void*> ptrs, int64_t ld) {
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16 != 0) return false;
  return ld % 8 == 0;
}

extern "C" int hstu_attn_fwd_a16(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                 int64_t ld_qkv, const int64_t* offsets, int B, int N, int max_len,
                                 int H, int d, const uint8_t* bucket_map, const float* pos_w,
                                 const float* ts_w, int num_buckets, const uint16_t* zrow,
                                 float* out, int64_t ld_out, void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && offsets && out && zrow, "hstu_attn_fwd_a16: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0, "hstu_attn_fwd_a16: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_fwd_a16: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(a16_shape(d) && a16_aligned({q, k, v, zrow}, ld_qkv) && ld_qkv >= (int64_t)H * d,
             "hstu_attn_fwd_a16: needs d %% 32 == 0 in (128, 256] and 16-byte aligned rows (d %d)", d);
  GR_REQUIRE(!bucket_map || (pos_w && ts_w && num_buckets > 0 && num_buckets < 256),
             "hstu_attn_fwd_a16: bucket_map given without pos_w/ts_w");
  if (B == 0 || max_len == 0) return 0;
  AttnFwdArgsW a{};
  a.qb = (const __bf16*)q; a.kb = (const __bf16*)k; a.vb = (const __bf16*)v;
  a.zrow = (const __bf16*)zrow;
  a.rsb_qkv = ld_qkv;
  a.offsets = offsets; a.B = B; a.N = N; a.H = H; a.d = d;
  a.map_qk = bucket_map; a.pos_w = pos_w; a.ts_w = ts_w; a.nb = bucket_map ? num_buckets : 0;
  a.out = out; a.ld_out = ld_out; a.inv_n = 1.0f / (float)N;
  hipStream_t st = (hipStream_t)stream;
  const int D32 = d / 32;
  if (D32 == 5) return launch_fwd_bf16w<5>(a, st, max_len);
  if (D32 == 6) return launch_fwd_bf16w<6>(a, st, max_len);
  if (D32 == 7) return launch_fwd_bf16w<7>(a, st, max_len);
  return launch_fwd_bf16w<8>(a, st, max_len);
}

extern "C" size_t hstu_attn_bwd_a16_workspace_size(int B, int N, int max_len, int H, int d,
                                                   int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0 || !a16_shape(d)) return 0;
  // bias slabs | dS blocks | P blocks (dO arrives in bf16: no copy, no zero row)
  return gr::al256(gr::bf16w_slab_bytes(B, N, max_len, H, num_buckets)) + 2 * gr::al256(gr::bf16w_ds_bytes(B, N, H));
}

extern "C" int hstu_attn_bwd_a16(const uint16_t* q, const uint16_t* k, const uint16_t* v,
                                 int64_t ld_qkv, const uint16_t* dout, int64_t ld_dout,
                                 const int64_t* offsets, int B, int N, int max_len, int H, int d,
                                 const uint8_t* bucket_map, const float* pos_w, const float* ts_w,
                                 int num_buckets, const uint16_t* hq, const uint16_t* hk,
                                 const uint16_t* hv, int64_t ld_h, uint16_t* dq, uint16_t* dk,
                                 uint16_t* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                                 const uint16_t* zrow, void* workspace, size_t ws_bytes,
                                 void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && dout && offsets && dq && dk && dvv && zrow, "hstu_attn_bwd_a16: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0, "hstu_attn_bwd_a16: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_bwd_a16: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(a16_shape(d) && a16_aligned({q, k, v, zrow}, ld_qkv) && ld_qkv >= (int64_t)H * d &&
                 a16_aligned({dout}, ld_dout) && ld_dout == (int64_t)H * d,
             "hstu_attn_bwd_a16: needs d %% 32 == 0 in (128, 256], 16-byte aligned rows and dout "
             "(bf16) with ld_dout = H d (d %d)", d);
  GR_REQUIRE((hq == nullptr) == (hk == nullptr) && (hk == nullptr) == (hv == nullptr),
             "hstu_attn_bwd_a16: hq/hk/hv must be all given or all NULL");
  if (bucket_map)
    GR_REQUIRE(pos_w && ts_w && dpos_w && dts_w && num_buckets > 0 && num_buckets < 256,
               "hstu_attn_bwd_a16: bucket_map given without pos_w/ts_w/dpos_w/dts_w");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0 || max_len == 0) {
    if (bucket_map) {
      zero_words_async(dpos_w, 2 * N - 1, st);
      zero_words_async(dts_w, num_buckets + 1, st);
    }
    return 0;
  }
  const size_t need = hstu_attn_bwd_a16_workspace_size(B, N, max_len, H, d, num_buckets);
  GR_REQUIRE(workspace && ws_bytes >= need, "hstu_attn_bwd_a16: workspace %zu B < %zu B", ws_bytes, need);
  const size_t slab_b = al256(bf16w_slab_bytes(B, N, max_len, H, num_buckets));
  const size_t ds_b = al256(bf16w_ds_bytes(B, N, H));
  AttnBwdArgsW a{};
  a.dout = nullptr; a.ld_dout = ld_dout;
  a.offsets = offsets; a.B = B; a.N = N; a.H = H; a.d = d;
  a.map_kq = bucket_map ? bucket_map + (size_t)B * attn_tiles_per_seq(N) * 4096 : nullptr;
  a.pos_w = pos_w; a.ts_w = ts_w; a.nb = bucket_map ? num_buckets : 0;
  // bf16 h / d through the fp32 pointer fields (a16 = 1, see store_dh)
  a.hq = (const float*)hq; a.hk = (const float*)hk; a.hv = (const float*)hv; a.ld_h = ld_h;
  a.dq = (float*)dq; a.dk = (float*)dk; a.dvv = (float*)dvv; a.ld_d = ld_d;
  a.a16 = 1;
  a.slabs = (float*)workspace;
  a.ds = (__bf16*)((char*)workspace + slab_b);
  a.pb = (__bf16*)((char*)workspace + slab_b + ds_b);
  a.ob = (__bf16*)dout;  // d_attn already in bf16, [row][head][d] (gate_o_bwd_a16): no copy
  a.qb = (__bf16*)q; a.kb = (__bf16*)k; a.vb = (__bf16*)v;  // read only
  a.rsb_qkv = ld_qkv;
  a.zrow = (__bf16*)zrow;
  a.total_rows = (int64_t)B * N;
  const int nb32 = ceil_div(N, 32);
  a.nbt = nb32 * (nb32 + 1) / 2;
  a.inv_n = 1.0f / (float)N;
  a.n_kt = ceil_div(max_len, WK);
  a.n_qt = ceil_div(max_len, WK);
  const int D32 = d / 32;
  if (D32 == 5) return launch_bwd_bf16w<5>(a, dpos_w, dts_w, st);
  if (D32 == 6) return launch_bwd_bf16w<6>(a, dpos_w, dts_w, st);
  if (D32 == 7) return launch_bwd_bf16w<7>(a, dpos_w, dts_w, st);
  return launch_bwd_bf16w<8>(a, dpos_w, dts_w, st);
}

#ifdef GR_STAMP
extern "C" __attribute__((visibility("default"))) int gr_stamp_bw_read(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gr::gr_stamp_bw_buf), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#endif
