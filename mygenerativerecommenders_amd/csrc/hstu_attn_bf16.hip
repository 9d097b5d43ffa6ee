// Jagged causal HSTU attention with bf16 MFMA operands and fp32 accumulation — gfx950
// (v_mfma_f32_16x16x32_bf16).  The opt-in bf16 compute mode of the encoder
// (HSTU(..., compute_dtype=torch.bfloat16)); the fp32 kernels stay the parity default.
//
// Same math and work decomposition as hstu_attn_fwd.hip (reference
// sequential_encoders/hstu.py:134-205 + the bias of hstu.py:96-128); what changes is the
// operand precision: Q, K, V are rounded to bf16 as they are staged, P = silu(S + bias)/N
// is rounded to bf16 as it becomes the A operand of P.V; S, the bias, silu and O are
// fp32.  One MFMA covers 32 of the head dims (16x the f32 MFMA's rate).
//
// Per 32-key chunk a wave computes
//   S^T (two 16-key blocks x 16 queries) = K_blk . Q^T   (A = K rows, bf16, from LDS;
//                                                          B = Q^T fragments in VGPRs)
// so lane (lr, lg) holds the 8 keys {4lg..4lg+3, 16+4lg..16+4lg+3} of query lr; those 8
// values, packed to bf16, are the A operand of  O += P . V  with that key order, and the
// B operand (V) is read from a TRANSPOSED bf16 tile (Vt[col][key]) as two 8-byte reads.
#include "attn_common.h"

#include "../../include/gr_hstu.h"

namespace gr {


struct AttnFwdArgsBf16 {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const int64_t* offsets;
  int B, N, H, dqk, dv, n_qtiles;
  const uint8_t* map_qk;  // null: no bias
  const float* pos_w;
  const float* ts_w;
  int nb;
  float* out;
  int64_t ld_out;
  float inv_n;
  int cus;  // CU count (snake_rank)
};


// Stages a ROWS x CP tile of a jagged fp32 column block as bf16 in LDS, NT threads.
// Columns >= ncols read 0 (out-of-range buffer offset); rows past the sequence read 0
// (descriptor range).
//   row-major  (K): item = (row, column pair), column pair fastest (coalesced reads);
//                   one packed dword at lds[row][2 cp]
//   transposed (V): item = (row pair, column pair); two packed dwords
//                   lds[2 cp][2 rp .. +1], lds[2 cp + 1][2 rp .. +1]
template <int CP, int ROWS, bool TRANS, int NT>
struct Bf16Stage {
  static constexpr int NP = CP / 2;
  static constexpr int RU = TRANS ? 2 : 1;  // rows per item
  static constexpr int ITEMS = ROWS / RU * NP;
  static constexpr int PER = (ITEMS + NT - 1) / NT;
  float v[PER][2 * RU];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int64_t ld, int r0, int ncols) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + NT * i;
      const int c = 2 * (id % NP), row = RU * (id / NP);
      const bool in = ITEMS % NT == 0 || id < ITEMS;
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int base = ((r0 + row + u) * (int)ld + c) * 4;
        v[i][2 * u] = buf_ld(r, in && c < ncols ? base : OOB_OFF, 0);
        v[i][2 * u + 1] = buf_ld(r, in && c + 1 < ncols ? base + 4 : OOB_OFF, 0);
      }
    }
  }
  __device__ __forceinline__ void store(__bf16* lds, int ldl) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + NT * i;
      if (ITEMS % NT != 0 && id >= ITEMS) continue;
      const int c = 2 * (id % NP), row = RU * (id / NP);
      if (TRANS) {
        *reinterpret_cast<uint32_t*>(lds + c * ldl + row) = pack_bf16(v[i][0], v[i][2]);
        *reinterpret_cast<uint32_t*>(lds + (c + 1) * ldl + row) = pack_bf16(v[i][1], v[i][3]);
      } else {
        *reinterpret_cast<uint32_t*>(lds + row * ldl + c) = pack_bf16(v[i][0], v[i][1]);
      }
    }
  }
};

// KC = 32-wide chunks of dqk, VT = 16-wide tiles of dv, TK = keys per LDS tile (mult. of 32)
template <int KC, int VT, int TK>
struct AttnBf16Cfg {
  static constexpr int KP = KC * 32;      // padded dqk
  static constexpr int VP = VT * 16;      // padded dv
  static constexpr int LDK = KP + 8;      // bf16 units: 16 B-aligned rows, rows 16 B apart mod 128
  static constexpr int LDV = TK + 8;      // transposed V rows (one per dv column)
  static constexpr size_t LDS_BYTES = 2 * ((size_t)TK * LDK + (size_t)VP * LDV);
  static constexpr int NCH = TK / 32;     // 32-key chunks per tile
};

// WAVES waves x 16 queries per workgroup: 8 at the wide heads, where every workgroup
// re-reads the K / V of all earlier keys (C3: ~2 GB per launch at 64 queries per
// workgroup), so twice the queries per staged tile halves that traffic.
template <int KC, int VT, int TK, int WAVES, bool HB>
__global__ __launch_bounds__(64 * WAVES) void hstu_attn_fwd_bf16_kernel(AttnFwdArgsBf16 a) {
  constexpr int NTH = 64 * WAVES, QT = 16 * WAVES;
  using C = AttnBf16Cfg<KC, VT, TK>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* Ks = reinterpret_cast<__bf16*>(smem);
  __bf16* Vt = Ks + TK * C::LDK;
  float* tsw = reinterpret_cast<float*>(smem + C::LDS_BYTES);  // nb + 1
  float* posw = tsw + (a.nb + 1);                              // 2N - 1

  const int BH = a.B * a.H;
  const int rank = snake_rank(blockIdx.x, a.cus);
  const int qt = a.n_qtiles - 1 - rank / BH;  // heaviest tiles first
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * QT;
  if (q0 >= L) return;

  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  if (HB) {
    for (int i = tid; i <= a.nb; i += NTH) tsw[i] = a.ts_w[i];
    for (int i = tid; i < 2 * a.N - 1; i += NTH) posw[i] = a.pos_w[i];
  }

  // this lane's query (S^T column) and its Q^T fragments: Q[qi][32c + 8lg .. +7]
  const int qi = q0 + w * 16 + lr;
  const bool q_ok = qi < L;
  u32x4_t qf[KC];
  {
    gptr<float> qrow = as_global(a.q) + (s0 + (q_ok ? qi : L - 1)) * a.ld_qk + h * a.dqk;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = 32 * c + 8 * lg + e;
        const float y = qrow[d < a.dqk ? d : a.dqk - 1];
        x[e] = d < a.dqk ? y : 0.f;
      }
      qf[c] = u32x4_t{pack_bf16(x[0], x[1]), pack_bf16(x[2], x[3]), pack_bf16(x[4], x[5]),
                      pack_bf16(x[6], x[7])};
    }
  }
  const int wq_lo = q0 + w * 16;  // first query of this wave
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_qk, b, attn_tiles_per_seq(a.N));
  const int map_voff = (((wq_lo & 63) + lr) * 16 + lg) * 4;  // 64 x 64 map tiles
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rv = seq_rsrc(a.v, a.ld_v, s0, h * a.dv, L, a.dv);

  f4 acc[VT];
#pragma unroll
  for (int ct = 0; ct < VT; ++ct) acc[ct] = f4_zero();

  Bf16Stage<C::KP, TK, false, NTH> kst;
  Bf16Stage<C::VP, TK, true, NTH> vst;
  kst.load(rk, a.ld_qk, 0, a.dqk);
  vst.load(rv, a.ld_v, 0, a.dv);
  kst.store(Ks, C::LDK);
  vst.store(Vt, C::LDV);
  __syncthreads();  // also publishes tsw / posw

  const int last_kt = min(q0 + QT - 1, L - 1) / TK;
  for (int kt = 0; kt <= last_kt; ++kt) {
    const int k0 = kt * TK;
    const bool more = kt < last_kt;
    if (more) {
      kst.load(rk, a.ld_qk, k0 + TK, a.dqk);
      vst.load(rv, a.ld_v, k0 + TK, a.dv);
    }
#pragma unroll
    for (int j = 0; j < C::NCH; ++j) {
      const int kc0 = k0 + 32 * j;
      if (kc0 > wq_lo + 15 || kc0 >= L) break;  // wave-uniform causal / length skip
      const bool two = kc0 + 16 <= wq_lo + 15 && kc0 + 16 < L;
      // bucket words of the two 16-key blocks (64 x 64 map tiles, query-major)
      uint32_t mw0 = 0, mw1 = 0;
      if (HB) {
        mw0 = buf_ld_u32(rmap, map_voff, map_soff(wq_lo, kc0, true));
        mw1 = two ? buf_ld_u32(rmap, map_voff, map_soff(wq_lo, kc0 + 16, true)) : 0u;
      }
      const __bf16* krow = Ks + (32 * j + lr) * C::LDK + 8 * lg;
      f4 s0v = f4_zero(), s1v = f4_zero();
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const u32x4_t ka = *reinterpret_cast<const u32x4_t*>(krow + 32 * c);
        s0v = mfma_bf16(ka, qf[c], s0v);
      }
      if (two) {
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          const u32x4_t ka = *reinterpret_cast<const u32x4_t*>(krow + 16 * C::LDK + 32 * c);
          s1v = mfma_bf16(ka, qf[c], s1v);
        }
      }
      // p[e]: e < 4 -> key kc0 + 4lg + e, e >= 4 -> key kc0 + 16 + 4lg + e - 4
      float p[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int hi = e >> 2, r = e & 3;
        const int kj = kc0 + 16 * hi + 4 * lg + r;
        float val = hi ? s1v[r] : s0v[r];
        if (HB) {
          const int bucket = ((hi ? mw1 : mw0) >> (8 * r)) & 0xFF;
          int pi = a.N - 1 + kj - qi;
          pi = pi < 0 ? 0 : (pi > 2 * a.N - 2 ? 2 * a.N - 2 : pi);
          val = val + (posw[pi] + tsw[bucket]);
        }
        p[e] = (q_ok && kj <= qi && (hi == 0 || two)) ? siluf_(val) * a.inv_n : 0.f;
      }
      const u32x4_t pa = u32x4_t{pack_bf16(p[0], p[1]), pack_bf16(p[2], p[3]),
                                 pack_bf16(p[4], p[5]), pack_bf16(p[6], p[7])};
      const __bf16* vcol = Vt + lr * C::LDV + 32 * j + 4 * lg;
#pragma unroll
      for (int ct = 0; ct < VT; ++ct) {
        const u32x2_t lo = *reinterpret_cast<const u32x2_t*>(vcol + ct * 16 * C::LDV);
        const u32x2_t hi = *reinterpret_cast<const u32x2_t*>(vcol + ct * 16 * C::LDV + 16);
        acc[ct] = mfma_bf16(pa, u32x4_t{lo.x, lo.y, hi.x, hi.y}, acc[ct]);
      }
    }
    if (more) {
      lds_barrier();
      kst.store(Ks, C::LDK);
      vst.store(Vt, C::LDV);
      lds_barrier();
    }
  }

  // ---- epilogue: acc[ct][r] = O[query wq_lo + 4lg + r][col ct*16 + lr]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qo = wq_lo + 4 * lg + r;
    if (qo >= L) continue;
    float* orow = a.out + (s0 + qo) * a.ld_out + h * a.dv;
#pragma unroll
    for (int ct = 0; ct < VT; ++ct) {
      const int c = ct * 16 + lr;
      if (c < a.dv) orow[c] = acc[ct][r];
    }
  }
}

template <int KC, int VT, int TK, int WAVES>
static int launch_fwd_bf16(AttnFwdArgsBf16 a, hipStream_t st) {
  using C = AttnBf16Cfg<KC, VT, TK>;
  a.n_qtiles = ceil_div(a.n_qtiles, 16 * WAVES);  // n_qtiles arrives as max_len
  a.cus = (int64_t)a.n_qtiles * a.B * a.H <= 2 * device_cus() ? device_cus() : (1 << 30);
  const int grid = a.n_qtiles * a.B * a.H;
  const size_t lds = C::LDS_BYTES + sizeof(float) * (a.nb + 1 + 2 * a.N - 1);
  GR_REQUIRE(lds <= 160 * 1024, "hstu_attn_fwd_bf16: LDS %zu B exceeds 160 KiB (N=%d)", lds, a.N);
  if (a.map_qk) {
    GR_TIMED("attn_fwd", st, hipLaunchKernelGGL((hstu_attn_fwd_bf16_kernel<KC, VT, TK, WAVES, true>), dim3(grid), dim3(64 * WAVES), lds, st, a));
  } else {
    GR_TIMED("attn_fwd", st, hipLaunchKernelGGL((hstu_attn_fwd_bf16_kernel<KC, VT, TK, WAVES, false>), dim3(grid), dim3(64 * WAVES), lds, st, a));
  }
  GR_LAUNCH_CHECK("hstu_attn_fwd_bf16");
  return 0;
}

}  // namespace gr

// wide heads (128 < d <= 256, dqk == dv): hstu_attn_bf16w.hip
size_t gr_attn_bf16w_copies_bytes(int B, int N, int H, int d);
int gr_attn_bf16w_copies(const float* q, const float* k, const float* v, int64_t ld_qk, int64_t ld_v,
                         const int64_t* offsets, int B, int N, int H, int d, void* copies,
                         hipStream_t st);
int gr_attn_fwd_bf16w(const void* copies, const int64_t* offsets, int B, int N, int max_len, int H,
                      int d, const uint8_t* map_qk, const float* pos_w, const float* ts_w,
                      int num_buckets, float* out, int64_t ld_out, hipStream_t st);
static bool bf16_wide(int dqk, int dv) { return dqk == dv && dqk > 128 && dqk <= 256; }

extern "C" size_t hstu_attn_bf16_copies_bytes(int B, int N, int H, int dqk, int dv) {
  if (B <= 0 || N <= 0 || H <= 0 || !bf16_wide(dqk, dv) || dqk % 2) return 0;
  return gr_attn_bf16w_copies_bytes(B, N, H, dqk);
}

extern "C" int hstu_attn_bf16_copies(const float* q, const float* k, const float* v, int64_t ld_qk,
                                     int64_t ld_v, const int64_t* offsets, int B, int N, int H,
                                     int dqk, int dv, void* copies, void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && offsets && copies, "hstu_attn_bf16_copies: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0, "hstu_attn_bf16_copies: bad sizes");
  GR_REQUIRE(bf16_wide(dqk, dv) && pair_aligned({q, k, v}, {ld_qk, ld_v, (int64_t)dqk}),
             "hstu_attn_bf16_copies: needs dqk == dv in (128, 256], even strides (dqk %d, dv %d)", dqk, dv);
  if (B == 0) return 0;
  return gr_attn_bf16w_copies(q, k, v, ld_qk, ld_v, offsets, B, N, H, dqk, copies, (hipStream_t)stream);
}

extern "C" int hstu_attn_fwd_bf16(const float* q, const float* k, const float* v, int64_t ld_qk,
                                  int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                                  int H, int dqk, int dv, const uint8_t* bucket_map,
                                  const float* pos_w, const float* ts_w, int num_buckets,
                                  float* out, int64_t ld_out, const void* copies, void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && offsets && out, "hstu_attn_fwd_bf16: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_fwd_bf16: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_fwd_bf16: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 256 && dv <= 256, "hstu_attn_fwd_bf16: dqk/dv > 256 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE(!bucket_map || (pos_w && ts_w && num_buckets > 0 && num_buckets < 256),
             "hstu_attn_fwd_bf16: bucket_map given without pos_w/ts_w");
  GR_REQUIRE(!copies || bf16_wide(dqk, dv),
             "hstu_attn_fwd_bf16: copies are for dqk == dv in (128, 256] (dqk %d, dv %d)", dqk, dv);
  if (B == 0 || max_len == 0) return 0;
  if (copies)
    return gr_attn_fwd_bf16w(copies, offsets, B, N, max_len, H, dqk, bucket_map, pos_w, ts_w,
                             num_buckets, out, ld_out, (hipStream_t)stream);
  AttnFwdArgsBf16 a{q, k, v, ld_qk, ld_v, offsets, B, N, H, dqk, dv, max_len,
                    bucket_map, pos_w, ts_w, bucket_map ? num_buckets : 0, out, ld_out,
                    1.0f / (float)N, 0};
  hipStream_t st = (hipStream_t)stream;
  const int d = dqk > dv ? dqk : dv;
  if (d <= 32) return launch_fwd_bf16<1, 2, 64, 4>(a, st);
  if (d <= 64) return launch_fwd_bf16<2, 4, 64, 4>(a, st);
  if (d <= 128) return launch_fwd_bf16<4, 8, 64, 8>(a, st);
  return launch_fwd_bf16<8, 16, 32, 8>(a, st);
}

// =================================================================== backward (bf16)
// Same passes as hstu_attn_bwd.hip with bf16 MFMA operands (fp32 accumulation, fp32
// elementwise):
//   * key-major (dK, dV, bias grads): WAVES x 16 keys per workgroup; per 32-query
//     chunk a wave computes S = Q K^T and dP = dO V^T (A = Q / dO rows from LDS, B = its
//     keys' K^T / V^T fragments in VGPRs), so lane (lr, lg) holds the 8 queries
//     {4lg..4lg+3, 16+4lg..16+4lg+3} of key lr -- directly the A operand (rows = keys,
//     k = queries) of dV += P^T dO and dK += dS^T Q, whose B operands come from
//     TRANSPOSED bf16 tiles of dO and Q;
//   * query-major (dQ): WAVES x 16 queries per workgroup; S^T = K Q^T, dP^T = V dO^T, and
//     dQ += dS K with B from a transposed K tile.
// Relative-bias gradients stay fp32 and deterministic: dts_w in per-wave LDS histograms;
// dpos_w per chunk as per-wave diagonal sums (47 bins) that one pass per tile adds, in
// wave order, into the workgroup's histogram; each workgroup writes one slab, reduced in
// a fixed order by the first workgroups of the dQ launch (bias_reduce_block).

namespace gr {

struct AttnBwdArgsBf16 {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const float* dout;
  int64_t ld_dout;
  const int64_t* offsets;
  int B, N, H, dqk, dv, max_len;
  const uint8_t* map_qk;
  const uint8_t* map_kq;
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
  float* slabs;  // [grid_kv][2N-1 + nb+1]
  float inv_n;
  int n_kt, n_qt;  // key / query tiles of the two passes
  int cus;
};

// A ROWS x CP fp32 tile loaded once, stored as bf16 row-major and / or transposed.
// Item = (row pair, column pair), column pair fastest.
template <int CP, int ROWS, int NT>
struct DualStage {
  static constexpr int NP = CP / 2;
  static constexpr int ITEMS = ROWS / 2 * NP;
  static constexpr int PER = (ITEMS + NT - 1) / NT;
  float v[PER][4];  // (r, c), (r, c+1), (r+1, c), (r+1, c+1)
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int64_t ld, int r0, int ncols) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = threadIdx.x + NT * i;
      const int c = 2 * (id % NP), row = 2 * (id / NP);
      const bool in = ITEMS % NT == 0 || id < ITEMS;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int base = ((r0 + row + u) * (int)ld + c) * 4;
        v[i][2 * u] = buf_ld(r, in && c < ncols ? base : OOB_OFF, 0);
        v[i][2 * u + 1] = buf_ld(r, in && c + 1 < ncols ? base + 4 : OOB_OFF, 0);
      }
    }
  }
  __device__ __forceinline__ void store_rows(__bf16* lds, int ldl) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = threadIdx.x + NT * i;
      if (ITEMS % NT != 0 && id >= ITEMS) continue;
      const int c = 2 * (id % NP), row = 2 * (id / NP);
      *reinterpret_cast<uint32_t*>(lds + row * ldl + c) = pack_bf16(v[i][0], v[i][1]);
      *reinterpret_cast<uint32_t*>(lds + (row + 1) * ldl + c) = pack_bf16(v[i][2], v[i][3]);
    }
  }
  __device__ __forceinline__ void store_trans(__bf16* lds, int ldl) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = threadIdx.x + NT * i;
      if (ITEMS % NT != 0 && id >= ITEMS) continue;
      const int c = 2 * (id % NP), row = 2 * (id / NP);
      *reinterpret_cast<uint32_t*>(lds + c * ldl + row) = pack_bf16(v[i][0], v[i][2]);
      *reinterpret_cast<uint32_t*>(lds + (c + 1) * ldl + row) = pack_bf16(v[i][1], v[i][3]);
    }
  }
};

// 8 bf16 of a row from global, zero past `n` (fragments held in VGPRs)
__device__ __forceinline__ u32x4_t row_frag(gptr<float> row, int d0, int n) {
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int d = d0 + e;
    const float y = row[d < n ? d : n - 1];
    x[e] = d < n ? y : 0.f;
  }
  return u32x4_t{pack_bf16(x[0], x[1]), pack_bf16(x[2], x[3]), pack_bf16(x[4], x[5]),
                 pack_bf16(x[6], x[7])};
}

// B operand of 8 permuted k-values from a transposed bf16 tile: [4g..4g+3] ++ [16+4g..]
__device__ __forceinline__ u32x4_t trans_frag(const __bf16* p) {
  const u32x2_t lo = *reinterpret_cast<const u32x2_t*>(p);
  const u32x2_t hi = *reinterpret_cast<const u32x2_t*>(p + 16);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}

template <int KC, int VC, int TQ>
struct BwdBf16Cfg {
  static constexpr int KP = KC * 32, VP = VC * 32;  // padded dqk, dv (32-wide chunks)
  static constexpr int KT = KP / 16, VT = VP / 16;  // 16-col output tiles
  static constexpr int LDK = KP + 8, LDV = VP + 8;  // row-major tiles (bf16 units)
  static constexpr int LDT = TQ + 8;                // transposed tiles (one row per column)
  static constexpr int NCH = TQ / 32;
};

constexpr int DIAG = 48;  // per-wave diagonal bins of one 32-query x 16-key chunk (47 used)

// PART: 0 = dV, dK and the bias gradients in one pass; at the wide heads (d > 128) the
// accumulators of both do not fit next to the fragments, so PART 1 computes dV (S, P)
// and PART 2 dK + bias gradients (S, dP, dS): S twice, no spills.
// PRIV: every wave keeps a private dpos_w histogram (short sequences: WAVES x (2N - 1)
// floats fit LDS) and adds each element directly -- no per-chunk ordered pass.
template <int KC, int VC, int TQ, int WAVES, bool HB, int PART, bool PRIV>
__global__ __launch_bounds__(64 * WAVES) void attn_bwd_bf16_dkv_kernel(AttnBwdArgsBf16 a) {
  using C = BwdBf16Cfg<KC, VC, TQ>;
  constexpr bool DO_V = PART != 2, DO_K = PART != 1;
  constexpr bool BIAS = HB && DO_K;
  constexpr int NTH = 64 * WAVES, KTILE = 16 * WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __bf16* Qs = reinterpret_cast<__bf16*>(smem);  // [TQ][LDK]
  __bf16* Qt = Qs + TQ * C::LDK;                 // [KP][LDT]
  __bf16* Ds = Qt + C::KP * C::LDT;              // [TQ][LDV]
  __bf16* Dt = Ds + TQ * C::LDV;                 // [VP][LDT]
  float* tsw = reinterpret_cast<float*>(Dt + C::VP * C::LDT);
  const int npos = 2 * a.N - 1;
  float* posw = tsw + (a.nb + 1);
  float* hpos = posw + npos;                     // dpos histogram(s) [PRIV ? WAVES : 1][npos]
  float* diag = hpos + (PRIV ? WAVES : 1) * npos;  // [WAVES][DIAG] (ordered mode)
  float* hts = diag + (PRIV ? 0 : WAVES * DIAG);   // [WAVES][nb + 1]

  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int rank = snake_rank(id, a.cus);
  const int kt = rank / BH;  // heaviest (first) key tiles first
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * KTILE;
  const int nbins = npos + a.nb + 1;
  float* slab = BIAS ? a.slabs + (int64_t)id * nbins : nullptr;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  if (k0 >= L) {
    if (BIAS)
      for (int i = tid; i < nbins; i += NTH) slab[i] = 0.f;
    return;
  }
  if (HB) {
    for (int i = tid; i <= a.nb; i += NTH) tsw[i] = a.ts_w[i];
    for (int i = tid; i < npos; i += NTH) posw[i] = a.pos_w[i];
    // hpos, diag and hts are contiguous
    const int nz = (PRIV ? WAVES : 1) * npos + (PRIV ? 0 : WAVES * DIAG) + WAVES * (a.nb + 1);
    for (int i = tid; i < nz; i += NTH) hpos[i] = 0.f;
  }
  const int wk_lo = k0 + 16 * w;
  const int kj = wk_lo + lr;  // this lane's key
  const bool k_ok = kj < L;
  u32x4_t kf[KC], vf[VC];
  {
    const int64_t row = s0 + (k_ok ? kj : L - 1);
    gptr<float> krow = as_global(a.k) + row * a.ld_qk + h * a.dqk;
    gptr<float> vrow = as_global(a.v) + row * a.ld_v + h * a.dv;
#pragma unroll
    for (int c = 0; c < KC; ++c) kf[c] = row_frag(krow, 32 * c + 8 * lg, a.dqk);
#pragma unroll
    for (int c = 0; c < VC; ++c) vf[c] = DO_K ? row_frag(vrow, 32 * c + 8 * lg, a.dv) : u32x4_t{};
  }
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_kq, b, attn_tiles_per_seq(a.N));
  const int map_voff = (((wk_lo & 63) + lr) * 16 + lg) * 4;  // key-major 64 x 64 tiles
  const __amdgpu_buffer_rsrc_t rq = seq_rsrc(a.q, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rdo = seq_rsrc(a.dout, a.ld_dout, s0, h * a.dv, L, a.dv);

  f4 dV[C::VT], dK[C::KT];
#pragma unroll
  for (int t = 0; t < C::VT; ++t) dV[t] = f4_zero();
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dK[t] = f4_zero();
  // dts: per-lane running (bucket, sum), flushed to the wave's histogram on change
  float* whts = hts + w * (a.nb + 1);
  float* wdiag = diag + w * DIAG;
  float* whpos = hpos + (PRIV ? w * npos : 0);
  int run_b = -1;
  float run_s = 0.f;

  DualStage<C::KP, TQ, NTH> qst;
  DualStage<C::VP, TQ, NTH> dst;
  const int qt0 = k0 / TQ, last_qt = (L - 1) / TQ;
  qst.load(rq, a.ld_qk, qt0 * TQ, a.dqk);
  dst.load(rdo, a.ld_dout, qt0 * TQ, a.dv);
  auto store_tiles = [&]() {
    qst.store_rows(Qs, C::LDK);
    if (DO_K) qst.store_trans(Qt, C::LDT);
    if (DO_K) dst.store_rows(Ds, C::LDV);
    if (DO_V) dst.store_trans(Dt, C::LDT);
  };
  store_tiles();
  __syncthreads();
  for (int qt = qt0; qt <= last_qt; ++qt) {
    const bool more = qt < last_qt;
    if (more) {
      qst.load(rq, a.ld_qk, (qt + 1) * TQ, a.dqk);
      dst.load(rdo, a.ld_dout, (qt + 1) * TQ, a.dv);
    }
    int dbase = 0;  // chunk diagonal base (for the ordered dpos pass below)
#pragma unroll
    for (int j = 0; j < C::NCH; ++j) {
      const int qc0 = qt * TQ + 32 * j;
      const bool act = qc0 + 31 >= wk_lo && qc0 < L;  // wave-uniform causal / length
      if (act) {
        uint32_t mw0 = 0, mw1 = 0;
        if (HB) {  // P needs the bias too
          mw0 = buf_ld_u32(rmap, map_voff, map_soff(qc0, wk_lo, false));
          mw1 = buf_ld_u32(rmap, map_voff, map_soff(qc0 + 16, wk_lo, false));
        }
        f4 sv[2] = {f4_zero(), f4_zero()}, dp[2] = {f4_zero(), f4_zero()};
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
          const __bf16* qrow = Qs + (32 * j + 16 * blk + lr) * C::LDK + 8 * lg;
          const __bf16* drow = Ds + (32 * j + 16 * blk + lr) * C::LDV + 8 * lg;
#pragma unroll
          for (int c = 0; c < KC; ++c)
            sv[blk] = mfma_bf16(*reinterpret_cast<const u32x4_t*>(qrow + 32 * c), kf[c], sv[blk]);
          if (DO_K) {
#pragma unroll
            for (int c = 0; c < VC; ++c)
              dp[blk] = mfma_bf16(*reinterpret_cast<const u32x4_t*>(drow + 32 * c), vf[c], dp[blk]);
          }
        }
        // element e: query qc0 + 16 (e >> 2) + 4lg + (e & 3), key kj
        float p[8], ds[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int hi = e >> 2, r = e & 3;
          const int qi = qc0 + 16 * hi + 4 * lg + r;
          const bool ok = k_ok && qi < L && kj <= qi;
          float x = sv[hi][r];
          const int bk = HB ? (int)(((hi ? mw1 : mw0) >> (8 * r)) & 0xFF) : 0;
          if (HB) {
            int pi = a.N - 1 + kj - qi;
            pi = pi < 0 ? 0 : (pi > npos - 1 ? npos - 1 : pi);
            x = x + (posw[pi] + tsw[bk]);
          }
          const float sg = sigmoidf_(x);
          p[e] = ok ? x * sg * a.inv_n : 0.f;
          ds[e] = ok ? dp[hi][r] * (sg * (1.0f + x * (1.0f - sg))) * a.inv_n : 0.f;
          if (BIAS) {
            if (ok) {
              if (bk != run_b) {  // queries walk in order: buckets change rarely
                if (run_b >= 0) atomicAdd(&whts[run_b], run_s);
                run_b = bk;
                run_s = 0.f;
              }
              run_s += ds[e];
              if (PRIV) {
                atomicAdd(&whpos[a.N - 1 + kj - qi], ds[e]);
              } else {  // diagonal kj - qi in [wk_lo - qc0 - 31, wk_lo - qc0 + 15]
                atomicAdd(&wdiag[kj - qi - (wk_lo - qc0 - 31)], ds[e]);
              }
            }
          }
        }
        const u32x4_t pa = u32x4_t{pack_bf16(p[0], p[1]), pack_bf16(p[2], p[3]),
                                   pack_bf16(p[4], p[5]), pack_bf16(p[6], p[7])};
        const u32x4_t da = u32x4_t{pack_bf16(ds[0], ds[1]), pack_bf16(ds[2], ds[3]),
                                   pack_bf16(ds[4], ds[5]), pack_bf16(ds[6], ds[7])};
        if (DO_V) {
#pragma unroll
          for (int t = 0; t < C::VT; ++t)
            dV[t] = mfma_bf16(pa, trans_frag(Dt + (16 * t + lr) * C::LDT + 32 * j + 4 * lg), dV[t]);
        }
        if (DO_K) {
#pragma unroll
          for (int t = 0; t < C::KT; ++t)
            dK[t] = mfma_bf16(da, trans_frag(Qt + (16 * t + lr) * C::LDT + 32 * j + 4 * lg), dK[t]);
        }
      }
      if (BIAS && !PRIV) {
        // ordered dpos: bins N-1 + (k0 - qc0 - 31) + t, t in [0, 16 WAVES + 47): wave w's
        // diagonal bin u covers t = 16 w + u; thread t adds the waves' bins in order
        __syncthreads();
        const int span = 16 * WAVES + DIAG - 1;
        const int base = a.N - 1 + (k0 - qc0 - 31);
        for (int t = tid; t < span; t += NTH) {
          float acc = 0.f;
#pragma unroll
          for (int ww = 0; ww < WAVES; ++ww) {
            const int u = t - 16 * ww;
            if (u >= 0 && u < DIAG) {
              acc += diag[ww * DIAG + u];
              diag[ww * DIAG + u] = 0.f;
            }
          }
          const int bin = base + t;
          if (bin >= 0 && bin < npos) hpos[bin] += acc;
        }
        __syncthreads();
      }
      (void)dbase;
    }
    if (more) {
      lds_barrier();
      store_tiles();
      lds_barrier();
    }
  }
  // ---- epilogue: rows = keys wk_lo + 4lg + r, cols = 16 t + lr (the silu'(h) inputs are
  // loaded here, all of a tensor's before any is used)
  if (DO_V)
    store_scaled<4, C::VT>([&](int i, int t) { return dV[t][i]; }, L, a.dv, s0, a.dvv, a.ld_d, a.hv,
                           a.ld_h, h * a.dv, [&](int i) { return wk_lo + 4 * lg + i; },
                           [&](int t) { return 16 * t + lr; });
  if (DO_K)
    store_scaled<4, C::KT>([&](int i, int t) { return dK[t][i]; }, L, a.dqk, s0, a.dk, a.ld_d, a.hk,
                           a.ld_h, h * a.dqk, [&](int i) { return wk_lo + 4 * lg + i; },
                           [&](int t) { return 16 * t + lr; });
  if (BIAS) {
    if (run_b >= 0) atomicAdd(&whts[run_b], run_s);
    __syncthreads();
    for (int i = tid; i < npos; i += NTH) {
      float acc = hpos[i];
      if (PRIV)
        for (int ww = 1; ww < WAVES; ++ww) acc += hpos[ww * npos + i];  // fixed wave order
      slab[i] = acc;
    }
    for (int i = tid; i <= a.nb; i += NTH) {
      float acc = 0.f;
      for (int ww = 0; ww < WAVES; ++ww) acc += hts[ww * (a.nb + 1) + i];
      slab[npos + i] = acc;
    }
  }
}

// The bias-gradient slabs of the dK/dV launch reduced by the first workgroups of the dQ
// launch (one launch fewer per layer): workgroup wg owns bins 16 wg .. 16 wg + 15, thread
// (bin, group g) sums slabs g, g + G, ... in order (8 loads in flight), then the G groups
// are added in order.  At 256 threads (G = 16) the order is that of the former reduce launch.
template <int NTH>
__device__ __forceinline__ void bias_reduce_block(const float* slabs, int n_slabs, int n_pos, int n_ts,
                                                  float* dpos_w, float* dts_w, int wg, float* part) {
  constexpr int G = NTH / 16;
  const int nbins = n_pos + n_ts;
  const int bl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int i = wg * 16 + bl;
  float acc = 0.f;
  if (i < nbins) {
    int j = g;
    for (; j + 7 * G < n_slabs; j += 8 * G) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slabs[(int64_t)(j + u * G) * nbins + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; j < n_slabs; j += G) acc += slabs[(int64_t)j * nbins + i];
  }
  part[g * 16 + bl] = acc;
  __syncthreads();
  if (g == 0 && i < nbins) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) s += part[k * 16 + bl];
    if (i < n_pos) dpos_w[i] = s;
    else dts_w[i - n_pos] = s;
  }
}

template <int KC, int VC, int TK, int WAVES, bool HB>
__global__ __launch_bounds__(64 * WAVES) void attn_bwd_bf16_dq_kernel(AttnBwdArgsBf16 a, int nbias,
                                                                     float* dpos_w, float* dts_w) {
  using C = BwdBf16Cfg<KC, VC, TK>;
  constexpr int NTH = 64 * WAVES, QT = 16 * WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (HB && (int)blockIdx.x < nbias) {
    bias_reduce_block<NTH>(a.slabs, a.n_kt * a.B * a.H, 2 * a.N - 1, a.nb + 1, dpos_w, dts_w,
                           blockIdx.x, reinterpret_cast<float*>(smem));
    return;
  }
  __bf16* Ks = reinterpret_cast<__bf16*>(smem);  // [TK][LDK]
  __bf16* Kt = Ks + TK * C::LDK;                 // [KP][LDT]
  __bf16* Vs = Kt + C::KP * C::LDT;              // [TK][LDV]
  float* tsw = reinterpret_cast<float*>(Vs + TK * C::LDV);
  float* posw = tsw + (a.nb + 1);

  const int BH = a.B * a.H;
  const int rank = snake_rank((int)blockIdx.x - nbias, a.cus);
  const int qt = a.n_qt - 1 - rank / BH;  // heaviest tiles first
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * QT;
  if (q0 >= L) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  if (HB) {
    for (int i = tid; i <= a.nb; i += NTH) tsw[i] = a.ts_w[i];
    for (int i = tid; i < 2 * a.N - 1; i += NTH) posw[i] = a.pos_w[i];
  }
  const int wq_lo = q0 + 16 * w;
  const int qi = wq_lo + lr;
  const bool q_ok = qi < L;
  u32x4_t qf[KC], df[VC];
  {
    const int64_t row = s0 + (q_ok ? qi : L - 1);
    gptr<float> qrow = as_global(a.q) + row * a.ld_qk + h * a.dqk;
    gptr<float> drow = as_global(a.dout) + row * a.ld_dout + h * a.dv;
#pragma unroll
    for (int c = 0; c < KC; ++c) qf[c] = row_frag(qrow, 32 * c + 8 * lg, a.dqk);
#pragma unroll
    for (int c = 0; c < VC; ++c) df[c] = row_frag(drow, 32 * c + 8 * lg, a.dv);
  }
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_qk, b, attn_tiles_per_seq(a.N));
  const int map_voff = (((wq_lo & 63) + lr) * 16 + lg) * 4;  // query-major 64 x 64 tiles
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rv = seq_rsrc(a.v, a.ld_v, s0, h * a.dv, L, a.dv);

  f4 dQ[C::KT];
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dQ[t] = f4_zero();
  DualStage<C::KP, TK, NTH> kst;
  DualStage<C::VP, TK, NTH> vst;
  kst.load(rk, a.ld_qk, 0, a.dqk);
  vst.load(rv, a.ld_v, 0, a.dv);
  kst.store_rows(Ks, C::LDK);
  kst.store_trans(Kt, C::LDT);
  vst.store_rows(Vs, C::LDV);
  __syncthreads();
  const int last_kt = min(q0 + QT - 1, L - 1) / TK;
  for (int kt = 0; kt <= last_kt; ++kt) {
    const bool more = kt < last_kt;
    if (more) {
      kst.load(rk, a.ld_qk, (kt + 1) * TK, a.dqk);
      vst.load(rv, a.ld_v, (kt + 1) * TK, a.dv);
    }
#pragma unroll
    for (int j = 0; j < C::NCH; ++j) {
      const int kc0 = kt * TK + 32 * j;
      if (kc0 > wq_lo + 15 || kc0 >= L) break;  // wave-uniform causal / length skip
      const bool two = kc0 + 16 <= wq_lo + 15 && kc0 + 16 < L;
      uint32_t mw0 = 0, mw1 = 0;
      if (HB) {
        mw0 = buf_ld_u32(rmap, map_voff, map_soff(wq_lo, kc0, true));
        mw1 = two ? buf_ld_u32(rmap, map_voff, map_soff(wq_lo, kc0 + 16, true)) : 0u;
      }
      f4 st[2] = {f4_zero(), f4_zero()}, dpt[2] = {f4_zero(), f4_zero()};
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        if (blk == 1 && !two) break;
        const __bf16* krow = Ks + (32 * j + 16 * blk + lr) * C::LDK + 8 * lg;
        const __bf16* vrow = Vs + (32 * j + 16 * blk + lr) * C::LDV + 8 * lg;
#pragma unroll
        for (int c = 0; c < KC; ++c)
          st[blk] = mfma_bf16(*reinterpret_cast<const u32x4_t*>(krow + 32 * c), qf[c], st[blk]);
#pragma unroll
        for (int c = 0; c < VC; ++c)
          dpt[blk] = mfma_bf16(*reinterpret_cast<const u32x4_t*>(vrow + 32 * c), df[c], dpt[blk]);
      }
      // element e: key kc0 + 16 (e >> 2) + 4lg + (e & 3), query qi
      float ds[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int hi = e >> 2, r = e & 3;
        const int kj = kc0 + 16 * hi + 4 * lg + r;
        const bool ok = q_ok && kj <= qi && (hi == 0 || two);
        float x = st[hi][r];
        if (HB) {
          const int bucket = ((hi ? mw1 : mw0) >> (8 * r)) & 0xFF;
          int pi = a.N - 1 + kj - qi;
          pi = pi < 0 ? 0 : (pi > 2 * a.N - 2 ? 2 * a.N - 2 : pi);
          x = x + (posw[pi] + tsw[bucket]);
        }
        ds[e] = ok ? dpt[hi][r] * silu_grad_(x) * a.inv_n : 0.f;
      }
      const u32x4_t da = u32x4_t{pack_bf16(ds[0], ds[1]), pack_bf16(ds[2], ds[3]),
                                 pack_bf16(ds[4], ds[5]), pack_bf16(ds[6], ds[7])};
#pragma unroll
      for (int t = 0; t < C::KT; ++t)
        dQ[t] = mfma_bf16(da, trans_frag(Kt + (16 * t + lr) * C::LDT + 32 * j + 4 * lg), dQ[t]);
    }
    if (more) {
      lds_barrier();
      kst.store_rows(Ks, C::LDK);
      kst.store_trans(Kt, C::LDT);
      vst.store_rows(Vs, C::LDV);
      lds_barrier();
    }
  }
  store_scaled<4, C::KT>([&](int i, int t) { return dQ[t][i]; }, L, a.dqk, s0, a.dq, a.ld_d, a.hq,
                         a.ld_h, h * a.dqk, [&](int i) { return wq_lo + 4 * lg + i; },
                         [&](int t) { return 16 * t + lr; });
}

// Deterministic slab reduction (fixed order): a workgroup owns 16 bins; thread (bin, g)
// sums slabs g, g + 16, ..., then the 16 partials are added in g order.
template <int KC, int VC, int TQ, int WAVES>
static size_t dkv_lds(const AttnBwdArgsBf16& a, bool priv) {
  using C = BwdBf16Cfg<KC, VC, TQ>;
  const size_t npos = 2 * a.N - 1;
  return 2 * ((size_t)TQ * C::LDK + (size_t)C::KP * C::LDT + (size_t)TQ * C::LDV + (size_t)C::VP * C::LDT) +
         sizeof(float) * ((a.nb + 1) + npos + (priv ? WAVES * npos : npos + WAVES * DIAG) +
                          WAVES * (a.nb + 1));
}
template <int WAVES>
static bool dkv_priv(const AttnBwdArgsBf16& a) { return (size_t)WAVES * (2 * a.N - 1) * 4 <= 40 * 1024; }
template <int KC, int VC, int TK>
static size_t dq_lds(const AttnBwdArgsBf16& a) {
  using C = BwdBf16Cfg<KC, VC, TK>;
  return 2 * ((size_t)TK * C::LDK + (size_t)C::KP * C::LDT + (size_t)TK * C::LDV) +
         sizeof(float) * ((a.nb + 1) + (2 * a.N - 1));
}

static size_t bwd_bf16_slab_bytes(int B, int N, int max_len, int H, int nb, int key_tile) {
  return sizeof(float) * (size_t)ceil_div(max_len, key_tile) * B * H * (size_t)(2 * N - 1 + nb + 1);
}

template <int KC, int VC, int T, int WAVES, bool HB, bool PRIV>
static void launch_dkv_bf16_p(const AttnBwdArgsBf16& a, int grid, size_t lds, hipStream_t st) {
  if constexpr (KC + VC > 8) {  // wide heads: dV and dK + bias as two passes
    GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL((attn_bwd_bf16_dkv_kernel<KC, VC, T, WAVES, HB, 1, PRIV>), dim3(grid), dim3(64 * WAVES), lds, st, a));
    GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL((attn_bwd_bf16_dkv_kernel<KC, VC, T, WAVES, HB, 2, PRIV>), dim3(grid), dim3(64 * WAVES), lds, st, a));
  } else {
    GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL((attn_bwd_bf16_dkv_kernel<KC, VC, T, WAVES, HB, 0, PRIV>), dim3(grid), dim3(64 * WAVES), lds, st, a));
  }
}
template <int KC, int VC, int T, int WAVES, bool HB>
static void launch_dkv_bf16(const AttnBwdArgsBf16& a, int grid, size_t lds, hipStream_t st) {
  if (dkv_priv<WAVES>(a)) launch_dkv_bf16_p<KC, VC, T, WAVES, HB, true>(a, grid, lds, st);
  else launch_dkv_bf16_p<KC, VC, T, WAVES, HB, false>(a, grid, lds, st);
}

template <int KC, int VC, int T, int WAVES>
static int launch_bwd_bf16(AttnBwdArgsBf16 a, float* dpos_w, float* dts_w, hipStream_t st) {
  a.n_kt = ceil_div(a.max_len, 16 * WAVES);
  a.n_qt = ceil_div(a.max_len, 16 * WAVES);
  const int grid = a.n_kt * a.B * a.H;
  const size_t l_kv = dkv_lds<KC, VC, T, WAVES>(a, dkv_priv<WAVES>(a)), l_q = dq_lds<KC, VC, T>(a);
  GR_REQUIRE(l_kv <= 160 * 1024 && l_q <= 160 * 1024,
             "hstu_attn_bwd_bf16: LDS (%zu, %zu B) exceeds 160 KiB (N=%d)", l_kv, l_q, a.N);
  a.cus = (int64_t)grid <= 2 * device_cus() ? device_cus() : (1 << 30);
  // the dQ launch's first workgroups reduce the dK/dV launch's bias slabs
  if (a.map_kq) {
    const int nbias = ceil_div(2 * a.N - 1 + a.nb + 1, 16);
    launch_dkv_bf16<KC, VC, T, WAVES, true>(a, grid, l_kv, st);
    GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL((attn_bwd_bf16_dq_kernel<KC, VC, T, WAVES, true>), dim3(nbias + grid), dim3(64 * WAVES),
                                                   std::max(l_q, sizeof(float) * 64 * WAVES), st, a, nbias, dpos_w, dts_w));
  } else {
    launch_dkv_bf16<KC, VC, T, WAVES, false>(a, grid, l_kv, st);
    GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL((attn_bwd_bf16_dq_kernel<KC, VC, T, WAVES, false>), dim3(grid), dim3(64 * WAVES), l_q, st, a,
                                                   0, dpos_w, dts_w));
  }
  GR_LAUNCH_CHECK("hstu_attn_bwd_bf16");
  return 0;
}

static int bwd_bf16_waves(int d) { return d <= 64 ? 4 : 8; }

}  // namespace gr

// wide heads (128 < d <= 256, dqk == dv): hstu_attn_bf16w.hip
size_t gr_attn_bwd_bf16w_workspace(int B, int N, int max_len, int H, int d, int num_buckets,
                                   bool with_copies);
int gr_attn_bwd_bf16w(const float* q, const float* k, const float* v, int64_t ld_qk, int64_t ld_v,
                      const float* dout, int64_t ld_dout, const int64_t* offsets, int B, int N,
                      int max_len, int H, int d, const uint8_t* map_kq, const float* pos_w,
                      const float* ts_w, int num_buckets, const float* hq, const float* hk,
                      const float* hv, int64_t ld_h, float* dq, float* dk, float* dvv, int64_t ld_d,
                      float* dpos_w, float* dts_w, const void* copies, void* workspace, hipStream_t st);
static bool bwd_bf16_wide(int dqk, int dv) { return bf16_wide(dqk, dv); }

extern "C" size_t hstu_attn_bwd_bf16_workspace_size(int B, int N, int max_len, int H, int dqk,
                                                    int dv, int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0 || dqk <= 0 || dv <= 0) return 0;
  if (bwd_bf16_wide(dqk, dv)) return gr_attn_bwd_bf16w_workspace(B, N, max_len, H, dqk, num_buckets, false);
  const int d = dqk > dv ? dqk : dv;
  return gr::bwd_bf16_slab_bytes(B, N, max_len, H, num_buckets, 16 * gr::bwd_bf16_waves(d));
}

extern "C" size_t hstu_attn_bwd_bf16_workspace_size_copies(int B, int N, int max_len, int H, int dqk,
                                                           int dv, int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0 || dqk <= 0 || dv <= 0) return 0;
  if (bwd_bf16_wide(dqk, dv)) return gr_attn_bwd_bf16w_workspace(B, N, max_len, H, dqk, num_buckets, true);
  return hstu_attn_bwd_bf16_workspace_size(B, N, max_len, H, dqk, dv, num_buckets);
}

extern "C" int hstu_attn_bwd_bf16(const float* q, const float* k, const float* v, int64_t ld_qk,
                                  int64_t ld_v, const float* dout, int64_t ld_dout,
                                  const int64_t* offsets, int B, int N, int max_len, int H,
                                  int dqk, int dv, const uint8_t* bucket_map, const float* pos_w,
                                  const float* ts_w, int num_buckets, const float* hq,
                                  const float* hk, const float* hv, int64_t ld_h, float* dq,
                                  float* dk, float* dvv, int64_t ld_d, float* dpos_w,
                                  float* dts_w, const void* copies, void* workspace, size_t ws_bytes,
                                  void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && dout && offsets && dq && dk && dvv, "hstu_attn_bwd_bf16: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_bwd_bf16: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_bwd_bf16: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 256 && dv <= 256, "hstu_attn_bwd_bf16: dqk/dv > 256 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE((hq == nullptr) == (hk == nullptr) && (hk == nullptr) == (hv == nullptr),
             "hstu_attn_bwd_bf16: hq/hk/hv must be all given or all NULL");
  const int d = dqk > dv ? dqk : dv;
  // wide heads need the workspace with or without the bias (the dS blocks live there)
  const bool wide = bwd_bf16_wide(dqk, dv) &&
                    pair_aligned({q, k, v, dout}, {ld_qk, ld_v, ld_dout, (int64_t)dqk, hq ? ld_h : 0});
  if (bucket_map) {
    GR_REQUIRE(pos_w && ts_w && dpos_w && dts_w && num_buckets > 0 && num_buckets < 256,
               "hstu_attn_bwd_bf16: bucket_map given without pos_w/ts_w/dpos_w/dts_w");
  }
  if (bucket_map || wide) {
    const size_t need = wide ? gr_attn_bwd_bf16w_workspace(B, N, max_len, H, dqk, num_buckets,
                                                           copies != nullptr)
                             : bwd_bf16_slab_bytes(B, N, max_len, H, num_buckets, 16 * bwd_bf16_waves(d));
    GR_REQUIRE(B == 0 || max_len == 0 || (workspace && ws_bytes >= need),
               "hstu_attn_bwd_bf16: workspace %zu B < %zu B", ws_bytes, need);
  }
  hipStream_t st = (hipStream_t)stream;
  if (B == 0 || max_len == 0) {
    if (bucket_map) {
      zero_words_async(dpos_w, 2 * N - 1, st);
      zero_words_async(dts_w, num_buckets + 1, st);
    }
    return 0;
  }
  const uint8_t* map_kq =
      bucket_map ? bucket_map + (size_t)B * attn_tiles_per_seq(N) * 4096 : nullptr;
  if (wide)
    return gr_attn_bwd_bf16w(q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, max_len, H, dqk,
                             map_kq, pos_w, ts_w, num_buckets, hq, hk, hv, ld_h, dq, dk, dvv, ld_d,
                             dpos_w, dts_w, copies, workspace, st);
  AttnBwdArgsBf16 a{q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, H, dqk, dv, max_len,
                    bucket_map, map_kq, pos_w, ts_w, bucket_map ? num_buckets : 0, hq, hk, hv,
                    ld_h, dq, dk, dvv, ld_d, bucket_map ? (float*)workspace : nullptr,
                    1.0f / (float)N, 0, 0, 0};
  if (d <= 32) return launch_bwd_bf16<1, 1, 64, 4>(a, dpos_w, dts_w, st);
  if (d <= 64) return launch_bwd_bf16<2, 2, 64, 4>(a, dpos_w, dts_w, st);
  if (d <= 128) return launch_bwd_bf16<4, 4, 32, 8>(a, dpos_w, dts_w, st);
  return launch_bwd_bf16<8, 8, 32, 8>(a, dpos_w, dts_w, st);
}
