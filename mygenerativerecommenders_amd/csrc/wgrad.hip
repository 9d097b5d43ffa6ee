// Weight gradients of the STU projections — gfx950, f32 MFMA.
//
//   C[ka][nb] = sum_m A'(m, ka) * Bm(m, nb),   A' = A or LayerNorm(A) from saved stats,
//   optional colsum[ka] = sum_m A'(m, ka)  (the bias gradient of _o).
// Replaces the mm-backward weight terms of reference hstu.py:303 (_uvqk) and
// hstu.py:404-413 (_o.weight, _o.bias).
//
// One launch computes BOTH weight gradients of a layer (the _uvqk and _o GEMMs are
// independent problems over the same jagged rows): grid = (row splits) x (output panels
// of problem 0, then of problem 1), and one reduce launch sums both problems' slabs.
// Split-K over rows: a workgroup streams its rows through LDS in chunks of 32 with the
// loads of WG_SUPER chunks in flight together (one HBM round trip per 4 chunks instead of
// one per chunk), and wave w accumulates ka-tile w & 3 of the panel against all NT
// nb-tiles over the k-steps of half w >> 2.  The column sum comes for free from a
// ones-column appended to Bm (padding column Nb).  Each split writes its panel to a
// workspace slab; wgrad_reduce sums the slabs in a fixed order (deterministic, no
// atomics) with 16 slab groups per output in parallel.
// The column sum (colsum, the _o bias gradient) is accumulated from the A operand the
// waves of the first nb-panel already hold (one add per k-step, a fixed-order lane and
// half reduction) and written as slab column Nb: no padding panel carries it (at C3 the
// ones column of Nb = 256 + 1 cost a second, all-padding panel of 256 columns).
#include "attn_common.h"
#include "mfma32.h"

#include "../../include/gr_hstu.h"

namespace gr {

constexpr int WG_KA = 64;   // ka rows per panel (4 waves x 16)
constexpr int WG_CH = 32;   // rows per chunk (8 MFMA k-steps)
constexpr int WG_SUPER = 4; // chunks whose loads are issued together
constexpr int WG_LDA = WG_KA + 16;  // == 16 mod 32: lane groups (4 rows apart) hit disjoint banks
constexpr int WG_THREADS = 512;     // 8 waves: wave w owns ka-tile w & 3, k-steps of half w >> 2

struct WgradProb {
  const float* a;
  int64_t lda;
  const float2* a_stats;
  const float* bm;
  int64_t ldb;
  int Ka, Nb, NC;     // NC = Nb (+1 with the ones column)
  int panels, panels_nb;
  float* slabs;       // [split][Ka][NC]
  float* c;           // reduce outputs
  float* colsum;
  int a16, b16;       // gr_wgrad_multi_a16: A / B rows are bf16 (the wide bf16 tile only)
};

// Up to WG_MAXP problems per launch (a layer's two, or every layer's of an encoder at
// once: gr_wgrad_multi).  Problems come in two panel classes (kind 0 / 1: NT0 / NT1 of
// the narrow kernels); pan0 / blk0 are the prefix sums of panels / reduce blocks.
constexpr int WG_MAXP = 16;
struct WgradArgs {
  WgradProb p[WG_MAXP];
  int np;
  int kind[WG_MAXP];
  int pan0[WG_MAXP + 1];
  int blk0[WG_MAXP + 1];
  const int64_t* offsets;
  int B;
  int64_t rows_per_split;
  int n_splits;
  int blkf0[WG_MAXP + 1];  // prefix of 256-output blocks (wgrad_reduce_few_kernel)
};

// problem owning item x of a prefix table (scalar: kernel arguments are wave-uniform)
__device__ __forceinline__ int wg_find(const int* pre, int np, int x) {
  int i = 0;
  while (i + 1 < np && x >= pre[i + 1]) ++i;
  return i;
}

// sum of a lane's partial column sum over its 4 lane groups (lanes lr, lr + 16, lr + 32,
// lr + 48 hold rows of the same column), fixed order
__device__ __forceinline__ float wg_colsum_lanes(float v) {
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int NT>
struct WgCfg {
  static constexpr int NP = NT * 16;
  static constexpr int LDB = (NP % 32 == 16) ? NP : NP + 16;  // == 16 mod 32
  static constexpr int NP2 = NP <= 64 ? 64 : NP <= 128 ? 128 : 256;  // staging column span
  static constexpr int BRPP = WG_THREADS / NP2;                   // B rows per pass
  static constexpr int BPER = WG_CH / BRPP;                       // B loads per thread
  static constexpr int APER = WG_CH * WG_KA / WG_THREADS;         // A loads per thread
  // chunks in flight: 4 at every panel width (NT 13: 211 VGPRs, NT 16: 230, no spills; the
  // workgroup is one per CU either way, 8 waves x > 128 VGPRs).  Two at NT 13/16 left one
  // chunk of MFMA work (~1.4 us) to cover each chunk's HBM round trip (~4.6 us at C2)
  static constexpr int SUPER = WG_SUPER;
  static constexpr size_t LDS = sizeof(float) * 2 * WG_CH * (WG_LDA + LDB + 2);
  static_assert(LDS >= sizeof(float) * (4 * NT * 4 * 64 + 4 * 16), "exchange area");
};

template <int NT>
__device__ __forceinline__ void wgrad_panel(const WgradProb& g, const int64_t* offsets, int B,
                                            int64_t rows_per_split, int split, int panel,
                                            char* smem) {
  using C = WgCfg<NT>;
  float (*As)[WG_CH * WG_LDA] = reinterpret_cast<float (*)[WG_CH * WG_LDA]>(smem);
  float (*Bs)[WG_CH * C::LDB] =
      reinterpret_cast<float (*)[WG_CH * C::LDB]>(smem + sizeof(float) * 2 * WG_CH * WG_LDA);
  // per-row LayerNorm (mean, rstd) of the chunk, applied as A is read (rows past the
  // split: (0, 0), so their zero A stays zero)
  float2 (*Ss)[WG_CH] = reinterpret_cast<float2 (*)[WG_CH]>(
      smem + sizeof(float) * 2 * WG_CH * (WG_LDA + C::LDB));
  const int pa = panel / g.panels_nb, pb = panel % g.panels_nb;
  const int ka0 = pa * WG_KA, nb0 = pb * C::NP;
  const int64_t total = offsets[B];
  const int64_t r0 = (int64_t)split * rows_per_split;
  const int64_t r1 = min(total, r0 + rows_per_split);
  const int tid = threadIdx.x, wv = wave_id(), lane = tid & 63;
  const int w = wv & 3, half = wv >> 2;
  const int lr = lane & 15, lg = lane >> 4;
  // wave-uniform (offsets[B] is loaded per lane; readfirstlane keeps the chunk loop and
  // its guards scalar instead of exec-mask branches around every load)
  const int n_ch = __builtin_amdgcn_readfirstlane(r1 > r0 ? (int)((r1 - r0 + WG_CH - 1) / WG_CH) : 0);

  // descriptors over this split's rows: rows past r1 load as 0
  const int64_t nrows = r1 > r0 ? r1 - r0 : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.a + r0 * g.lda), 0, nrows ? (int)(((nrows - 1) * g.lda + g.Ka) * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.bm + r0 * g.ldb), 0, nrows ? (int)(((nrows - 1) * g.ldb + g.Nb) * 4) : 0, 0x00020000);

  // staging coordinates
  const int ac = tid & 63, ar = tid >> 6;               // A: col ka0 + ac, rows ar + 8i
  const int bc = tid % C::NP2, br = tid / C::NP2;       // B: col nb0 + bc, rows br + BRPP i
  const int aka = ka0 + ac, bnb = nb0 + bc;
  const bool a_ok = aka < g.Ka;
  const bool b_in = bnb < g.Nb;
  const bool do_cs = g.NC > g.Nb && pb == 0;  // this panel also sums A' over its rows
  float csum = 0.f;
  float ra_v[C::SUPER][C::APER], rb_v[C::SUPER][C::BPER];
  float2 st_v[C::SUPER];
  auto load = [&](int u, int ch) {
    const int rr0 = ch * WG_CH;
#pragma unroll
    for (int i = 0; i < C::APER; ++i) {
      const int rr = rr0 + ar + (WG_THREADS / 64) * i;
      ra_v[u][i] = buf_ld(ra, a_ok ? (int)((rr * g.lda + aka) * 4) : OOB_OFF, 0);
    }
    if (g.a_stats && tid < WG_CH) st_v[u] = ld_f2(g.a_stats, min(r0 + rr0 + tid, total - 1));
#pragma unroll
    for (int i = 0; i < C::BPER; ++i) {
      const int rr = rr0 + br + C::BRPP * i;
      rb_v[u][i] = buf_ld(rb, b_in ? (int)((rr * g.ldb + bnb) * 4) : OOB_OFF, 0);
    }
  };
  auto store = [&](int u, int buf, int ch) {
    const int rr0 = ch * WG_CH;
#pragma unroll
    for (int i = 0; i < C::APER; ++i) {
      const int rr = ar + (WG_THREADS / 64) * i;
      As[buf][rr * WG_LDA + ac] = (a_ok && r0 + rr0 + rr < r1) ? ra_v[u][i] : 0.f;
    }
    if (tid < WG_CH)
      Ss[buf][tid] = g.a_stats && r0 + rr0 + tid < r1 ? st_v[u] : make_float2(0.f, 1.f);
    if (bc < C::NP) {
#pragma unroll
      for (int i = 0; i < C::BPER; ++i) {
        const int rr = br + C::BRPP * i;
        Bs[buf][rr * C::LDB + bc] = rb_v[u][i];  // rows past r1 meet a zero A
      }
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  // SUPER register slots rotate over the chunks: chunk c is staged from slot c % SUPER
  // into LDS buffer c & 1, and the slot is refilled with chunk c + SUPER right away, so
  // SUPER - 1 chunks of compute cover each load (issuing a whole super-chunk's loads only
  // after the previous one was computed exposed one HBM round trip per SUPER chunks:
  // C2 rows-per-split sweeps showed ~4.6 us per chunk against ~1.4 us of MFMA).  One
  // barrier per chunk: the store into a buffer follows the barrier after the previous
  // chunk's store, which every wave reaches only after computing on that buffer two
  // chunks ago.
#pragma unroll
  for (int u = 0; u < C::SUPER; ++u)
    if (u < n_ch) load(u, u);
  for (int sc = 0; sc < n_ch; sc += C::SUPER) {
#pragma unroll
    for (int u = 0; u < C::SUPER; ++u) {
      if (sc + u < n_ch) {
        const int ch = sc + u, buf = ch & 1;
        store(u, buf, ch);
        if (ch + C::SUPER < n_ch) load(u, ch + C::SUPER);
        __syncthreads();
        const float* Ab = As[buf];
        const float* Bb = Bs[buf];
        const float2* Sb = Ss[buf];
        // operands of k-step ks + 1 are read from LDS while the MFMAs of ks run (one
        // read -> wait -> MFMA round trip per operand otherwise)
        constexpr int KS = WG_CH / 8;
        const int ks0 = half * KS;
        float av[2], bv[2][NT];
        float2 sv[2];
        auto rd = [&](int slot, int ks) {
          sv[slot] = Sb[4 * ks + lg];
          av[slot] = Ab[(4 * ks + lg) * WG_LDA + 16 * w + lr];
#pragma unroll
          for (int t = 0; t < NT; ++t) bv[slot][t] = Bb[(4 * ks + lg) * C::LDB + 16 * t + lr];
        };
        rd(0, ks0);
#pragma unroll
        for (int j = 0; j < KS; ++j) {
          if (j + 1 < KS) rd((j + 1) & 1, ks0 + j + 1);
          __builtin_amdgcn_sched_barrier(0);
          const float a = (av[j & 1] - sv[j & 1].x) * sv[j & 1].y;
          if (do_cs) csum += a;  // A'[row 4ks + lg][ka 16w + lr]
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(a, bv[j & 1][t], acc[t]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
  __syncthreads();  // LDS is reused for the exchange below
  // the two halves' partial sums meet in LDS (fixed order: half 0 + half 1)
  float* xch = reinterpret_cast<float*>(smem);  // [4 waves][NT][4][64], then [4][16] colsums
  if (do_cs) csum = wg_colsum_lanes(csum);
  if (half == 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[((w * NT + t) * 4 + r) * 64 + lane] = acc[t][r];
    if (do_cs && lg == 0) xch[4 * NT * 4 * 64 + 16 * w + lr] = csum;
  }
  __syncthreads();
  if (half == 1) return;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[t][r] += xch[((w * NT + t) * 4 + r) * 64 + lane];
  // acc[t][r] = C[ka0 + 16w + 4lg + r][nb0 + 16t + lr]
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
  if (do_cs && lg == 0 && ka0 + 16 * w + lr < g.Ka)
    slab[(int64_t)(ka0 + 16 * w + lr) * g.NC + g.Nb] = csum + xch[4 * NT * 4 * 64 + 16 * w + lr];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ka = ka0 + 16 * w + 4 * lg + r;
    if (ka >= g.Ka) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int nb = nb0 + 16 * t + lr;
      if (nb < g.Nb) slab[(int64_t)ka * g.NC + nb] = acc[t][r];  // column Nb: colsum above
    }
  }
}

template <int NT0, int NT1>
__global__ __launch_bounds__(WG_THREADS) void wgrad_partial_kernel(WgradArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int panel = blockIdx.y;
  const int i = wg_find(g.pan0, g.np, panel);
  if (g.kind[i] == 0)
    wgrad_panel<NT0>(g.p[i], g.offsets, g.B, g.rows_per_split, blockIdx.x, panel - g.pan0[i], smem);
  else
    wgrad_panel<NT1>(g.p[i], g.offsets, g.B, g.rows_per_split, blockIdx.x, panel - g.pan0[i], smem);
}

// ---------------------------------------------------------------------------- bf16
// bf16-operand panel (autocast_dtype = bfloat16), v_mfma_f32_16x16x32_bf16.  Chunks of
// WGB_CH = 64 rows; both operands are staged TRANSPOSED as bf16 images (A'^T [ka][row]
// with the LayerNorm applied in fp32 before rounding, Bm^T [nb][row]) so a lane's 8
// consecutive rows are one 16-byte LDS read.  A thread stages 8 consecutive rows of one
// A column (8 coalesced row loads, one 16-byte LDS store) and RB consecutive rows of one
// B column.  Wave w: ka-tile w & 3, k-step (rows 32 half .. +31) of half w >> 2; the
// halves and the slab write are as in the f32 panel.
constexpr int WGB_CH = 64;
constexpr int WGB_LDT = WGB_CH + 8;  // bf16 per image row: 144 B, 16 lanes -> 16 bank groups

template <int NT>
struct WgCfgB {
  static constexpr int NP = NT * 16;
  static constexpr int NP2 = NP <= 64 ? 64 : NP <= 128 ? 128 : 256;
  static constexpr int BG = WG_THREADS / NP2;  // row groups of the B image
  static constexpr int RB = WGB_CH / BG;       // B rows per thread (8, 16, 32)
  static constexpr size_t STAGE = 2 * (size_t)WGB_LDT * (WG_KA + NP);
  static constexpr size_t XCH = sizeof(float) * (4 * NT * 4 * 64 + 4 * 16);
  static constexpr size_t LDS = STAGE > XCH ? STAGE : XCH;
};

template <int NT>
__device__ __forceinline__ void wgrad_panel_bf16(const WgradProb& g, const int64_t* offsets, int B,
                                                 int64_t rows_per_split, int split, int panel,
                                                 char* smem) {
  using C = WgCfgB<NT>;
  __bf16* At = reinterpret_cast<__bf16*>(smem);   // [WG_KA][WGB_LDT]
  __bf16* Bt = At + WG_KA * WGB_LDT;               // [NP][WGB_LDT]
  const int pa = panel / g.panels_nb, pb = panel % g.panels_nb;
  const int ka0 = pa * WG_KA, nb0 = pb * C::NP;
  const int64_t total = offsets[B];
  const int64_t r0 = (int64_t)split * rows_per_split;
  const int64_t r1 = min(total, r0 + rows_per_split);
  const int tid = threadIdx.x, wv = wave_id(), lane = tid & 63;
  const int w = wv & 3, half = wv >> 2;
  const int lr = lane & 15, lg = lane >> 4;
  const int n_ch = __builtin_amdgcn_readfirstlane(r1 > r0 ? (int)((r1 - r0 + WGB_CH - 1) / WGB_CH) : 0);
  const int64_t nrows = r1 > r0 ? r1 - r0 : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.a + r0 * g.lda), 0, nrows ? (int)(((nrows - 1) * g.lda + g.Ka) * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.bm + r0 * g.ldb), 0, nrows ? (int)(((nrows - 1) * g.ldb + g.Nb) * 4) : 0, 0x00020000);
  const int ac = tid & 63, ag = tid >> 6;            // A: column ka0 + ac, rows 8 ag .. +7
  const int bc = tid % C::NP2, bg = tid / C::NP2;    // B: column nb0 + bc, rows RB bg .. +RB-1
  const int aka = ka0 + ac, bnb = nb0 + bc;
  const bool a_ok = aka < g.Ka;
  const bool b_in = bnb < g.Nb;
  const bool do_cs = g.NC > g.Nb && pb == 0;  // this panel also sums bf16(A') over its rows
  float csum = 0.f;
  float av_[8], bv_[C::RB];
  float2 sv_[8];
  auto load = [&](int ch) {
    const int rr0 = ch * WGB_CH;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = rr0 + 8 * ag + i;
      av_[i] = buf_ld(ra, a_ok ? (int)((rr * g.lda + aka) * 4) : OOB_OFF, 0);
      sv_[i] = g.a_stats ? ld_f2(g.a_stats, min(r0 + rr, total - 1)) : make_float2(0.f, 1.f);
    }
#pragma unroll
    for (int i = 0; i < C::RB; ++i) {
      const int rr = rr0 + C::RB * bg + i;
      bv_[i] = buf_ld(rb, b_in ? (int)((rr * g.ldb + bnb) * 4) : OOB_OFF, 0);
    }
  };
  auto store = [&](int ch) {
    const int rr0 = ch * WGB_CH;
    uint32_t pk[4];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      const bool ok0 = a_ok && r0 + rr0 + 8 * ag + i < r1, ok1 = a_ok && r0 + rr0 + 8 * ag + i + 1 < r1;
      pk[i / 2] = pack_bf16(ok0 ? (av_[i] - sv_[i].x) * sv_[i].y : 0.f,
                            ok1 ? (av_[i + 1] - sv_[i + 1].x) * sv_[i + 1].y : 0.f);
    }
    *reinterpret_cast<u32x4_t*>(At + ac * WGB_LDT + 8 * ag) = u32x4_t{pk[0], pk[1], pk[2], pk[3]};
    if (bc < C::NP) {
#pragma unroll
      for (int q = 0; q < C::RB; q += 8) {
        uint32_t pb2[4];
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          pb2[i / 2] = pack_bf16(bv_[q + i], bv_[q + i + 1]);  // rows past r1 meet a zero A
        }
        *reinterpret_cast<u32x4_t*>(Bt + bc * WGB_LDT + C::RB * bg + q) =
            u32x4_t{pb2[0], pb2[1], pb2[2], pb2[3]};
      }
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  if (n_ch > 0) load(0);
  for (int ch = 0; ch < n_ch; ++ch) {
    store(ch);
    __syncthreads();
    if (ch + 1 < n_ch) load(ch + 1);  // next chunk's rows fly during the MFMAs
    const int k0 = 32 * half + 8 * lg;
    const u32x4_t a = *reinterpret_cast<const u32x4_t*>(At + (16 * w + lr) * WGB_LDT + k0);
    if (do_cs) {  // the 8 rounded values of rows k0 .. k0 + 7, column ka 16w + lr
#pragma unroll
      for (int e = 0; e < 4; ++e)
        csum += __uint_as_float(a[e] << 16) + __uint_as_float(a[e] & 0xffff0000u);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const u32x4_t b = *reinterpret_cast<const u32x4_t*>(Bt + (16 * t + lr) * WGB_LDT + k0);
      acc[t] = mfma_bf16(a, b, acc[t]);
    }
    __syncthreads();
  }
  // the two halves' partial sums meet in LDS (fixed order: half 0 + half 1)
  float* xch = reinterpret_cast<float*>(smem);  // [4 waves][NT][4][64], then [4][16] colsums
  if (do_cs) csum = wg_colsum_lanes(csum);
  if (half == 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[((w * NT + t) * 4 + r) * 64 + lane] = acc[t][r];
    if (do_cs && lg == 0) xch[4 * NT * 4 * 64 + 16 * w + lr] = csum;
  }
  __syncthreads();
  if (half == 1) return;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[t][r] += xch[((w * NT + t) * 4 + r) * 64 + lane];
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
  if (do_cs && lg == 0 && ka0 + 16 * w + lr < g.Ka)
    slab[(int64_t)(ka0 + 16 * w + lr) * g.NC + g.Nb] = csum + xch[4 * NT * 4 * 64 + 16 * w + lr];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ka = ka0 + 16 * w + 4 * lg + r;
    if (ka >= g.Ka) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int nb = nb0 + 16 * t + lr;
      if (nb < g.Nb) slab[(int64_t)ka * g.NC + nb] = acc[t][r];  // column Nb: colsum above
    }
  }
}

template <int NT0, int NT1>
__global__ __launch_bounds__(WG_THREADS) void wgrad_partial_bf16_kernel(WgradArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int panel = blockIdx.y;
  const int i = wg_find(g.pan0, g.np, panel);
  if (g.kind[i] == 0)
    wgrad_panel_bf16<NT0>(g.p[i], g.offsets, g.B, g.rows_per_split, blockIdx.x, panel - g.pan0[i], smem);
  else
    wgrad_panel_bf16<NT1>(g.p[i], g.offsets, g.B, g.rows_per_split, blockIdx.x, panel - g.pan0[i], smem);
}

// ------------------------------------------------------------------ bf16, wide (Ka <= 256)
// 256 (ka) x 256 (nb) output tile per workgroup, v_mfma_f32_32x32x16_bf16: A is read once
// per nb tile instead of once per 64-wide ka panel and B once instead of once per ka panel
// (C3 _uvqk: 0.67 GB of operand traffic per layer instead of 1.7 GB).  Chunks of 32 rows:
// each thread loads 4 float4 of A and 4 of B (one chunk ahead, in registers), applies the
// LayerNorm to A in fp32, rounds both to bf16 and writes row-major LDS tiles; the MFMA
// operands are transposed reads of those tiles (A^T: lanes = ka; B: lanes = nb, both with
// k = rows).  Wave w: ka rows 64 (w & 3) .. +63, nb columns 128 (w >> 2) .. +127 (8 tiles).
constexpr int WGW_T = 256;            // tile edge
constexpr int WGW_RS = WGW_T + 8;     // LDS row stride (bf16)
constexpr size_t WGW_LDS = 2 * 2 * 32 * WGW_RS * 2;

// A16 / B16: that operand's rows are bf16 in HBM (gr_wgrad_multi_a16): a thread loads its 4
// columns as one 8-byte piece and writes the bits to LDS unchanged (A16 has no row stats)
template <bool A16, bool B16>
__device__ __forceinline__ void wgrad_tile_bf16w(const WgradProb& g, const int64_t* offsets, int B,
                                                 int64_t rows_per_split, int split, int tile,
                                                 char* smem) {
  __bf16* lds = reinterpret_cast<__bf16*>(smem);  // [2 buffers][A, B][32][WGW_RS]
  const int nb0 = tile * WGW_T;
  const int64_t total = offsets[B];
  const int64_t r0 = (int64_t)split * rows_per_split;
  const int64_t r1 = min(total, r0 + rows_per_split);
  const int tid = threadIdx.x, wv = wave_id(), lane = tid & 63;
  const int n_ch = __builtin_amdgcn_readfirstlane(r1 > r0 ? (int)((r1 - r0 + 31) / 32) : 0);
  const int64_t nrows = r1 > r0 ? r1 - r0 : 0;
  constexpr int EA = A16 ? 2 : 4, EB = B16 ? 2 : 4;  // bytes per element
  const char* abase = (const char*)g.a + r0 * g.lda * EA;
  const char* bbase = (const char*)g.bm + r0 * g.ldb * EB;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)abase, 0, nrows ? (int)(((nrows - 1) * g.lda + g.Ka) * EA) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)bbase, 0, nrows ? (int)(((nrows - 1) * g.ldb + g.Nb) * EB) : 0, 0x00020000);
  // staging: thread t owns columns 4 (t % 64) .. +3 of rows t / 64 + 8 i (i < 4)
  const int sc = 4 * (tid & 63), sr = tid >> 6;
  const bool a_ok = sc < g.Ka, b_ok = nb0 + sc < g.Nb;  // Ka, Nb multiples of 4 (host check)
  const int aoff = a_ok ? sc * EA : OOB_OFF, boff = b_ok ? (nb0 + sc) * EB : OOB_OFF;
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v av[A16 ? 1 : 4], bv[B16 ? 1 : 4];
  u32x2_t ah[A16 ? 4 : 1], bh[B16 ? 4 : 1];
  float2 stv[4];
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = 32 * ch + sr + 8 * i;
      if constexpr (A16)
        ah[i] = __builtin_amdgcn_raw_buffer_load_b64(ra, aoff + rr * (int)g.lda * 2, 0, 0);
      else
        av[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff + rr * (int)g.lda * 4, 0, 0));
      if constexpr (B16)
        bh[i] = __builtin_amdgcn_raw_buffer_load_b64(rb, boff + rr * (int)g.ldb * 2, 0, 0);
      else
        bv[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rb, boff + rr * (int)g.ldb * 4, 0, 0));
      if constexpr (!A16) stv[i] = g.a_stats ? ld_f2(g.a_stats, min(r0 + rr, total - 1)) : make_float2(0.f, 1.f);
    }
  };
  const bool do_cs = g.NC > g.Nb && tile == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};  // bf16(A') column sums of this thread's 4 columns
  auto store = [&](int ch, int buf) {
    __bf16* At = lds + buf * 2 * 32 * WGW_RS;
    __bf16* Bt = At + 32 * WGW_RS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = sr + 8 * i;
      const bool ok = r0 + 32 * ch + rr < r1;
      uint32_t p0, p1;
      if constexpr (A16) {  // rows >= r1 read 0 (descriptor range)
        p0 = ah[i].x;
        p1 = ah[i].y;
      } else {
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = ok ? (av[A16 ? 0 : i][e] - stv[i].x) * stv[i].y : 0.f;
        p0 = pack_bf16(x[0], x[1]);
        p1 = pack_bf16(x[2], x[3]);
      }
      if (do_cs) {
        cs[0] += __uint_as_float(p0 << 16);
        cs[1] += __uint_as_float(p0 & 0xffff0000u);
        cs[2] += __uint_as_float(p1 << 16);
        cs[3] += __uint_as_float(p1 & 0xffff0000u);
      }
      *reinterpret_cast<u32x2_t*>(At + rr * WGW_RS + sc) = u32x2_t{p0, p1};
      if constexpr (B16)
        *reinterpret_cast<u32x2_t*>(Bt + rr * WGW_RS + sc) = bh[i];
      else  // rows past r1 meet a zero A
        *reinterpret_cast<u32x2_t*>(Bt + rr * WGW_RS + sc) =
            u32x2_t{pack_bf16(bv[B16 ? 0 : i][0], bv[B16 ? 0 : i][1]),
                    pack_bf16(bv[B16 ? 0 : i][2], bv[B16 ? 0 : i][3])};
    }
  };
  const int wka = 64 * (wv & 3), wnb = 128 * (wv >> 2);
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f16_zero();
  if (n_ch > 0) {
    load(0);
    store(0, 0);
  }
  __syncthreads();
  for (int ch = 0; ch < n_ch; ++ch) {
    const bool more = ch + 1 < n_ch;
    if (more) load(ch + 1);  // the next chunk's rows fly during the MFMAs
    const __bf16* At = lds + (ch & 1) * 2 * 32 * WGW_RS;
    const __bf16* Bt = At + 32 * WGW_RS;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4_t af[2], bf[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = trB_nat(At, WGW_RS, s, wka + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = trB_nat(Bt, WGW_RS, s, wnb + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(af[i], bf[j], acc[i][j]);
    }
    if (more) store(ch + 1, (ch + 1) & 1);
    __syncthreads();
  }
  // acc[i][j][rr] = C[ka wka + 32 i + (rr & 3) + 8 (rr >> 2) + 4 (lane >> 5)][nb nb0 + wnb + 32 j + lane % 32]
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int ka = wka + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
      if (ka >= g.Ka) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nb = nb0 + wnb + 32 * j + lr;
        if (nb < g.Nb) slab[(int64_t)ka * g.NC + nb] = acc[i][j][rr];
      }
    }
  if (do_cs) {  // the 8 row groups' partial column sums, added in wave order
    float* xs = reinterpret_cast<float*>(smem);  // [8][256]
#pragma unroll
    for (int e = 0; e < 4; ++e) xs[sr * WGW_T + sc + e] = cs[e];
    __syncthreads();
    if (tid < WGW_T && tid < g.Ka) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += xs[r * WGW_T + tid];
      slab[(int64_t)tid * g.NC + g.Nb] = t;
    }
  }
}

// fp32 form of the same tile (gr_wgrad2 at wide heads): v_mfma_f32_32x32x2_f32 straight
// from fp32 LDS tiles (A' with the LayerNorm applied, B), 16-row chunks; an A (B) fragment
// is one float per lane: row 2 s + lane / 32, column lane % 32 of the tile.
constexpr int WGF_CH = 16;
constexpr size_t WGF_LDS = 2 * 2 * WGF_CH * WGW_T * 4;

__device__ __forceinline__ f32x16 mfma32f(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void wgrad_tile_f32w(const WgradProb& g, const int64_t* offsets, int B,
                                                int64_t rows_per_split, int split, int tile,
                                                char* smem) {
  float* lds = reinterpret_cast<float*>(smem);  // [2 buffers][A, B][WGF_CH][256]
  const int nb0 = tile * WGW_T;
  const int64_t total = offsets[B];
  const int64_t r0 = (int64_t)split * rows_per_split;
  const int64_t r1 = min(total, r0 + rows_per_split);
  const int tid = threadIdx.x, wv = wave_id(), lane = tid & 63;
  const int n_ch = __builtin_amdgcn_readfirstlane(r1 > r0 ? (int)((r1 - r0 + WGF_CH - 1) / WGF_CH) : 0);
  const int64_t nrows = r1 > r0 ? r1 - r0 : 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.a + r0 * g.lda), 0, nrows ? (int)(((nrows - 1) * g.lda + g.Ka) * 4) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.bm + r0 * g.ldb), 0, nrows ? (int)(((nrows - 1) * g.ldb + g.Nb) * 4) : 0, 0x00020000);
  // staging: thread t owns columns 4 (t % 64) .. +3 of rows t / 64 + 8 i (i < 2)
  const int sc = 4 * (tid & 63), sr = tid >> 6;
  const bool a_ok = sc < g.Ka, b_ok = nb0 + sc < g.Nb;
  const int aoff = a_ok ? sc * 4 : OOB_OFF, boff = b_ok ? (nb0 + sc) * 4 : OOB_OFF;
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v av[2], bv[2];
  float2 stv[2];
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = WGF_CH * ch + sr + 8 * i;
      av[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff + rr * (int)g.lda * 4, 0, 0));
      bv[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rb, boff + rr * (int)g.ldb * 4, 0, 0));
      stv[i] = g.a_stats ? ld_f2(g.a_stats, min(r0 + rr, total - 1)) : make_float2(0.f, 1.f);
    }
  };
  const bool do_cs = g.NC > g.Nb && tile == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  auto store = [&](int ch, int buf) {
    float* At = lds + buf * 2 * WGF_CH * WGW_T;
    float* Bt = At + WGF_CH * WGW_T;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = sr + 8 * i;
      const bool ok = r0 + WGF_CH * ch + rr < r1;
      f4v x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = ok ? (av[i][e] - stv[i].x) * stv[i].y : 0.f;
        if (do_cs) cs[e] += x[e];
      }
      *reinterpret_cast<f4v*>(At + rr * WGW_T + sc) = x;
      *reinterpret_cast<f4v*>(Bt + rr * WGW_T + sc) = bv[i];  // rows past r1 meet a zero A
    }
  };
  const int wka = 64 * (wv & 3), wnb = 128 * (wv >> 2);
  const int lr = lane & 31, lh = lane >> 5;
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f16_zero();
  if (n_ch > 0) {
    load(0);
    store(0, 0);
  }
  __syncthreads();
  for (int ch = 0; ch < n_ch; ++ch) {
    const bool more = ch + 1 < n_ch;
    if (more) load(ch + 1);
    const float* At = lds + (ch & 1) * 2 * WGF_CH * WGW_T + lh * WGW_T + lr;
    const float* Bt = At + WGF_CH * WGW_T;
#pragma unroll
    for (int s = 0; s < WGF_CH / 2; ++s) {
      float af[2], bf[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = At[2 * s * WGW_T + wka + 32 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = Bt[2 * s * WGW_T + wnb + 32 * j];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32f(af[i], bf[j], acc[i][j]);
    }
    if (more) store(ch + 1, (ch + 1) & 1);
    __syncthreads();
  }
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int ka = wka + 32 * i + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
      if (ka >= g.Ka) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nb = nb0 + wnb + 32 * j + lr;
        if (nb < g.Nb) slab[(int64_t)ka * g.NC + nb] = acc[i][j][rr];
      }
    }
  if (do_cs) {
    float* xs = reinterpret_cast<float*>(smem);  // [8][256]
#pragma unroll
    for (int e = 0; e < 4; ++e) xs[sr * WGW_T + sc + e] = cs[e];
    __syncthreads();
    if (tid < WGW_T && tid < g.Ka) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += xs[r * WGW_T + tid];
      slab[(int64_t)tid * g.NC + g.Nb] = t;
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(WG_THREADS) void wgrad_partial_wide_kernel(WgradArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int P = g.pan0[g.np];
  const int x = blockIdx.x & 7, sl = blockIdx.x >> 3;
  const int split = (sl / P) * 8 + x, tile = sl % P;
  if (split >= g.n_splits) return;
  const int i = wg_find(g.pan0, g.np, tile);
  const WgradProb& p = g.p[i];
  const int t = tile - g.pan0[i];
  if (BF16) {
    if (p.a16) {
      if (p.b16) wgrad_tile_bf16w<true, true>(p, g.offsets, g.B, g.rows_per_split, split, t, smem);
      else wgrad_tile_bf16w<true, false>(p, g.offsets, g.B, g.rows_per_split, split, t, smem);
    } else {
      if (p.b16) wgrad_tile_bf16w<false, true>(p, g.offsets, g.B, g.rows_per_split, split, t, smem);
      else wgrad_tile_bf16w<false, false>(p, g.offsets, g.B, g.rows_per_split, split, t, smem);
    }
  } else {
    wgrad_tile_f32w(p, g.offsets, g.B, g.rows_per_split, split, t, smem);
  }
}

// out = sum over splits (fixed order): a workgroup owns 16 outputs of one problem; thread
// (o, grp) sums splits grp, grp+16, ... 8-deep, then the 16 partials are added in grp
// order.  Blocks [blk0[i], blk0[i + 1]) reduce problem i.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WgradArgs g) {
  __shared__ float part[16][17];
  const int pi = wg_find(g.blk0, g.np, blockIdx.x);
  const WgradProb& p = g.p[pi];
  const int blk = blockIdx.x - g.blk0[pi];
  const int64_t ne = (int64_t)p.Ka * p.NC;
  const int o = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blk * 16 + o;
  const int64_t ic = i < ne ? i : ne - 1;
  gptr<float> src = as_global(p.slabs);
  const int n_splits = g.n_splits;
  float acc = 0.f;
  int j = grp;
  for (; j + 112 < n_splits; j += 128) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(j + 16 * u) * ne + ic];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; j < n_splits; j += 16) acc += src[(int64_t)j * ne + ic];
  part[grp][o] = acc;
  __syncthreads();
  if (grp == 0 && i < ne) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += part[k][o];
    const int ka = (int)(i / p.NC), nb = (int)(i - (int64_t)ka * p.NC);
    if (nb < p.Nb) p.c[(int64_t)ka * p.Nb + nb] = s;
    else if (p.colsum) p.colsum[ka] = s;
  }
}

// n_splits <= 16 (the wide plans): one thread per output, the splits summed in order --
// the same additions in the same order as wgrad_reduce_kernel (whose 16 groups then hold
// one split each, added in group order), without its 16-output workgroups (C3: 2.6 M
// outputs x 8 splits took 154 us per step as 164 K workgroups).
__global__ __launch_bounds__(256) void wgrad_reduce_few_kernel(WgradArgs g) {
  const int pi = wg_find(g.blkf0, g.np, blockIdx.x);
  const WgradProb& p = g.p[pi];
  const int64_t ne = (int64_t)p.Ka * p.NC;
  const int64_t i = (int64_t)(blockIdx.x - g.blkf0[pi]) * 256 + threadIdx.x;
  if (i >= ne) return;
  gptr<float> src = as_global(p.slabs);
  const int n = g.n_splits;
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = src[(int64_t)(j < n ? j : 0) * ne + i];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += j < n ? v[j] : 0.f;
  const int ka = (int)(i / p.NC), nb = (int)(i - (int64_t)ka * p.NC);
  if (nb < p.Nb) p.c[(int64_t)ka * p.Nb + nb] = s;
  else if (p.colsum) p.colsum[ka] = s;
}

static int wgrad_nt(int nc) {
  const int nt = ceil_div(nc, 16);
  if (nt <= 4) return 4;
  if (nt <= 8) return 8;
  if (nt <= 13) return 13;
  return 16;
}

struct WgPlan {
  int nt[2];                       // narrow panel width class of kind 0 / 1
  int np, kind[WG_MAXP], panels[WG_MAXP], panels_nb[WG_MAXP];
  int n_splits;
  int64_t rps;
  size_t slab_bytes[WG_MAXP];
  size_t need;                     // workspace bytes (slab regions, 256-aligned)
  bool ok;                         // the problems fit two narrow panel classes
};

static void wg_finish(WgPlan& pl, int64_t max_rows, int64_t rps, const int* Ka, const int* Nb) {
  pl.rps = rps;
  pl.n_splits = (int)((max_rows + rps - 1) / rps);
  if (pl.n_splits < 1) pl.n_splits = 1;
  pl.need = 0;
  for (int i = 0; i < pl.np; ++i) {
    pl.slab_bytes[i] = Ka[i] > 0 ? sizeof(float) * (size_t)pl.n_splits * Ka[i] * (Nb[i] + 1) : 0;
    pl.need += (pl.slab_bytes[i] + 255) & ~(size_t)255;
  }
}

// Panels cover the Nb columns of a problem; the slabs hold Nb + 1 (the workspace query has
// no colsum flag: column Nb is only written when a colsum is requested).  Splits so that
// splits x panels ~ one workgroup per CU, each split a multiple of WG_CH rows.
// Problems with Ka <= 0 are absent (no panels, no slabs).
static WgPlan wgrad_plan(int64_t max_rows, const int* Ka, const int* Nb, int np) {
  WgPlan pl{};
  pl.np = np;
  pl.ok = true;
  pl.nt[0] = pl.nt[1] = 0;
  int total_panels = 0;
  for (int i = 0; i < np; ++i) {
    if (Ka[i] <= 0) continue;
    const int nt = wgrad_nt(Nb[i]);
    int k = nt == pl.nt[0] ? 0 : nt == pl.nt[1] ? 1 : pl.nt[0] == 0 ? 0 : pl.nt[1] == 0 ? 1 : -1;
    if (k < 0) { pl.ok = false; k = 0; }
    pl.nt[k] = nt;
    pl.kind[i] = k;
    const int pa = ceil_div(Ka[i], WG_KA), pb = ceil_div(Nb[i], nt * 16);
    pl.panels[i] = pa * pb;
    pl.panels_nb[i] = pb;
    total_panels += pl.panels[i];
  }
  if (pl.nt[0] == 0) pl.nt[0] = 4;
  if (pl.nt[1] == 0) pl.nt[1] = 4;
  // ~2 workgroups per CU over the launch (one resident at a time: ~190 VGPRs x 8 waves),
  // >= 4 chunks each (C2 sweep of rows per split, grouped launch: 64 -> 33 us, 128 -> 30,
  // 256 -> 37, 512 -> 63, 1024 -> 116; the per-CU f32 MFMA time of a chunk is ~1.4 us)
  int target = 2 * device_cus() / (total_panels > 0 ? total_panels : 1);
  if (target < 1) target = 1;
  int64_t rps = (max_rows + target - 1) / target;
  // many problems over few rows (the encoder's layers in one gr_wgrad_multi launch at C2:
  // 8 problems x 27 K rows): shorter splits while the grid stays within 8 workgroups per
  // CU -- every split is a latency chain of chunks (C2, 8 problems, rows per split
  // 448 (the rule above) -> 111 us partial + reduce, 256 -> 102, 192 -> 95, 128 -> 98)
  constexpr int64_t RPS_SHORT = 192;
  if (rps > RPS_SHORT && (max_rows + RPS_SHORT - 1) / RPS_SHORT * total_panels <= 8 * device_cus())
    rps = RPS_SHORT;
  if (option(GR_OPT_WGRAD_ROWS) > 0) rps = option(GR_OPT_WGRAD_ROWS);
  rps = ((rps + WGB_CH - 1) / WGB_CH) * WGB_CH;  // whole chunks of either panel kind
  if (rps < 4 * WG_CH) rps = 4 * WG_CH;
  wg_finish(pl, max_rows, rps, Ka, Nb);
  return pl;
}

static size_t align256w(size_t v) { return (v + 255) & ~(size_t)255; }

template <int NT0>
static void launch_partial_nt1(int nt1, const dim3& grid, size_t lds, hipStream_t st, const WgradArgs& g) {
  switch (nt1) {
    case 4: hipLaunchKernelGGL((wgrad_partial_kernel<NT0, 4>), grid, dim3(WG_THREADS), lds, st, g); break;
    case 8: hipLaunchKernelGGL((wgrad_partial_kernel<NT0, 8>), grid, dim3(WG_THREADS), lds, st, g); break;
    case 13: hipLaunchKernelGGL((wgrad_partial_kernel<NT0, 13>), grid, dim3(WG_THREADS), lds, st, g); break;
    default: hipLaunchKernelGGL((wgrad_partial_kernel<NT0, 16>), grid, dim3(WG_THREADS), lds, st, g); break;
  }
}

template <int NT0>
static void launch_partial_bf16_nt1(int nt1, const dim3& grid, size_t lds, hipStream_t st, const WgradArgs& g) {
  switch (nt1) {
    case 4: hipLaunchKernelGGL((wgrad_partial_bf16_kernel<NT0, 4>), grid, dim3(WG_THREADS), lds, st, g); break;
    case 8: hipLaunchKernelGGL((wgrad_partial_bf16_kernel<NT0, 8>), grid, dim3(WG_THREADS), lds, st, g); break;
    case 13: hipLaunchKernelGGL((wgrad_partial_bf16_kernel<NT0, 13>), grid, dim3(WG_THREADS), lds, st, g); break;
    default: hipLaunchKernelGGL((wgrad_partial_bf16_kernel<NT0, 16>), grid, dim3(WG_THREADS), lds, st, g); break;
  }
}

static size_t lds_of_bf16(int nt) {
  switch (nt) {
    case 4: return WgCfgB<4>::LDS;
    case 8: return WgCfgB<8>::LDS;
    case 13: return WgCfgB<13>::LDS;
    default: return WgCfgB<16>::LDS;
  }
}

static size_t lds_of(int nt) {
  switch (nt) {
    case 4: return WgCfg<4>::LDS;
    case 8: return WgCfg<8>::LDS;
    case 13: return WgCfg<13>::LDS;
    default: return WgCfg<16>::LDS;
  }
}

// wide plan (wgrad_tile_bf16w / _f32w): Ka <= 256, one 256-wide tile per 256 columns of Nb;
// splits a multiple of 8 (XCD groups) with ~one workgroup per CU over the launch.
static bool wgrad_wide_ok(const WgradProb* in, int np) {
  int kmax = 0;
  for (int i = 0; i < np; ++i) {
    if (!in[i].a) continue;
    const WgradProb& p = in[i];
    if (p.Ka > WGW_T || p.Ka % 4 || p.Nb % 4 || p.lda % 4 || p.ldb % 4 ||
        (uintptr_t)p.a % (p.a16 ? 8 : 16) || (uintptr_t)p.bm % (p.b16 ? 8 : 16))
      return false;
    kmax = std::max(kmax, p.Ka);
  }
  return kmax > 128;
}
static bool wgrad_any16(const WgradProb* in, int np) {
  for (int i = 0; i < np; ++i)
    if (in[i].a && (in[i].a16 || in[i].b16)) return true;
  return false;
}
static WgPlan wgrad_plan_wide(int64_t max_rows, const int* Ka, const int* Nb, int np) {
  WgPlan pl{};
  pl.np = np;
  pl.ok = true;
  int tiles = 0;
  for (int i = 0; i < np; ++i) {
    if (Ka[i] <= 0) continue;
    pl.panels[i] = ceil_div(Nb[i], WGW_T);
    pl.panels_nb[i] = pl.panels[i];
    tiles += pl.panels[i];
  }
  int target = device_cus() / (tiles > 0 ? tiles : 1);
  target = std::max(8, (target / 8) * 8);
  int64_t rps = (max_rows + target - 1) / target;
  rps = std::max<int64_t>(((rps + 31) / 32) * 32, 128);
  wg_finish(pl, max_rows, rps, Ka, Nb);
  return pl;
}

static bool ws_fits(const WgradProb* in, int np);
static int wgrad_run_stream(const WgradProb* in, int np, const int64_t* offsets, int B,
                            int64_t max_rows, void* workspace, size_t ws_bytes, hipStream_t st);

static int wgrad_run(const WgradProb* in, int np, const int64_t* offsets, int B, int64_t max_rows,
                     void* workspace, size_t ws_bytes, hipStream_t st, bool bf16 = false) {
  GR_REQUIRE(np >= 1 && np <= WG_MAXP, "gr_wgrad: %d problems (1..%d)", np, WG_MAXP);
  int Ka[WG_MAXP], Nb[WG_MAXP];
  for (int i = 0; i < np; ++i) {
    Ka[i] = in[i].a ? in[i].Ka : 0;
    Nb[i] = in[i].a ? in[i].Nb : 0;
  }
  if (max_rows == 0) {
    for (int i = 0; i < np; ++i) {
      if (Ka[i] <= 0) continue;
      zero_words_async(in[i].c, (int64_t)Ka[i] * Nb[i], st);
      if (in[i].colsum) zero_words_async(in[i].colsum, Ka[i], st);
    }
    return 0;
  }
  // f32 at Ka <= 64, Nb <= 256: the streaming form (GR_OPT_WGRAD_STREAM, default on)
  if (!bf16 && option(GR_OPT_WGRAD_STREAM) != 0 && ws_fits(in, np))
    return wgrad_run_stream(in, np, offsets, B, max_rows, workspace, ws_bytes, st);
  const bool any16 = wgrad_any16(in, np);
  // bf16 operands: only the wide bf16 tile reads them (the caller checked its shape rules)
  const bool wide = any16 || wgrad_wide_ok(in, np);
  const WgPlan pl = wide ? wgrad_plan_wide(max_rows, Ka, Nb, np) : wgrad_plan(max_rows, Ka, Nb, np);
  GR_REQUIRE(pl.ok, "gr_wgrad: the problems need more than two panel widths");
  GR_REQUIRE(workspace && ws_bytes >= pl.need, "gr_wgrad: workspace %zu B < %zu B", ws_bytes, pl.need);
  WgradArgs g{};
  g.offsets = offsets;
  g.B = B;
  g.rows_per_split = pl.rps;
  g.n_splits = pl.n_splits;
  g.np = np;
  char* ws = (char*)workspace;
  size_t off = 0;
  g.pan0[0] = g.blk0[0] = 0;
  for (int i = 0; i < np; ++i) {
    g.p[i] = in[i];
    g.kind[i] = pl.kind[i];
    int blocks = 0;
    if (Ka[i] <= 0) {
      g.p[i].panels = 0;
    } else {
      g.p[i].NC = in[i].Nb + (in[i].colsum ? 1 : 0);
      g.p[i].panels = pl.panels[i];
      g.p[i].panels_nb = pl.panels_nb[i];
      g.p[i].slabs = (float*)(ws + off);
      off += align256w(pl.slab_bytes[i]);
      blocks = (int)(((int64_t)Ka[i] * g.p[i].NC + 15) / 16);
    }
    g.pan0[i + 1] = g.pan0[i] + g.p[i].panels;
    g.blk0[i + 1] = g.blk0[i] + blocks;
  }
  const int P = g.pan0[np];
  if (wide) {
    const dim3 grid(ceil_div(pl.n_splits, 8) * 8 * P);  // XCD groups, see wgrad_partial_wide_kernel
    if (bf16)
      GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_wide_kernel<true>, grid, dim3(WG_THREADS), WGW_LDS, st, g));
    else
      GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_wide_kernel<false>, grid, dim3(WG_THREADS), WGF_LDS, st, g));
    GR_LAUNCH_CHECK("gr_wgrad(partial, wide)");
  } else {
    const int nt0 = pl.nt[0], nt1 = pl.nt[1];
    const size_t l0 = bf16 ? lds_of_bf16(nt0) : lds_of(nt0), l1 = bf16 ? lds_of_bf16(nt1) : lds_of(nt1);
    const size_t lds = l0 > l1 ? l0 : l1;
    const dim3 grid(pl.n_splits, P);
    if (bf16) {
      GR_TIMED("wgrad_partial", st, {
        switch (nt0) {
          case 4: launch_partial_bf16_nt1<4>(nt1, grid, lds, st, g); break;
          case 8: launch_partial_bf16_nt1<8>(nt1, grid, lds, st, g); break;
          case 13: launch_partial_bf16_nt1<13>(nt1, grid, lds, st, g); break;
          default: launch_partial_bf16_nt1<16>(nt1, grid, lds, st, g); break;
        }
      });
    } else {
      GR_TIMED("wgrad_partial", st, {
        switch (nt0) {
          case 4: launch_partial_nt1<4>(nt1, grid, lds, st, g); break;
          case 8: launch_partial_nt1<8>(nt1, grid, lds, st, g); break;
          case 13: launch_partial_nt1<13>(nt1, grid, lds, st, g); break;
          default: launch_partial_nt1<16>(nt1, grid, lds, st, g); break;
        }
      });
    }
    GR_LAUNCH_CHECK("gr_wgrad(partial)");
  }
  if (g.n_splits <= 16) {
    g.blkf0[0] = 0;
    for (int i = 0; i < np; ++i)
      g.blkf0[i + 1] = g.blkf0[i] + (g.p[i].panels ? (int)(((int64_t)Ka[i] * g.p[i].NC + 255) / 256) : 0);
    GR_TIMED("wgrad_reduce", st, hipLaunchKernelGGL(wgrad_reduce_few_kernel, dim3(g.blkf0[np]), dim3(256), 0, st, g));
  } else {
    GR_TIMED("wgrad_reduce", st, hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(g.blk0[np]), dim3(256), 0, st, g));
  }
  GR_LAUNCH_CHECK("gr_wgrad(reduce)");
  return 0;
}

// ---------------------------------------------------------------- narrow streaming form
// Ka <= 64, Nb <= 256, even widths and strides, f32 (ml-1m: per layer _uvqk 50 x 200 over
// LN(x) rows and _o 50 x 50 over dy rows; the 8 problems of an encoder backward in one
// launch).  No LDS staging: a lane loads its MFMA operands straight from the row-major
// operands as 8- / 16-byte pieces, with the columns PERMUTED so that one piece feeds four
// MFMAs:
//   A fragment of ka-tile ct:  lane (lr, lg) = A'[row 4 s + lg][ka 4 lr + ct]
//   B fragment of nb-tile t of 64-column group gi:  B[row 4 s + lg][64 gi + 4 lr + t]
// so a lane's float4 of A (two 8-byte loads) and of B (one 16-byte load, or two 8-byte)
// are the operands of the 16 MFMAs (ct, t) of the k-step, and accumulator (ct, t) holds
// C[ka 16 lg + 4 r + ct][nb 64 gi + 4 lr + t].  Workgroup = one (problem, row split), 8
// waves = NG column groups x P row phases (NG = ceil(Nb / 64), P = 8 / NG); wave (gi, ph)
// takes k-steps ph, ph + P, ..., WS_DEPTH of them in flight.  The phases meet in LDS by a
// fixed pairwise tree and the workgroup writes one slab; ws_reduce sums each problem's
// slabs in split order.  Splits per problem are proportional to its column groups (MFMA
// work per row), ~one workgroup per CU in total.  Deterministic: k-ordered MFMA chains, a
// fixed tree, a fixed split order.  Measured at C2 (scripts/wgrad_micro.py, 8 problems):
// 52 us against 79 us for the LDS-staged panels; a dword-per-lane mapping (four 64-byte
// row segments per instruction, B re-read per ka-tile) 61 us, 16 waves with 8 MFMAs each
// 57 us, a 4-deep LDS-DMA ring of 32-row chunks 85 us.
constexpr int WS_THREADS = 512;
constexpr int WS_DEPTH = 4;

struct WsProb {
  const float* a;
  int64_t lda;
  const float2* a_stats;
  const float* bm;
  int64_t ldb;
  int Ka, Nb, NC;  // NC = Nb + 1: slab column Nb holds the column sum of A'
  int ng;          // 64-column groups of Nb (1, 2, 4)
  int vb;          // B piece: 4 = one 16-byte load (Nb, ldb % 4 == 0, 16-byte base), 2 = two 8-byte
  int splits;      // row splits = workgroups of this problem
  float* slabs;    // [splits][Ka][NC]
  float* c;
  float* colsum;
};
struct WsArgs {
  WsProb p[WG_MAXP];
  int np;
  int wg0[WG_MAXP + 1];   // prefix of workgroups (main launch)
  int blk0[WG_MAXP + 1];  // prefix of reduce blocks
  const int64_t* offsets;
  int B;
};

constexpr int WS_XCH = 68;  // floats per lane in the phase exchange: 64 accumulators + 4 column sums

template <int P, int VB, int DEPTH>
__device__ __forceinline__ void ws_body(const WsProb& g, int64_t total, int split, char* smem) {
  constexpr int NG = 8 / P;
  const int w = wave_id(), lane = threadIdx.x & 63;
  const int gi = w % NG, ph = w / NG;
  const int lr = lane & 15, lg = lane >> 4;
  // this split's rows [r0, r1); r0 a multiple of 4 P (the phases' k-steps align)
  const int64_t step = 4 * P;
  const int64_t rps = ((total + g.splits - 1) / g.splits + step - 1) / step * step;
  const int64_t r0 = (int64_t)split * rps;
  const int64_t r1 = min(total, r0 + rps);
  const int nks = __builtin_amdgcn_readfirstlane(r1 > r0 ? (int)((r1 - r0 + 3) >> 2) : 0);
  const int mine = nks > ph ? (nks - ph + P - 1) / P : 0;
  // rows >= total read 0 (per-dword range check): A, its stats and B, so A' = 0 there
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.a, 0, (int)(total * g.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.bm, 0, (int)(total * g.ldb * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.a_stats ? (const void*)g.a_stats : (const void*)g.a), 0,
      g.a_stats ? (int)(total * 8) : 0, 0x00020000);
  constexpr int OOBW = OOB_OFF;
  const int acol = 4 * lr, bcol = 64 * gi + 4 * lr;
  const bool a_lo = acol < g.Ka, a_hi = acol + 2 < g.Ka;  // Ka even: 8-byte pieces in or out
  const bool b_lo = bcol < g.Nb, b_hi = bcol + 2 < g.Nb;

  f4 av[DEPTH], bv[DEPTH];
  float2 sv[DEPTH];
  auto issue = [&](int u, int j) {
    const bool in = j < mine;
    const int row = (int)(r0 + 4 * (ph + P * j)) + lg;
    const int ao = row * (int)g.lda + acol, bo = row * (int)g.ldb + bcol;
    const u32x2_t a0 = __builtin_amdgcn_raw_buffer_load_b64(ra, in && a_lo ? ao * 4 : OOBW, 0, 0);
    const u32x2_t a1 = __builtin_amdgcn_raw_buffer_load_b64(ra, in && a_hi ? ao * 4 + 8 : OOBW, 0, 0);
    av[u] = f4{__uint_as_float(a0.x), __uint_as_float(a0.y), __uint_as_float(a1.x), __uint_as_float(a1.y)};
    if (g.a_stats) {
      const u32x2_t st = __builtin_amdgcn_raw_buffer_load_b64(rs, in ? row * 8 : OOBW, 0, 0);
      sv[u] = make_float2(__uint_as_float(st.x), __uint_as_float(st.y));
    } else {
      sv[u] = make_float2(0.f, 1.f);
    }
    if constexpr (VB == 4) {
      const u32x4_t b = __builtin_amdgcn_raw_buffer_load_b128(rb, in && b_lo ? bo * 4 : OOBW, 0, 0);
      bv[u] = f4{__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w)};
    } else {
      const u32x2_t b0 = __builtin_amdgcn_raw_buffer_load_b64(rb, in && b_lo ? bo * 4 : OOBW, 0, 0);
      const u32x2_t b1 = __builtin_amdgcn_raw_buffer_load_b64(rb, in && b_hi ? bo * 4 + 8 : OOBW, 0, 0);
      bv[u] = f4{__uint_as_float(b0.x), __uint_as_float(b0.y), __uint_as_float(b1.x), __uint_as_float(b1.y)};
    }
  };

  f4 acc[4][4];  // [ct][t]
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[ct][t] = f4_zero();
  f4 csum = f4_zero();  // A'[row][4 lr + ct] summed over this wave's rows (the _o bias gradient)
  if (mine > 0) {
#pragma unroll
    for (int u = 0; u < DEPTH; ++u) issue(u, u);
    const int iters = (mine + DEPTH - 1) / DEPTH * DEPTH;
    for (int j0 = 0; j0 < iters; j0 += DEPTH) {
#pragma unroll
      for (int u = 0; u < DEPTH; ++u) {
        f4 a = av[u];
        if (g.a_stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] = (a[e] - sv[u].x) * sv[u].y;  // rows out of range: 0 * 0
        }
        csum += a;
        const f4 b = bv[u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[ct][t] = mfma16x16x4(a[ct], b[t], acc[ct][t]);
        __builtin_amdgcn_sched_barrier(0);
        issue(u, j0 + u + DEPTH);
      }
    }
  }
  // column sums over the k-step rows (lanes lr, lr + 16, lr + 32, lr + 48), fixed order
#pragma unroll
  for (int e = 0; e < 4; ++e) csum[e] = wg_colsum_lanes(csum[e]);
  // phases meet pairwise in LDS: round s, phases s .. 2s - 1 hand their sums to phase - s
  float* xch = reinterpret_cast<float*>(smem);  // [P / 2 slots][NG][WS_XCH][64]
#pragma unroll
  for (int s = P / 2; s >= 1; s >>= 1) {
    if (ph >= s && ph < 2 * s) {
      float* x = xch + ((ph - s) * NG + gi) * WS_XCH * 64 + lane;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) x[((ct * 4 + t) * 4 + r) * 64] = acc[ct][t][r];
#pragma unroll
      for (int e = 0; e < 4; ++e) x[(64 + e) * 64] = csum[e];
    }
    __syncthreads();
    if (ph < s) {
      const float* x = xch + (ph * NG + gi) * WS_XCH * 64 + lane;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[ct][t][r] += x[((ct * 4 + t) * 4 + r) * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[e] += x[(64 + e) * 64];
    }
    __syncthreads();
  }
  if (ph != 0) return;
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
  // column sums of ka 4 lr .. 4 lr + 3 (a lane whose B columns lie past Nb still owns them)
  if (g.colsum && gi == 0 && lg == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (acol + e < g.Ka) slab[(int64_t)(acol + e) * g.NC + g.Nb] = csum[e];
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ka = 16 * lg + 4 * r + ct;
      if (ka >= g.Ka) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (bcol + t < g.Nb) slab[(int64_t)ka * g.NC + bcol + t] = acc[ct][t][r];
    }
}

__global__ __launch_bounds__(WS_THREADS) void wgrad_stream_kernel(WsArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int i = wg_find(g.wg0, g.np, blockIdx.x);
  const WsProb& p = g.p[i];
  const int split = blockIdx.x - g.wg0[i];
  const int64_t total = g.offsets[g.B];
  const int P = 8 / p.ng;
  if (p.vb == 4) {
    if (P == 8) ws_body<8, 4, WS_DEPTH>(p, total, split, smem);
    else if (P == 4) ws_body<4, 4, WS_DEPTH>(p, total, split, smem);
    else ws_body<2, 4, WS_DEPTH>(p, total, split, smem);
  } else {
    if (P == 8) ws_body<8, 2, WS_DEPTH>(p, total, split, smem);
    else if (P == 4) ws_body<4, 2, WS_DEPTH>(p, total, split, smem);
    else ws_body<2, 2, WS_DEPTH>(p, total, split, smem);
  }
}

// out = sum over a problem's splits in split order: thread (o, grp) of a 256-thread block
// sums splits grp, grp + 16, ... of output o, then the 16 partials are added in grp order
__global__ __launch_bounds__(256) void ws_reduce_kernel(WsArgs g) {
  __shared__ float part[16][17];
  const int pi = wg_find(g.blk0, g.np, blockIdx.x);
  const WsProb& p = g.p[pi];
  const int blk = blockIdx.x - g.blk0[pi];
  const int64_t ne = (int64_t)p.Ka * p.NC;
  const int o = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blk * 16 + o;
  const int64_t ic = i < ne ? i : ne - 1;
  gptr<float> src = as_global(p.slabs);
  float acc = 0.f;
  int j = grp;
  for (; j + 112 < p.splits; j += 128) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(j + 16 * u) * ne + ic];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; j < p.splits; j += 16) acc += src[(int64_t)j * ne + ic];
  part[grp][o] = acc;
  __syncthreads();
  if (grp == 0 && i < ne) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += part[k][o];
    const int ka = (int)(i / p.NC), nb = (int)(i - (int64_t)ka * p.NC);
    if (nb < p.Nb) p.c[(int64_t)ka * p.Nb + nb] = s;
    else if (p.colsum) p.colsum[ka] = s;
  }
}

static int ws_ng(int nb) { return nb <= 64 ? 1 : nb <= 128 ? 2 : 4; }
// the streaming form: every problem Ka <= 64, Nb <= 256, even widths and strides, 8-byte
// aligned bases
static bool ws_fits_shapes(const int* Ka, const int* Nb, int np) {
  for (int i = 0; i < np; ++i)
    if (Ka[i] > 0 && (Ka[i] > 64 || Nb[i] > 256 || (Ka[i] | Nb[i]) & 1)) return false;
  return true;
}
static bool ws_fits(const WgradProb* in, int np) {
  int Ka[WG_MAXP], Nb[WG_MAXP];
  for (int i = 0; i < np; ++i) {
    const WgradProb& p = in[i];
    Ka[i] = p.a ? p.Ka : 0;
    Nb[i] = p.a ? p.Nb : 0;
    if (!p.a) continue;
    if ((p.lda | p.ldb) & 1 || (uintptr_t)p.a % 8 || (uintptr_t)p.bm % 8 ||
        (p.a_stats && (uintptr_t)p.a_stats % 8))
      return false;
  }
  return ws_fits_shapes(Ka, Nb, np);
}
static size_t ws_lds(int ng) { return sizeof(float) * (size_t)(8 / ng / 2) * ng * WS_XCH * 64; }

struct WsPlan {
  int splits[WG_MAXP];
  size_t slab_bytes[WG_MAXP];
  size_t need;
};
// splits per problem proportional to its column groups, ~one workgroup per CU in total,
// each split >= 64 rows
static WsPlan ws_plan(int64_t max_rows, const int* Ka, const int* Nb, int np) {
  WsPlan pl{};
  int csum = 0;
  for (int i = 0; i < np; ++i)
    if (Ka[i] > 0) csum += ws_ng(Nb[i]);
  const int G = device_cus();
  const int64_t cap = std::max<int64_t>(1, (max_rows + 63) / 64);
  for (int i = 0; i < np; ++i) {
    if (Ka[i] <= 0) continue;
    int64_t s = ((int64_t)G * ws_ng(Nb[i]) + csum / 2) / std::max(csum, 1);
    s = std::max<int64_t>(1, std::min(s, cap));
    pl.splits[i] = (int)s;
    pl.slab_bytes[i] = sizeof(float) * (size_t)s * Ka[i] * (Nb[i] + 1);
    pl.need += (pl.slab_bytes[i] + 255) & ~(size_t)255;
  }
  return pl;
}

static int wgrad_run_stream(const WgradProb* in, int np, const int64_t* offsets, int B,
                            int64_t max_rows, void* workspace, size_t ws_bytes, hipStream_t st) {
  int Ka[WG_MAXP], Nb[WG_MAXP];
  for (int i = 0; i < np; ++i) {
    Ka[i] = in[i].a ? in[i].Ka : 0;
    Nb[i] = in[i].a ? in[i].Nb : 0;
  }
  const WsPlan pl = ws_plan(max_rows, Ka, Nb, np);
  GR_REQUIRE(workspace && ws_bytes >= pl.need, "gr_wgrad: workspace %zu B < %zu B", ws_bytes, pl.need);
  WsArgs g{};
  g.offsets = offsets;
  g.B = B;
  g.np = 0;
  char* ws = (char*)workspace;
  size_t off = 0, lds = 0;
  g.wg0[0] = g.blk0[0] = 0;
  for (int i = 0; i < np; ++i) {
    if (Ka[i] <= 0) continue;
    WsProb& p = g.p[g.np];
    p.a = in[i].a;
    p.lda = in[i].lda;
    p.a_stats = in[i].a_stats;
    p.bm = in[i].bm;
    p.ldb = in[i].ldb;
    p.Ka = Ka[i];
    p.Nb = Nb[i];
    p.NC = Nb[i] + 1;
    p.ng = ws_ng(Nb[i]);
    p.vb = (Nb[i] % 4 == 0 && p.ldb % 4 == 0 && (uintptr_t)p.bm % 16 == 0) ? 4 : 2;
    p.splits = pl.splits[i];
    p.slabs = (float*)(ws + off);
    off += (pl.slab_bytes[i] + 255) & ~(size_t)255;
    p.c = in[i].c;
    p.colsum = in[i].colsum;
    lds = std::max(lds, ws_lds(p.ng));
    g.wg0[g.np + 1] = g.wg0[g.np] + p.splits;
    g.blk0[g.np + 1] = g.blk0[g.np] + (int)(((int64_t)p.Ka * p.NC + 15) / 16);
    ++g.np;
  }
  if (g.np == 0) return 0;
  GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_stream_kernel, dim3(g.wg0[g.np]), dim3(WS_THREADS), lds, st, g));
  GR_LAUNCH_CHECK("gr_wgrad(stream)");
  GR_TIMED("wgrad_reduce", st, hipLaunchKernelGGL(ws_reduce_kernel, dim3(g.blk0[g.np]), dim3(256), 0, st, g));
  GR_LAUNCH_CHECK("gr_wgrad(stream reduce)");
  return 0;
}

// workspace of a problem list: the largest of the narrow, streaming and (when it may be
// taken) wide plans
static size_t wgrad_ws_need(const int* Ka, const int* Nb, int np, int64_t max_rows) {
  size_t need = wgrad_plan(max_rows, Ka, Nb, np).need;
  int kmax = 0;
  for (int i = 0; i < np; ++i) kmax = std::max(kmax, Ka[i]);
  if (kmax <= WGW_T) need = std::max(need, wgrad_plan_wide(max_rows, Ka, Nb, np).need);
  if (ws_fits_shapes(Ka, Nb, np)) need = std::max(need, ws_plan(max_rows, Ka, Nb, np).need);
  return need;
}

}  // namespace gr

using namespace gr;

extern "C" size_t gr_wgrad_workspace_size(int64_t max_rows, int Ka, int Nb) {
  if (max_rows <= 0 || Ka <= 0 || Nb <= 0) return 0;
  const int ka[1] = {Ka}, nb[1] = {Nb};
  return wgrad_ws_need(ka, nb, 1, max_rows);
}

extern "C" size_t gr_wgrad2_workspace_size(int64_t max_rows, int Ka0, int Nb0, int Ka1, int Nb1) {
  if (max_rows <= 0 || Ka0 <= 0 || Nb0 <= 0 || Ka1 < 0 || Nb1 < 0) return 0;
  const int ka[2] = {Ka0, Nb1 > 0 ? Ka1 : 0}, nb[2] = {Nb0, Ka1 > 0 ? Nb1 : 0};
  return wgrad_ws_need(ka, nb, 2, max_rows);
}

extern "C" int gr_wgrad(const float* a, int64_t lda, const float* a_stats, const float* bm,
                        int64_t ldb, const int64_t* offsets, int B, int64_t max_rows, int Ka,
                        int Nb, float* c, float* a_colsum, void* workspace, size_t ws_bytes,
                        void* stream) {
  GR_REQUIRE(a && bm && offsets && c, "gr_wgrad: null pointer");
  GR_REQUIRE(Ka > 0 && Nb > 0 && B >= 0 && max_rows >= 0, "gr_wgrad: bad sizes");
  GR_REQUIRE(max_rows * (lda > ldb ? lda : ldb) * 4 < 0x7fffffffLL,
             "gr_wgrad: %lld rows exceed the 32-bit buffer range", (long long)max_rows);
  WgradProb p[1] = {};
  p[0] = WgradProb{a, lda, (const float2*)a_stats, bm, ldb, Ka, Nb, 0, 0, 0, nullptr, c, a_colsum};
  return wgrad_run(p, 1, offsets, B, max_rows, workspace, ws_bytes, (hipStream_t)stream);
}

static int gr_wgrad2_impl(bool bf16, const float* a0, int64_t lda0, const float* a_stats0, const float* b0,
                         int64_t ldb0, int Ka0, int Nb0, float* c0, float* colsum0,
                         const float* a1, int64_t lda1, const float* a_stats1, const float* b1,
                         int64_t ldb1, int Ka1, int Nb1, float* c1, float* colsum1,
                         const int64_t* offsets, int B, int64_t max_rows, void* workspace,
                         size_t ws_bytes, void* stream) {
  GR_REQUIRE(a0 && b0 && c0 && a1 && b1 && c1 && offsets, "gr_wgrad2: null pointer");
  GR_REQUIRE(Ka0 > 0 && Nb0 > 0 && Ka1 > 0 && Nb1 > 0 && B >= 0 && max_rows >= 0,
             "gr_wgrad2: bad sizes");
  const int64_t ld = std::max(std::max(lda0, ldb0), std::max(lda1, ldb1));
  GR_REQUIRE(max_rows * ld * 4 < 0x7fffffffLL,
             "gr_wgrad2: %lld rows exceed the 32-bit buffer range", (long long)max_rows);
  WgradProb p[2] = {};
  p[0] = WgradProb{a0, lda0, (const float2*)a_stats0, b0, ldb0, Ka0, Nb0, 0, 0, 0, nullptr, c0, colsum0};
  p[1] = WgradProb{a1, lda1, (const float2*)a_stats1, b1, ldb1, Ka1, Nb1, 0, 0, 0, nullptr, c1, colsum1};
  return wgrad_run(p, 2, offsets, B, max_rows, workspace, ws_bytes, (hipStream_t)stream, bf16);
}
extern "C" int gr_wgrad2(const float* a0, int64_t lda0, const float* a_stats0, const float* b0,
                         int64_t ldb0, int Ka0, int Nb0, float* c0, float* colsum0,
                         const float* a1, int64_t lda1, const float* a_stats1, const float* b1,
                         int64_t ldb1, int Ka1, int Nb1, float* c1, float* colsum1,
                         const int64_t* offsets, int B, int64_t max_rows, void* workspace,
                         size_t ws_bytes, void* stream) {
  return gr_wgrad2_impl(false, a0, lda0, a_stats0, b0, ldb0, Ka0, Nb0, c0, colsum0, a1, lda1, a_stats1, b1, ldb1, Ka1, Nb1, c1, colsum1, offsets, B, max_rows, workspace, ws_bytes, stream);
}
extern "C" int gr_wgrad2_bf16(const float* a0, int64_t lda0, const float* a_stats0, const float* b0,
                         int64_t ldb0, int Ka0, int Nb0, float* c0, float* colsum0,
                         const float* a1, int64_t lda1, const float* a_stats1, const float* b1,
                         int64_t ldb1, int Ka1, int Nb1, float* c1, float* colsum1,
                         const int64_t* offsets, int B, int64_t max_rows, void* workspace,
                         size_t ws_bytes, void* stream) {
  return gr_wgrad2_impl(true, a0, lda0, a_stats0, b0, ldb0, Ka0, Nb0, c0, colsum0, a1, lda1, a_stats1, b1, ldb1, Ka1, Nb1, c1, colsum1, offsets, B, max_rows, workspace, ws_bytes, stream);
}

// ---------------------------------------------------------------- many problems at once
// desc: 9 int64 per problem {a, lda, a_stats, b, ldb, Ka, Nb, c, colsum} (pointers as
// integers, a_stats / colsum may be 0).
static int wg_parse(const int64_t* desc, int np, WgradProb* p, int* Ka, int* Nb, int64_t* ldmax) {
  GR_REQUIRE(desc && np >= 1 && np <= WG_MAXP, "gr_wgrad_multi: %d problems (1..%d)", np, WG_MAXP);
  *ldmax = 0;
  for (int i = 0; i < np; ++i) {
    const int64_t* d = desc + 9 * i;
    p[i] = WgradProb{(const float*)d[0], d[1], (const float2*)d[2], (const float*)d[3], d[4],
                     (int)d[5], (int)d[6], 0, 0, 0, nullptr, (float*)d[7], (float*)d[8]};
    GR_REQUIRE(p[i].a && p[i].bm && p[i].c && p[i].Ka > 0 && p[i].Nb > 0,
               "gr_wgrad_multi: problem %d has a null pointer or an empty shape", i);
    Ka[i] = p[i].Ka;
    Nb[i] = p[i].Nb;
    *ldmax = std::max(*ldmax, std::max(d[1], d[4]));
  }
  return 0;
}

extern "C" size_t gr_wgrad_multi_workspace_size(const int64_t* desc, int n_problems, int64_t max_rows) {
  if (!desc || n_problems < 1 || n_problems > WG_MAXP || max_rows <= 0) return 0;
  int Ka[WG_MAXP], Nb[WG_MAXP];
  for (int i = 0; i < n_problems; ++i) {
    Ka[i] = (int)desc[9 * i + 5];
    Nb[i] = (int)desc[9 * i + 6];
  }
  return wgrad_ws_need(Ka, Nb, n_problems, max_rows);
}

// desc: 10 int64 per problem, gr_wgrad_multi's 9 plus flags (bit 0: A rows bf16, bit 1: B
// rows bf16); bf16 MFMA operands, the wide tile (Ka <= 256, 4-aligned widths and strides,
// bf16 operands 8-byte aligned; A in bf16 takes no row stats).
extern "C" size_t gr_wgrad_multi_a16_workspace_size(const int64_t* desc, int n_problems, int64_t max_rows) {
  if (!desc || n_problems < 1 || n_problems > WG_MAXP || max_rows <= 0) return 0;
  int Ka[WG_MAXP], Nb[WG_MAXP];
  for (int i = 0; i < n_problems; ++i) {
    Ka[i] = (int)desc[10 * i + 5];
    Nb[i] = (int)desc[10 * i + 6];
    if (Ka[i] > WGW_T) return 0;
  }
  return wgrad_plan_wide(max_rows, Ka, Nb, n_problems).need;
}

extern "C" int gr_wgrad_multi_a16(const int64_t* desc, int n_problems, const int64_t* offsets, int B,
                                  int64_t max_rows, void* workspace, size_t ws_bytes, void* stream) {
  GR_REQUIRE(desc && n_problems >= 1 && n_problems <= WG_MAXP, "gr_wgrad_multi_a16: %d problems (1..%d)",
             n_problems, WG_MAXP);
  WgradProb p[WG_MAXP] = {};
  int64_t ld = 0;
  for (int i = 0; i < n_problems; ++i) {
    const int64_t* d = desc + 10 * i;
    p[i] = WgradProb{(const float*)d[0], d[1], (const float2*)d[2], (const float*)d[3], d[4],
                     (int)d[5], (int)d[6], 0, 0, 0, nullptr, (float*)d[7], (float*)d[8],
                     (int)(d[9] & 1), (int)((d[9] >> 1) & 1)};
    const WgradProb& q = p[i];
    GR_REQUIRE(q.a && q.bm && q.c && q.Ka > 0 && q.Nb > 0,
               "gr_wgrad_multi_a16: problem %d has a null pointer or an empty shape", i);
    GR_REQUIRE(!(q.a16 && q.a_stats), "gr_wgrad_multi_a16: problem %d: bf16 A takes no row stats", i);
    GR_REQUIRE(q.Ka <= WGW_T && q.Ka % 4 == 0 && q.Nb % 4 == 0 && q.lda % 4 == 0 && q.ldb % 4 == 0 &&
                   (uintptr_t)q.a % (q.a16 ? 8 : 16) == 0 && (uintptr_t)q.bm % (q.b16 ? 8 : 16) == 0,
               "gr_wgrad_multi_a16: problem %d needs Ka <= 256, 4-aligned widths / strides and aligned rows", i);
    ld = std::max(ld, std::max(d[1], d[4]));
  }
  GR_REQUIRE(offsets && B >= 0 && max_rows >= 0, "gr_wgrad_multi_a16: bad sizes");
  GR_REQUIRE(max_rows * ld * 4 < 0x7fffffffLL,
             "gr_wgrad_multi_a16: %lld rows exceed the 32-bit buffer range", (long long)max_rows);
  return wgrad_run(p, n_problems, offsets, B, max_rows, workspace, ws_bytes, (hipStream_t)stream, true);
}

extern "C" int gr_wgrad_multi(const int64_t* desc, int n_problems, const int64_t* offsets, int B,
                              int64_t max_rows, int bf16, void* workspace, size_t ws_bytes,
                              void* stream) {
  WgradProb p[WG_MAXP] = {};
  int Ka[WG_MAXP], Nb[WG_MAXP];
  int64_t ld = 0;
  if (const int rc = wg_parse(desc, n_problems, p, Ka, Nb, &ld)) return rc;
  GR_REQUIRE(offsets && B >= 0 && max_rows >= 0, "gr_wgrad_multi: bad sizes");
  GR_REQUIRE(max_rows * ld * 4 < 0x7fffffffLL,
             "gr_wgrad_multi: %lld rows exceed the 32-bit buffer range", (long long)max_rows);
  return wgrad_run(p, n_problems, offsets, B, max_rows, workspace, ws_bytes, (hipStream_t)stream,
                   bf16 != 0);
}
