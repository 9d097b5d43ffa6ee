// Weight gradients of the STU projections — gfx950, f32 MFMA.
//
//   C[ka][nb] = sum_m A'(m, ka) * Bm(m, nb),   A' = A or LayerNorm(A) from saved stats,
//   optional colsum[ka] = sum_m A'(m, ka)  (the bias gradient of _o).
// Replaces the mm-backward weight terms of reference hstu.py:303 (_uvqk) and
// hstu.py:404-413 (_o.weight, _o.bias).
//
// Split-K over rows: grid = (row splits) x (output panels of 64 ka x NT*16 nb).  A
// workgroup streams its rows through LDS in chunks of 32 (double-buffered; the next
// chunk is loaded into registers through buffer descriptors while the current one runs)
// and wave w accumulates ka-tile w of the panel against all NT nb-tiles.  The column sum
// comes for free from a ones-column appended to Bm (padding column Nb).  Each split
// writes its panel to a workspace slab; wgrad_reduce sums the slabs in a fixed order
// (deterministic, no atomics) with 16 slab groups per output in parallel.
#include "attn_common.h"

#include "../../include/gr_hstu.h"

namespace gr {

constexpr int WG_KA = 64;   // ka rows per panel (4 waves x 16)
constexpr int WG_CH = 32;   // rows per chunk (8 MFMA k-steps)
constexpr int WG_LDA = WG_KA + 16;  // == 16 mod 32: lane groups (4 rows apart) hit disjoint banks
constexpr int WG_THREADS = 512;     // 8 waves: wave w owns ka-tile w & 3, k-steps of half w >> 2

struct WgradArgs {
  const float* a;
  int64_t lda;
  const float2* a_stats;
  const float* bm;
  int64_t ldb;
  const int64_t* offsets;
  int B, Ka, Nb, NC;  // NC = Nb (+1 with the ones column)
  int64_t rows_per_split;
  int n_splits, panels_nb;
  float* slabs;  // [split][Ka][NC]
};

template <int NT>
struct WgCfg {
  static constexpr int NP = NT * 16;
  static constexpr int LDB = (NP % 32 == 16) ? NP : NP + 16;  // == 16 mod 32
  static constexpr int NP2 = NP <= 64 ? 64 : NP <= 128 ? 128 : 256;  // staging column span
  static constexpr int BRPP = WG_THREADS / NP2;                   // B rows per pass
  static constexpr int BPER = WG_CH / BRPP;                       // B loads per thread
  static constexpr int APER = WG_CH * WG_KA / WG_THREADS;         // A loads per thread
  static constexpr size_t LDS = sizeof(float) * 2 * WG_CH * (WG_LDA + LDB);
};

template <int NT>
__global__ __launch_bounds__(WG_THREADS) void wgrad_partial_kernel(WgradArgs g) {
  using C = WgCfg<NT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float (*As)[WG_CH * WG_LDA] = reinterpret_cast<float (*)[WG_CH * WG_LDA]>(smem);
  float (*Bs)[WG_CH * C::LDB] =
      reinterpret_cast<float (*)[WG_CH * C::LDB]>(smem + sizeof(float) * 2 * WG_CH * WG_LDA);
  const int split = blockIdx.x;
  const int pa = blockIdx.y / g.panels_nb, pb = blockIdx.y % g.panels_nb;
  const int ka0 = pa * WG_KA, nb0 = pb * C::NP;
  const int64_t total = g.offsets[g.B];
  const int64_t r0 = (int64_t)split * g.rows_per_split;
  const int64_t r1 = min(total, r0 + g.rows_per_split);
  const int tid = threadIdx.x, wv = wave_id(), lane = tid & 63;
  const int w = wv & 3, half = wv >> 2;
  const int lr = lane & 15, lg = lane >> 4;
  const int n_ch = r1 > r0 ? (int)((r1 - r0 + WG_CH - 1) / WG_CH) : 0;

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
  const bool b_in = bnb < g.Nb, b_one = bnb == g.Nb && g.NC > g.Nb;
  float ra_v[C::APER], rb_v[C::BPER];
  float2 st_v[C::APER];
  auto load = [&](int ch) {
    const int rr0 = ch * WG_CH;
#pragma unroll
    for (int i = 0; i < C::APER; ++i) {
      const int rr = rr0 + ar + (WG_THREADS / 64) * i;
      ra_v[i] = buf_ld(ra, a_ok ? (int)((rr * g.lda + aka) * 4) : 0x40000000, 0);
      if (g.a_stats) st_v[i] = ld_f2(g.a_stats, min(r0 + rr, total - 1));
    }
#pragma unroll
    for (int i = 0; i < C::BPER; ++i) {
      const int rr = rr0 + br + C::BRPP * i;
      rb_v[i] = buf_ld(rb, b_in ? (int)((rr * g.ldb + bnb) * 4) : 0x40000000, 0);
    }
  };
  auto store = [&](int buf, int ch) {
    const int rr0 = ch * WG_CH;
#pragma unroll
    for (int i = 0; i < C::APER; ++i) {
      const int rr = ar + (WG_THREADS / 64) * i;
      float v = ra_v[i];
      if (g.a_stats) v = (v - st_v[i].x) * st_v[i].y;
      As[buf][rr * WG_LDA + ac] = (a_ok && r0 + rr0 + rr < r1) ? v : 0.f;
    }
    if (bc < C::NP) {
#pragma unroll
      for (int i = 0; i < C::BPER; ++i) {
        const int rr = br + C::BRPP * i;
        const bool row_ok = r0 + rr0 + rr < r1;
        Bs[buf][rr * C::LDB + bc] = b_one ? (row_ok ? 1.f : 0.f) : rb_v[i];
      }
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  if (n_ch > 0) {
    load(0);
    store(0, 0);
  }
  __syncthreads();
  for (int ch = 0; ch < n_ch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < n_ch) load(ch + 1);
    const float* Ab = As[buf];
    const float* Bb = Bs[buf];
#pragma unroll
    for (int ks = half * (WG_CH / 8); ks < (half + 1) * (WG_CH / 8); ++ks) {
      const float av = Ab[(4 * ks + lg) * WG_LDA + 16 * w + lr];
      float bv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[t] = Bb[(4 * ks + lg) * C::LDB + 16 * t + lr];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(av, bv[t], acc[t]);
    }
    if (ch + 1 < n_ch) store(buf ^ 1, ch + 1);
    lds_barrier();
  }
  // the two halves' partial sums meet in LDS (fixed order: half 0 + half 1)
  float* xch = reinterpret_cast<float*>(smem);  // [4 waves][NT][4][64]
  if (half == 1) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[((w * NT + t) * 4 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  if (half == 1) return;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[t][r] += xch[((w * NT + t) * 4 + r) * 64 + lane];
  // acc[t][r] = C[ka0 + 16w + 4lg + r][nb0 + 16t + lr]
  float* slab = g.slabs + (int64_t)split * g.Ka * g.NC;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ka = ka0 + 16 * w + 4 * lg + r;
    if (ka >= g.Ka) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int nb = nb0 + 16 * t + lr;
      if (nb < g.NC) slab[(int64_t)ka * g.NC + nb] = acc[t][r];
    }
  }
}

// out = sum over splits (fixed order): a workgroup owns 16 outputs; thread (o, grp) sums
// splits grp, grp+16, ... 8-deep, then the 16 partials are added in grp order.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* slabs, int n_splits, int Ka,
                                                           int Nb, int NC, float* c,
                                                           float* colsum) {
  __shared__ float part[16][17];
  const int64_t ne = (int64_t)Ka * NC;
  const int o = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + o;
  const int64_t ic = i < ne ? i : ne - 1;
  gptr<float> src = as_global(slabs);
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
    const int ka = (int)(i / NC), nb = (int)(i - (int64_t)ka * NC);
    if (nb < Nb) c[(int64_t)ka * Nb + nb] = s;
    else if (colsum) colsum[ka] = s;
  }
}

static int wgrad_nt(int nc) {
  const int nt = ceil_div(nc, 16);
  if (nt <= 4) return 4;
  if (nt <= 8) return 8;
  if (nt <= 13) return 13;
  return 16;
}

static int wg_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// Splits so that splits x panels ~ one workgroup per CU, >= 4 chunks per split.
static void wgrad_plan(int64_t max_rows, int Ka, int NC, int* n_splits, int64_t* rows_per_split,
                       int* panels, int* panels_nb, int* nt) {
  *nt = wgrad_nt(NC);
  const int pa = ceil_div(Ka, WG_KA), pb = ceil_div(NC, *nt * 16);
  *panels = pa * pb;
  *panels_nb = pb;
  int target = ceil_div(wg_num_cus(), *panels);
  int64_t rps = (max_rows + target - 1) / target;
  rps = ((rps + WG_CH - 1) / WG_CH) * WG_CH;
  if (rps < 4 * WG_CH) rps = 4 * WG_CH;
  *rows_per_split = rps;
  *n_splits = (int)((max_rows + rps - 1) / rps);
  if (*n_splits < 1) *n_splits = 1;
}

}  // namespace gr

using namespace gr;

extern "C" size_t gr_wgrad_workspace_size(int64_t max_rows, int Ka, int Nb) {
  if (max_rows <= 0 || Ka <= 0 || Nb <= 0) return 0;
  int n_splits, panels, pnb, nt;
  int64_t rps;
  wgrad_plan(max_rows, Ka, Nb + 1, &n_splits, &rps, &panels, &pnb, &nt);
  return sizeof(float) * (size_t)n_splits * (size_t)Ka * (Nb + 1);
}

extern "C" int gr_wgrad(const float* a, int64_t lda, const float* a_stats, const float* bm,
                        int64_t ldb, const int64_t* offsets, int B, int64_t max_rows, int Ka,
                        int Nb, float* c, float* a_colsum, void* workspace, size_t ws_bytes,
                        void* stream) {
  GR_REQUIRE(a && bm && offsets && c, "gr_wgrad: null pointer");
  GR_REQUIRE(Ka > 0 && Nb > 0 && B >= 0 && max_rows >= 0, "gr_wgrad: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (max_rows == 0) {
    zero_words_async(c, (int64_t)Ka * Nb, st);
    if (a_colsum) zero_words_async(a_colsum, Ka, st);
    return 0;
  }
  GR_REQUIRE(max_rows * (lda > ldb ? lda : ldb) * 4 < 0x7fffffffLL,
             "gr_wgrad: %lld rows exceed the 32-bit buffer range", (long long)max_rows);
  const int NC = Nb + (a_colsum ? 1 : 0);
  int n_splits, panels, pnb, nt;
  int64_t rps;
  // one plan for both column counts (the workspace query has no colsum flag): panels
  // cover Nb + 1 columns, the ones column is only filled when a_colsum is requested
  wgrad_plan(max_rows, Ka, Nb + 1, &n_splits, &rps, &panels, &pnb, &nt);
  const size_t need = sizeof(float) * (size_t)n_splits * Ka * NC;
  GR_REQUIRE(workspace && ws_bytes >= need, "gr_wgrad: workspace %zu B < %zu B", ws_bytes, need);
  WgradArgs g{a, lda, (const float2*)a_stats, bm, ldb, offsets, B, Ka, Nb, NC, rps, n_splits, pnb,
              (float*)workspace};
  const dim3 grid(n_splits, panels);
  switch (nt) {
    case 4: GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_kernel<4>, grid, dim3(WG_THREADS), WgCfg<4>::LDS, st, g)); break;
    case 8: GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_kernel<8>, grid, dim3(WG_THREADS), WgCfg<8>::LDS, st, g)); break;
    case 13: GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_kernel<13>, grid, dim3(WG_THREADS), WgCfg<13>::LDS, st, g)); break;
    default: GR_TIMED("wgrad_partial", st, hipLaunchKernelGGL(wgrad_partial_kernel<16>, grid, dim3(WG_THREADS), WgCfg<16>::LDS, st, g)); break;
  }
  GR_LAUNCH_CHECK("gr_wgrad(partial)");
  const int64_t ne = (int64_t)Ka * NC;
  GR_TIMED("wgrad_reduce", st, hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((ne + 15) / 16)), dim3(256), 0, st,
                                                  (const float*)workspace, n_splits, Ka, Nb, NC, c, a_colsum));
  GR_LAUNCH_CHECK("gr_wgrad(reduce)");
  return 0;
}
