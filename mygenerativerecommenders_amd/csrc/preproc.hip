// Input-features preprocessor, forward and backward, one pass each.
//
// Replaces LearnablePositionalEmbeddingInputFeaturesPreprocessor.forward
// (preprocessors/learnable_positional_embedding.py:42-58):
//   y = dropout(x * sqrt(D) + pos_emb[n]) * (past_ids != 0)
// which PyTorch runs as ~7 elementwise / gather kernels forward and as many backward.
// Dropout keeps an element when hash(seed + *seed_off, element) >= p * 2^32 (the same
// counter hash as the STU layers), so the backward regenerates the mask instead of
// storing it and a captured graph draws a fresh mask per replay (the caller bumps
// *seed_off on the device).
//
// Backward:  dx = dy * keep/(1-p) * valid * sqrt(D);
//            dpos[n] = sum_b dy[b, n] * keep/(1-p) * valid  (fixed b order: deterministic).
// Layout: (B, N, D) contiguous; a 16-lane group per (b, n) row, 4 rows per wave.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

__device__ __forceinline__ float pre_keep(uint64_t seed, int64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t hsh = hash_u32(seed, (uint64_t)idx);
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  return hsh >= thr ? 1.f / (1.f - p) : 0.f;
}

__global__ __launch_bounds__(256) void preproc_fwd_kernel(const float* x, const int64_t* ids,
                                                          const float* pos, int64_t rows, int N,
                                                          int D, float scale, float p, uint64_t seed,
                                                          const int64_t* seed_off, float* y) {
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (r >= rows) return;
  const int sub = threadIdx.x & 15;
  const int n = (int)(r % N);
  const uint64_t sd = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  const bool valid = ids[r] != 0;
  gptr<float> xr = as_global(x) + r * D;
  gptr<float> pr = as_global(pos) + (int64_t)n * D;
  float* yr = y + r * D;
  for (int c = sub; c < D; c += 16) {
    const float v = fmaf(xr[c], scale, pr[c]);
    yr[c] = valid ? v * pre_keep(sd, r * D + c, p) : 0.f;
  }
}

__global__ __launch_bounds__(256) void preproc_bwd_x_kernel(const float* dy, const int64_t* ids,
                                                            int64_t rows, int D, float scale, float p,
                                                            uint64_t seed, const int64_t* seed_off,
                                                            float* dx) {
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (r >= rows) return;
  const int sub = threadIdx.x & 15;
  const uint64_t sd = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  const bool valid = ids[r] != 0;
  gptr<float> gr_ = as_global(dy) + r * D;
  float* dr = dx + r * D;
  for (int c = sub; c < D; c += 16)
    dr[c] = valid ? gr_[c] * pre_keep(sd, r * D + c, p) * scale : 0.f;
}

// dpos[n][c]: a workgroup owns 16 consecutive outputs i = n * D + c; thread (o, grp)
// sums b = grp, grp + 16, ... in order (8 loads in flight), then the 16 partials are
// added in grp order (deterministic, no atomics).  Splitting B over 16 groups gives
// N * D / 16 workgroups (660 at ml-1m) instead of N * D / 256 (42), each with a
// 16x shorter dependent chain.
constexpr int kPosGroups = 16;
__global__ __launch_bounds__(256) void preproc_bwd_pos_kernel(const float* dy, const int64_t* ids,
                                                              int B, int N, int D, float p,
                                                              uint64_t seed, const int64_t* seed_off,
                                                              float* dpos) {
  __shared__ float part[kPosGroups][17];
  const int o = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + o;
  const int64_t nd = (int64_t)N * D;
  const int64_t ic = i < nd ? i : nd - 1;
  const int n = (int)(ic / D), c = (int)(ic % D);
  const uint64_t sd = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  float acc = 0.f;
  int b = grp;
  for (; b + 7 * kPosGroups < B; b += 8 * kPosGroups) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t r = (int64_t)(b + kPosGroups * u) * N + n;
      v[u] = ids[r] != 0 ? dy[r * D + c] * pre_keep(sd, r * D + c, p) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; b < B; b += kPosGroups) {
    const int64_t r = (int64_t)b * N + n;
    acc += ids[r] != 0 ? dy[r * D + c] * pre_keep(sd, r * D + c, p) : 0.f;
  }
  part[grp][o] = acc;
  __syncthreads();
  if (grp == 0 && i < nd) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kPosGroups; ++k) s += part[k][o];
    dpos[i] = s;
  }
}

}  // namespace gr

extern "C" {

int gr_preproc_fwd(const float* x, const int64_t* past_ids, const float* pos_w, int B, int N, int D,
                   float scale, float dropout_p, uint64_t seed, const int64_t* seed_offset, float* y,
                   void* stream) {
  GR_REQUIRE(B >= 0 && N > 0 && D > 0 && dropout_p >= 0.f && dropout_p < 1.f,
             "gr_preproc_fwd: bad args (B=%d N=%d D=%d p=%f)", B, N, D, dropout_p);
  const int64_t rows = (int64_t)B * N;
  if (rows == 0) return 0;
  GR_REQUIRE(x && past_ids && pos_w && y, "gr_preproc_fwd: null pointer");
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("preproc", st,
           hipLaunchKernelGGL(gr::preproc_fwd_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0,
                              st, x, past_ids, pos_w, rows, N, D, scale, dropout_p, seed, seed_offset,
                              y));
  GR_LAUNCH_CHECK("gr_preproc_fwd");
  return 0;
}

int gr_preproc_bwd(const float* dy, const int64_t* past_ids, int B, int N, int D, float scale,
                   float dropout_p, uint64_t seed, const int64_t* seed_offset, float* dx, float* dpos_w,
                   void* stream) {
  GR_REQUIRE(B >= 0 && N > 0 && D > 0 && dropout_p >= 0.f && dropout_p < 1.f,
             "gr_preproc_bwd: bad args (B=%d N=%d D=%d p=%f)", B, N, D, dropout_p);
  const hipStream_t st = (hipStream_t)stream;
  const int64_t rows = (int64_t)B * N;
  GR_REQUIRE(dy && past_ids && (dx || dpos_w) || rows == 0, "gr_preproc_bwd: null pointer");
  if (dx && rows > 0) {
    GR_TIMED("preproc", st,
             hipLaunchKernelGGL(gr::preproc_bwd_x_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256),
                                0, st, dy, past_ids, rows, D, scale, dropout_p, seed, seed_offset, dx));
    GR_LAUNCH_CHECK("gr_preproc_bwd(dx)");
  }
  if (dpos_w) {
    const int64_t nd = (int64_t)N * D;
    GR_TIMED("preproc", st,
             hipLaunchKernelGGL(gr::preproc_bwd_pos_kernel, dim3((unsigned)((nd + 15) / 16)), dim3(256),
                                0, st, dy, past_ids, B, N, D, dropout_p, seed, seed_offset, dpos_w));
    GR_LAUNCH_CHECK("gr_preproc_bwd(dpos)");
  }
  return 0;
}

}  // extern "C"
