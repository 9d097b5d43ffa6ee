// Jagged <-> padded layout kernels and the offsets scan.
// Replace reference utils/ops.py:18-114 (fbgemm asynchronous_complete_cumsum /
// dense_to_jagged / jagged_to_padded_dense, whose CPU fallback is a per-row Python
// loop).  All are stream-ordered and sync-free: the total row count is read from
// offsets[B] on the device.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

// single workgroup exclusive scan: offsets[0] = 0, offsets[b+1] = sum_{<=b} lengths
__global__ __launch_bounds__(1024) void cumsum_kernel(const int64_t* lengths, int B,
                                                     int64_t* offsets) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (B + 1023) / 1024;
  const int lo = t * per, hi = min(B, lo + per);
  int64_t s = 0;
  for (int i = lo; i < hi; ++i) s += lengths[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    int64_t v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  if (t == 0) offsets[0] = 0;
  for (int i = lo; i < hi; ++i) {
    run += lengths[i];
    offsets[i + 1] = run;
  }
}

// one wave per padded row (b, p)
__global__ __launch_bounds__(256) void dense_to_jagged_kernel(const float* dense,
                                                              const int64_t* offsets, int B,
                                                              int N, int D, float* jagged) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * N) return;
  const int b = (int)(row / N), p = (int)(row - (int64_t)b * N);
  const int64_t s0 = offsets[b];
  if (p >= offsets[b + 1] - s0) return;
  const float* src = dense + row * D;
  float* dst = jagged + (s0 + p) * D;
  for (int c = threadIdx.x & 63; c < D; c += 64) dst[c] = src[c];
}

__global__ __launch_bounds__(256) void jagged_to_padded_kernel(const float* jagged,
                                                               const int64_t* offsets, int B,
                                                               int N, int D, float* dense) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (int64_t)B * N) return;
  const int b = (int)(row / N), p = (int)(row - (int64_t)b * N);
  const int64_t s0 = offsets[b];
  const bool valid = p < offsets[b + 1] - s0;
  const float* src = jagged + (s0 + p) * D;
  float* dst = dense + row * D;
  for (int c = threadIdx.x & 63; c < D; c += 64) dst[c] = valid ? src[c] : 0.f;
}

// Row-wise L2 normalisation y = x / max(||x||, eps): 16 lanes per row, 4 rows per wave.
// Replaces postprocessors.py:47-56 (L2NormEmbeddingPostprocessor) and
// negative_sampler.py:31-37.  `gather` (optional): row r reads x[gather_row(r)], with
// gather_row(r) = r * N + lengths[r] - 1 (utils/ops.py:171-187 get_current_embeddings).
__global__ __launch_bounds__(256) void l2norm_kernel(const float* x, int64_t ldx, int64_t rows, int D,
                                                     float eps, const int64_t* lengths, int N,
                                                     int normalize, float* y, int64_t ldy) {
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  const int64_t rc = r < rows ? r : rows - 1;
  const int64_t src = lengths ? rc * N + (lengths[rc] > 0 ? lengths[rc] - 1 : 0) : rc;
  gptr<float> xr = as_global(x) + src * ldx;
  float ss = 0.f;
  for (int c = sub; c < D; c += 16) {
    const float v = xr[c];
    ss += v * v;
  }
  ss = sum16(ss);
  const float inv = normalize ? 1.f / fmaxf(sqrtf(ss), eps) : 1.f;
  if (r < rows)
    for (int c = sub; c < D; c += 16) y[r * ldy + c] = xr[c] * inv;
}

// dx = (dy - y (y . dy)) / ||x||   (||x|| > eps),   dy / eps   otherwise
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* x, int64_t ldx, const float* dy,
                                                         int64_t lddy, int64_t rows, int D, float eps,
                                                         float* dx, int64_t lddx) {
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  const int64_t rc = r < rows ? r : rows - 1;
  gptr<float> xr = as_global(x) + rc * ldx;
  gptr<float> gr_ = as_global(dy) + rc * lddy;
  float ss = 0.f, xg = 0.f;
  for (int c = sub; c < D; c += 16) {
    const float v = xr[c], g = gr_[c];
    ss += v * v;
    xg += v * g;
  }
  ss = sum16(ss);
  xg = sum16(xg);
  const float n = sqrtf(ss);
  if (r >= rows) return;
  if (n > eps) {
    const float inv = 1.f / n;
    const float proj = xg * inv * inv;  // (y . dy) / ||x||
    for (int c = sub; c < D; c += 16) dx[r * lddx + c] = (gr_[c] - xr[c] * proj) * inv;
  } else {
    for (int c = sub; c < D; c += 16) dx[r * lddx + c] = gr_[c] / eps;
  }
}

}  // namespace gr

extern "C" {

int gr_l2_normalize(const float* x, int64_t ld_x, int64_t rows, int D, float eps, float* out,
                    int64_t ld_out, void* stream) {
  GR_REQUIRE(rows >= 0 && D > 0, "gr_l2_normalize: bad args");
  if (rows == 0) return 0;
  GR_REQUIRE(x && out, "gr_l2_normalize: null pointer");
  GR_TIMED("l2_normalize", (hipStream_t)stream,
           hipLaunchKernelGGL(gr::l2norm_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0,
                              (hipStream_t)stream, x, ld_x, rows, D, eps, nullptr, 0, 1, out, ld_out));
  GR_LAUNCH_CHECK("gr_l2_normalize");
  return 0;
}

int gr_l2_normalize_bwd(const float* x, int64_t ld_x, const float* dy, int64_t ld_dy, int64_t rows,
                        int D, float eps, float* dx, int64_t ld_dx, void* stream) {
  GR_REQUIRE(rows >= 0 && D > 0, "gr_l2_normalize_bwd: bad args");
  if (rows == 0) return 0;
  GR_REQUIRE(x && dy && dx, "gr_l2_normalize_bwd: null pointer");
  GR_TIMED("l2_normalize", (hipStream_t)stream,
           hipLaunchKernelGGL(gr::l2norm_bwd_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0,
                              (hipStream_t)stream, x, ld_x, dy, ld_dy, rows, D, eps, dx, ld_dx));
  GR_LAUNCH_CHECK("gr_l2_normalize_bwd");
  return 0;
}

int gr_current_embeddings(const float* encoded, const int64_t* lengths, int B, int N, int D,
                          int normalize, float eps, float* out, void* stream) {
  GR_REQUIRE(encoded && lengths && out && B >= 0 && N > 0 && D > 0,
             "gr_current_embeddings: bad args");
  if (B == 0) return 0;
  GR_TIMED("current_embeddings", (hipStream_t)stream,
           hipLaunchKernelGGL(gr::l2norm_kernel, dim3((unsigned)((B + 15) / 16)), dim3(256), 0,
                              (hipStream_t)stream, encoded, (int64_t)D, (int64_t)B, D, eps, lengths,
                              N, normalize, out, (int64_t)D));
  GR_LAUNCH_CHECK("gr_current_embeddings");
  return 0;
}


int gr_complete_cumsum(const int64_t* lengths, int B, int64_t* offsets, void* stream) {
  GR_REQUIRE(offsets && (B == 0 || lengths) && B >= 0, "gr_complete_cumsum: bad args");
  GR_TIMED("cumsum", (hipStream_t)stream, hipLaunchKernelGGL(gr::cumsum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, lengths,
                     B, offsets));
  GR_LAUNCH_CHECK("gr_complete_cumsum");
  return 0;
}

int gr_dense_to_jagged(const float* dense, const int64_t* offsets, int B, int N, int D,
                       int64_t max_rows, float* jagged, void* stream) {
  (void)max_rows;
  GR_REQUIRE(dense && offsets && jagged && B >= 0 && N >= 0 && D > 0,
             "gr_dense_to_jagged: bad args");
  const int64_t rows = (int64_t)B * N;
  if (rows == 0) return 0;
  GR_TIMED("dense_to_jagged", (hipStream_t)stream, hipLaunchKernelGGL(gr::dense_to_jagged_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256),
                     0, (hipStream_t)stream, dense, offsets, B, N, D, jagged));
  GR_LAUNCH_CHECK("gr_dense_to_jagged");
  return 0;
}

int gr_jagged_to_padded(const float* jagged, const int64_t* offsets, int B, int N, int D,
                        float* dense, void* stream) {
  GR_REQUIRE(dense && offsets && jagged && B >= 0 && N >= 0 && D > 0,
             "gr_jagged_to_padded: bad args");
  const int64_t rows = (int64_t)B * N;
  if (rows == 0) return 0;
  GR_TIMED("jagged_to_padded", (hipStream_t)stream, hipLaunchKernelGGL(gr::jagged_to_padded_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256),
                     0, (hipStream_t)stream, jagged, offsets, B, N, D, dense));
  GR_LAUNCH_CHECK("gr_jagged_to_padded");
  return 0;
}

}  // extern "C"
