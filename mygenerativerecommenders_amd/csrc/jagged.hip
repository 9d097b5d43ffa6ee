// Jagged <-> padded layout kernels and the offsets scan.
// Replace reference utils/ops.py:18-114 (fbgemm asynchronous_complete_cumsum /
// dense_to_jagged / jagged_to_padded_dense, whose CPU fallback is a per-row Python
// loop).  All are stream-ordered and sync-free: the total row count is read from
// offsets[B] on the device.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

// single workgroup exclusive scan: offsets[0] = 0, offsets[b+1] = sum_{<=b} lengths
__global__ __launch_bounds__(256) void cumsum_kernel(const int64_t* lengths, int B,
                                                    int64_t* offsets) {
  offsets_scan(lengths, B, offsets);
}

// Sequence b's valid rows are one contiguous span of L_b * D floats on both sides
// (dense[b, 0:L_b, :] <-> jagged[s0_b : s0_b + L_b, :]), so each copy is a flat,
// fully coalesced stream in units of V (float2 when D is even; rows of 4*D bytes keep
// both sides 8-byte aligned).  Grid: x = chunks of JG_CHUNK units within a sequence,
// y = sequences (strided for B > 65535).  Each thread issues its JG_PER loads before
// any store.
constexpr int JG_PER = 4;
constexpr int JG_CHUNK = 256 * JG_PER;

// Bounded by max_rows (the jagged buffer's row count): nothing is written at or past it.
// zero_fill: the rows of sequence b that the copy does not reach (a length above N is
// truncated, as fbgemm's dense_to_jagged gradient does) and the rows [offsets[B],
// max_rows) are zeroed -- the virtual sequence b == B covers the latter.
template <typename V>
__global__ __launch_bounds__(256) void dense_to_jagged_kernel(const V* dense, const int64_t* offsets,
                                                              int B, int N, int64_t row_units,
                                                              int64_t max_rows, int zero_fill,
                                                              V* jagged) {
  for (int b = blockIdx.y; b <= B; b += gridDim.y) {
    // the first chunk's dense loads do not depend on the offsets (the padded rows of b are
    // always in range): issued before the offsets are read, so the two round trips overlap
    const int64_t nd = (int64_t)N * row_units;
    const V* src = dense + (int64_t)min(b, B - 1) * nd;
    const int64_t base0 = (int64_t)blockIdx.x * JG_CHUNK;
    V v0[JG_PER];
#pragma unroll
    for (int k = 0; k < JG_PER; ++k) {
      const int64_t i = base0 + threadIdx.x + 256 * k;
      v0[k] = b < B && i < nd ? src[i] : V{};
    }
    const int64_t s0 = offsets[b];
    const int64_t s1 = b < B ? offsets[b + 1] : max_rows;
    if (s0 >= max_rows || s0 < 0 || (b == B && !zero_fill)) continue;
    const int64_t end = min(s1, max_rows);                           // rows this span owns
    const int64_t L = b < B ? min(min(s1 - s0, (int64_t)N), end - s0) : 0;  // rows copied
    const int64_t n_copy = L * row_units;
    const int64_t n = (zero_fill ? end - s0 : L) * row_units;
    V* dst = jagged + s0 * row_units;
    for (int64_t base = base0; base < n; base += (int64_t)gridDim.x * JG_CHUNK) {
      V v[JG_PER];
#pragma unroll
      for (int k = 0; k < JG_PER; ++k) {
        const int64_t i = base + threadIdx.x + 256 * k;
        v[k] = i < n_copy ? (base == base0 ? v0[k] : src[i]) : V{};
      }
#pragma unroll
      for (int k = 0; k < JG_PER; ++k) {
        const int64_t i = base + threadIdx.x + 256 * k;
        if (i < n) dst[i] = v[k];
      }
    }
  }
}

template <typename V>
__global__ __launch_bounds__(256) void jagged_to_padded_kernel(const V* jagged, const int64_t* offsets,
                                                               int B, int N, int64_t row_units,
                                                               V* dense) {
  const int64_t n = (int64_t)N * row_units;
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const int64_t s0 = offsets[b];
    const int64_t valid = min(offsets[b + 1] - s0, (int64_t)N) * row_units;
    const V* src = jagged + s0 * row_units;
    V* dst = dense + (int64_t)b * n;
    for (int64_t base = (int64_t)blockIdx.x * JG_CHUNK; base < n; base += (int64_t)gridDim.x * JG_CHUNK) {
      V v[JG_PER];
#pragma unroll
      for (int k = 0; k < JG_PER; ++k) {
        const int64_t i = base + threadIdx.x + 256 * k;
        v[k] = i < valid ? src[i] : V{};
      }
#pragma unroll
      for (int k = 0; k < JG_PER; ++k) {
        const int64_t i = base + threadIdx.x + 256 * k;
        if (i < n) dst[i] = v[k];
      }
    }
  }
}

template <typename V>
static void launch_jagged_copy(bool to_jagged, const float* src, const int64_t* offsets, int B, int N,
                               int D, float* dst, hipStream_t st, int64_t max_rows = 0,
                               int zero_fill = 0) {
  const int64_t units = (int64_t)D * sizeof(float) / sizeof(V);
  const int64_t chunks = ((int64_t)N * units + JG_CHUNK - 1) / JG_CHUNK;
  const int ny = to_jagged && zero_fill ? B + 1 : B;
  const dim3 grid((unsigned)(chunks > 0 ? chunks : 1), (unsigned)(ny < 65535 ? ny : 65535));
  if (to_jagged)
    GR_TIMED("dense_to_jagged", st,
             hipLaunchKernelGGL(dense_to_jagged_kernel<V>, grid, dim3(256), 0, st,
                                reinterpret_cast<const V*>(src), offsets, B, N, units, max_rows,
                                zero_fill, reinterpret_cast<V*>(dst)));
  else
    GR_TIMED("jagged_to_padded", st,
             hipLaunchKernelGGL(jagged_to_padded_kernel<V>, grid, dim3(256), 0, st,
                                reinterpret_cast<const V*>(src), offsets, B, N, units,
                                reinterpret_cast<V*>(dst)));
}

static bool aligned8(const void* a, const void* b) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 7) == 0;
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
  GR_TIMED("cumsum", (hipStream_t)stream, hipLaunchKernelGGL(gr::cumsum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, lengths,
                     B, offsets));
  GR_LAUNCH_CHECK("gr_complete_cumsum");
  return 0;
}

int gr_dense_to_jagged(const float* dense, const int64_t* offsets, int B, int N, int D,
                       int64_t max_rows, int zero_fill, float* jagged, void* stream) {
  GR_REQUIRE(dense && offsets && jagged && B >= 0 && N >= 0 && D > 0 && max_rows >= 0,
             "gr_dense_to_jagged: bad args");
  if (max_rows == 0 || (B == 0 && !zero_fill)) return 0;
  if (B == 0 || N == 0) {
    if (zero_fill) gr::zero_words_async(jagged, max_rows * D, (hipStream_t)stream);
    GR_LAUNCH_CHECK("gr_dense_to_jagged");
    return 0;
  }
  if (D % 2 == 0 && gr::aligned8(dense, jagged))
    gr::launch_jagged_copy<float2>(true, dense, offsets, B, N, D, jagged, (hipStream_t)stream,
                                   max_rows, zero_fill);
  else
    gr::launch_jagged_copy<float>(true, dense, offsets, B, N, D, jagged, (hipStream_t)stream,
                                  max_rows, zero_fill);
  GR_LAUNCH_CHECK("gr_dense_to_jagged");
  return 0;
}

int gr_jagged_to_padded(const float* jagged, const int64_t* offsets, int B, int N, int D,
                        float* dense, void* stream) {
  GR_REQUIRE(dense && offsets && jagged && B >= 0 && N >= 0 && D > 0,
             "gr_jagged_to_padded: bad args");
  const int64_t rows = (int64_t)B * N;
  if (rows == 0) return 0;
  if (D % 2 == 0 && gr::aligned8(jagged, dense))
    gr::launch_jagged_copy<float2>(false, jagged, offsets, B, N, D, dense, (hipStream_t)stream);
  else
    gr::launch_jagged_copy<float>(false, jagged, offsets, B, N, D, dense, (hipStream_t)stream);
  GR_LAUNCH_CHECK("gr_jagged_to_padded");
  return 0;
}

}  // extern "C"
