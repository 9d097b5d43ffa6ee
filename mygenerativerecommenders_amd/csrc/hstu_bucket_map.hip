// Relative-time bucket map, computed ONCE per batch and shared by every layer's
// attention forward and backward (the timestamps do not change across layers).
//
// Reference: sequential_encoders/hstu.py:111-123 builds an int64 (B, N, N) bucket tensor
// per layer (45.6 MB at ml-1m) and re-derives it in every layer.  Here the causal
// 64 x 64 tiles of each sequence are stored as uint8 in two orientations:
//   map_qk[b][tile(qt, kt)][q][k]  -- read by the query-major kernels (fwd, dQ): a lane
//                                     loads the 4 keys 4g..4g+3 of its query as 1 dword
//   map_kq[b][tile(qt, kt)][k][q]  -- read by the key-major kernel (dK, dV)
// tile(qt, kt) = qt (qt + 1) / 2 + kt, kt <= qt.  bucket(i, j) = max{b : thr[b] <=
// |ts_next(i) - ts(j)|} with ts_next(i) = ts[i + 1] (ts[N - 1] for i = N - 1),
// hstu.py:113-119; entries outside the sequence are 0 (masked by the consumers).
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

__host__ __device__ inline int tiles_per_seq(int N) {
  const int T = (N + 63) / 64;
  return T * (T + 1) / 2;
}

__global__ __launch_bounds__(256) void bucket_map_kernel(const int64_t* ts, const int64_t* offsets,
                                                         int B, int N, const int64_t* thr_g,
                                                         int nb, uint8_t* map_qk,
                                                         uint8_t* map_kq) {
  __shared__ int64_t thr[256];
  __shared__ int64_t tsq[64], tsk[64];
  __shared__ uint32_t tile[64][17];  // [q][k/4] packed bytes, padded row
  const int tpb = tiles_per_seq(N);
  const int b = blockIdx.x / tpb;
  const int t = blockIdx.x % tpb;
  int qt = 0;
  while ((qt + 1) * (qt + 2) / 2 <= t) ++qt;
  const int kt = t - qt * (qt + 1) / 2;
  const int tid = threadIdx.x;
  const int64_t s0 = offsets[b];
  const int L = (int)(offsets[b + 1] - s0);
  for (int i = tid; i <= nb; i += 256) thr[i] = thr_g[i];
  if (tid < 64) {
    const int q = qt * 64 + tid;
    const int nx = q + 1 < N ? q + 1 : N - 1;
    const int qc = q < N ? q : N - 1;
    tsq[tid] = ts[(int64_t)b * N + (q < N ? nx : qc)];
  } else if (tid < 128) {
    const int k = kt * 64 + tid - 64;
    tsk[tid - 64] = ts[(int64_t)b * N + (k < N ? k : N - 1)];
  }
  __syncthreads();
  // thread -> (q = tid / 4, 16 keys = 4 dwords)
  const int ql = tid >> 2, part = tid & 3;
  const int q = qt * 64 + ql;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kl = part * 16 + d * 4 + e;
      const int k = kt * 64 + kl;
      uint32_t bk = 0;
      if (q < L && k <= q) bk = (uint32_t)time_bucket(tsq[ql] - tsk[kl], thr, nb);
      word |= bk << (8 * e);
    }
    tile[ql][part * 4 + d] = word;
  }
  __syncthreads();
  const int64_t base = ((int64_t)b * tpb + t) * 4096;
  // map_qk: row q = 16 dwords
  uint32_t* dst_qk = reinterpret_cast<uint32_t*>(map_qk + base);
  for (int i = tid; i < 64 * 16; i += 256) dst_qk[i] = tile[i >> 4][i & 15];
  // map_kq: row k holds the 64 queries' bytes
  uint32_t* dst_kq = reinterpret_cast<uint32_t*>(map_kq + base);
  for (int i = tid; i < 64 * 16; i += 256) {
    const int kl = i >> 4, qd = i & 15;
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ql2 = qd * 4 + e;
      const uint32_t w = tile[ql2][kl >> 2];
      word |= ((w >> (8 * (kl & 3))) & 0xFFu) << (8 * e);
    }
    dst_kq[i] = word;
  }
}

}  // namespace gr

extern "C" size_t hstu_bucket_map_bytes(int B, int N) {
  if (B <= 0 || N <= 0) return 0;
  return (size_t)2 * B * gr::tiles_per_seq(N) * 4096;
}

extern "C" int hstu_bucket_map(const int64_t* ts, const int64_t* offsets, int B, int N,
                               const int64_t* bucket_thr, int num_buckets, uint8_t* map,
                               void* stream) {
  GR_REQUIRE(ts && offsets && bucket_thr && map, "hstu_bucket_map: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && num_buckets > 0 && num_buckets < 256,
             "hstu_bucket_map: bad sizes (num_buckets must be < 256)");
  if (B == 0) return 0;
  const int tpb = gr::tiles_per_seq(N);
  uint8_t* map_kq = map + (size_t)B * tpb * 4096;
  GR_TIMED("bucket_map", (hipStream_t)stream, hipLaunchKernelGGL(gr::bucket_map_kernel, dim3(B * tpb), dim3(256), 0, (hipStream_t)stream, ts,
                     offsets, B, N, bucket_thr, num_buckets, map, map_kq));
  GR_LAUNCH_CHECK("hstu_bucket_map");
  return 0;
}

// ------------------------------------------------------------------ materialised bias
// RelativeBucketedTimeAndPositionBasedBias.forward (hstu.py:96-128) for callers that
// want the (B, N, N) tensor itself (debug hooks, the module called on its own); the
// attention kernels never use it.  bias[b, i, j] = pos_w[N - 1 + j - i]
//   + ts_w[bucket(ts_next(b, i) - ts(b, j))] over ALL (i, j), causal or not, as the
// reference computes it.  Backward: d_pos_w by diagonal (one thread per offset, b and i
// in order) and d_ts_w by per-row bucket sums (slabs, then a fixed-order reduce): both
// deterministic, no float atomics.
namespace gr {

__global__ __launch_bounds__(256) void rel_bias_fwd_kernel(const int64_t* ts, int B, int N,
                                                           const int64_t* thr_g, int nb,
                                                           const float* pos_w, const float* ts_w,
                                                           float* out) {
  __shared__ int64_t thr[256];
  for (int i = threadIdx.x; i <= nb; i += 256) thr[i] = thr_g[i];
  __syncthreads();
  const int64_t row = blockIdx.x;  // (b, i)
  const int b = (int)(row / N), i = (int)(row % N);
  const int64_t tq = ts[(int64_t)b * N + (i + 1 < N ? i + 1 : N - 1)];
  for (int j = threadIdx.x; j < N; j += 256) {
    const int bk = time_bucket(tq - ts[(int64_t)b * N + j], thr, nb);
    out[row * N + j] = pos_w[N - 1 + j - i] + ts_w[bk];
  }
}

__global__ __launch_bounds__(256) void rel_bias_dpos_kernel(const float* dout, int B, int N,
                                                            float* d_pos) {
  const int r = blockIdx.x * 256 + threadIdx.x;  // j - i + N - 1
  if (r >= 2 * N - 1) return;
  const int dlt = r - (N - 1);
  const int i0 = dlt < 0 ? -dlt : 0, i1 = dlt < 0 ? N : N - dlt;
  float acc = 0.f;
  for (int b = 0; b < B; ++b)
    for (int i = i0; i < i1; ++i) acc += dout[((int64_t)b * N + i) * N + i + dlt];
  d_pos[r] = acc;
}

// one workgroup per (b, i) row: bucket sums of the row in j order -> slab[row][nb + 1]
__global__ __launch_bounds__(256) void rel_bias_dts_rows_kernel(const int64_t* ts, const float* dout,
                                                                int B, int N, const int64_t* thr_g,
                                                                int nb, float* slabs) {
  __shared__ int64_t thr[256];
  __shared__ uint8_t bk[1024];
  __shared__ float val[1024];
  for (int i = threadIdx.x; i <= nb; i += 256) thr[i] = thr_g[i];
  const int64_t row = blockIdx.x;
  const int b = (int)(row / N), i = (int)(row % N);
  const int64_t tq = ts[(int64_t)b * N + (i + 1 < N ? i + 1 : N - 1)];
  float acc = 0.f;  // thread t <= nb: bucket t
  for (int j0 = 0; j0 < N; j0 += 1024) {
    __syncthreads();
    for (int j = threadIdx.x; j < 1024 && j0 + j < N; j += 256) {
      bk[j] = (uint8_t)time_bucket(tq - ts[(int64_t)b * N + j0 + j], thr, nb);
      val[j] = dout[row * N + j0 + j];
    }
    __syncthreads();
    if ((int)threadIdx.x <= nb) {
      const int n = N - j0 < 1024 ? N - j0 : 1024;
      for (int j = 0; j < n; ++j)
        if (bk[j] == threadIdx.x) acc += val[j];
    }
  }
  if ((int)threadIdx.x <= nb) slabs[row * (nb + 1) + threadIdx.x] = acc;
}

// one workgroup per bucket: thread t sums slab rows t, t + 256, ... in order, then a
// fixed-order tree over the 256 partials
__global__ __launch_bounds__(256) void rel_bias_dts_reduce_kernel(const float* slabs, int64_t rows,
                                                                  int nb, float* d_ts) {
  __shared__ float part[256];
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int64_t r = threadIdx.x; r < rows; r += 256) acc += slabs[r * (nb + 1) + c];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) d_ts[c] = part[0];
}

}  // namespace gr

extern "C" int hstu_rel_bias_fwd(const int64_t* ts, int B, int N, const int64_t* bucket_thr,
                                 int num_buckets, const float* pos_w, const float* ts_w,
                                 float* out, void* stream) {
  GR_REQUIRE(ts && bucket_thr && pos_w && ts_w && out, "hstu_rel_bias_fwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && num_buckets > 0 && num_buckets < 256,
             "hstu_rel_bias_fwd: bad sizes (num_buckets must be < 256)");
  GR_REQUIRE((int64_t)B * N < 0x7fffffff, "hstu_rel_bias_fwd: B * N too large");
  if (B == 0) return 0;
  hipLaunchKernelGGL(gr::rel_bias_fwd_kernel, dim3(B * N), dim3(256), 0, (hipStream_t)stream, ts,
                     B, N, bucket_thr, num_buckets, pos_w, ts_w, out);
  GR_LAUNCH_CHECK("hstu_rel_bias_fwd");
  return 0;
}

extern "C" size_t hstu_rel_bias_bwd_workspace_size(int B, int N, int num_buckets) {
  if (B <= 0 || N <= 0 || num_buckets <= 0) return 0;
  return sizeof(float) * (size_t)B * N * (num_buckets + 1);
}

extern "C" int hstu_rel_bias_bwd(const int64_t* ts, int B, int N, const int64_t* bucket_thr,
                                 int num_buckets, const float* dout, float* d_pos_w,
                                 float* d_ts_w, void* workspace, size_t ws_bytes, void* stream) {
  GR_REQUIRE(ts && bucket_thr && dout && d_pos_w && d_ts_w, "hstu_rel_bias_bwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && num_buckets > 0 && num_buckets < 256,
             "hstu_rel_bias_bwd: bad sizes (num_buckets must be < 256)");
  GR_REQUIRE((int64_t)B * N < 0x7fffffff, "hstu_rel_bias_bwd: B * N too large");
  const hipStream_t st = (hipStream_t)stream;
  if (B == 0) {
    gr::zero_words_async(d_pos_w, 2 * N - 1, st);
    gr::zero_words_async(d_ts_w, num_buckets + 1, st);
    return 0;
  }
  const size_t need = hstu_rel_bias_bwd_workspace_size(B, N, num_buckets);
  GR_REQUIRE(workspace && ws_bytes >= need, "hstu_rel_bias_bwd: workspace %zu B < %zu B",
             ws_bytes, need);
  float* slabs = (float*)workspace;
  hipLaunchKernelGGL(gr::rel_bias_dpos_kernel, dim3((2 * N - 1 + 255) / 256), dim3(256), 0, st,
                     dout, B, N, d_pos_w);
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dpos)");
  hipLaunchKernelGGL(gr::rel_bias_dts_rows_kernel, dim3(B * N), dim3(256), 0, st, ts, dout, B, N,
                     bucket_thr, num_buckets, slabs);
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dts rows)");
  hipLaunchKernelGGL(gr::rel_bias_dts_reduce_kernel, dim3(num_buckets + 1), dim3(256), 0, st,
                     slabs, (int64_t)B * N, num_buckets, d_ts_w);
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dts reduce)");
  return 0;
}
