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
