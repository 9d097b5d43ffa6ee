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

// Tile t (causal order) of sequence b, L = its length: both orientations of the tile.
__device__ __forceinline__ void bucket_tile(const int64_t* ts, int b, int t, int L, int N, int tpb,
                                            const int64_t* thr_g, int nb, uint8_t* map_qk,
                                            uint8_t* map_kq) {
  __shared__ int64_t thr[256];
  __shared__ int64_t tsq[64], tsk[64];
  __shared__ uint32_t tile_kq[64][17];  // [k][q/4] packed bytes, padded row
  int qt = (int)((sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);  // t = qt (qt + 1) / 2 + kt
  while (qt > 0 && qt * (qt + 1) / 2 > t) --qt;
  while ((qt + 1) * (qt + 2) / 2 <= t) ++qt;
  const int kt = t - qt * (qt + 1) / 2;
  const int tid = threadIdx.x;
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
  // thread -> a 4 x 4 block: queries 4 qb .. 4 qb + 3, keys 4 kb .. 4 kb + 3.  Its four
  // query-major words (4 keys each) are stored as they are; the four key-major words
  // (4 queries each) are the same 16 bytes transposed in registers, staged through LDS
  // for a coalesced store (conflict-free: row stride 17 dwords)
  const int kb = tid & 15, qb = tid >> 4;
  uint32_t bk[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ql = 4 * qb + i, q = qt * 64 + ql;
    const int64_t tq = tsq[ql];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kl = 4 * kb + e, k = kt * 64 + kl;
      bk[i][e] = (q < L && k <= q) ? (uint32_t)time_bucket(tq - tsk[kl], thr, nb) : 0u;
    }
  }
  const int64_t base = ((int64_t)b * tpb + t) * 4096;
  uint32_t* dst_qk = reinterpret_cast<uint32_t*>(map_qk + base);  // row q = 16 dwords
#pragma unroll
  for (int i = 0; i < 4; ++i)
    dst_qk[(4 * qb + i) * 16 + kb] = bk[i][0] | (bk[i][1] << 8) | (bk[i][2] << 16) | (bk[i][3] << 24);
#pragma unroll
  for (int e = 0; e < 4; ++e)
    tile_kq[4 * kb + e][qb] = bk[0][e] | (bk[1][e] << 8) | (bk[2][e] << 16) | (bk[3][e] << 24);
  __syncthreads();
  // map_kq: row k holds the 64 queries' bytes
  uint32_t* dst_kq = reinterpret_cast<uint32_t*>(map_kq + base);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = tid + 256 * j;
    dst_kq[i] = tile_kq[i >> 4][i & 15];
  }
}

__global__ __launch_bounds__(256) void bucket_map_kernel(const int64_t* ts, const int64_t* offsets,
                                                         int B, int N, const int64_t* thr_g,
                                                         int nb, uint8_t* map_qk,
                                                         uint8_t* map_kq) {
  const int tpb = tiles_per_seq(N);
  const int b = blockIdx.x / tpb;
  bucket_tile(ts, b, blockIdx.x % tpb, (int)(offsets[b + 1] - offsets[b]), N, tpb, thr_g, nb,
              map_qk, map_kq);
}

// ------------------------------------------------------------------ encoder prologue
// The batch setup of an encoder forward as one launch (hstu.py:502, utils/ops.py:18-64,
// and the bucket map above): x_offsets = complete_cumsum(lengths), the padded input rows
// -> jagged rows, the bucket map, and one step of the dropout counter.  Three kinds of
// workgroup, none waiting for another:
//   [0, n_bucket)               bucket tiles (L = lengths[b]),
//   [n_bucket, + n_copy)        copy chunks: each wave sums lengths[0 .. b) itself for the
//                               destination row s0; the chunk's padded rows are loaded
//                               before that sum is known (they are always in range),
//   last                        the offsets scan, then step += 1.
// Copies as gr_dense_to_jagged with zero_fill = 0: min(L, N) rows of sequence b, none at
// or past max_rows.
struct PrologueArgs {
  const int64_t* lengths;
  int B, N;
  const void* x;      // [B][N][row_units] units of V
  int64_t row_units;
  int64_t max_rows;
  int chunks;         // copy workgroups per sequence
  const int64_t* ts;  // [B][N] (bucket map) or null
  const int64_t* thr;
  int nb, tpb;
  int n_bucket, n_copy;
  int64_t* offsets;
  void* xj;           // [max_rows][row_units]
  uint8_t* map_qk;
  uint8_t* map_kq;
  int64_t* step;      // dropout step counter or null
};

constexpr int PRO_PER = 4;
constexpr int PRO_CHUNK = 256 * PRO_PER;

template <typename V>
__global__ __launch_bounds__(256) void encoder_prologue_kernel(PrologueArgs a) {
  const int id = blockIdx.x;
  if (id < a.n_bucket) {
    const int b = id / a.tpb;
    bucket_tile(a.ts, b, id % a.tpb, (int)a.lengths[b], a.N, a.tpb, a.thr, a.nb, a.map_qk, a.map_kq);
    return;
  }
  const int j = id - a.n_bucket;
  if (j < a.n_copy) {
    const int b = j / a.chunks;
    const int64_t nd = (int64_t)a.N * a.row_units;
    const V* src = reinterpret_cast<const V*>(a.x) + (int64_t)b * nd;
    const int64_t base = (int64_t)(j % a.chunks) * PRO_CHUNK;
    V v[PRO_PER];
#pragma unroll
    for (int k = 0; k < PRO_PER; ++k) {
      const int64_t i = base + threadIdx.x + 256 * k;
      v[k] = i < nd ? src[i] : V{};
    }
    const int lane = threadIdx.x & 63;
    int64_t s0 = 0;
    for (int i = lane; i < b; i += 64) s0 += a.lengths[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s0 += __shfl_xor(s0, o, 64);
    const int64_t len = a.lengths[b];
    if (s0 < 0 || s0 >= a.max_rows || len <= 0) return;
    const int64_t L = min(min(len, (int64_t)a.N), a.max_rows - s0);
    const int64_t n_copy = L * a.row_units;
    V* dst = reinterpret_cast<V*>(a.xj) + s0 * a.row_units;
#pragma unroll
    for (int k = 0; k < PRO_PER; ++k) {
      const int64_t i = base + threadIdx.x + 256 * k;
      if (i < n_copy) dst[i] = v[k];
    }
    return;
  }
  offsets_scan(a.lengths, a.B, a.offsets);
  if (threadIdx.x == 0 && a.step) a.step[0] = a.step[0] + 1;
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

extern "C" int hstu_encoder_prologue(const int64_t* lengths, int B, int N, const float* x, int D,
                                     int64_t max_rows, const int64_t* ts, const int64_t* bucket_thr,
                                     int num_buckets, int64_t* offsets, float* x_jagged,
                                     uint8_t* map, int64_t* step, void* stream) {
  GR_REQUIRE(offsets && B >= 0 && N >= 0 && D > 0 && max_rows >= 0,
             "hstu_encoder_prologue: bad args");
  GR_REQUIRE(B == 0 || (lengths && x && x_jagged), "hstu_encoder_prologue: null pointer");
  GR_REQUIRE(!map || (ts && bucket_thr && N > 0 && num_buckets > 0 && num_buckets < 256),
             "hstu_encoder_prologue: bucket map needs ts, the threshold table, N > 0 and "
             "0 < num_buckets < 256");
  gr::PrologueArgs a{};
  a.lengths = lengths;
  a.B = B;
  a.N = N;
  a.x = x;
  a.max_rows = max_rows;
  a.ts = ts;
  a.thr = bucket_thr;
  a.nb = num_buckets;
  a.offsets = offsets;
  a.xj = x_jagged;
  a.step = step;
  const bool v2 = D % 2 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(x_jagged)) & 7) == 0;
  a.row_units = v2 ? D / 2 : D;
  a.chunks = (int)((int64_t)N * a.row_units + gr::PRO_CHUNK - 1) / gr::PRO_CHUNK;
  a.tpb = N > 0 ? gr::tiles_per_seq(N) : 0;
  a.n_bucket = map && B > 0 ? B * a.tpb : 0;
  a.n_copy = max_rows > 0 ? B * a.chunks : 0;
  if (map) {
    a.map_qk = map;
    a.map_kq = map + (size_t)B * a.tpb * 4096;
  }
  const dim3 grid((unsigned)(a.n_bucket + a.n_copy + 1));
  const hipStream_t st = (hipStream_t)stream;
  if (v2)
    GR_TIMED("encoder_prologue", st, hipLaunchKernelGGL(gr::encoder_prologue_kernel<float2>, grid, dim3(256), 0, st, a));
  else
    GR_TIMED("encoder_prologue", st, hipLaunchKernelGGL(gr::encoder_prologue_kernel<float>, grid, dim3(256), 0, st, a));
  GR_LAUNCH_CHECK("hstu_encoder_prologue");
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

// one workgroup per diagonal r = j - i + N - 1: threads stride over its B * len entries in a
// fixed order, then a fixed-order tree (deterministic)
__global__ __launch_bounds__(256) void rel_bias_dpos_kernel(const float* dout, int B, int N,
                                                            float* d_pos) {
  __shared__ float part[256];
  const int r = blockIdx.x;
  const int dlt = r - (N - 1);
  const int i0 = dlt < 0 ? -dlt : 0, i1 = dlt < 0 ? N : N - dlt;
  const int len = i1 - i0;
  const int total = B * len;  // B * N < 2^31 (checked by the entry)
  // 4 partial sums (entries t, t + 256, t + 512, t + 768 of each group of 1024): 4 loads in
  // flight instead of a chain of dependent adds
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int b = threadIdx.x / len, i = threadIdx.x - b * len;
  const int bs = 256 / len, is = 256 - bs * len;  // the stride 256 as (b, i) steps
  int q = 0;
  for (int t = threadIdx.x; t < total; t += 256) {
    const float v = dout[((int64_t)b * N + i0 + i) * N + i0 + i + dlt];
    acc[0] += q == 0 ? v : 0.f;
    acc[1] += q == 1 ? v : 0.f;
    acc[2] += q == 2 ? v : 0.f;
    acc[3] += q == 3 ? v : 0.f;
    q = (q + 1) & 3;
    b += bs;
    i += is;
    if (i >= len) {
      i -= len;
      ++b;
    }
  }
  part[threadIdx.x] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) d_pos[r] = part[0];
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
  // 4 partial sums over rows t + 1024 k + 256 q, q = 0..3 (4 loads in flight)
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int64_t r = threadIdx.x;
  for (; r + 768 < rows; r += 1024) {
    a0 += slabs[r * (nb + 1) + c];
    a1 += slabs[(r + 256) * (nb + 1) + c];
    a2 += slabs[(r + 512) * (nb + 1) + c];
    a3 += slabs[(r + 768) * (nb + 1) + c];
  }
  for (; r < rows; r += 256) a0 += slabs[r * (nb + 1) + c];
  part[threadIdx.x] = (a0 + a1) + (a2 + a3);
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
  GR_TIMED("rel_bias_fwd", (hipStream_t)stream,
           hipLaunchKernelGGL(gr::rel_bias_fwd_kernel, dim3(B * N), dim3(256), 0,
                              (hipStream_t)stream, ts, B, N, bucket_thr, num_buckets, pos_w, ts_w,
                              out));
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
  GR_TIMED("rel_bias_bwd", st,
           hipLaunchKernelGGL(gr::rel_bias_dpos_kernel, dim3(2 * N - 1), dim3(256), 0, st, dout,
                              B, N, d_pos_w));
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dpos)");
  GR_TIMED("rel_bias_bwd", st,
           hipLaunchKernelGGL(gr::rel_bias_dts_rows_kernel, dim3(B * N), dim3(256), 0, st, ts,
                              dout, B, N, bucket_thr, num_buckets, slabs));
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dts rows)");
  GR_TIMED("rel_bias_bwd", st,
           hipLaunchKernelGGL(gr::rel_bias_dts_reduce_kernel, dim3(num_buckets + 1), dim3(256), 0,
                              st, slabs, (int64_t)B * N, num_buckets, d_ts_w));
  GR_LAUNCH_CHECK("hstu_rel_bias_bwd(dts reduce)");
  return 0;
}
