// Cached (incremental) HSTU decoding: the delta_x_offsets / cache branch of
// sequential_encoders/hstu.py (:151-177, :293-298, :321-322, :393-423).
//
// The reference re-encodes the rows x[delta_x_offsets[0]] only, writes their v into the
// jagged v cache and their q / k into the padded (B, n, .) caches (index_copy_), then runs
// the WHOLE (B, h, n, n) attention over the caches and keeps the delta rows
// (hstu.py:393-397).  Only those rows reach the output, so hstu_decode_attn computes just
// them: one workgroup per (delta row, head) streams the cached keys 0 .. p of the row's
// sequence (p = its position) and their values — an HBM-bound pass over K and V of
// 4 (p + 1) (dqk + dv) bytes per (row, head), no (n, n) scores.  gr_rows_copy does the
// row gathers / scatters (x[delta], the three cache updates, the output rows).
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

// dst[row_d(e)] = src[row_s(e)], width floats, e < n; row(e) = index ? index[e] + e * step
// : e.  Rows outside [0, rows) are skipped (the host validates them; no access past the
// buffers either way).
__global__ __launch_bounds__(256) void rows_copy_kernel(const float* src, int64_t ld_src,
                                                        const int64_t* src_index, int64_t src_step,
                                                        int64_t src_rows, float* dst, int64_t ld_dst,
                                                        const int64_t* dst_index, int64_t dst_step,
                                                        int64_t dst_rows, int width) {
  const int64_t e = blockIdx.x;
  const int64_t rs = src_index ? src_index[e] + e * src_step : e;
  const int64_t rd = dst_index ? dst_index[e] + e * dst_step : e;
  if (rs < 0 || rs >= src_rows || rd < 0 || rd >= dst_rows) return;
  const float* s = src + rs * ld_src;
  float* d = dst + rd * ld_dst;
  for (int c = threadIdx.x; c < width; c += 256) d[c] = s[c];
}

struct DecodeArgs {
  const float* q;  // padded (B, N, ld_qk) caches
  const float* k;
  int64_t ld_qk;
  const float* v;  // jagged (v_rows, ld_v) cache
  int64_t ld_v, v_rows;
  const int64_t* offsets;
  int B;
  const int64_t* rows;  // jagged row of each delta entry
  int N, H, dqk, dv;
  const int64_t* ts;  // (B, N) or NULL (no relative bias)
  const int64_t* thr;
  int nb;
  const float* pos_w;
  const float* ts_w;
  float* out;
  int64_t ld_out;
};

constexpr int kKeysPerPass = 4;  // keys per wave per pass of the score loop

// Workgroup (e, h): row r = rows[e] of sequence b (offsets[b] <= r < offsets[b + 1]) at
// position p = r - offsets[b]; query = q cache (b, p), keys j = 0 .. p (causal; p < L_b,
// so every such key is a real item) from the k cache (b, j), values v[offsets[b] + j]:
//   out[e, h] = sum_j silu(q . k_j + pos_w[N - 1 + j - p] + ts_w[bucket]) / N * v_j
// (hstu.py:186-205: bias shared across heads; bucket of ts[b, p + 1] - ts[b, j] with
// ts[b, N] = ts[b, N - 1], hstu.py:113-123).  LDS: thresholds | q | weights [N] | partial
// sums [4][dv].
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeArgs a) {
  extern __shared__ int64_t smem_i64[];
  const int e = blockIdx.x, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool bias = a.ts != nullptr;
  int64_t* thr = smem_i64;
  float* qs = reinterpret_cast<float*>(thr + (bias ? a.nb + 1 : 0));
  float* wts = qs + a.dqk;
  float* part = wts + a.N;
  float* orow = a.out + (int64_t)e * a.ld_out + (int64_t)h * a.dv;
  const int64_t r = a.rows[e];
  const int64_t total = a.offsets[a.B];
  if (r < 0 || r >= total) {  // validated by the host; zeros rather than a stray read
    for (int c = tid; c < a.dv; c += 256) orow[c] = 0.f;
    return;
  }
  int lo = 0, hi = a.B;  // offsets[lo] <= r < offsets[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (a.offsets[mid] <= r) lo = mid;
    else hi = mid;
  }
  const int b = lo;
  const int64_t s0 = a.offsets[b];
  const int p = (int)(r - s0);
  if (p >= a.N) {
    for (int c = tid; c < a.dv; c += 256) orow[c] = 0.f;
    return;
  }
  if (bias)
    for (int i = tid; i <= a.nb; i += 256) thr[i] = a.thr[i];
  const int64_t qk0 = (int64_t)b * a.N;
  const int hq = h * a.dqk;
  for (int d = tid; d < a.dqk; d += 256) qs[d] = a.q[(qk0 + p) * a.ld_qk + hq + d];
  __syncthreads();
  const int64_t tq = bias ? a.ts[qk0 + (p + 1 < a.N ? p + 1 : a.N - 1)] : 0;
  const float inv_n = 1.0f / (float)a.N;
  // scores: wave w takes keys w*4 .. w*4+3, then +16; lanes split the head dim
  for (int j0 = kKeysPerPass * w; j0 <= p; j0 += 4 * kKeysPerPass) {
    float acc[kKeysPerPass];
#pragma unroll
    for (int u = 0; u < kKeysPerPass; ++u) {
      acc[u] = 0.f;
      const int j = j0 + u;
      if (j <= p) {
        const float* kr = a.k + (qk0 + j) * a.ld_qk + hq;
        for (int d = lane; d < a.dqk; d += 64) acc[u] += qs[d] * kr[d];
      }
    }
#pragma unroll
    for (int u = 0; u < kKeysPerPass; ++u) acc[u] = wave_sum(acc[u]);
    if (lane < kKeysPerPass) {
      const int j = j0 + lane;
      float x = lane == 0 ? acc[0] : lane == 1 ? acc[1] : lane == 2 ? acc[2] : acc[3];
      if (j <= p) {
        if (bias)
          x = x + (a.pos_w[a.N - 1 + j - p] +
                   a.ts_w[time_bucket(tq - a.ts[qk0 + j], thr, a.nb)]);
        wts[j] = siluf_(x) * inv_n;
      }
    }
  }
  __syncthreads();
  // out[c] = sum_j wts[j] v[s0 + j][h dv + c]: wave w sums keys j = w mod 4, lanes over c
  const int hv = h * a.dv;
  // keys whose value rows lie in the cache (all of 0 .. p once the host has validated it)
  const int pe = (int)(s0 + p < a.v_rows ? p : a.v_rows - 1 - s0);
  for (int c0 = 0; c0 < a.dv; c0 += 64) {
    const int c = c0 + lane;
    float acc0 = 0.f, acc1 = 0.f;
    if (c < a.dv) {
      int j = w;
      for (; j + 4 <= pe; j += 8) {
        acc0 += wts[j] * a.v[(s0 + j) * a.ld_v + hv + c];
        acc1 += wts[j + 4] * a.v[(s0 + j + 4) * a.ld_v + hv + c];
      }
      if (j <= pe) acc0 += wts[j] * a.v[(s0 + j) * a.ld_v + hv + c];
      part[w * a.dv + c] = acc0 + acc1;
    }
  }
  __syncthreads();
  for (int c = tid; c < a.dv; c += 256)
    orow[c] = (part[c] + part[a.dv + c]) + (part[2 * a.dv + c] + part[3 * a.dv + c]);
}

}  // namespace gr

extern "C" int gr_rows_copy(const float* src, int64_t ld_src, const int64_t* src_index,
                            int64_t src_step, int64_t src_rows, float* dst, int64_t ld_dst,
                            const int64_t* dst_index, int64_t dst_step, int64_t dst_rows, int n,
                            int width, void* stream) {
  GR_REQUIRE(src && dst, "gr_rows_copy: null pointer");
  GR_REQUIRE(n >= 0 && width >= 0 && ld_src >= width && ld_dst >= width && src_rows >= 0 &&
                 dst_rows >= 0,
             "gr_rows_copy: bad sizes (n %d, width %d, ld %lld / %lld)", n, width,
             (long long)ld_src, (long long)ld_dst);
  if (n == 0 || width == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("rows_copy", st,
           hipLaunchKernelGGL(gr::rows_copy_kernel, dim3(n), dim3(256), 0, st, src, ld_src,
                              src_index, src_step, src_rows, dst, ld_dst, dst_index, dst_step,
                              dst_rows, width));
  GR_LAUNCH_CHECK("gr_rows_copy");
  return 0;
}

extern "C" size_t hstu_decode_attn_lds_bytes(int N, int dqk, int dv, int num_buckets) {
  if (N <= 0 || dqk <= 0 || dv <= 0) return 0;
  return sizeof(int64_t) * (size_t)(num_buckets > 0 ? num_buckets + 1 : 0) +
         sizeof(float) * ((size_t)dqk + (size_t)N + 4 * (size_t)dv);
}

extern "C" int hstu_decode_attn(const float* q_cache, const float* k_cache, int64_t ld_qk,
                                const float* v_cache, int64_t ld_v, int64_t v_rows,
                                const int64_t* offsets, int B, const int64_t* rows, int n_rows,
                                int N, int H, int dqk, int dv, const int64_t* ts,
                                const int64_t* bucket_thr, int num_buckets, const float* pos_w,
                                const float* ts_w, float* out, int64_t ld_out, void* stream) {
  GR_REQUIRE(q_cache && k_cache && v_cache && offsets && rows && out,
             "hstu_decode_attn: null pointer");
  GR_REQUIRE(B > 0 && N > 0 && H > 0 && dqk > 0 && dv > 0 && n_rows >= 0 && v_rows >= 0,
             "hstu_decode_attn: bad sizes (B %d, N %d, H %d, dqk %d, dv %d)", B, N, H, dqk, dv);
  GR_REQUIRE(ld_qk >= (int64_t)H * dqk && ld_v >= (int64_t)H * dv && ld_out >= (int64_t)H * dv,
             "hstu_decode_attn: bad strides");
  GR_REQUIRE(!ts || (bucket_thr && pos_w && ts_w && num_buckets > 0 && num_buckets < 256),
             "hstu_decode_attn: timestamps given without bucket_thr / pos_w / ts_w");
  const size_t lds = hstu_decode_attn_lds_bytes(N, dqk, dv, ts ? num_buckets : 0);
  GR_REQUIRE(lds <= 64 * 1024, "hstu_decode_attn: N %d too large (%zu B of LDS)", N, lds);
  if (n_rows == 0) return 0;
  gr::DecodeArgs a{q_cache, k_cache, ld_qk, v_cache, ld_v, v_rows, offsets, B, rows, N, H, dqk,
                   dv, ts, bucket_thr, num_buckets, pos_w, ts_w, out, ld_out};
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("decode_attn", st,
           hipLaunchKernelGGL(gr::decode_attn_kernel, dim3(n_rows, H), dim3(256), (uint32_t)lds,
                              st, a));
  GR_LAUNCH_CHECK("hstu_decode_attn");
  return 0;
}
