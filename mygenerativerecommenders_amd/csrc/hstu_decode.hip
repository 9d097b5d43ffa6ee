// Cached (incremental) HSTU decoding: the delta_x_offsets / cache branch of
// sequential_encoders/hstu.py (:151-177, :293-298, :321-322, :393-423).
//
// The reference re-encodes the rows x[delta_x_offsets[0]] only, writes their v into the
// jagged v cache and their q / k into the padded (B, n, .) caches (index_copy_), then runs
// the WHOLE (B, h, n, n) attention over the caches and keeps the delta rows
// (hstu.py:393-397).  Only those rows reach the output, so hstu_decode_attn computes just
// them: workgroups of 64 cached keys (chunk, head, delta row) stream the keys 0 .. p of the
// row's sequence (p = its position) and their values — an HBM-bound pass over K and V of
// 4 (p + 1) (dqk + dv) bytes per (row, head), no (n, n) scores — and a second launch sums
// the chunks' partial rows in chunk order (SiLU attention has no row normaliser, so the
// chunks' sums simply add).  hstu_decode_scatter writes the three cache updates in one
// launch; gr_rows_copy does the other row moves (x[delta], the output rows).
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

// v_cache[rows[e]] = v_e, q_cache[pos[e] + e N] = q_e, k_cache[pos[e] + e N] = k_e for the
// e-th re-encoded row (u | v | q | k columns of uvqk): the three index_copy_ of
// hstu.py:321-322 and :160-177 in one launch.
__global__ __launch_bounds__(256) void decode_scatter_kernel(const float* uvqk, int64_t ld_u, int hv,
                                                             int hq, const int64_t* rows,
                                                             const int64_t* pos, int N,
                                                             float* v_cache, int64_t v_rows,
                                                             float* q_cache, float* k_cache,
                                                             int64_t qk_rows) {
  const int64_t e = blockIdx.x;
  const float* src = uvqk + e * ld_u + hv;  // v | q | k
  const int64_t rv = rows[e], rq = pos[e] + e * N;
  const bool v_ok = rv >= 0 && rv < v_rows, qk_ok = pos[e] >= 0 && pos[e] < N && rq < qk_rows;
  for (int c = threadIdx.x; c < hv + 2 * hq; c += 256) {
    const float x = src[c];
    if (c < hv) {
      if (v_ok) v_cache[rv * hv + c] = x;
    } else if (qk_ok) {
      if (c < hv + hq) q_cache[rq * hq + (c - hv)] = x;
      else k_cache[rq * hq + (c - hv - hq)] = x;
    }
  }
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
  int n_rows;
  int N, H, dqk, dv;
  const int64_t* ts;  // (B, N) or NULL (no relative bias)
  const int64_t* thr;
  int nb;
  const float* pos_w;
  const float* ts_w;
  float* part;  // [chunks][n_rows][H dv] partial sums
  float* out;
  int64_t ld_out;
};

constexpr int kDecKeys = 64;  // keys per workgroup (one chunk of a row's keys)

// (sequence, position) of jagged row r: offsets[b] <= r < offsets[b + 1]; false when r is
// outside [0, offsets[B]) or the position is not below N.
__device__ __forceinline__ bool decode_locate(const DecodeArgs& a, int64_t r, int& b, int& p) {
  if (r < 0 || r >= a.offsets[a.B]) return false;
  int lo = 0, hi = a.B;  // offsets[lo] <= r < offsets[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (a.offsets[mid] <= r) lo = mid;
    else hi = mid;
  }
  b = lo;
  p = (int)(r - a.offsets[lo]);
  return p < a.N;
}

// Workgroup (chunk c, head h, delta row e): keys j in [64 c, 64 c + 64) with j <= p of row
// r = rows[e] (sequence b, position p; every such key is a real item as p < L_b):
//   part[c][e][h dv + col] = sum_j silu(q . k_j + pos_w[N - 1 + j - p] + ts_w[bucket]) / N
//                                  * v[offsets[b] + j][h dv + col]
// (hstu.py:186-205: bias shared across heads; bucket of ts[b, p + 1] - ts[b, j] with
// ts[b, N] = ts[b, N - 1], hstu.py:113-123).  Scores: 16-lane groups per key (16 keys in
// flight per pass), lanes over the head dim, a DPP sum; values: threads over columns
// (coalesced v rows), key subsets per thread group, an LDS reduce.  Chunks past p write
// nothing (the reduce reads only the chunks a row has).
template <int VEC>
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeArgs a) {
  extern __shared__ int64_t smem_i64[];
  const int c = blockIdx.x, h = blockIdx.y, e = blockIdx.z;
  const int tid = threadIdx.x;
  int b, p;
  if (!decode_locate(a, a.rows[e], b, p)) return;
  const int j0 = c * kDecKeys;
  if (j0 > p) return;
  const int nk = p - j0 + 1 < kDecKeys ? p - j0 + 1 : kDecKeys;
  const bool bias = a.ts != nullptr;
  int64_t* thr = smem_i64;
  float* qs = reinterpret_cast<float*>(thr + (bias ? (a.nb + 2) & ~1 : 0));  // 16-byte aligned
  float* wts = qs + ((a.dqk + 3) & ~3);
  float* red = wts + kDecKeys;  // [4][dv] group partials
  if (bias)
    for (int i = tid; i <= a.nb; i += 256) thr[i] = a.thr[i];
  const int64_t qk0 = (int64_t)b * a.N;
  const int hq = h * a.dqk;
  for (int d = tid; d < a.dqk; d += 256) qs[d] = a.q[(qk0 + p) * a.ld_qk + hq + d];
  __syncthreads();
  const int g = tid >> 4, l16 = tid & 15;
  const int64_t tq = bias ? a.ts[qk0 + (p + 1 < a.N ? p + 1 : a.N - 1)] : 0;
  const float inv_n = 1.0f / (float)a.N;
#pragma unroll
  for (int t = 0; t < kDecKeys / 16; ++t) {
    const int jj = g + 16 * t;  // key within the chunk
    float acc = 0.f;
    if (jj < nk) {
      const float* kr = a.k + (qk0 + j0 + jj) * a.ld_qk + hq;
      if (VEC == 4) {
        for (int d = 4 * l16; d < a.dqk; d += 64) {
          const float4 kv = *reinterpret_cast<const float4*>(kr + d);
          const float4 qv = *reinterpret_cast<const float4*>(qs + d);
          acc += qv.x * kv.x + qv.y * kv.y + qv.z * kv.z + qv.w * kv.w;
        }
      } else {
        for (int d = l16; d < a.dqk; d += 16) acc += qs[d] * kr[d];
      }
    }
    acc = sum16(acc);
    if (l16 == 0 && jj < kDecKeys) {
      float w = 0.f;
      if (jj < nk) {
        const int j = j0 + jj;
        float x = acc;
        if (bias)
          x = x + (a.pos_w[a.N - 1 + j - p] + a.ts_w[time_bucket(tq - a.ts[qk0 + j], thr, a.nb)]);
        w = siluf_(x) * inv_n;
      }
      wts[jj] = w;
    }
  }
  __syncthreads();
  // values: column groups of dvp = 64 ceil(dv / 64) threads (dv <= 256: 256 / dvp groups
  // split the chunk's keys; wider: one group loops over the columns)
  const int dvp = a.dv <= 64 ? 64 : a.dv <= 128 ? 128 : 256;
  const int ng = 256 / dvp, grp = tid / dvp, lc = tid % dvp;
  const int64_t vrow0 = a.offsets[b] + j0;
  // keys whose value rows lie in the cache (all nk once the host has validated it)
  const int nkv = (int)(vrow0 + nk <= a.v_rows ? nk : (a.v_rows > vrow0 ? a.v_rows - vrow0 : 0));
  const int hv = h * a.dv;
  float* prow = a.part + ((int64_t)c * a.n_rows + e) * ((int64_t)a.H * a.dv) + hv;
  for (int col0 = 0; col0 < a.dv; col0 += dvp) {
    const int col = col0 + lc;
    float acc0 = 0.f, acc1 = 0.f;
    if (col < a.dv) {
      // 4 independent loads in flight per step
      const float* vp = a.v + vrow0 * a.ld_v + hv + col;
      float acc2 = 0.f, acc3 = 0.f;
      int jj = grp;
      for (; jj + 3 * ng < nkv; jj += 4 * ng) {
        const float v0 = vp[(int64_t)jj * a.ld_v], v1 = vp[(int64_t)(jj + ng) * a.ld_v];
        const float v2 = vp[(int64_t)(jj + 2 * ng) * a.ld_v], v3 = vp[(int64_t)(jj + 3 * ng) * a.ld_v];
        acc0 += wts[jj] * v0;
        acc1 += wts[jj + ng] * v1;
        acc2 += wts[jj + 2 * ng] * v2;
        acc3 += wts[jj + 3 * ng] * v3;
      }
      for (; jj < nkv; jj += ng) acc0 += wts[jj] * vp[(int64_t)jj * a.ld_v];
      acc0 += acc2;
      acc1 += acc3;
    }
    if (ng == 1) {
      if (col < a.dv) prow[col] = acc0 + acc1;
    } else {
      if (col < a.dv) red[grp * a.dv + col] = acc0 + acc1;
      __syncthreads();
      for (int cc = tid; cc < a.dv; cc += 256) {
        float s = 0.f;
        for (int q2 = 0; q2 < ng; ++q2) s += red[q2 * a.dv + cc];
        prow[cc] = s;
      }
      __syncthreads();
    }
  }
}

// out[e][col] = sum over the row's chunks of part[c][e][col], in chunk order (deterministic);
// zeros for rows outside the batch.
__global__ __launch_bounds__(64) void decode_reduce_kernel(DecodeArgs a) {
  const int e = blockIdx.y;
  const int w = a.H * a.dv;
  const int col = blockIdx.x * 64 + threadIdx.x;
  int b, p;
  const bool ok = decode_locate(a, a.rows[e], b, p);
  const int nc = ok ? p / kDecKeys + 1 : 0;
  if (col >= w) return;
  const int64_t cs = (int64_t)a.n_rows * w;  // chunk stride
  const float* src = a.part + (int64_t)e * w + col;
  // chunk order fixed (deterministic): 4 partial sums over chunks c = 0, 1, 2, 3 mod 4
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int c = 0;
  for (; c + 3 < nc; c += 4) {
    s0 += src[c * cs];
    s1 += src[(c + 1) * cs];
    s2 += src[(c + 2) * cs];
    s3 += src[(c + 3) * cs];
  }
  for (; c < nc; ++c) s0 += src[c * cs];
  a.out[(int64_t)e * a.ld_out + col] = (s0 + s1) + (s2 + s3);
}

// ---------------------------------------------------------------- small-M projections
// The decode step's projections have one row per sequence (M = B: 32 at the C3 width).
// The training GEMMs tile 64 rows per workgroup, which leaves 4 workgroups at M = 32;
// these tile 16 rows x 16 output columns with both operands staged in LDS, so a
// (1024-column, 32-row) projection runs as 128 workgroups, each reading its 16 weight
// columns once (coalesced) and one output per thread.

constexpr int kSmRows = 16, kSmCols = 16;

// LayerNorm (no affine, biased variance, hstu.py:258-259) of rows r0 .. r0 + 15 of x into
// LDS xn[16][D] (D <= 512); wave w normalises rows 4 w .. 4 w + 3, whose loads are all
// issued before the first reduction.
__device__ __forceinline__ void sm_layernorm(const float* x, int64_t ld_x, int n, int r0, int D,
                                             float eps, float* xn) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float v[4][8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + 4 * w + q;
    const float* xr = x + (int64_t)(r < n ? r : 0) * ld_x;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = lane + 64 * m;
      v[q][m] = r < n && d < D ? xr[d] : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = 4 * w + q;
    if (r0 + rr >= n) break;
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += v[q][m];
    const float mean = wave_sum(s) / (float)D;
    float var = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float t = lane + 64 * m < D ? v[q][m] - mean : 0.f;
      var += t * t;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(var) / (float)D + eps);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = lane + 64 * m;
      if (d < D) xn[rr * D + d] = (v[q][m] - mean) * rstd;
    }
  }
}

// sum_k a[k] b[k * sb] over LDS rows, 4 partial sums
__device__ __forceinline__ float sm_dot(const float* a, const float* b, int sb, int K) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 3 < K; k += 4) {
    s0 += a[k] * b[k * sb];
    s1 += a[k + 1] * b[(k + 1) * sb];
    s2 += a[k + 2] * b[(k + 2) * sb];
    s3 += a[k + 3] * b[(k + 3) * sb];
  }
  for (; k < K; ++k) s0 += a[k] * b[k * sb];
  return (s0 + s1) + (s2 + s3);
}

// uvqk[r][c] = act(LN(x[r]) . w_uvqk[:, c])  (hstu.py:300-305), w_uvqk (D, n_out) row-major.
// LDS: xn[16][D] | wl[D][16]; thread (row tid / 16, column tid % 16).
__global__ __launch_bounds__(256) void sm_ln_uvqk_kernel(const float* x, int64_t ld_x, int n,
                                                         int D, const float* w, int n_out,
                                                         float eps, int activation, float* out,
                                                         int64_t ld_out) {
  extern __shared__ float sm_l[];
  float* xn = sm_l;
  float* wl = sm_l + kSmRows * D;
  const int c0 = blockIdx.x * kSmCols, r0 = blockIdx.y * kSmRows;
  const int rr = threadIdx.x >> 4, cc = threadIdx.x & 15;
  {  // 16 rows of 16 columns per step (64-byte runs), all loads issued before the stores
    float t[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int d = rr + kSmRows * i;
      t[i] = d < D && c0 + cc < n_out ? w[(int64_t)d * n_out + c0 + cc] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int d = rr + kSmRows * i;
      if (d < D) wl[d * kSmCols + cc] = t[i];
    }
  }
  sm_layernorm(x, ld_x, n, r0, D, eps, xn);
  __syncthreads();
  const int r = r0 + rr, c = c0 + cc;
  if (r >= n || c >= n_out) return;
  const float h = sm_dot(xn + rr * D, wl + cc, kSmCols, D);
  out[(int64_t)r * ld_out + c] = activation ? siluf_(h) : h;
}

// y[r][c] = (u[r] * LN(attn[r])) . w_o[c] + b_o[c] + x_res[r][c]  (hstu.py:393-413 without
// dropout), w_o (D, hdv) row-major (nn.Linear.weight).  LDS: oin[16][hdv] | wt[16][hdv + 1].
__global__ __launch_bounds__(256) void sm_gate_o_kernel(const float* u, int64_t ld_u,
                                                        const float* attn, int64_t ld_attn, int n,
                                                        int hdv, int D, const float* w_o,
                                                        const float* b_o, const float* x_res,
                                                        int64_t ld_x, float eps, float* y,
                                                        int64_t ld_y) {
  extern __shared__ float sm_g[];
  float* oin = sm_g;
  float* wt = sm_g + kSmRows * hdv;
  const int c0 = blockIdx.x * kSmCols, r0 = blockIdx.y * kSmRows;
  {  // one k per thread (hdv <= 256), the 16 rows' loads issued before the stores
    const int k = threadIdx.x;
    float t[kSmCols];
#pragma unroll
    for (int cc = 0; cc < kSmCols; ++cc)
      t[cc] = k < hdv && c0 + cc < D ? w_o[(int64_t)(c0 + cc) * hdv + k] : 0.f;
    if (k < hdv) {
#pragma unroll
      for (int cc = 0; cc < kSmCols; ++cc) wt[cc * (hdv + 1) + k] = t[cc];
    }
  }
  sm_layernorm(attn, ld_attn, n, r0, hdv, eps, oin);
  __syncthreads();
  {
    const int k = threadIdx.x;
    float t[kSmRows];
#pragma unroll
    for (int rr = 0; rr < kSmRows; ++rr)
      t[rr] = k < hdv && r0 + rr < n ? u[(int64_t)(r0 + rr) * ld_u + k] : 0.f;
    if (k < hdv) {
#pragma unroll
      for (int rr = 0; rr < kSmRows; ++rr) oin[rr * hdv + k] *= t[rr];
    }
  }
  __syncthreads();
  const int rr = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int r = r0 + rr, c = c0 + cc;
  if (r >= n || c >= D) return;
  const float acc = sm_dot(oin + rr * hdv, wt + cc * (hdv + 1), 1, hdv);
  y[(int64_t)r * ld_y + c] =
      (acc + (b_o ? b_o[c] : 0.f)) + (x_res ? x_res[(int64_t)r * ld_x + c] : 0.f);
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

extern "C" int hstu_decode_scatter(const float* uvqk, int64_t ld_u, int hv, int hq,
                                   const int64_t* rows, const int64_t* pos, int n, int N,
                                   float* v_cache, int64_t v_rows, float* q_cache,
                                   float* k_cache, int64_t qk_rows, void* stream) {
  GR_REQUIRE(uvqk && rows && pos && v_cache && q_cache && k_cache,
             "hstu_decode_scatter: null pointer");
  GR_REQUIRE(n >= 0 && N > 0 && hv > 0 && hq > 0 && ld_u >= hv + 2 * (int64_t)hq + hv,
             "hstu_decode_scatter: bad sizes (n %d, N %d, hv %d, hq %d)", n, N, hv, hq);
  if (n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("decode_scatter", st,
           hipLaunchKernelGGL(gr::decode_scatter_kernel, dim3(n), dim3(256), 0, st, uvqk, ld_u,
                              hv, hq, rows, pos, N, v_cache, v_rows, q_cache, k_cache, qk_rows));
  GR_LAUNCH_CHECK("hstu_decode_scatter");
  return 0;
}

extern "C" size_t hstu_decode_attn_workspace_size(int n_rows, int N, int H, int dv) {
  if (n_rows <= 0 || N <= 0 || H <= 0 || dv <= 0) return 0;
  return sizeof(float) * (size_t)((N + gr::kDecKeys - 1) / gr::kDecKeys) * n_rows * H * dv;
}

extern "C" int hstu_decode_attn(const float* q_cache, const float* k_cache, int64_t ld_qk,
                                const float* v_cache, int64_t ld_v, int64_t v_rows,
                                const int64_t* offsets, int B, const int64_t* rows, int n_rows,
                                int N, int H, int dqk, int dv, const int64_t* ts,
                                const int64_t* bucket_thr, int num_buckets, const float* pos_w,
                                const float* ts_w, float* out, int64_t ld_out, void* workspace,
                                size_t ws_bytes, void* stream) {
  GR_REQUIRE(q_cache && k_cache && v_cache && offsets && rows && out,
             "hstu_decode_attn: null pointer");
  GR_REQUIRE(B > 0 && N > 0 && H > 0 && dqk > 0 && dv > 0 && n_rows >= 0 && v_rows >= 0,
             "hstu_decode_attn: bad sizes (B %d, N %d, H %d, dqk %d, dv %d)", B, N, H, dqk, dv);
  GR_REQUIRE(ld_qk >= (int64_t)H * dqk && ld_v >= (int64_t)H * dv && ld_out >= (int64_t)H * dv,
             "hstu_decode_attn: bad strides");
  GR_REQUIRE(!ts || (bucket_thr && pos_w && ts_w && num_buckets > 0 && num_buckets < 256),
             "hstu_decode_attn: timestamps given without bucket_thr / pos_w / ts_w");
  GR_REQUIRE(n_rows <= 65535, "hstu_decode_attn: %d rows (at most 65535 per call)", n_rows);
  if (n_rows == 0) return 0;
  const size_t need = hstu_decode_attn_workspace_size(n_rows, N, H, dv);
  GR_REQUIRE(workspace && ws_bytes >= need, "hstu_decode_attn: workspace %zu B < %zu B",
             ws_bytes, need);
  const int dvr = dv <= 256 ? dv : 256;  // the group-partial rows (dv > 256: one group)
  const size_t lds = sizeof(int64_t) * (size_t)(ts ? (num_buckets + 2) & ~1 : 0) +
                     sizeof(float) * ((size_t)((dqk + 3) & ~3) + gr::kDecKeys + 4 * (size_t)dvr);
  GR_REQUIRE(lds <= 64 * 1024, "hstu_decode_attn: head dims too large (%zu B of LDS)", lds);
  gr::DecodeArgs a{q_cache, k_cache, ld_qk, v_cache, ld_v, v_rows, offsets, B, rows, n_rows,
                   N, H, dqk, dv, ts, bucket_thr, num_buckets, pos_w, ts_w, (float*)workspace,
                   out, ld_out};
  const bool vec = dqk % 4 == 0 && ld_qk % 4 == 0 && ((uintptr_t)q_cache & 15) == 0 &&
                   ((uintptr_t)k_cache & 15) == 0;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((N + gr::kDecKeys - 1) / gr::kDecKeys, H, n_rows);
  GR_TIMED("decode_attn", st, {
    if (vec)
      hipLaunchKernelGGL(gr::decode_attn_kernel<4>, grid, dim3(256), (uint32_t)lds, st, a);
    else
      hipLaunchKernelGGL(gr::decode_attn_kernel<1>, grid, dim3(256), (uint32_t)lds, st, a);
  });
  GR_LAUNCH_CHECK("hstu_decode_attn");
  GR_TIMED("decode_attn", st,
           hipLaunchKernelGGL(gr::decode_reduce_kernel, dim3((H * dv + 63) / 64, n_rows), dim3(64),
                              0, st, a));
  GR_LAUNCH_CHECK("hstu_decode_attn(reduce)");
  return 0;
}

extern "C" int hstu_decode_ln_uvqk(const float* x, int64_t ld_x, int n, int D, const float* w_uvqk,
                                   int n_out, float eps, int activation, float* uvqk,
                                   int64_t ld_out, void* stream) {
  GR_REQUIRE(x && w_uvqk && uvqk, "hstu_decode_ln_uvqk: null pointer");
  GR_REQUIRE(n >= 0 && D > 0 && D <= 512 && n_out > 0 && ld_x >= D && ld_out >= n_out &&
                 (activation == 0 || activation == 1),
             "hstu_decode_ln_uvqk: bad sizes (n %d, D %d, n_out %d)", n, D, n_out);
  if (n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((n_out + gr::kSmCols - 1) / gr::kSmCols, (n + gr::kSmRows - 1) / gr::kSmRows);
  GR_REQUIRE(grid.y <= 65535, "hstu_decode_ln_uvqk: %d rows", n);
  GR_TIMED("ln_uvqk_fwd", st,
           hipLaunchKernelGGL(gr::sm_ln_uvqk_kernel, grid, dim3(256),
                              (uint32_t)(sizeof(float) * (gr::kSmRows + gr::kSmCols) * D), st,
                              x, ld_x, n, D,
                              w_uvqk, n_out, eps, activation, uvqk, ld_out));
  GR_LAUNCH_CHECK("hstu_decode_ln_uvqk");
  return 0;
}

extern "C" int hstu_decode_gate_o(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                  int n, int hdv, int D, const float* w_o, const float* b_o,
                                  const float* x_res, int64_t ld_x, float eps, float* y,
                                  int64_t ld_y, void* stream) {
  GR_REQUIRE(u && attn && w_o && y, "hstu_decode_gate_o: null pointer");
  GR_REQUIRE(n >= 0 && hdv > 0 && hdv <= 256 && D > 0 && ld_u >= hdv && ld_attn >= hdv &&
                 ld_y >= D && (!x_res || ld_x >= D),
             "hstu_decode_gate_o: bad sizes (n %d, hdv %d, D %d)", n, hdv, D);
  if (n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((D + gr::kSmCols - 1) / gr::kSmCols, (n + gr::kSmRows - 1) / gr::kSmRows);
  GR_REQUIRE(grid.y <= 65535, "hstu_decode_gate_o: %d rows", n);
  const size_t lds = sizeof(float) * ((size_t)gr::kSmRows * hdv + (size_t)gr::kSmCols * (hdv + 1));
  GR_TIMED("gate_o_fwd", st,
           hipLaunchKernelGGL(gr::sm_gate_o_kernel, grid, dim3(256), (uint32_t)lds, st, u, ld_u,
                              attn, ld_attn, n, hdv, D, w_o, b_o, x_res, ld_x, eps, y, ld_y));
  GR_LAUNCH_CHECK("hstu_decode_gate_o");
  return 0;
}
