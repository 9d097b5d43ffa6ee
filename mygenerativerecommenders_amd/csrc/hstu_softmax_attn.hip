// The normalization="softmax_rel_bias" attention of SequentialTransductionUnitJagged
// (sequential_encoders/hstu.py:341-389, non-cached branch) and its backward.
//
// Reference semantics, kept exactly: the scores use all heads' columns at once
// (einsum "bnd,bmd->bnm" over the padded (B, n, h dqk) q / k), the bias (when given) is
// added before the 1 / sqrt(attention_dim) scale, the softmax runs over ALL n keys of a
// row — padded keys (k = 0: their score is the bias alone) and future keys included —
// and only then is the causal mask applied, so rows are not renormalised.  Query rows
// past a sequence's length are dropped by the reference's dense_to_jagged and are not
// computed here.
//
// One wave per (sequence, query row): the scores of the row's n keys live in the wave's
// LDS slice (lanes over keys), the value sum runs with lanes over the output columns
// (coalesced rows of v).  The backward is two launches: a row pass (recomputed
// probabilities A, dS = A (dA - D) / sqrt(d) with D = dO . O, stored as the (B, n, n)
// bias gradient, and dQ) and a key pass (dK = dS^T Q, dV = (A * mask)^T dO).  fp32 FMA:
// the branch is used by no configuration, so it is built for parity, not for the MFMA.
#include <math.h>

#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

struct SoftmaxAttnArgs {
  const float* q;  // jagged rows, columns 0 .. hdq of each row
  const float* k;
  int64_t ld_qk;
  const float* v;
  int64_t ld_v;
  const int64_t* offsets;
  int B, N, hdq, hdv;
  float sqrt_d;
  const float* bias;  // (B, N, N) or NULL
  float* out;
  int64_t ld_out;
  float* stats;  // (rows, 2): row max and sum of exp of the scaled scores
  // backward
  const float* dout;
  int64_t ld_do;
  const float* hq;  // pre-activations (silu' applied to dq / dk / dv) or NULL
  const float* hk;
  const float* hv;
  int64_t ld_h;
  float* dq;
  float* dk;
  float* dv;
  int64_t ld_d;
  float* g;  // (B, N, N): d loss / d (qk + bias), i.e. the bias gradient
  float* p;  // (B, N, N): A * causal mask, rows of valid queries
};

constexpr int kSmWaves = 4;  // waves (query or key rows) per workgroup

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// the wave's own LDS writes become visible to all its lanes
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (dot(q_i, k_j) [+ bias]) / sqrt(d) for key j of a sequence with L rows (k_j = 0 for j >= L)
__device__ __forceinline__ float sm_score(const SoftmaxAttnArgs& a, const float* qs, int64_t s0,
                                          int L, const float* brow, int j) {
  float dot = 0.f;
  if (j < L) {
    const float* kr = a.k + (s0 + j) * a.ld_qk;
    for (int d = 0; d < a.hdq; ++d) dot += qs[d] * kr[d];
  }
  const float x = brow ? dot + brow[j] : dot;
  return x / a.sqrt_d;
}

__device__ __forceinline__ float silu_scale(const float* h, int64_t ld, int64_t r, int c) {
  return h ? silu_grad_(h[r * ld + c]) : 1.f;
}

__global__ __launch_bounds__(256) void softmax_attn_fwd_kernel(SoftmaxAttnArgs a) {
  extern __shared__ float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kSmWaves + w;  // b * N + i
  if (row >= (int64_t)a.B * a.N) return;
  const int b = (int)(row / a.N), i = (int)(row % a.N);
  const int64_t s0 = a.offsets[b];
  const int64_t len = a.offsets[b + 1] - s0;
  const int L = len < a.N ? (int)len : a.N;
  if (i >= L) return;
  float* qs = sm + w * (a.hdq + a.N);
  float* sc = qs + a.hdq;
  const float* qrow = a.q + (s0 + i) * a.ld_qk;
  for (int d = lane; d < a.hdq; d += 64) qs[d] = qrow[d];
  wave_sync();
  const float* brow = a.bias ? a.bias + row * a.N : nullptr;
  float mx = -INFINITY;
  for (int j = lane; j < a.N; j += 64) {
    const float x = sm_score(a, qs, s0, L, brow, j);
    sc[j] = x;
    mx = fmaxf(mx, x);
  }
  mx = wave_max(mx);
  float z = 0.f;
  for (int j = lane; j < a.N; j += 64) {
    const float e = __expf(sc[j] - mx);
    sc[j] = e;
    z += e;
  }
  z = wave_sum(z);
  wave_sync();
  const float inv_z = 1.f / z;
  float* orow = a.out + (s0 + i) * a.ld_out;
  for (int c = lane; c < a.hdv; c += 64) {
    float acc0 = 0.f, acc1 = 0.f;
    int j = 0;
    for (; j + 1 <= i; j += 2) {
      acc0 += (sc[j] * inv_z) * a.v[(s0 + j) * a.ld_v + c];
      acc1 += (sc[j + 1] * inv_z) * a.v[(s0 + j + 1) * a.ld_v + c];
    }
    if (j <= i) acc0 += (sc[j] * inv_z) * a.v[(s0 + j) * a.ld_v + c];
    orow[c] = acc0 + acc1;
  }
  if (lane == 0) {
    a.stats[2 * (s0 + i)] = mx;
    a.stats[2 * (s0 + i) + 1] = z;
  }
}

// Row pass of the backward: one wave per (b, i).  Rows i >= L only zero their g row.
__global__ __launch_bounds__(256) void softmax_attn_bwd_rows_kernel(SoftmaxAttnArgs a) {
  extern __shared__ float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kSmWaves + w;
  if (row >= (int64_t)a.B * a.N) return;
  const int b = (int)(row / a.N), i = (int)(row % a.N);
  const int64_t s0 = a.offsets[b];
  const int64_t len = a.offsets[b + 1] - s0;
  const int L = len < a.N ? (int)len : a.N;
  float* grow = a.g + row * a.N;
  if (i >= L) {
    for (int j = lane; j < a.N; j += 64) grow[j] = 0.f;
    return;
  }
  float* qs = sm + w * (a.hdq + a.hdv + a.N);
  float* dos = qs + a.hdq;
  float* gs = dos + a.hdv;
  const int64_t r = s0 + i;
  for (int d = lane; d < a.hdq; d += 64) qs[d] = a.q[r * a.ld_qk + d];
  float dd = 0.f;  // D = dO_i . O_i
  for (int c = lane; c < a.hdv; c += 64) {
    const float o = a.dout[r * a.ld_do + c];
    dos[c] = o;
    dd += o * a.out[r * a.ld_out + c];
  }
  dd = wave_sum(dd);
  wave_sync();
  const float mx = a.stats[2 * r], inv_z = 1.f / a.stats[2 * r + 1];
  const float* brow = a.bias ? a.bias + row * a.N : nullptr;
  float* prow = a.p + row * a.N;
  for (int j = lane; j < a.N; j += 64) {
    const float A = __expf(sm_score(a, qs, s0, L, brow, j) - mx) * inv_z;
    float da = 0.f;
    if (j <= i) {
      const float* vr = a.v + (s0 + j) * a.ld_v;
      for (int c = 0; c < a.hdv; ++c) da += dos[c] * vr[c];
      prow[j] = A;
    }
    const float gv = A * (da - dd) / a.sqrt_d;
    grow[j] = gv;
    gs[j] = gv;
  }
  wave_sync();
  for (int c = lane; c < a.hdq; c += 64) {
    float acc0 = 0.f, acc1 = 0.f;
    int j = 0;
    for (; j + 1 < L; j += 2) {
      acc0 += gs[j] * a.k[(s0 + j) * a.ld_qk + c];
      acc1 += gs[j + 1] * a.k[(s0 + j + 1) * a.ld_qk + c];
    }
    if (j < L) acc0 += gs[j] * a.k[(s0 + j) * a.ld_qk + c];
    a.dq[r * a.ld_d + c] = (acc0 + acc1) * silu_scale(a.hq, a.ld_h, r, c);
  }
}

// Key pass: one wave per (b, j), j < L: dK_j = sum_{i<L} g[b,i,j] q_i,
// dV_j = sum_{j<=i<L} p[b,i,j] dO_i.
__global__ __launch_bounds__(256) void softmax_attn_bwd_cols_kernel(SoftmaxAttnArgs a) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kSmWaves + w;
  if (row >= (int64_t)a.B * a.N) return;
  const int b = (int)(row / a.N), j = (int)(row % a.N);
  const int64_t s0 = a.offsets[b];
  const int64_t len = a.offsets[b + 1] - s0;
  const int L = len < a.N ? (int)len : a.N;
  if (j >= L) return;
  const int64_t base = (int64_t)b * a.N * a.N + j;  // + i * N: column j of row i
  const int64_t r = s0 + j;
  for (int c = lane; c < a.hdq; c += 64) {
    float acc0 = 0.f, acc1 = 0.f;
    int i = 0;
    for (; i + 1 < L; i += 2) {
      acc0 += a.g[base + (int64_t)i * a.N] * a.q[(s0 + i) * a.ld_qk + c];
      acc1 += a.g[base + (int64_t)(i + 1) * a.N] * a.q[(s0 + i + 1) * a.ld_qk + c];
    }
    if (i < L) acc0 += a.g[base + (int64_t)i * a.N] * a.q[(s0 + i) * a.ld_qk + c];
    a.dk[r * a.ld_d + c] = (acc0 + acc1) * silu_scale(a.hk, a.ld_h, r, c);
  }
  for (int c = lane; c < a.hdv; c += 64) {
    float acc0 = 0.f, acc1 = 0.f;
    int i = j;
    for (; i + 1 < L; i += 2) {
      acc0 += a.p[base + (int64_t)i * a.N] * a.dout[(s0 + i) * a.ld_do + c];
      acc1 += a.p[base + (int64_t)(i + 1) * a.N] * a.dout[(s0 + i + 1) * a.ld_do + c];
    }
    if (i < L) acc0 += a.p[base + (int64_t)i * a.N] * a.dout[(s0 + i) * a.ld_do + c];
    a.dv[r * a.ld_d + c] = (acc0 + acc1) * silu_scale(a.hv, a.ld_h, r, c);
  }
}

}  // namespace gr

namespace {
size_t nn_bytes(int B, int N) { return sizeof(float) * (size_t)B * N * N; }
size_t align256(size_t v) { return (v + 255) / 256 * 256; }

int check_common(const char* who, const float* q, const float* k, int64_t ld_qk, const float* v,
                 int64_t ld_v, const int64_t* offsets, int B, int N, int hdq, int hdv,
                 float sqrt_d, int64_t ld_out, size_t lds) {
  GR_REQUIRE(q && k && v && offsets, "%s: null pointer", who);
  GR_REQUIRE(B > 0 && N > 0 && hdq > 0 && hdv > 0 && sqrt_d > 0.f,
             "%s: bad sizes (B %d, N %d, hdq %d, hdv %d)", who, B, N, hdq, hdv);
  GR_REQUIRE(ld_qk >= hdq && ld_v >= hdv && ld_out >= hdv, "%s: bad strides", who);
  GR_REQUIRE((int64_t)B * N < 0x7fffffff, "%s: B * N too large", who);
  GR_REQUIRE(lds <= 64 * 1024, "%s: N + head columns too large (%zu B of LDS)", who, lds);
  return 0;
}
}  // namespace

extern "C" size_t hstu_softmax_attn_bwd_workspace_size(int B, int N, int with_dbias) {
  if (B <= 0 || N <= 0) return 0;
  return align256(nn_bytes(B, N)) + (with_dbias ? 0 : align256(nn_bytes(B, N)));
}

extern "C" int hstu_softmax_attn_fwd(const float* q, const float* k, int64_t ld_qk, const float* v,
                                     int64_t ld_v, const int64_t* offsets, int B, int N, int hdq,
                                     int hdv, float sqrt_d, const float* bias, float* out,
                                     int64_t ld_out, float* stats, void* stream) {
  const size_t lds = sizeof(float) * gr::kSmWaves * ((size_t)hdq + N);
  if (int rc = check_common("hstu_softmax_attn_fwd", q, k, ld_qk, v, ld_v, offsets, B, N, hdq,
                            hdv, sqrt_d, ld_out, lds))
    return rc;
  GR_REQUIRE(out && stats, "hstu_softmax_attn_fwd: null pointer");
  gr::SoftmaxAttnArgs a{};
  a.q = q; a.k = k; a.ld_qk = ld_qk; a.v = v; a.ld_v = ld_v; a.offsets = offsets;
  a.B = B; a.N = N; a.hdq = hdq; a.hdv = hdv; a.sqrt_d = sqrt_d; a.bias = bias;
  a.out = out; a.ld_out = ld_out; a.stats = stats;
  const hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)(((int64_t)B * N + gr::kSmWaves - 1) / gr::kSmWaves);
  GR_TIMED("softmax_attn_fwd", st,
           hipLaunchKernelGGL(gr::softmax_attn_fwd_kernel, dim3(grid), dim3(256), (uint32_t)lds,
                              st, a));
  GR_LAUNCH_CHECK("hstu_softmax_attn_fwd");
  return 0;
}

extern "C" int hstu_softmax_attn_bwd(const float* q, const float* k, int64_t ld_qk, const float* v,
                                     int64_t ld_v, const int64_t* offsets, int B, int N, int hdq,
                                     int hdv, float sqrt_d, const float* bias, const float* out,
                                     int64_t ld_out, const float* stats, const float* dout,
                                     int64_t ld_do, const float* hq, const float* hk,
                                     const float* hv, int64_t ld_h, float* dq, float* dk,
                                     float* dv, int64_t ld_d, float* dbias, void* workspace,
                                     size_t ws_bytes, void* stream) {
  const size_t lds = sizeof(float) * gr::kSmWaves * ((size_t)hdq + hdv + N);
  if (int rc = check_common("hstu_softmax_attn_bwd", q, k, ld_qk, v, ld_v, offsets, B, N, hdq,
                            hdv, sqrt_d, ld_out, lds))
    return rc;
  GR_REQUIRE(out && stats && dout && dq && dk && dv, "hstu_softmax_attn_bwd: null pointer");
  GR_REQUIRE(ld_do >= hdv && ld_d >= hdq && ld_d >= hdv && (!(hq || hk || hv) || (hq && hk && hv)),
             "hstu_softmax_attn_bwd: bad strides or a partial set of pre-activations");
  const size_t need = hstu_softmax_attn_bwd_workspace_size(B, N, dbias ? 1 : 0);
  GR_REQUIRE(workspace && ws_bytes >= need, "hstu_softmax_attn_bwd: workspace %zu B < %zu B",
             ws_bytes, need);
  gr::SoftmaxAttnArgs a{};
  a.q = q; a.k = k; a.ld_qk = ld_qk; a.v = v; a.ld_v = ld_v; a.offsets = offsets;
  a.B = B; a.N = N; a.hdq = hdq; a.hdv = hdv; a.sqrt_d = sqrt_d; a.bias = bias;
  a.out = const_cast<float*>(out); a.ld_out = ld_out; a.stats = const_cast<float*>(stats);
  a.dout = dout; a.ld_do = ld_do; a.hq = hq; a.hk = hk; a.hv = hv; a.ld_h = ld_h;
  a.dq = dq; a.dk = dk; a.dv = dv; a.ld_d = ld_d;
  char* ws = (char*)workspace;
  a.p = (float*)ws;
  a.g = dbias ? dbias : (float*)(ws + align256(nn_bytes(B, N)));
  const hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)(((int64_t)B * N + gr::kSmWaves - 1) / gr::kSmWaves);
  GR_TIMED("softmax_attn_bwd", st,
           hipLaunchKernelGGL(gr::softmax_attn_bwd_rows_kernel, dim3(grid), dim3(256),
                              (uint32_t)lds, st, a));
  GR_LAUNCH_CHECK("hstu_softmax_attn_bwd(rows)");
  GR_TIMED("softmax_attn_bwd", st,
           hipLaunchKernelGGL(gr::softmax_attn_bwd_cols_kernel, dim3(grid), dim3(256), 0, st, a));
  GR_LAUNCH_CHECK("hstu_softmax_attn_bwd(keys)");
  return 0;
}
