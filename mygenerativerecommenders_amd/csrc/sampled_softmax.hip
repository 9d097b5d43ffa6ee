// Fused sampled-softmax loss over a local negatives table (forward + backward).
//
// Replaces, for one training step, the chain
//   LocalNegativesSampler.forward      (negative_sampler.py:105-131: randint offsets ->
//                                       ids -> get_item_embeddings -> L2 norm)
//   DotProductSimilarity.forward       (dot_product.py:31-64: bmm (M,R,D) x (M,D,1))
//   SampledSoftmaxLoss.jagged_forward  (autoregressive_losses.py:259-306: /T, -5e4
//                                       collision mask, -log_softmax(cat[pos, neg])[:, 0])
// which materialises an (M, R, D) gathered tensor (655 MB at ml-1m C2).  Here the
// negatives are rows of the (already L2-normalised) per-catalog-row table, gathered
// by sampled offset straight from L2/MALL, and nothing of size M*R*D is written.
//
// Row layout: a sample's row is read by L lanes (L = 1, 2, 4, 8, 16 for D <= 16L), each
// holding 4 float4 at d = 4j + 4Lk (j = lane % L, k < 4).  The gathers are 16-byte
// buffer loads (rows only need 4-byte alignment; past-the-table reads return 0 from the
// range check, and out_t is zeroed for d >= D so in-row overreads contribute nothing),
// which is what the texture path needs: with one dword per lane the kernels were bound
// by vector-memory instruction issue, not by bytes.  Dot products reduce over the L
// lanes with DPP.
//
// Token-major kernels (forward, backward pass 1): one wave per token t; per step the
// wave scores G = 64/L samples (group g = lane / L takes sample G*i + g of the 64-sample
// chunk); the chunk's offsets are loaded lane-parallel once (one ballot gives the
// id-collision mask) and handed to the groups by lane shuffles; 4 steps of gathers are
// issued back to back before any dot product is reduced.
//
// Backward (dloss_t = the per-token upstream gradient, c_{t,r} = dlogit_{t,r} / T):
//   p_r = exp(logit_r - lse_t),  dlogit_0 = g (p_0 - 1),  dlogit_r = g p_r (0 if masked)
//   d_out[t]  = c_{t,0} pos_t + sum_r c_{t,r} E[off_r]       (pass 1, token-major)
//   d_pos[t]  = c_{t,0} out_t                                (pass 1)
//   d_table[v] = sum_{(t,r): off_{t,r} = v} c_{t,r} out_t     (row-major reduce)
// The table gradient is a transpose of the sampling: a counting sort of the M*R offsets
// (LDS-histogram count with in-bucket ranks, scan, scatter of {t, c}) orders the
// samples by catalog row, and a segmented reduction sums c * out_t per row in
// registers with one fp32 atomic flush per (wave, row) — ~M*R*D/256 atomics instead of
// the M*R*D of a direct scatter-add, which ran ~1.1 ms at C2 on gfx950 (global) and
// ~1.8 ms as LDS atomics into an LDS-resident table slice: float atomics resolve about
// one lane per clock.  In-bucket order follows integer atomics, so the summation order
// is not fixed.
#include "common.h"

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "../../include/gr_hstu.h"

namespace gr {

typedef float f4v __attribute__((ext_vector_type(4)));

struct SsmArgs {
  const float* out;
  int64_t ld_out;
  const float* pos;
  int64_t ld_pos;
  const int64_t* sup_ids;
  const float* table;
  int64_t ld_table;
  int64_t V;
  const int64_t* all_ids;  // nullable: sampled id == offset
  const int64_t* offsets;  // (M, R) row-major
  int64_t M;
  int R;
  int D;
  float temperature;
  float* loss;  // (M,)
  float* lse;   // (M,)
  // backward
  const float* dloss;  // (M,)
  float* d_out;
  int64_t ld_dout;
  float* d_pos;
  int64_t ld_dpos;
  int2* rec;  // (M, R) {offset, bits of c_{t,r}}
};

constexpr float kCollisionLogit = -5e4f;  // autoregressive_losses.py:296-300
constexpr int kK4 = 4;                    // float4 per lane per row
constexpr int kStepsInFlight = 4;         // gather steps issued before reducing

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* base, int64_t rows,
                                                            int64_t ld) {
  const int64_t bytes = rows * ld * 4;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0,
                                           (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
}

__device__ __forceinline__ f4v buf_ld4(__amdgpu_buffer_rsrc_t r, int voff) {
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const u4v x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return f4v{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
}

// sum over the L lanes of a sample group (lanes of a group hold equal partials after
// each step, so the half-row / row mirrors act as xor 4 / xor 8)
template <int L>
__device__ __forceinline__ float sumL(float v) {
  if constexpr (L >= 2) v += dpp_mov<0xB1>(v);
  if constexpr (L >= 4) v += dpp_mov<0x4E>(v);
  if constexpr (L >= 8) v += dpp_mov<0x141>(v);
  if constexpr (L >= 16) v += dpp_mov<0x140>(v);
  return v;
}

// sum over the G = 64/L groups (lanes with the same j)
template <int L>
__device__ __forceinline__ float sum_groups(float v) {
#pragma unroll
  for (int o = L; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float dot4(f4v a, f4v b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}

__device__ __forceinline__ int clamp_off(int64_t off, int64_t V) {
  return (int)(off < 0 ? 0 : (off >= V ? V - 1 : off));
}

// this lane's float4 slots of a length-D row, zero for d >= D
template <int L>
__device__ __forceinline__ void load_vec(__amdgpu_buffer_rsrc_t r, int64_t row, int64_t ld, int j, int D,
                                         f4v (&x)[kK4]) {
#pragma unroll
  for (int k = 0; k < kK4; ++k) {
    const int d = 4 * j + 4 * L * k;
    f4v v = buf_ld4(r, (int)((row * ld + d) * 4));
    v.x = d < D ? v.x : 0.f;
    v.y = d + 1 < D ? v.y : 0.f;
    v.z = d + 2 < D ? v.z : 0.f;
    v.w = d + 3 < D ? v.w : 0.f;
    x[k] = v;
  }
}

template <int L>
struct TokenState {
  f4v o[kK4];  // out_t, this lane's slots (0 past D)
  f4v p[kK4];  // pos_t
  float pos_logit;
  int64_t sup;
};

template <int L>
__device__ __forceinline__ void load_token(const SsmArgs& a, int64_t t, int j, TokenState<L>& s) {
  load_vec<L>(rows_rsrc(a.out, a.M, a.ld_out), t, a.ld_out, j, a.D, s.o);
  load_vec<L>(rows_rsrc(a.pos, a.M, a.ld_pos), t, a.ld_pos, j, a.D, s.p);
  float pl = 0.f;
#pragma unroll
  for (int k = 0; k < kK4; ++k) pl = dot4(s.o[k], s.p[k], pl);
  s.pos_logit = sumL<L>(pl) / a.temperature;
  s.sup = a.sup_ids[t];
}

// Chunk of samples r0 .. r0+63: lane l loads sample r0 + l (clamped offset, 0 past R);
// bit l of the ballot marks an id collision with the positive.
__device__ __forceinline__ int load_chunk(const SsmArgs& a, int64_t t, int r0, int lane,
                                          int64_t sup, uint64_t& mask) {
  const int r = r0 + lane;
  int off = 0;
  if (r < a.R) off = clamp_off(a.offsets[t * a.R + r], a.V);
  const int64_t id = a.all_ids ? a.all_ids[off] : (int64_t)off;
  mask = __ballot(r < a.R && id == sup);
  return off;
}

// Gathers the rows of steps i0 .. i0+S-1 (chunk sample G*i + g) and their dots with out_t.
template <int L, int S>
__device__ __forceinline__ void gather_dots(__amdgpu_buffer_rsrc_t tr, int64_t ld, int loff, int i0,
                                            int g, int j, const f4v (&o)[kK4],
                                            f4v (&row)[S][kK4], float (&dot)[S]) {
  constexpr int G = 64 / L;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int off = __shfl(loff, G * (i0 + i) + g, 64);
    const int base = (int)(((int64_t)off * ld + 4 * j) * 4);
#pragma unroll
    for (int k = 0; k < kK4; ++k) row[i][k] = buf_ld4(tr, base + 16 * L * k);
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < kK4; ++k) acc = dot4(o[k], row[i][k], acc);
    dot[i] = sumL<L>(acc);
  }
}

template <int L>
__global__ __launch_bounds__(256) void ssm_fwd_kernel(SsmArgs a) {
  constexpr int G = 64 / L, S = L < kStepsInFlight ? L : kStepsInFlight;
  const int64_t t = (int64_t)blockIdx.x * 4 + wave_id();
  if (t >= a.M) return;
  const int lane = threadIdx.x & 63, g = lane / L, j = lane % L;
  TokenState<L> s;
  load_token<L>(a, t, j, s);
  const __amdgpu_buffer_rsrc_t tr = rows_rsrc(a.table, a.V, a.ld_table);

  float m = -INFINITY, sum = 0.f;
  for (int r0 = 0; r0 < a.R; r0 += 64) {
    uint64_t mask;
    const int loff = load_chunk(a, t, r0, lane, s.sup, mask);
    const int n = min(64, a.R - r0);
#pragma unroll
    for (int i0 = 0; i0 < L; i0 += S) {
      f4v row[S][kK4];
      float dot[S];
      gather_dots<L, S>(tr, a.ld_table, loff, i0, g, j, s.o, row, dot);
      float lg[S];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int rr = G * (i0 + i) + g;
        const float x = ((mask >> rr) & 1ull) ? kCollisionLogit : dot[i] / a.temperature;
        lg[i] = rr < n ? x : -INFINITY;
      }
      float cm = lg[0];
#pragma unroll
      for (int i = 1; i < S; ++i) cm = fmaxf(cm, lg[i]);
      const float mn = fmaxf(m, cm);
      if (mn != -INFINITY) {  // this group has scored at least one sample
        float cs = 0.f;
#pragma unroll
        for (int i = 0; i < S; ++i) cs += expf(lg[i] - mn);
        sum = (m == -INFINITY ? 0.f : sum * expf(m - mn)) + cs;
        m = mn;
      }
    }
  }
  // merge the G sample groups, then fold in the positive logit
#pragma unroll
  for (int o = L; o < 64; o <<= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sum, o, 64);
    const float mn = fmaxf(m, m2);
    sum = (m == -INFINITY ? 0.f : sum * expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * expf(m2 - mn));
    m = mn;
  }
  const float mn = fmaxf(m, s.pos_logit);
  sum = (m == -INFINITY ? 0.f : sum * expf(m - mn)) + expf(s.pos_logit - mn);
  const float lse = mn + logf(sum);
  if (lane == 0) {
    a.lse[t] = lse;
    a.loss[t] = lse - s.pos_logit;
  }
}

// masked row store of this lane's float4 slots
template <int L>
__device__ __forceinline__ void store_vec(float* row, int j, int D, const f4v (&x)[kK4]) {
#pragma unroll
  for (int k = 0; k < kK4; ++k) {
    const int d = 4 * j + 4 * L * k;
    if (d < D) row[d] = x[k].x;
    if (d + 1 < D) row[d + 1] = x[k].y;
    if (d + 2 < D) row[d + 2] = x[k].z;
    if (d + 3 < D) row[d + 3] = x[k].w;
  }
}

// Backward pass 1 (token-major): d_out, d_pos and the coefficients c_{t,r}.
template <int L>
__global__ __launch_bounds__(256) void ssm_bwd_token_kernel(SsmArgs a) {
  constexpr int G = 64 / L, S = L < kStepsInFlight ? L : kStepsInFlight;
  const int64_t t = (int64_t)blockIdx.x * 4 + wave_id();
  if (t >= a.M) return;
  const int lane = threadIdx.x & 63, g = lane / L, j = lane % L;
  const float gt = a.dloss[t];
  float* dorow = a.d_out + t * a.ld_dout;
  float* dprow = a.d_pos + t * a.ld_dpos;
  int2* rrow = a.rec + t * a.R;
  if (gt == 0.f) {  // masked-out supervision position (weight 0): no gradient anywhere
    for (int d = lane; d < a.D; d += 64) {
      dorow[d] = 0.f;
      dprow[d] = 0.f;
    }
    for (int r = lane; r < a.R; r += 64) rrow[r] = make_int2(0, 0);
    return;
  }
  TokenState<L> s;
  load_token<L>(a, t, j, s);
  const __amdgpu_buffer_rsrc_t tr = rows_rsrc(a.table, a.V, a.ld_table);
  const float lse = a.lse[t];
  const float c0 = gt * (expf(s.pos_logit - lse) - 1.f) / a.temperature;

  f4v acc[kK4];
#pragma unroll
  for (int k = 0; k < kK4; ++k) acc[k] = f4v{0.f, 0.f, 0.f, 0.f};
  for (int r0 = 0; r0 < a.R; r0 += 64) {
    uint64_t mask;
    const int loff = load_chunk(a, t, r0, lane, s.sup, mask);
    const int n = min(64, a.R - r0);
    float mine = 0.f;  // c of chunk sample `lane` (held by group lane % G at step lane / G)
#pragma unroll
    for (int i0 = 0; i0 < L; i0 += S) {
      f4v row[S][kK4];
      float dot[S];
      gather_dots<L, S>(tr, a.ld_table, loff, i0, g, j, s.o, row, dot);
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int rr = G * (i0 + i) + g;
        const bool live = rr < n && !((mask >> rr) & 1ull);
        const float c = live ? gt * expf(dot[i] / a.temperature - lse) / a.temperature : 0.f;
#pragma unroll
        for (int k = 0; k < kK4; ++k) acc[k] += c * row[i][k];
        const float cb = __shfl(c, (lane % G) * L, 64);
        mine = lane / G == i0 + i ? cb : mine;
      }
    }
    if (lane < n) rrow[r0 + lane] = make_int2(loff, __float_as_int(mine));
  }
#pragma unroll
  for (int k = 0; k < kK4; ++k) {
    acc[k].x = sum_groups<L>(acc[k].x);
    acc[k].y = sum_groups<L>(acc[k].y);
    acc[k].z = sum_groups<L>(acc[k].z);
    acc[k].w = sum_groups<L>(acc[k].w);
  }
  if (g == 0) {
    f4v dpv[kK4];
#pragma unroll
    for (int k = 0; k < kK4; ++k) {
      acc[k] += c0 * s.p[k];
      dpv[k] = c0 * s.o[k];
    }
    store_vec<L>(dorow, j, a.D, acc);
    store_vec<L>(dprow, j, a.D, dpv);
  }
}

// ---- transpose of the sampling (counting sort by catalog row)
// Count: each workgroup ranks its chunk of kCountChunk samples in an LDS histogram
// (LDS atomics), then claims its range inside every bucket with one global atomic per
// non-empty bucket; rank[p] = bucket-local position of sample p.  Catalogs too large for
// LDS (V > kLdsBins) rank with global atomics directly.
constexpr int kCountThreads = 1024;
constexpr int kCountPer = 32;
constexpr int64_t kCountChunk = (int64_t)kCountThreads * kCountPer;
constexpr int64_t kLdsBins = 32768;

// Sort key of sample p = t * R + r: (token range of t) * V + catalog row.  With kRanges = 8
// the tokens split into one contiguous range per XCD (blocks b, b + 8 share an XCD) so
// an XCD's out_t gathers stay in its L2; measured at ml-1m C2 that cost more (8x the
// buckets: more flushes, a 126 KB count histogram) than it saved: 168 -> 372 us.
constexpr int kRanges = 1;

__device__ __forceinline__ int sort_key(int2 x, int64_t p, int R, int64_t M, int64_t V) {
  const int64_t t = p / R;
  return (int)((t * kRanges / M) * V + x.x);
}

template <bool LDS>
__global__ __launch_bounds__(kCountThreads) void ssm_count_kernel(const int2* rec, int64_t n, int R,
                                                                  int64_t M, int64_t V, int64_t K,
                                                                  int* cnt, int* rank) {
  if constexpr (LDS) {
    extern __shared__ int hist[];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kCountChunk;
    for (int64_t v = tid; v < K; v += kCountThreads) hist[v] = 0;
    __syncthreads();
    int vv[kCountPer], lr[kCountPer];
#pragma unroll
    for (int k = 0; k < kCountPer; ++k) {
      const int64_t p = base + (int64_t)k * kCountThreads + tid;
      const int key = p < n ? sort_key(rec[p], p, R, M, V) : -1;
      vv[k] = key >= 0 && key < K ? key : -1;  // out-of-range rows: dropped (fill flags them)
    }
#pragma unroll
    for (int k = 0; k < kCountPer; ++k) lr[k] = vv[k] >= 0 ? atomicAdd(hist + vv[k], 1) : 0;
    __syncthreads();
    for (int64_t v = tid; v < K; v += kCountThreads) {
      const int c = hist[v];
      hist[v] = c ? atomicAdd(cnt + v, c) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kCountPer; ++k) {
      const int64_t p = base + (int64_t)k * kCountThreads + threadIdx.x;
      if (vv[k] >= 0) rank[p] = hist[vv[k]] + lr[k];
    }
  } else {
    for (int64_t p = (int64_t)blockIdx.x * kCountThreads + threadIdx.x; p < n;
         p += (int64_t)gridDim.x * kCountThreads) {
      const int key = sort_key(rec[p], p, R, M, V);
      rank[p] = key >= 0 && key < K ? atomicAdd(cnt + key, 1) : 0;
    }
  }
}

// exclusive scan of cnt[0..V) into start[0..V] (start[V] = total), one workgroup
__global__ __launch_bounds__(1024) void ssm_scan_kernel(const int* cnt, int64_t V, int* start) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int64_t per = (V + 1023) / 1024;
  const int64_t b = min(V, tid * per), e = min(V, b + per);
  int s = 0;
  for (int64_t v = b; v < e; ++v) s += cnt[v];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const int x = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  int run = part[tid] - s;
  for (int64_t v = b; v < e; ++v) {
    start[v] = run;
    run += cnt[v];
  }
  if (tid == 1023) start[V] = part[1023];
}

// Scatter: sorted[start[key] + rank[p]] = {t, c} of sample p = t * R + r.  A slot outside
// its key's [start[key], start[key + 1]) (or a key outside [0, K)) is never written: the
// sample is dropped and the status word flags it.
__global__ __launch_bounds__(256) void ssm_fill_kernel(const int2* rec, int64_t n, int R, int64_t M,
                                                       int64_t V, int64_t K, const int* start,
                                                       const int* rank, int2* sorted, int* status) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const int2 x = rec[p];
    const int key = sort_key(x, p, R, M, V);
    if (key < 0 || key >= K || x.x < 0 || x.x >= V) {
      atomicOr(status, 1);
      continue;
    }
    const int64_t dst = (int64_t)start[key] + rank[p];
    if (rank[p] < 0 || dst >= start[key + 1] || dst >= n) {
      atomicOr(status, 2);
      continue;
    }
    sorted[dst] = make_int2((int)(p / R), x.y);
  }
}

// d_table[v] += sum over row v's samples of c * out_t.  One wave per kTgSeg consecutive
// sorted samples; group g of the wave owns the contiguous run g*P .. g*P+P-1 of them
// (P = kTgSeg / G), so a group crosses few catalog rows.  Per batch, lane l loads the
// {t, c} of sample (l / L)*P + b*L + l % L (runs of L, the next batch prefetched) and
// group g takes its run's sample b*L + i in step i.  Rows come from the boundaries
// start[] that fall inside the segment (scalar loads; usually none or one).  A group
// accumulates in registers while its row stays the same and flushes with fp32 atomics
// when it changes; at the end the groups merge into one flush when they all sit on the
// same row.  The caller zeroes d_table.
constexpr int kTgSeg = 256;

template <int L>
__device__ __forceinline__ void tg_flush(float* d_table, int64_t ld_dt, int v, int j, int D,
                                         const f4v (&acc)[kK4]) {
  float* dst = d_table + (int64_t)v * ld_dt;
#pragma unroll
  for (int k = 0; k < kK4; ++k) {
    const int d = 4 * j + 4 * L * k;
    if (d < D) atomicAdd(dst + d, acc[k].x);
    if (d + 1 < D) atomicAdd(dst + d + 1, acc[k].y);
    if (d + 2 < D) atomicAdd(dst + d + 2, acc[k].z);
    if (d + 3 < D) atomicAdd(dst + d + 3, acc[k].w);
  }
}

// first row v with start[v + 1] > q (start is non-decreasing, start[V] = n > q)
__device__ __forceinline__ int row_of(const int* start, int64_t V, int64_t q) {
  int64_t lo = 0, hi = V - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (start[mid + 1] > q) hi = mid; else lo = mid + 1;
  }
  return (int)lo;
}

template <int L>
__global__ __launch_bounds__(256) void ssm_table_grad_kernel(const float* out, int64_t ld_out,
                                                             int64_t M, int D, int64_t V, int64_t n,
                                                             const int* start, const int2* sorted,
                                                             float* d_table, int64_t ld_dt) {
  constexpr int G = 64 / L, S = L < kStepsInFlight ? L : kStepsInFlight, P = kTgSeg / G;
  // token range x = blockIdx % kRanges (blocks b and b + 8 share an XCD)
  const int x = blockIdx.x % kRanges;
  const int64_t rbeg = start[x * V], rend = start[(x + 1) * V];
  const int64_t w = (int64_t)(blockIdx.x / kRanges) * 4 + wave_id();
  const int64_t q0 = rbeg + w * kTgSeg;
  if (q0 >= rend) return;
  const int lane = threadIdx.x & 63, g = lane / L, j = lane % L;
  const int64_t qend = min(rend, q0 + kTgSeg);
  const int vfirst = __builtin_amdgcn_readfirstlane(row_of(start, kRanges * V, q0));
  const __amdgpu_buffer_rsrc_t orr = rows_rsrc(out, M, ld_out);
  f4v acc[kK4];
#pragma unroll
  for (int k = 0; k < kK4; ++k) acc[k] = f4v{0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  const int64_t qlane = q0 + (int64_t)(lane / L) * P + lane % L;  // batch 0
  int2 nxt = qlane < qend ? sorted[qlane] : make_int2(0, 0);
#pragma unroll 1
  for (int b = 0; b < P / L; ++b) {
    const int64_t q = qlane + (int64_t)b * L;
    const int2 x = nxt;
    if (b + 1 < P / L) nxt = q + L < qend ? sorted[q + L] : make_int2(0, 0);
    const bool valid = q < qend;
    // row of this lane's sample: vfirst + number of row boundaries <= q in the segment
    int vq = vfirst;
    for (int v = vfirst;; ++v) {
      const int bnd = start[v + 1];  // wave-uniform scalar load
      if (bnd >= qend) break;
      vq += q >= bnd ? 1 : 0;
    }
    vq = valid ? vq : -1;
    const int tq = x.x;
    const float cq = valid ? __int_as_float(x.y) : 0.f;
#pragma unroll
    for (int i0 = 0; i0 < L; i0 += S) {
      f4v row[S][kK4];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int t = __shfl(tq, g * L + i0 + i, 64);
        const int base = (int)(((int64_t)t * ld_out + 4 * j) * 4);
#pragma unroll
        for (int k = 0; k < kK4; ++k) row[i][k] = buf_ld4(orr, base + 16 * L * k);
      }
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int v = __shfl(vq, g * L + i0 + i, 64);
        const float c = __shfl(cq, g * L + i0 + i, 64);
        if (v != cur) {  // uniform within the group
          if (cur >= 0) tg_flush<L>(d_table, ld_dt, cur % (int)V, j, D, acc);
#pragma unroll
          for (int k = 0; k < kK4; ++k) acc[k] = f4v{0.f, 0.f, 0.f, 0.f};
          cur = v;
        }
#pragma unroll
        for (int k = 0; k < kK4; ++k) acc[k] += c * row[i][k];
      }
    }
  }
  const int c0 = __builtin_amdgcn_readfirstlane(cur);
  if (__ballot(cur != c0) == 0) {
#pragma unroll
    for (int k = 0; k < kK4; ++k) {
      acc[k].x = sum_groups<L>(acc[k].x);
      acc[k].y = sum_groups<L>(acc[k].y);
      acc[k].z = sum_groups<L>(acc[k].z);
      acc[k].w = sum_groups<L>(acc[k].w);
    }
    if (g == 0 && cur >= 0) tg_flush<L>(d_table, ld_dt, cur % (int)V, j, D, acc);
  } else if (cur >= 0) {
    tg_flush<L>(d_table, ld_dt, cur % (int)V, j, D, acc);
  }
}

// Deterministic mode: keys[p] = catalog row of sample p, vals[p] = p (sort input).
__global__ __launch_bounds__(256) void ssm_det_keys_kernel(const int2* rec, int64_t n, int64_t V,
                                                           int* keys, int* vals, int* status) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const int v = rec[p].x;
    if (v < 0 || v >= V) atomicOr(status, 1);
    keys[p] = v < 0 || v >= V ? (int)V : v;  // out-of-range rows sort past every real row
    vals[p] = (int)p;
  }
}

// first position e in skeys[0 .. n) with skeys[e] >= v
__device__ __forceinline__ int64_t lower_bound_i32(const int* skeys, int64_t n, int v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skeys[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// One wave per catalog row: d_table[v] = sum over its samples, in sample order, of
// c * out_t (lanes over the D columns; 8 samples' rows loaded ahead of their adds).
__global__ __launch_bounds__(256) void ssm_table_grad_det_kernel(const float* out, int64_t ld_out,
                                                                 int D, int64_t V, int R, int64_t n,
                                                                 const int2* rec, const int* skeys,
                                                                 const int* svals, float* d_table,
                                                                 int64_t ld_dt) {
  const int64_t v = (int64_t)blockIdx.x * 4 + wave_id();
  if (v >= V) return;
  const int lane = threadIdx.x & 63;
  const int64_t lo = lower_bound_i32(skeys, n, (int)v), hi = lower_bound_i32(skeys, n, (int)v + 1);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // columns lane + 64 j (D <= 256)
  constexpr int U = 8;
  for (int64_t e0 = lo; e0 < hi; e0 += U) {
    float c[U], x[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u < hi ? e0 + u : hi - 1;
      const int p = svals[e];
      const int2 r = rec[p];
      c[u] = e0 + u < hi ? __int_as_float(r.y) : 0.f;
      const float* orow = out + (int64_t)(p / R) * ld_out;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int d = lane + 64 * j;
        x[u][j] = d < D ? orow[d] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += c[u] * x[u][j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = lane + 64 * j;
    if (d < D) d_table[v * ld_dt + d] = acc[j];
  }
}

// d_table[v][0 .. D) = 0 for every row (a strided memset as a kernel: the graph-captured
// step then holds no 2-D memset node)
__global__ __launch_bounds__(256) void ssm_zero_rows_kernel(float* p, int64_t ld, int64_t rows, int D) {
  const int64_t total = rows * D;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / D;
    p[r * ld + (e - r * D)] = 0.f;
  }
}

inline int lanes_per_row(int D) { return D <= 16 ? 1 : D <= 32 ? 2 : D <= 64 ? 4 : D <= 128 ? 8 : 16; }

#define GR_SSM_DISPATCH(L, KERNEL, ...)                          \
  switch (L) {                                                   \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;   \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;   \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;   \
    default: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break; \
  }

inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// GR_OPT_DETERMINISTIC: the table gradient from a STABLE radix sort of the samples by
// catalog row (hipcub, keys = row, values = sample index in sample order), then one wave
// per row summing its samples in sample order -- no atomics, a fixed summation order.
inline size_t ssm_det_sort_bytes(int64_t n, int64_t V) {
  size_t tb = 0;
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) <= V) ++bits;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const int*)nullptr, (int*)nullptr,
                                           (const int*)nullptr, (int*)nullptr, (int)n, 0, bits);
  return tb;
}
inline size_t ssm_det_bytes(int64_t n, int64_t V) {
  return option(GR_OPT_DETERMINISTIC) != 0 ? align256(n * 4) + align256(ssm_det_sort_bytes(n, V)) : 0;
}

// workspace: rec[n] (int2) | sorted[n] (int2) | cnt[K] | start[K+1] | rank[n] (int32)
// [| vals[n] | sort temp  (deterministic mode)] | status word, K = kRanges * V sort keys
inline size_t ssm_ws_bytes(int64_t M, int R, int64_t V, int D) {
  (void)D;
  const int64_t n = M * (int64_t)R, K = kRanges * V;
  return 2 * align256(n * 8) + align256(K * 4) + align256((K + 1) * 4) + align256(n * 4) +
         ssm_det_bytes(n, V) + 256;
}
// byte offset of the status word (last 256 B of the workspace): 0 after a clean backward;
// bit 0 = a sample's catalog row outside [0, V), bit 1 = a scatter slot outside its row's
// range (stale counters) -- such samples are dropped instead of written out of bounds
inline size_t ssm_status_offset(int64_t M, int R, int64_t V, int D) {
  return ssm_ws_bytes(M, R, V, D) - 256;
}

inline bool fits_buffer(int64_t rows, int64_t ld) { return rows * ld * 4 < 0x7fffffff; }

}  // namespace gr

extern "C" {

size_t gr_sampled_softmax_workspace_size(int64_t M, int R, int64_t V, int D) {
  return gr::ssm_ws_bytes(M, R, V, D);
}

size_t gr_sampled_softmax_status_offset(int64_t M, int R, int64_t V, int D) {
  return gr::ssm_status_offset(M, R, V, D);
}

int gr_sampled_softmax_fwd(const float* out, int64_t ld_out, const float* pos, int64_t ld_pos,
                           const int64_t* sup_ids, const float* table, int64_t ld_table, int64_t V,
                           const int64_t* all_ids, const int64_t* offsets, int64_t M, int R, int D,
                           float temperature, float* loss, float* lse, void* stream) {
  GR_REQUIRE(M >= 0 && R >= 0 && D > 0 && D <= 256 && V > 0 && temperature != 0.f,
             "gr_sampled_softmax_fwd: bad sizes (M=%lld R=%d D=%d V=%lld)", (long long)M, R, D,
             (long long)V);
  GR_REQUIRE(gr::fits_buffer(V, ld_table) && gr::fits_buffer(M, ld_out) && gr::fits_buffer(M, ld_pos),
             "gr_sampled_softmax_fwd: table / rows must be < 2 GiB");
  if (M == 0) return 0;
  GR_REQUIRE(out && pos && sup_ids && table && loss && lse && (offsets || R == 0),
             "gr_sampled_softmax_fwd: null pointer");
  gr::SsmArgs a{};
  a.out = out; a.ld_out = ld_out; a.pos = pos; a.ld_pos = ld_pos; a.sup_ids = sup_ids;
  a.table = table; a.ld_table = ld_table; a.V = V; a.all_ids = all_ids; a.offsets = offsets;
  a.M = M; a.R = R; a.D = D; a.temperature = temperature; a.loss = loss; a.lse = lse;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((M + 3) / 4)), block(256);
  GR_TIMED("sampled_softmax_fwd", st,
           GR_SSM_DISPATCH(gr::lanes_per_row(D), gr::ssm_fwd_kernel, grid, block, 0, st, a));
  GR_LAUNCH_CHECK("gr_sampled_softmax_fwd");
  return 0;
}

int gr_sampled_softmax_bwd(const float* out, int64_t ld_out, const float* pos, int64_t ld_pos,
                           const int64_t* sup_ids, const float* table, int64_t ld_table, int64_t V,
                           const int64_t* all_ids, const int64_t* offsets, int64_t M, int R, int D,
                           float temperature, const float* lse, const float* dloss, float* d_out,
                           int64_t ld_dout, float* d_pos, int64_t ld_dpos, float* d_table,
                           int64_t ld_dtable, void* workspace, size_t workspace_bytes,
                           void* stream) {
  GR_REQUIRE(M >= 0 && R >= 0 && D > 0 && D <= 256 && V > 0 && temperature != 0.f,
             "gr_sampled_softmax_bwd: bad sizes (M=%lld R=%d D=%d V=%lld)", (long long)M, R, D,
             (long long)V);
  GR_REQUIRE(M * (int64_t)R < ((int64_t)1 << 31) && V * 8 < ((int64_t)1 << 31),
             "gr_sampled_softmax_bwd: M*R and V must fit int32");
  GR_REQUIRE(gr::fits_buffer(V, ld_table) && gr::fits_buffer(M, ld_out) && gr::fits_buffer(M, ld_pos),
             "gr_sampled_softmax_bwd: table / rows must be < 2 GiB");
  GR_REQUIRE(d_table && ld_dtable >= D, "gr_sampled_softmax_bwd: bad d_table");
  const hipStream_t st = (hipStream_t)stream;
  const int64_t n = M * (int64_t)R;
  {  // the row reduction accumulates into d_table
    const int64_t zt = V * D;
    const unsigned zg = (unsigned)std::min<int64_t>((zt + 255) / 256, 4 * gr::device_cus());
    hipLaunchKernelGGL(gr::ssm_zero_rows_kernel, dim3(zg), dim3(256), 0, st, d_table, ld_dtable, V, D);
    GR_LAUNCH_CHECK("gr_sampled_softmax_bwd (zero d_table)");
  }
  if (M == 0) return 0;
  GR_REQUIRE(out && pos && sup_ids && table && lse && dloss && d_out && d_pos && (offsets || R == 0),
             "gr_sampled_softmax_bwd: null pointer");
  GR_REQUIRE(workspace && workspace_bytes >= gr::ssm_ws_bytes(M, R, V, D),
             "gr_sampled_softmax_bwd: workspace too small (%zu < %zu)", workspace_bytes,
             gr::ssm_ws_bytes(M, R, V, D));
  char* w = (char*)workspace;
  int2* rec = (int2*)w;
  w += gr::align256(n * 8);

  gr::SsmArgs a{};
  a.out = out; a.ld_out = ld_out; a.pos = pos; a.ld_pos = ld_pos; a.sup_ids = sup_ids;
  a.table = table; a.ld_table = ld_table; a.V = V; a.all_ids = all_ids; a.offsets = offsets;
  a.M = M; a.R = R; a.D = D; a.temperature = temperature; a.lse = const_cast<float*>(lse);
  a.dloss = dloss; a.d_out = d_out; a.ld_dout = ld_dout; a.d_pos = d_pos; a.ld_dpos = ld_dpos;
  a.rec = rec;
  const int L = gr::lanes_per_row(D);
  const dim3 tgrid((unsigned)((M + 3) / 4)), block(256);
  GR_TIMED("sampled_softmax_bwd", st,
           GR_SSM_DISPATCH(L, gr::ssm_bwd_token_kernel, tgrid, block, 0, st, a));
  GR_LAUNCH_CHECK("gr_sampled_softmax_bwd");
  if (n == 0) return 0;
  int2* sorted = (int2*)w;
  w += gr::align256(n * 8);
  const int64_t K = gr::kRanges * V;
  int* cnt = (int*)w;
  w += gr::align256(K * 4);
  int* start = (int*)w;
  w += gr::align256((K + 1) * 4);
  int* rank = (int*)w;
  const unsigned sgrid = (unsigned)std::min<int64_t>((n + 255) / 256, 4 * gr::device_cus());
  if (gr::option(GR_OPT_DETERMINISTIC) != 0) {
    GR_REQUIRE(D <= 256 && n < 0x7fffffffLL && V < 0x7fffffffLL,
               "gr_sampled_softmax_bwd: deterministic mode needs D <= 256 and < 2^31 samples");
    int* status = (int*)((char*)workspace + gr::ssm_status_offset(M, R, V, D));
    int* keys_in = rank;                               // rank[n] region
    int* vals_in = (int*)(w + gr::align256(n * 4));    // deterministic extra region
    void* temp = (char*)vals_in + gr::align256(n * 4);
    size_t temp_bytes = gr::ssm_det_sort_bytes(n, V);
    int* keys_out = (int*)sorted;                      // sorted[n] (int2) region: 2 x n ints
    int* vals_out = keys_out + n;
    int bits = 1;
    while (bits < 31 && ((int64_t)1 << bits) <= V) ++bits;
    hipError_t srt = hipSuccess;
    GR_TIMED("sampled_softmax_csr", st, {
      gr::zero_words_async(status, 1, st);
      hipLaunchKernelGGL(gr::ssm_det_keys_kernel, dim3(sgrid), dim3(256), 0, st, rec, n, V, keys_in,
                         vals_in, status);
      srt = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in,
                                               vals_out, (int)n, 0, bits, st);
    });
    GR_REQUIRE(srt == hipSuccess, "gr_sampled_softmax_bwd: radix sort failed");
    GR_LAUNCH_CHECK("gr_sampled_softmax_bwd (deterministic sort)");
    GR_TIMED("sampled_softmax_table_grad", st,
             hipLaunchKernelGGL(gr::ssm_table_grad_det_kernel, dim3((unsigned)((V + 3) / 4)), dim3(256), 0,
                                st, out, ld_out, D, V, R, n, rec, keys_out, vals_out, d_table,
                                ld_dtable));
    GR_LAUNCH_CHECK("gr_sampled_softmax_bwd (deterministic table grad)");
    return 0;
  }
  const bool lds = K <= gr::kLdsBins;
  const unsigned cgrid = lds ? (unsigned)((n + gr::kCountChunk - 1) / gr::kCountChunk)
                             : (unsigned)std::min<int64_t>((n + 1023) / 1024, 4 * gr::device_cus());
  int* status = (int*)((char*)workspace + gr::ssm_status_offset(M, R, V, D));
  GR_TIMED("sampled_softmax_csr", st, {
    gr::zero_words_async(cnt, K, st);
    gr::zero_words_async(status, 1, st);
    if (lds)
      hipLaunchKernelGGL(gr::ssm_count_kernel<true>, dim3(cgrid), dim3(gr::kCountThreads),
                         (size_t)K * 4, st, rec, n, R, M, V, K, cnt, rank);
    else
      hipLaunchKernelGGL(gr::ssm_count_kernel<false>, dim3(cgrid), dim3(gr::kCountThreads), 0, st,
                         rec, n, R, M, V, K, cnt, rank);
    hipLaunchKernelGGL(gr::ssm_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, K, start);
    hipLaunchKernelGGL(gr::ssm_fill_kernel, dim3(sgrid), dim3(256), 0, st, rec, n, R, M, V, K, start,
                       rank, sorted, status);
  });
  GR_LAUNCH_CHECK("gr_sampled_softmax_bwd (csr)");
  // every token range holds exactly (its tokens) * R samples: at most ceil(M / 8) * R
  const int64_t per_range = (M + gr::kRanges - 1) / gr::kRanges * R;
  const int64_t wgs = (per_range + 4 * gr::kTgSeg - 1) / (4 * gr::kTgSeg);
  const dim3 wgrid((unsigned)(wgs * gr::kRanges));
  GR_TIMED("sampled_softmax_table_grad", st,
           GR_SSM_DISPATCH(L, gr::ssm_table_grad_kernel, wgrid, block, 0, st, out, ld_out, M, D, V, n,
                           start, sorted, d_table, ld_dtable));
  GR_LAUNCH_CHECK("gr_sampled_softmax_bwd (table grad)");
  return 0;
}

}  // extern "C"
