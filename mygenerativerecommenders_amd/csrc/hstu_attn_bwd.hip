// Jagged causal HSTU attention, backward — gfx950, f32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Replaces the autograd backward of reference sequential_encoders/hstu.py:134-205 and
// of the bias module hstu.py:96-128 (bmm-backward x4, silu_backward, the index_add_
// of 5.7 M updates into the 129-bin _ts_w and the slice/pad backward into _pos_w).
// HSTU attention has no softmax, so there is no LSE/delta: with
//   S = Q K^T + bias,  P = silu(S) / N (causal),  O = P V
// the gradients are  dP = dO V^T,  dS = dP * silu'(S) / N,
//   dV = P^T dO,  dK = dS^T Q,  dQ = dS K,  dbias[i, j] = sum_h dS[h, i, j].
// Two atomic-free, deterministic kernels recompute S:
//   * key-major  (dK, dV, bias grads): a workgroup owns 64 keys and walks the query
//     tiles at or after it; per-wave LDS histograms for dpos_w (2N-1 bins) and dts_w
//     (129 bins) are summed in a fixed order into one slab per workgroup, and a third
//     kernel reduces the slabs in a fixed order;
//   * query-major (dQ): a workgroup owns 64 queries and walks key tiles 0..qt.
// Optional fused epilogue: the gradients are multiplied by silu'(h) of the UVQK
// pre-activation (hstu.py:303-305), so the caller gets d(pre-activation) directly.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

struct AttnBwdArgs {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const float* dout;
  int64_t ld_dout;
  const int64_t* offsets;
  int B, N, H, dqk, dv, n_tiles;
  const int64_t* ts;
  const float* pos_w;
  const float* ts_w;
  const int64_t* thr;
  int nb;
  const float* hq;
  const float* hk;
  const float* hv;
  int64_t ld_h;
  float* dq;
  float* dk;
  float* dvv;
  int64_t ld_d;
  float* slabs;  // [grid][2N-1 + nb+1]
  float inv_n;
};

template <int KSTEPS, int VTILES>
struct AttnBwdCfg {
  static constexpr int KP = KSTEPS * 4;          // padded dqk (k-steps of the QK product)
  static constexpr int KT = (KP + 15) / 16;      // 16-col tiles of dK / dQ
  static constexpr int KPT = KT * 16;            // dqk padded to the output tile width
  static constexpr int VP = VTILES * 16;         // padded dv
  static constexpr int VSTEPS = VP / 4;          // k-steps of the dO V^T product
  // row strides: == 4 mod 8 keeps the 4-row-apart B reads conflict-free; the 16-row
  // A reads are then 2-way (LDS is not the limiter at 32-cycle MFMAs).
  static constexpr int LDQ = (KPT > KP ? KPT : KP) + 4;
  static constexpr int LDV = VP + 4;
};

__device__ __forceinline__ float attn_bias(int64_t tsn, int64_t tsk, int i, int j,
                                           const int64_t* thr, const float* tsw,
                                           const float* posw, int N, int nb) {
  const int bucket = time_bucket(tsn - tsk, thr, nb);
  int pi = N - 1 + j - i;
  pi = pi < 0 ? 0 : (pi > 2 * N - 2 ? 2 * N - 2 : pi);
  return posw[pi] + tsw[bucket];
}

// ------------------------------------------------------------------ key-major: dK, dV
template <int KSTEPS, int VTILES>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnBwdArgs a) {
  using C = AttnBwdCfg<KSTEPS, VTILES>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Qs = reinterpret_cast<float*>(smem);              // [64][LDQ]
  float* Ds = Qs + 64 * C::LDQ;                            // dO tile [64][LDV]
  int64_t* tsn = reinterpret_cast<int64_t*>(Ds + 64 * C::LDV);  // 64 query next-ts
  int64_t* thr = tsn + 64;                                 // nb + 1
  float* tsw = reinterpret_cast<float*>(thr + (a.nb + 1)); // nb + 1
  float* posw = tsw + (a.nb + 1);                          // 2N - 1
  const int nbins = 2 * a.N - 1 + a.nb + 1;
  float* hist = posw + (2 * a.N - 1);                      // [4 waves][nbins]

  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int kt = id / BH;  // kt = 0 (the most query tiles) first
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int k0 = kt * 64;
  const bool has_bias = a.ts != nullptr;
  float* slab = a.slabs ? a.slabs + (int64_t)id * nbins : nullptr;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;

  if (k0 >= L) {  // this workgroup still owns a (zero) slab
    if (has_bias && slab)
      for (int i = tid; i < nbins; i += 256) slab[i] = 0.f;
    return;
  }
  if (has_bias) {
    for (int i = tid; i <= a.nb; i += 256) {
      thr[i] = a.thr[i];
      tsw[i] = a.ts_w[i];
    }
    for (int i = tid; i < 2 * a.N - 1; i += 256) posw[i] = a.pos_w[i];
    for (int i = tid; i < 4 * nbins; i += 256) hist[i] = 0.f;
  }
  float* whist = hist + w * nbins;

  // this lane's key (as the column of S and dP) and its K^T / V^T fragments
  const int kj = k0 + w * 16 + lr;
  const bool k_ok = kj < L;
  float kreg[KSTEPS], vreg[C::VSTEPS];
  {
    const float* krow = a.k + (s0 + (k_ok ? kj : 0)) * a.ld_qk + h * a.dqk;
    const float* vrow = a.v + (s0 + (k_ok ? kj : 0)) * a.ld_v + h * a.dv;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      kreg[st] = (k_ok && d < a.dqk) ? krow[d] : 0.f;
    }
#pragma unroll
    for (int st = 0; st < C::VSTEPS; ++st) {
      const int d = 4 * st + lg;
      vreg[st] = (k_ok && d < a.dv) ? vrow[d] : 0.f;
    }
  }
  const int64_t ts_k = (has_bias && k_ok) ? a.ts[(int64_t)b * a.N + kj] : 0;
  const int vsteps = (a.dv + 3) / 4;

  f4 dV[VTILES], dK[C::KT];
#pragma unroll
  for (int t = 0; t < VTILES; ++t) dV[t] = f4_zero();
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dK[t] = f4_zero();

  const int wk_lo = k0 + w * 16;
  const int last_qt = (L - 1) / 64;
  for (int qt = kt; qt <= last_qt; ++qt) {
    const int q0 = qt * 64;
    __syncthreads();
    for (int e = tid; e < 64 * C::KPT; e += 256) {
      const int r = e / C::KPT, c = e - r * C::KPT;
      const int qi = q0 + r;
      float val = 0.f;
      if (qi < L && c < a.dqk) val = a.q[(s0 + qi) * a.ld_qk + h * a.dqk + c];
      Qs[r * C::LDQ + c] = val;
    }
    for (int e = tid; e < 64 * C::VP; e += 256) {
      const int r = e / C::VP, c = e - r * C::VP;
      const int qi = q0 + r;
      float val = 0.f;
      if (qi < L && c < a.dv) val = a.dout[(s0 + qi) * a.ld_dout + h * a.dv + c];
      Ds[r * C::LDV + c] = val;
    }
    if (has_bias && tid < 64) {
      const int qi = q0 + tid;
      const int nx = qi + 1 < a.N ? qi + 1 : a.N - 1;
      tsn[tid] = qi < L ? a.ts[(int64_t)b * a.N + nx] : 0;
    }
    __syncthreads();

#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      const int qb0 = q0 + qb * 16;
      if (qb0 >= L) break;                   // past the sequence
      if (qb0 + 15 < wk_lo) continue;        // all queries before this wave's keys
      // S[query 4lg + r][key lr] and dP alike
      f4 s = f4_zero(), dp = f4_zero();
      const float* qrow = Qs + (qb * 16 + lr) * C::LDQ + lg;
#pragma unroll
      for (int st = 0; st < KSTEPS; ++st) s = mfma16x16x4(qrow[4 * st], kreg[st], s);
      const float* drow = Ds + (qb * 16 + lr) * C::LDV + lg;
#pragma unroll
      for (int st = 0; st < C::VSTEPS; ++st) {
        if (st < vsteps) dp = mfma16x16x4(drow[4 * st], vreg[st], dp);
      }
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = qb0 + 4 * lg + r;
        const bool ok = k_ok && qi < L && kj <= qi;
        float x = s[r];
        int bucket = 0;
        if (has_bias && ok) {
          bucket = time_bucket(tsn[qb * 16 + 4 * lg + r] - ts_k, thr, a.nb);
          x = x + (posw[a.N - 1 + kj - qi] + tsw[bucket]);
        }
        const float sg = sigmoidf_(x);
        p[r] = ok ? x * sg * a.inv_n : 0.f;
        ds[r] = ok ? dp[r] * (sg * (1.0f + x * (1.0f - sg))) * a.inv_n : 0.f;
        if (has_bias && ok) {
          atomicAdd(&whist[a.N - 1 + kj - qi], ds[r]);
          atomicAdd(&whist[2 * a.N - 1 + bucket], ds[r]);
        }
      }
      // dV[key][c] += P^T dO ; dK[key][d] += dS^T Q   (k-step r: queries 4g + r)
      const float* dcol = Ds + (qb * 16 + 4 * lg) * C::LDV + lr;
      const float* qcol = Qs + (qb * 16 + 4 * lg) * C::LDQ + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int t = 0; t < VTILES; ++t)
          dV[t] = mfma16x16x4(p[r], dcol[r * C::LDV + t * 16], dV[t]);
#pragma unroll
        for (int t = 0; t < C::KT; ++t)
          dK[t] = mfma16x16x4(ds[r], qcol[r * C::LDQ + t * 16], dK[t]);
      }
    }
  }

  // ---- epilogue: rows = keys wk_lo + 4lg + r, cols = lr + 16 t
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = wk_lo + 4 * lg + r;
    if (key >= L) continue;
    const int64_t row = s0 + key;
#pragma unroll
    for (int t = 0; t < VTILES; ++t) {
      const int c = t * 16 + lr;
      if (c < a.dv) {
        float g = dV[t][r];
        if (a.hv) g *= silu_grad_(a.hv[row * a.ld_h + h * a.dv + c]);
        a.dvv[row * a.ld_d + h * a.dv + c] = g;
      }
    }
#pragma unroll
    for (int t = 0; t < C::KT; ++t) {
      const int c = t * 16 + lr;
      if (c < a.dqk) {
        float g = dK[t][r];
        if (a.hk) g *= silu_grad_(a.hk[row * a.ld_h + h * a.dqk + c]);
        a.dk[row * a.ld_d + h * a.dqk + c] = g;
      }
    }
  }
  if (has_bias && slab) {
    __syncthreads();
    for (int i = tid; i < nbins; i += 256)
      slab[i] = ((hist[i] + hist[nbins + i]) + hist[2 * nbins + i]) + hist[3 * nbins + i];
  }
}

// ------------------------------------------------------------------ query-major: dQ
template <int KSTEPS, int VTILES>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  using C = AttnBwdCfg<KSTEPS, VTILES>;
  constexpr int LDK = C::LDQ;
  constexpr int LDV = 32 * ((C::VP - 2 + 31) / 32) + 2;  // A-operand reads only
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);          // [64][LDK]
  float* Vs = Ks + 64 * LDK;                           // [64][LDV]
  int64_t* tsk = reinterpret_cast<int64_t*>(Vs + 64 * LDV);
  int64_t* thr = tsk + 64;
  float* tsw = reinterpret_cast<float*>(thr + (a.nb + 1));
  float* posw = tsw + (a.nb + 1);

  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qt = a.n_tiles - 1 - id / BH;
  const int bh = id % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * 64;
  if (q0 >= L) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const bool has_bias = a.ts != nullptr;
  if (has_bias) {
    for (int i = tid; i <= a.nb; i += 256) {
      thr[i] = a.thr[i];
      tsw[i] = a.ts_w[i];
    }
    for (int i = tid; i < 2 * a.N - 1; i += 256) posw[i] = a.pos_w[i];
  }
  const int qi = q0 + w * 16 + lr;
  const bool q_ok = qi < L;
  float qreg[KSTEPS], doreg[C::VSTEPS];
  {
    const float* qrow = a.q + (s0 + (q_ok ? qi : 0)) * a.ld_qk + h * a.dqk;
    const float* drow = a.dout + (s0 + (q_ok ? qi : 0)) * a.ld_dout + h * a.dv;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      qreg[st] = (q_ok && d < a.dqk) ? qrow[d] : 0.f;
    }
#pragma unroll
    for (int st = 0; st < C::VSTEPS; ++st) {
      const int d = 4 * st + lg;
      doreg[st] = (q_ok && d < a.dv) ? drow[d] : 0.f;
    }
  }
  int64_t ts_next = 0;
  if (has_bias && q_ok) {
    const int nx = qi + 1 < a.N ? qi + 1 : a.N - 1;
    ts_next = a.ts[(int64_t)b * a.N + nx];
  }
  const int vsteps = (a.dv + 3) / 4;
  f4 dQ[C::KT];
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dQ[t] = f4_zero();
  const int wq_lo = q0 + w * 16;

  for (int kt = 0; kt <= qt; ++kt) {
    const int k0 = kt * 64;
    __syncthreads();
    for (int e = tid; e < 64 * C::KPT; e += 256) {
      const int r = e / C::KPT, c = e - r * C::KPT;
      const int key = k0 + r;
      float val = 0.f;
      if (key < L && c < a.dqk) val = a.k[(s0 + key) * a.ld_qk + h * a.dqk + c];
      Ks[r * LDK + c] = val;
    }
    for (int e = tid; e < 64 * C::VP; e += 256) {
      const int r = e / C::VP, c = e - r * C::VP;
      const int key = k0 + r;
      float val = 0.f;
      if (key < L && c < a.dv) val = a.v[(s0 + key) * a.ld_v + h * a.dv + c];
      Vs[r * LDV + c] = val;
    }
    if (has_bias && tid < 64) {
      const int key = k0 + tid;
      tsk[tid] = key < L ? a.ts[(int64_t)b * a.N + key] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int kb0 = k0 + kb * 16;
      if (kb0 > wq_lo + 15 || kb0 >= L) break;
      f4 s = f4_zero(), dpt = f4_zero();
      const float* krow = Ks + (kb * 16 + lr) * LDK + lg;
#pragma unroll
      for (int st = 0; st < KSTEPS; ++st) s = mfma16x16x4(krow[4 * st], qreg[st], s);
      const float* vrow = Vs + (kb * 16 + lr) * LDV + lg;
#pragma unroll
      for (int st = 0; st < C::VSTEPS; ++st)
        if (st < vsteps) dpt = mfma16x16x4(vrow[4 * st], doreg[st], dpt);
      // s[r] = S^T[key kb0 + 4lg + r][query qi]
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = kb0 + 4 * lg + r;
        const bool ok = q_ok && kj <= qi;
        float x = s[r];
        if (has_bias && ok)
          x = x + attn_bias(ts_next, tsk[kb * 16 + 4 * lg + r], qi, kj, thr, tsw, posw, a.N, a.nb);
        ds[r] = ok ? dpt[r] * silu_grad_(x) * a.inv_n : 0.f;
      }
      const float* kcol = Ks + (kb * 16 + 4 * lg) * LDK + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int t = 0; t < C::KT; ++t)
          dQ[t] = mfma16x16x4(ds[r], kcol[r * LDK + t * 16], dQ[t]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qo = wq_lo + 4 * lg + r;
    if (qo >= L) continue;
    const int64_t row = s0 + qo;
#pragma unroll
    for (int t = 0; t < C::KT; ++t) {
      const int c = t * 16 + lr;
      if (c < a.dqk) {
        float g = dQ[t][r];
        if (a.hq) g *= silu_grad_(a.hq[row * a.ld_h + h * a.dqk + c]);
        a.dq[row * a.ld_d + h * a.dqk + c] = g;
      }
    }
  }
}

// ------------------------------------------------------------------ slab reduce
__global__ __launch_bounds__(256) void bias_grad_reduce_kernel(const float* slabs, int n_slabs,
                                                               int n_pos, int n_ts,
                                                               float* dpos_w, float* dts_w) {
  const int nbins = n_pos + n_ts;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nbins) return;
  float s = 0.f;
  for (int j = 0; j < n_slabs; ++j) s += slabs[(int64_t)j * nbins + i];
  if (i < n_pos) dpos_w[i] = s;
  else dts_w[i - n_pos] = s;
}

static size_t bwd_slab_bytes(int B, int N, int max_len, int H, int nb) {
  const int n_tiles = ceil_div(max_len, 64);
  return sizeof(float) * (size_t)n_tiles * B * H * (size_t)(2 * N - 1 + nb + 1);
}

template <int KS, int VT>
static int launch_bwd(const AttnBwdArgs& a, float* dpos_w, float* dts_w, hipStream_t st) {
  using C = AttnBwdCfg<KS, VT>;
  const int grid = a.n_tiles * a.B * a.H;
  const int nbins = 2 * a.N - 1 + a.nb + 1;
  const size_t tail = sizeof(int64_t) * (64 + a.nb + 1) + sizeof(float) * (a.nb + 1 + 2 * a.N - 1);
  const size_t lds_kv = sizeof(float) * (64 * C::LDQ + 64 * C::LDV) + tail +
                        (a.ts ? sizeof(float) * 4 * nbins : 0);
  constexpr int LDV_Q = 32 * ((C::VP - 2 + 31) / 32) + 2;
  const size_t lds_q = sizeof(float) * (64 * C::LDQ + 64 * LDV_Q) + tail;
  GR_REQUIRE(lds_kv <= 160 * 1024 && lds_q <= 160 * 1024,
             "hstu_attn_bwd: LDS (%zu, %zu B) exceeds 160 KiB (N=%d)", lds_kv, lds_q, a.N);
  hipLaunchKernelGGL((attn_bwd_dkv_kernel<KS, VT>), dim3(grid), dim3(256), lds_kv, st, a);
  GR_LAUNCH_CHECK("hstu_attn_bwd(dkv)");
  hipLaunchKernelGGL((attn_bwd_dq_kernel<KS, VT>), dim3(grid), dim3(256), lds_q, st, a);
  GR_LAUNCH_CHECK("hstu_attn_bwd(dq)");
  if (a.ts) {
    hipLaunchKernelGGL(bias_grad_reduce_kernel, dim3(ceil_div(nbins, 256)), dim3(256), 0, st,
                       a.slabs, grid, 2 * a.N - 1, a.nb + 1, dpos_w, dts_w);
    GR_LAUNCH_CHECK("hstu_attn_bwd(bias reduce)");
  }
  return 0;
}

}  // namespace gr

extern "C" size_t hstu_attn_bwd_workspace_size(int B, int N, int max_len, int H,
                                               int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0) return 0;
  return gr::bwd_slab_bytes(B, N, max_len, H, num_buckets);
}

extern "C" int hstu_attn_bwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                             int64_t ld_v, const float* dout, int64_t ld_dout,
                             const int64_t* offsets, int B, int N, int max_len, int H, int dqk,
                             int dv, const int64_t* ts, const float* pos_w, const float* ts_w,
                             const int64_t* bucket_thr, int num_buckets, const float* hq,
                             const float* hk, const float* hv, int64_t ld_h, float* dq,
                             float* dk, float* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                             void* workspace, size_t ws_bytes, void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && dout && offsets && dq && dk && dvv, "hstu_attn_bwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_bwd: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_bwd: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 128 && dv <= 128, "hstu_attn_bwd: dqk/dv > 128 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE((hq == nullptr) == (hk == nullptr) && (hk == nullptr) == (hv == nullptr),
             "hstu_attn_bwd: hq/hk/hv must be all given or all NULL");
  if (ts) {
    GR_REQUIRE(pos_w && ts_w && bucket_thr && dpos_w && dts_w && num_buckets > 0 && num_buckets < 1024,
               "hstu_attn_bwd: ts given without pos_w/ts_w/bucket_thr/dpos_w/dts_w");
    const size_t need = bwd_slab_bytes(B, N, max_len, H, num_buckets);
    GR_REQUIRE(workspace && ws_bytes >= need, "hstu_attn_bwd: workspace %zu B < %zu B", ws_bytes, need);
  }
  hipStream_t st = (hipStream_t)stream;
  if (B == 0 || max_len == 0) {
    if (ts) {
      (void)hipMemsetAsync(dpos_w, 0, sizeof(float) * (2 * N - 1), st);
      (void)hipMemsetAsync(dts_w, 0, sizeof(float) * (num_buckets + 1), st);
    }
    return 0;
  }
  AttnBwdArgs a{q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, H, dqk, dv,
                ceil_div(max_len, 64), ts, pos_w, ts_w, bucket_thr, ts ? num_buckets : 0,
                hq, hk, hv, ld_h, dq, dk, dvv, ld_d, ts ? (float*)workspace : nullptr,
                1.0f / (float)N};
  const int d = dqk > dv ? dqk : dv;
  if (d <= 8) return launch_bwd<2, 1>(a, dpos_w, dts_w, st);
  if (d <= 16) return launch_bwd<4, 1>(a, dpos_w, dts_w, st);
  if (d <= 32) return launch_bwd<8, 2>(a, dpos_w, dts_w, st);
  if (d <= 52) return launch_bwd<13, 4>(a, dpos_w, dts_w, st);
  if (d <= 64) return launch_bwd<16, 4>(a, dpos_w, dts_w, st);
  return launch_bwd<32, 8>(a, dpos_w, dts_w, st);
}
