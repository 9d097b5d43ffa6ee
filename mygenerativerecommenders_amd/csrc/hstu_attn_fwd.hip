// Jagged causal HSTU attention, forward — gfx950, f32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Replaces reference sequential_encoders/hstu.py:134-205 (pad q/k/v, bmm QK^T, + bias,
// silu / N, causal mask, bmm AV, unpad) and the (B, N, N) bias materialisation of
// hstu.py:96-128.  Nothing N x N is ever written: the bias is rebuilt per tile from
// timestamps (int64 deltas -> integer threshold table) and pos_w held in LDS.
//
// Work decomposition: one workgroup = 4 waves = 64 queries of one (sequence, head);
// wave w owns queries q0+16w .. q0+16w+15.  The workgroup walks key tiles of 64
// (causal: tiles 0..qt) staged in LDS.  Per 16-key block a wave computes
//   S^T (16 keys x 16 queries) = K_blk . Q^T  (A = K rows from LDS, B = Q^T in VGPRs)
// so each lane holds 4 keys of ONE query; those 4 values are directly the A operand
// of the next product  O += P . V  with the key order permuted per k-step
// (k-step r uses keys 4g + r, g = lane>>4) — no LDS round trip for P.
// Blocks are issued heaviest-first (largest query tile first) for causal balance.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

struct AttnFwdArgs {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const int64_t* offsets;
  int B, N, H, dqk, dv, n_qtiles;
  const int64_t* ts;
  const float* pos_w;
  const float* ts_w;
  const int64_t* thr;
  int nb;
  float* out;
  int64_t ld_out;
  float inv_n;
};

template <int KSTEPS, int VTILES>
struct AttnFwdCfg {
  static constexpr int KP = KSTEPS * 4;                      // padded dqk
  static constexpr int VP = VTILES * 16;                     // padded dv
  static constexpr int LDK = 32 * ((KP - 2 + 31) / 32) + 2;  // == 2 mod 32: conflict-free A reads
  static constexpr int LDV = VP + 4;                         // == 4 mod 8: conflict-free B reads
  static constexpr int LDS_FLOATS = 64 * LDK + 64 * LDV;
};

template <int KSTEPS, int VTILES>
__global__ __launch_bounds__(256) void hstu_attn_fwd_kernel(AttnFwdArgs a) {
  using C = AttnFwdCfg<KSTEPS, VTILES>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);
  float* Vs = Ks + 64 * C::LDK;
  int64_t* tsk = reinterpret_cast<int64_t*>(Vs + 64 * C::LDV);  // 64 key timestamps
  int64_t* thr = tsk + 64;                                       // nb + 1
  float* tsw = reinterpret_cast<float*>(thr + (a.nb + 1));        // nb + 1
  float* posw = tsw + (a.nb + 1);                                // 2N - 1

  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int qt = a.n_qtiles - 1 - id / BH;  // heaviest tiles first
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

  // this lane's query (as the S^T column) and its Q^T fragments
  const int qi = q0 + w * 16 + lr;
  const bool q_ok = qi < L;
  float qreg[KSTEPS];
  {
    const float* qrow = a.q + (s0 + (q_ok ? qi : 0)) * a.ld_qk + h * a.dqk;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      qreg[st] = (q_ok && d < a.dqk) ? qrow[d] : 0.f;
    }
  }
  int64_t ts_next = 0;
  if (has_bias && q_ok) {
    const int nx = qi + 1 < a.N ? qi + 1 : a.N - 1;  // ext_ts[N] = ts[N-1] (hstu.py:113-115)
    ts_next = a.ts[(int64_t)b * a.N + nx];
  }

  f4 acc[VTILES];
#pragma unroll
  for (int ct = 0; ct < VTILES; ++ct) acc[ct] = f4_zero();

  const int wq_lo = q0 + w * 16;  // first query of this wave
  for (int kt = 0; kt <= qt; ++kt) {
    const int k0 = kt * 64;
    __syncthreads();
    // ---- stage K, V tiles (zero-filled past L / past d) and key timestamps
    for (int e = tid; e < 64 * C::KP; e += 256) {
      const int r = e / C::KP, c = e - r * C::KP;
      const int key = k0 + r;
      float val = 0.f;
      if (key < L && c < a.dqk) val = a.k[(s0 + key) * a.ld_qk + h * a.dqk + c];
      Ks[r * C::LDK + c] = val;
    }
    for (int e = tid; e < 64 * C::VP; e += 256) {
      const int r = e / C::VP, c = e - r * C::VP;
      const int key = k0 + r;
      float val = 0.f;
      if (key < L && c < a.dv) val = a.v[(s0 + key) * a.ld_v + h * a.dv + c];
      Vs[r * C::LDV + c] = val;
    }
    if (has_bias && tid < 64) {
      const int key = k0 + tid;
      tsk[tid] = key < L ? a.ts[(int64_t)b * a.N + key] : 0;
    }
    __syncthreads();

#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int kb0 = k0 + kb * 16;
      if (kb0 > wq_lo + 15 || kb0 >= L) break;  // wave-uniform causal / length skip
      f4 s = f4_zero();
      const float* krow = Ks + (kb * 16 + lr) * C::LDK + lg;
#pragma unroll
      for (int st = 0; st < KSTEPS; ++st) s = mfma16x16x4(krow[4 * st], qreg[st], s);
      // s[r] = S^T[key kb0 + 4lg + r][query qi]
      float p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = kb0 + 4 * lg + r;
        float val = s[r];
        if (has_bias) {
          const int bucket = time_bucket(ts_next - tsk[kb * 16 + 4 * lg + r], thr, a.nb);
          const int pi = a.N - 1 + kj - qi;
          const float bias = posw[pi < 0 ? 0 : (pi > 2 * a.N - 2 ? 2 * a.N - 2 : pi)] + tsw[bucket];
          val = val + bias;
        }
        p[r] = (q_ok && kj <= qi) ? siluf_(val) * a.inv_n : 0.f;
      }
      const float* vrow = Vs + (kb * 16 + 4 * lg) * C::LDV + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int ct = 0; ct < VTILES; ++ct)
          acc[ct] = mfma16x16x4(p[r], vrow[r * C::LDV + ct * 16], acc[ct]);
      }
    }
  }

  // ---- epilogue: acc[ct][r] = O[query wq_lo + 4lg + r][col ct*16 + lr]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qo = wq_lo + 4 * lg + r;
    if (qo >= L) continue;
    float* orow = a.out + (s0 + qo) * a.ld_out + h * a.dv;
#pragma unroll
    for (int ct = 0; ct < VTILES; ++ct) {
      const int c = ct * 16 + lr;
      if (c < a.dv) orow[c] = acc[ct][r];
    }
  }
}

// (KSTEPS, VTILES) instantiation ladder, chosen by max(dqk, dv) bracket
template <int KS, int VT>
static int launch_fwd(const AttnFwdArgs& a, int grid, hipStream_t st) {
  using C = AttnFwdCfg<KS, VT>;
  size_t lds = sizeof(float) * C::LDS_FLOATS + sizeof(int64_t) * (64 + a.nb + 1) +
               sizeof(float) * (a.nb + 1 + 2 * a.N - 1);
  GR_REQUIRE(lds <= 160 * 1024, "hstu_attn_fwd: LDS %zu B exceeds 160 KiB (N=%d)", lds, a.N);
  hipLaunchKernelGGL((hstu_attn_fwd_kernel<KS, VT>), dim3(grid), dim3(256), lds, st, a);
  GR_LAUNCH_CHECK("hstu_attn_fwd");
  return 0;
}

}  // namespace gr

extern "C" int hstu_attn_fwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                             int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                             int H, int dqk, int dv, const int64_t* ts, const float* pos_w,
                             const float* ts_w, const int64_t* bucket_thr, int num_buckets,
                             float* out, int64_t ld_out, void* stream) {
  using namespace gr;
  GR_REQUIRE(q && k && v && offsets && out, "hstu_attn_fwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_fwd: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_fwd: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 128 && dv <= 128, "hstu_attn_fwd: dqk/dv > 128 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE(!ts || (pos_w && ts_w && bucket_thr && num_buckets > 0 && num_buckets < 1024),
             "hstu_attn_fwd: ts given without pos_w/ts_w/bucket_thr");
  if (B == 0 || max_len == 0) return 0;
  AttnFwdArgs a{q, k, v, ld_qk, ld_v, offsets, B, N, H, dqk, dv, ceil_div(max_len, 64),
                ts, pos_w, ts_w, bucket_thr, ts ? num_buckets : 0, out, ld_out, 1.0f / (float)N};
  const int grid = a.n_qtiles * B * H;
  hipStream_t st = (hipStream_t)stream;
  const int d = dqk > dv ? dqk : dv;
  if (d <= 8) return launch_fwd<2, 1>(a, grid, st);
  if (d <= 16) return launch_fwd<4, 1>(a, grid, st);
  if (d <= 32) return launch_fwd<8, 2>(a, grid, st);
  if (d <= 52) return launch_fwd<13, 4>(a, grid, st);
  if (d <= 64) return launch_fwd<16, 4>(a, grid, st);
  return launch_fwd<32, 8>(a, grid, st);
}
