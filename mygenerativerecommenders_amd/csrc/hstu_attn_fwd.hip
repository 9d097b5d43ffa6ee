// Jagged causal HSTU attention, forward — gfx950, f32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Replaces reference sequential_encoders/hstu.py:134-205 (pad q/k/v, bmm QK^T, + bias,
// silu / N, causal mask, bmm AV, unpad) and the (B, N, N) bias materialisation of
// hstu.py:96-128.  Nothing N x N is written per layer: the bias is rebuilt per tile
// from pos_w / ts_w (LDS) and the per-batch uint8 bucket map (hstu_bucket_map).
//
// Work decomposition: one workgroup = 4 waves = 64 queries of one (sequence, head);
// wave w owns queries q0+16w .. q0+16w+15.  The workgroup walks key tiles of 64
// (causal: tiles 0..qt) through LDS; tile kt+1 is loaded into registers while tile kt
// is computed (LDS-only barriers keep the prefetch in flight).  Per 16-key block a
// wave computes
//   S^T (16 keys x 16 queries) = K_blk . Q^T  (A = K rows from LDS, B = Q^T in VGPRs)
// so each lane holds 4 keys of ONE query; those 4 values are directly the A operand
// of the next product  O += P . V  with the key order permuted per k-step
// (k-step r uses keys 4g + r, g = lane>>4) — no LDS round trip for P.
// Blocks are issued heaviest-first (largest query tile first) for causal balance.
#include "attn_common.h"
#include "rowwave.h"

#include "../../include/gr_hstu.h"

namespace gr {

struct AttnFwdArgs {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const int64_t* offsets;
  int B, N, H, dqk, dv, n_qtiles;
  const uint8_t* map_qk;  // null: no bias
  const float* pos_w;
  const float* ts_w;
  int nb;
  float* out;
  int64_t ld_out;
  float inv_n;
  int vec2;  // 8-byte pair staging (aligned rows, even widths)
  int cus;   // CU count (snake_rank)
};

// TK = keys per LDS tile (64, or 16 for the wide head dims where a 64-key register
// stage would not fit next to the Q fragments and accumulators).
template <int KSTEPS, int VTILES, int TK>
struct AttnFwdCfg {
  static constexpr int KP = KSTEPS * 4;                      // padded dqk
  static constexpr int VP = VTILES * 16;                     // padded dv
  static constexpr int LDK = 32 * ((KP - 2 + 31) / 32) + 2;  // == 2 mod 32: conflict-free A reads
  static constexpr int LDV = VP + 4;                         // == 4 mod 8: conflict-free B reads
  static constexpr int LDS_FLOATS = TK * LDK + TK * LDV;
  static constexpr int KB = TK / 16;                         // 16-key blocks per tile
};

// V2: pair staging fixed at compile time (see BWD_V2 in hstu_attn_bwd.hip)
// Returns false when the workgroup's query tile is past its sequence (the whole workgroup
// returns), else the tile's first query q0, the sequence's first row s0 and length L.
template <int KSTEPS, int VTILES, int TK, bool HB, bool V2>
__device__ __forceinline__ bool hstu_attn_fwd_body(const AttnFwdArgs& a, int* q0_out = nullptr,
                                                   int* L_out = nullptr, int64_t* s0_out = nullptr) {
  using C = AttnFwdCfg<KSTEPS, VTILES, TK>;
  const bool v2 = V2 || a.vec2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);
  float* Vs = Ks + TK * C::LDK;
  float* tsw = Vs + TK * C::LDV;   // nb + 1
  float* posw = tsw + (a.nb + 1);  // 2N - 1

  const int BH = a.B * a.H;
  const int id = blockIdx.x;
  const int rank = snake_rank(id, a.cus);
  const int qt = a.n_qtiles - 1 - rank / BH;  // heaviest tiles first
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * 64;
  if (q0 >= L) return false;
  if (q0_out) {
    *q0_out = q0;
    *L_out = L;
    *s0_out = s0;
  }

  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr bool has_bias = HB;  // compile-time: the bias gathers of a lane issue together

  if (has_bias) {
    for (int i = tid; i <= a.nb; i += 256) tsw[i] = a.ts_w[i];
    for (int i = tid; i < 2 * a.N - 1; i += 256) posw[i] = a.pos_w[i];
  }

  // this lane's query (as the S^T column) and its Q^T fragments
  const int qi = q0 + w * 16 + lr;
  const bool q_ok = qi < L;
  float qreg[KSTEPS];
  {
    gptr<float> qrow = as_global(a.q) + (s0 + (q_ok ? qi : L - 1)) * a.ld_qk + h * a.dqk;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      const float x = qrow[d < a.dqk ? d : a.dqk - 1];
      qreg[st] = d < a.dqk ? x : 0.f;
    }
  }
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_qk, b, attn_tiles_per_seq(a.N));
  const int map_voff = ((w * 16 + lr) * 16 + lg) * 4;
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rv = seq_rsrc(a.v, a.ld_v, s0, h * a.dv, L, a.dv);

  f4 acc[VTILES];
#pragma unroll
  for (int ct = 0; ct < VTILES; ++ct) acc[ct] = f4_zero();

  BufTile<C::KP, TK> kst;
  BufTile<C::VP, TK> vst;
  uint32_t mw[C::KB], mwn[C::KB];
  auto load_tile = [&](int kt, uint32_t (&m)[C::KB]) {
    kst.load(rk, a.ld_qk, kt * TK, a.dqk, v2);
    vst.load(rv, a.ld_v, kt * TK, a.dv, v2);
#pragma unroll
    for (int kb = 0; kb < C::KB; ++kb)
      m[kb] = buf_ld_u32(rmap, map_voff, map_soff(q0, kt * TK + kb * 16, true));
  };

  load_tile(0, mw);
  kst.store(Ks, C::LDK, v2);
  vst.store(Vs, C::LDV, v2);
  __syncthreads();  // also publishes tsw / posw

  const int wq_lo = q0 + w * 16;  // first query of this wave
  const int last_kt = min(q0 + 63, L - 1) / TK;
  // consume the first tile's map words before the loop (see the dK/dV body of the backward:
  // a load pending at the loop entry makes every tile's blocks wait for the next prefetch)
#pragma unroll
  for (int kb = 0; kb < C::KB; ++kb) asm volatile("" ::"v"(mw[kb]));
  for (int kt = 0; kt <= last_kt; ++kt) {
    const int k0 = kt * TK;
    const bool more = kt < last_kt;
    if (more) load_tile(kt + 1, mwn);
    // key blocks in pairs: the two S = K Q^T chains interleave (one 13-deep chain of
    // dependent MFMAs alone is latency-bound); each block's arithmetic is unchanged
#pragma unroll
    for (int kb = 0; kb < C::KB; kb += 2) {
      const int kb0 = k0 + kb * 16;
      if (kb0 > wq_lo + 15 || kb0 >= L) break;  // wave-uniform causal / length skip
      const bool two = kb + 1 < C::KB && kb0 + 16 <= wq_lo + 15 && kb0 + 16 < L;
      f4 s0 = f4_zero(), s1 = f4_zero();
      const float* krow = Ks + (kb * 16 + lr) * C::LDK + lg;
      if (two) {
#pragma unroll
        for (int st = 0; st < KSTEPS; ++st) {
          s0 = mfma16x16x4(krow[4 * st], qreg[st], s0);
          s1 = mfma16x16x4(krow[16 * C::LDK + 4 * st], qreg[st], s1);
        }
      } else {
#pragma unroll
        for (int st = 0; st < KSTEPS; ++st) s0 = mfma16x16x4(krow[4 * st], qreg[st], s0);
      }
      // s[r] = S^T[key kb0 + 16 j + 4lg + r][query qi]
      float p[2][4];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = kb0 + 16 * j + 4 * lg + r;
          float val = j ? s1[r] : s0[r];
          if (has_bias) {
            const int bucket = (mw[kb + (j && kb + 1 < C::KB ? 1 : 0)] >> (8 * r)) & 0xFF;
            int pi = a.N - 1 + kj - qi;
            pi = pi < 0 ? 0 : (pi > 2 * a.N - 2 ? 2 * a.N - 2 : pi);
            val = val + (posw[pi] + tsw[bucket]);
          }
          p[j][r] = (q_ok && kj <= qi) ? siluf_(val) * a.inv_n : 0.f;
        }
      const float* vrow = Vs + (kb * 16 + 4 * lg) * C::LDV + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int ct = 0; ct < VTILES; ++ct)
          acc[ct] = mfma16x16x4(p[0][r], vrow[r * C::LDV + ct * 16], acc[ct]);
      }
      if (two) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int ct = 0; ct < VTILES; ++ct)
            acc[ct] = mfma16x16x4(p[1][r], vrow[(16 + r) * C::LDV + ct * 16], acc[ct]);
        }
      }
    }
    if (more) {
      lds_barrier();
      kst.store(Ks, C::LDK, v2);
      vst.store(Vs, C::LDV, v2);
#pragma unroll
      for (int kb = 0; kb < C::KB; ++kb) mw[kb] = mwn[kb];
      lds_barrier();
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
  return true;
}

template <int KSTEPS, int VTILES, int TK, bool HB>
__global__ __launch_bounds__(256) void hstu_attn_fwd_kernel(AttnFwdArgs a) {
  if (a.vec2) hstu_attn_fwd_body<KSTEPS, VTILES, TK, HB, true>(a);
  else hstu_attn_fwd_body<KSTEPS, VTILES, TK, HB, false>(a);
}

// Attention forward with the layer boundary as its epilogue (hstu_attn_fwd_bnd, H == 1):
// once a workgroup's 64 query rows of attention output are stored, the K / V tile area is
// re-staged with the boundary's weight panels (gate_o's W_o, the next layer's W_uvqk) and
// each wave runs the row-wave boundary unit of its 16 rows -- y = x + gate(u, LN(attn))
// W_o^T + b, then LN(y) W_uvqk of the next layer -- or, OP2 = false (the last layer),
// gate_o alone.  Rows past the sequence fall outside the ops' descriptors.
template <int KSTEPS, int VTILES, bool HB, int NT2, bool OP2>
__global__ __launch_bounds__(256) void hstu_attn_fwd_bnd_kernel(AttnFwdArgs a, RwGateO<4, 4, 2> op1,
                                                                RwLnUvqk<4, NT2, 2> op2) {
  // the weight panels' loads are issued first and land while the attention runs; they
  // reach LDS once the K / V tiles they overwrite are done with
  RwStage<4, 4, RwGateO<4, 4, 2>> st1;
  RwStage<4, NT2, RwLnUvqk<4, NT2, 2>> st2;
  st1.load(op1);
  if constexpr (OP2) st2.load(op2);
  int q0 = 0, L = 0;
  int64_t s0 = 0;
  const bool live = a.vec2 ? hstu_attn_fwd_body<KSTEPS, VTILES, 64, HB, true>(a, &q0, &L, &s0)
                           : hstu_attn_fwd_body<KSTEPS, VTILES, 64, HB, false>(a, &q0, &L, &s0);
  if (!live) return;  // uniform over the workgroup
  using C1 = RowWaveCfg<4, 4>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* W1 = reinterpret_cast<float*>(smem);
  float* W2 = W1 + C1::KP * C1::LDW;
  __syncthreads();  // every wave is done with the K / V tiles the panels overwrite
  st1.store(W1);
  if constexpr (OP2) st2.store(W2);
  __syncthreads();
  // this wave's attention rows have landed before its unit reads them back
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int w = wave_id(), lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  op1.setup(s0 + L);
  op1.rd_aux = 16;  // attn rows: L2, not an L1 line a neighbouring wave filled before our store
  if constexpr (OP2) op2.setup(s0 + L);
  const int r = q0 + 16 * w + lr;
  if (q0 + 16 * w >= L) return;  // wave-uniform: no rows of this wave
  if constexpr (OP2) rw2_unit<4, 4, NT2>(op1, op2, W1, W2, s0 + r, r < L, lr, lg);
  else rw1_unit<4, 4>(op1, W1, s0 + r, r < L, lr, lg);
}

struct BndFwdCtx {
  RwArgsGateO a1;
  RwArgsLnUvqk a2;
  bool op2;
  int nt2;     // 13 | 16
  bool fused;
};

template <int KS, int VT, bool HB, int NT2, bool OP2>
static int launch_fwd_bnd_k(const AttnFwdArgs& a, int grid, BndFwdCtx& bc, hipStream_t st) {
  using C = AttnFwdCfg<KS, VT, 64>;
  RwGateO<4, 4, 2> o1{};
  RwLnUvqk<4, NT2, 2> o2{};
  bc.a1.fill(o1);
  if (OP2) bc.a2.fill(o2);
  const size_t lds_attn = sizeof(float) * (C::LDS_FLOATS + a.nb + 1 + 2 * a.N - 1);
  const size_t lds_w = RowWaveCfg<4, 4>::LDS_BYTES + (OP2 ? RowWaveCfg<4, NT2>::LDS_BYTES : 0);
  const size_t lds = lds_attn > lds_w ? lds_attn : lds_w;
  GR_REQUIRE(lds <= 160 * 1024, "hstu_attn_fwd_bnd: LDS %zu B exceeds 160 KiB (N=%d)", lds, a.N);
  GR_TIMED(OP2 ? "attn_fwd_bnd" : "attn_fwd_bnd1", st, hipLaunchKernelGGL((hstu_attn_fwd_bnd_kernel<KS, VT, HB, NT2, OP2>), dim3(grid),
                                              dim3(256), lds, st, a, o1, o2));
  GR_LAUNCH_CHECK("hstu_attn_fwd_bnd");
  bc.fused = true;
  return 0;
}
template <int KS, int VT, bool HB>
static int launch_fwd_bnd_h(const AttnFwdArgs& a, int grid, BndFwdCtx& bc, hipStream_t st) {
  if (!bc.op2) return launch_fwd_bnd_k<KS, VT, HB, 13, false>(a, grid, bc, st);
  return bc.nt2 == 13 ? launch_fwd_bnd_k<KS, VT, HB, 13, true>(a, grid, bc, st)
                      : launch_fwd_bnd_k<KS, VT, HB, 16, true>(a, grid, bc, st);
}

template <int KS, int VT, int TK = 64>
static int launch_fwd(const AttnFwdArgs& a, int grid, hipStream_t st, BndFwdCtx* bnd = nullptr) {
  if constexpr (TK == 64 && VT == 4 && (KS == 13 || KS == 16)) {
    if (bnd && a.H == 1)
      return a.map_qk ? launch_fwd_bnd_h<KS, VT, true>(a, grid, *bnd, st)
                      : launch_fwd_bnd_h<KS, VT, false>(a, grid, *bnd, st);
  }
  using C = AttnFwdCfg<KS, VT, TK>;
  size_t lds = sizeof(float) * (C::LDS_FLOATS + a.nb + 1 + 2 * a.N - 1);
  GR_REQUIRE(lds <= 160 * 1024, "hstu_attn_fwd: LDS %zu B exceeds 160 KiB (N=%d)", lds, a.N);
  if (a.map_qk) {
    GR_TIMED("attn_fwd", st, hipLaunchKernelGGL((hstu_attn_fwd_kernel<KS, VT, TK, true>), dim3(grid), dim3(256), lds, st, a));
  } else {
    GR_TIMED("attn_fwd", st, hipLaunchKernelGGL((hstu_attn_fwd_kernel<KS, VT, TK, false>), dim3(grid), dim3(256), lds, st, a));
  }
  GR_LAUNCH_CHECK("hstu_attn_fwd");
  return 0;
}

}  // namespace gr

namespace gr {
static int attn_fwd_impl(const float* q, const float* k, const float* v, int64_t ld_qk,
                         int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                         int H, int dqk, int dv, const uint8_t* bucket_map,
                         const float* pos_w, const float* ts_w, int num_buckets, float* out,
                         int64_t ld_out, void* stream, BndFwdCtx* bnd) {
  GR_REQUIRE(q && k && v && offsets && out, "hstu_attn_fwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_fwd: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_fwd: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 256 && dv <= 256, "hstu_attn_fwd: dqk/dv > 256 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE(!bucket_map || (pos_w && ts_w && num_buckets > 0 && num_buckets < 256),
             "hstu_attn_fwd: bucket_map given without pos_w/ts_w");
  if (B == 0 || max_len == 0) return 0;
  AttnFwdArgs a{q, k, v, ld_qk, ld_v, offsets, B, N, H, dqk, dv, ceil_div(max_len, 64),
                bucket_map, pos_w, ts_w, bucket_map ? num_buckets : 0, out, ld_out,
                1.0f / (float)N, 0};
  // snake pairing only when the grid is resident in <= 2 rounds; otherwise plain
  // heaviest-first (dynamic dispatch = longest-processing-time order)
  a.cus = (int64_t)a.n_qtiles * B * H <= 2 * device_cus() ? device_cus() : (1 << 30);
  a.vec2 = pair_aligned({q, k, v}, {ld_qk, ld_v, dqk, dv});
  const int grid = a.n_qtiles * B * H;
  hipStream_t st = (hipStream_t)stream;
  const int d = dqk > dv ? dqk : dv;
  if (d <= 8) return launch_fwd<2, 1>(a, grid, st, bnd);
  if (d <= 16) return launch_fwd<4, 1>(a, grid, st, bnd);
  if (d <= 32) return launch_fwd<8, 2>(a, grid, st, bnd);
  if (d <= 52) return launch_fwd<13, 4>(a, grid, st, bnd);
  if (d <= 64) return launch_fwd<16, 4>(a, grid, st, bnd);
  if (d <= 128) return launch_fwd<32, 8>(a, grid, st, bnd);
  return launch_fwd<64, 16, 16>(a, grid, st, bnd);
}
}  // namespace gr

extern "C" int hstu_attn_fwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                             int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                             int H, int dqk, int dv, const uint8_t* bucket_map,
                             const float* pos_w, const float* ts_w, int num_buckets, float* out,
                             int64_t ld_out, void* stream) {
  return gr::attn_fwd_impl(q, k, v, ld_qk, ld_v, offsets, B, N, max_len, H, dqk, dv, bucket_map,
                           pos_w, ts_w, num_buckets, out, ld_out, stream, nullptr);
}

extern "C" int hstu_attn_fwd_bnd(const float* q, const float* k, const float* v, int64_t ld_qk,
                                 int64_t ld_v, const int64_t* offsets, int B, int N, int max_len,
                                 int H, int dqk, int dv, const uint8_t* bucket_map,
                                 const float* pos_w, const float* ts_w, int num_buckets, float* out,
                                 int64_t ld_out, const GrBoundaryFwd* bnd, void* stream) {
  using namespace gr;
  GR_REQUIRE(bnd, "hstu_attn_fwd_bnd: null boundary");
  const GrBoundaryFwd& g = *bnd;
  GR_REQUIRE(g.u && g.w_o && g.y && g.attn_stats && g.hdv > 0 && g.D > 0,
             "hstu_attn_fwd_bnd: boundary null pointer or bad sizes");
  GR_REQUIRE(!g.w_uvqk || (g.uvqk && g.x_stats && g.n_out > 0),
             "hstu_attn_fwd_bnd: next-layer LN / UVQK null pointer");
  BndFwdCtx bc{};
  bc.a1 = RwArgsGateO{offsets, B, g.hdv, g.D, g.u, g.ld_u, out, ld_out, g.w_o, g.b_o, g.x_res,
                      g.ld_x, g.eps, g.dropout_p, g.seed, g.seed_offset, (float2*)g.attn_stats,
                      g.o_in, g.y, g.ld_y};
  bc.op2 = g.w_uvqk != nullptr;
  if (bc.op2)
    bc.a2 = RwArgsLnUvqk{offsets, B, g.D, g.n_out, g.y, g.ld_y, g.w_uvqk, g.eps, g.activation,
                         (float2*)g.x_stats, g.h_pre, g.uvqk, g.ld_out};
  const int ng = bc.op2 ? ceil_div(g.n_out, 16) : 13;
  bc.nt2 = ng > 8 && ng <= 13 ? 13 : ng > 13 && ng <= 16 ? 16 : -1;
  auto in_w4 = [](int x) { return x > 32 && x <= 64; };  // the W = 4 (64-column) instantiation
  const bool aligned = pair_aligned({g.u, out, g.x_res, g.o_in, g.y, g.h_pre, g.uvqk},
                                    {g.ld_u, ld_out, g.ld_x, g.ld_y, g.ld_out, g.hdv, g.D,
                                     bc.op2 ? g.n_out : 2});
  const bool fuse = option(GR_OPT_BOUNDARY_FUSE) != 0 && option(GR_OPT_ROWWAVE) != 0 && H == 1 &&
                    bc.nt2 > 0 && in_w4(g.D) && in_w4(g.hdv) && g.hdv == H * dv && aligned &&
                    g.max_rows * 4 * 1024 <= 0x7fffffffLL;
  if (int rc = attn_fwd_impl(q, k, v, ld_qk, ld_v, offsets, B, N, max_len, H, dqk, dv, bucket_map,
                             pos_w, ts_w, num_buckets, out, ld_out, stream, fuse ? &bc : nullptr))
    return rc;
  if (bc.fused) return 0;
  if (bc.op2)
    return hstu_boundary_fwd(g.u, g.ld_u, out, ld_out, offsets, B, g.max_rows, g.hdv, g.D, g.w_o,
                             g.b_o, g.x_res, g.ld_x, g.eps, g.dropout_p, g.seed, g.seed_offset,
                             g.attn_stats, g.o_in, g.y, g.ld_y, g.w_uvqk, g.n_out, g.activation,
                             g.x_stats, g.h_pre, g.uvqk, g.ld_out, stream);
  return hstu_gate_o_fwd(g.u, g.ld_u, out, ld_out, offsets, B, g.max_rows, g.hdv, g.D, g.w_o, g.b_o,
                         g.x_res, g.ld_x, g.eps, g.dropout_p, g.seed, g.seed_offset, g.attn_stats,
                         g.o_in, g.y, g.ld_y, stream);
}
