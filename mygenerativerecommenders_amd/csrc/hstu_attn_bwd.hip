// Jagged causal HSTU attention, backward — gfx950, f32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Replaces the autograd backward of reference sequential_encoders/hstu.py:134-205 and
// of the bias module hstu.py:96-128 (bmm-backward x4, silu_backward, the index_add_
// of 5.7 M updates into the 129-bin _ts_w and the slice/pad backward into _pos_w).
// HSTU attention has no softmax, so there is no LSE/delta: with
//   S = Q K^T + bias,  P = silu(S) / N (causal),  O = P V
// the gradients are  dP = dO V^T,  dS = dP * silu'(S) / N,
//   dV = P^T dO,  dK = dS^T Q,  dQ = dS K,  dbias[i, j] = sum_h dS[h, i, j].
// Two atomic-free (global), deterministic kernels recompute S:
//   * key-major  (dK, dV, bias grads): a workgroup owns 64 keys and walks the query
//     tiles at or after it; per-wave LDS histograms for dpos_w (2N-1 bins) and dts_w
//     (129 bins) are summed in a fixed order into one slab per workgroup, and a third
//     kernel reduces the slabs in a fixed order;
//   * query-major (dQ): a workgroup owns 64 queries and walks key tiles 0..qt.
// Tiles are register-prefetched one step ahead (LDS-only barriers), buckets come from
// the per-batch map of hstu_bucket_map.  Optional fused epilogue: the gradients are
// multiplied by silu'(h) of the UVQK pre-activation (hstu.py:303-305), so the caller
// gets d(pre-activation) directly.
#include "attn_common.h"
#include "rowwave.h"

#include "../../include/gr_hstu.h"

namespace gr {

#ifdef GR_STAMP
// Diagnostic build only (-DGR_STAMP): per-wave phase cycle sums of the dK/dV kernel.
__device__ unsigned long long gr_stamp_buf[1 << 16];
__device__ __forceinline__ unsigned long long gr_stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define GR_ST(acc, dep)                                \
  do {                                                 \
    asm volatile("" ::"v"(dep));                       \
    const unsigned long long t1_ = gr_stamp();         \
    acc += t1_ - st_t0;                                \
    st_t0 = t1_;                                       \
  } while (0)
#else
#define GR_ST(acc, dep) do { } while (0)
#endif

#ifdef GR_STAMP
// Workgroup timeline (diagnostic build): [wg][entry, exit, HW_ID | XCC_ID << 32, kind]
__device__ unsigned long long gr_tl_buf[1 << 15];
#define GR_TL_BEGIN() const unsigned long long tl0_ = __builtin_amdgcn_s_memrealtime()
#define GR_TL_END(slot, kind)                                                              \
  do {                                                                                   \
    if (threadIdx.x == 0 && (slot) * 4 + 4 <= (1 << 15)) {                               \
      const unsigned long long hw_ = __builtin_amdgcn_s_getreg((31 << 11) | 4);          \
      const unsigned long long xcc_ = __builtin_amdgcn_s_getreg((15 << 11) | 20);        \
      gr_tl_buf[(slot) * 4 + 0] = tl0_;                                                  \
      gr_tl_buf[(slot) * 4 + 1] = __builtin_amdgcn_s_memrealtime();                      \
      gr_tl_buf[(slot) * 4 + 2] = hw_ | (xcc_ << 32);                                    \
      gr_tl_buf[(slot) * 4 + 3] = (kind);                                                \
    }                                                                                    \
  } while (0)
#else
#define GR_TL_BEGIN() do { } while (0)
#define GR_TL_END(slot, kind) do { } while (0)
#endif

struct AttnBwdArgs {
  const float* q;
  const float* k;
  const float* v;
  int64_t ld_qk, ld_v;
  const float* dout;
  int64_t ld_dout;
  const int64_t* offsets;
  int B, N, H, dqk, dv, n_tiles;
  const uint8_t* map_qk;
  const uint8_t* map_kq;
  const float* pos_w;
  const float* ts_w;
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
  int vec2;   // 8-byte pair staging (aligned rows, even widths)
  int cus;    // CU count (snake_rank)
  int vec2h;  // the same for the hq / hk / hv rows
  int paired; // workgroups run tile pairs (p, T-1-p); grid = B*H*ceil(T/2) per kind
  float* ds;  // non-null: the dK/dV pass stores dS as 16 x 16 tiles for the dQ pass
  int ds_tps; // dS tiles per (sequence, head): NB (NB + 1) / 2, NB = ceil(N / 16)
  uint32_t* ds_flags;  // one-launch form: [bh][key tile] = 1 once that tile's dS is published
};

// TT = rows per streamed LDS tile (queries in dK/dV, keys in dQ): 64, or 16 for the
// wide head dims (d > 128) where a 64-row register stage would not fit.
template <int KSTEPS, int VTILES, int TT>
struct AttnBwdCfg {
  static constexpr int TB = TT / 16;             // 16-row blocks per tile
  static constexpr int KP = KSTEPS * 4;          // padded dqk (k-steps of the QK product)
  static constexpr int KT = (KP + 15) / 16;      // 16-col tiles of dK / dQ
  static constexpr int KPT = KT * 16;            // dqk padded to the output tile width
  static constexpr int VP = VTILES * 16;         // padded dv
  // row strides: == 4 mod 8 keeps the 4-row-apart B reads conflict-free; the 16-row
  // A reads are then 2-way (LDS is not the limiter at 32-cycle MFMAs).
  static constexpr int LDQ = KPT + 4;
  static constexpr int LDV = VP + 4;
};


// ------------------------------------------------------------------ key-major: dK, dV
// Per 16 x 16 (query, key) block a wave computes S and dP (A = Q / dO rows from LDS,
// B = its keys' K^T / V^T fragments in VGPRs), the elementwise P / dS in registers
// (branch-free; wave-uniform block skips are scalar branches), the relative-bias
// gradients as LDS float adds into the wave's private histograms (dpos: one add per
// element, <= 4-way address conflicts; dts: equal consecutive buckets of a lane merged
// first), then dV += P^T dO and dK += dS^T Q (k-step r = queries 4g + r).
#ifndef GR_DTS_COPIES
#define GR_DTS_COPIES 4
#endif
// dts_w histogram: GR_DTS_COPIES copies per wave (lane lr uses copy lr % copies) so
// lanes flushing the same bucket together mostly hit different addresses; stride == 1
// mod 32.
__host__ __device__ constexpr int dts_stride(int nb1) { return ((nb1 + 30) / 32) * 32 + 1; }

// KIND: 0 = dK, dV and the bias gradients in one pass; 1 = dV only (S, P, dV += P^T dO);
// 2 = dK only (S, dP, dS, dK += dS^T Q, the bias gradients, the stored dS).  The wide
// heads (d > 128) run kinds 1 and 2 as separate workgroups: one pass holding the K and V
// fragments, both accumulators and the block's operands needed ~460 registers (one wave
// per SIMD and ~370 AGPR copies per block); a kind holds about half (two waves per SIMD)
// for 25 % more MFMA work (S is formed by both kinds).
template <int KSTEPS, int VTILES, int TT, bool HB, bool V2, int KIND = 0>
__device__ __forceinline__ void attn_bwd_dkv_body(const AttnBwdArgs& a, const int id) {
  // V2: 8-byte pair staging known at compile time (see BWD_V2 below)
  const bool v2 = V2 || a.vec2, v2h = V2 || a.vec2h;
  constexpr bool DO_V = KIND != 2, DO_K = KIND != 1;
  // A-operand (Q / dO rows) reads of a block: all before the first MFMA, or for the wide
  // heads a window of PW k-steps read ahead of the MFMAs (64 + 64 operands in registers
  // at d = 256 otherwise)
  constexpr int PW = KSTEPS > 16 ? 8 : KSTEPS;
  using C = AttnBwdCfg<KSTEPS, VTILES, TT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Qs = reinterpret_cast<float*>(smem);  // [TT][LDQ]
  float* Ds = Qs + TT * C::LDQ;                // dO tile [TT][LDV]
  float* tsw = Ds + TT * C::LDV;               // nb + 1
  float* posw = tsw + (a.nb + 1);              // 2N - 1
  const int npos = 2 * a.N - 1;
  const int nbins = npos + a.nb + 1;
  const int tss = dts_stride(a.nb + 1);
  const int wbins = npos + GR_DTS_COPIES * tss;  // per wave: dpos bins, dts copies
  float* hist = posw + npos;                   // [4 waves][wbins]

#ifdef GR_STAMP
  const unsigned long long st_entry = gr_stamp();
#endif
  const int BH = a.B * a.H;
  // paired: workgroup (p, bh) runs key tiles p and T-1-p of one sequence (the causal work
  // of the pair is T+1 tiles for every p, so a one-round grid is balanced); otherwise one
  // tile per workgroup, heaviest first
  int kt_a, kt_b = -1, bh;
  if (a.paired) {
    kt_a = id / BH;
    bh = id % BH;
    kt_b = a.n_tiles - 1 - kt_a;
    if (kt_b == kt_a) kt_b = -1;
  } else {
    const int rank = snake_rank(id, a.cus);
    kt_a = rank / BH;  // kt = 0 (the most query tiles) first
    bh = rank % BH;
  }
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  constexpr bool has_bias = HB && DO_K;  // compile-time: the 4 bias gathers of a lane issue together
  constexpr bool bias_in_s = HB;          // S includes the bias in both kinds
  float* slab = a.slabs && DO_K ? a.slabs + (int64_t)id * nbins : nullptr;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;

  if (kt_a * 64 >= L) {  // this workgroup still owns a (zero) slab (kt_b > kt_a: also past L)
    if (has_bias && slab)
      for (int i = tid; i < nbins; i += 256) slab[i] = 0.f;
    return;
  }
  if (bias_in_s) {
    for (int i = tid; i <= a.nb; i += 256) tsw[i] = a.ts_w[i];
    for (int i = tid; i < npos; i += 256) posw[i] = a.pos_w[i];
  }
  if (has_bias)
    for (int i = tid; i < 4 * wbins; i += 256) hist[i] = 0.f;
  float* whist = hist + w * wbins;
  float* wts = whist + npos + (lr % GR_DTS_COPIES) * tss;
  float carry = 0.f;   // dpos: diagonal partial sums handed to the next block
  int last_db = 0;
  // dts: a lane walks its key's queries in order, and the relative-time bucket of
  // (query, key) is non-decreasing along that walk for time-ordered sequences, so the
  // lane keeps a running (bucket, sum) and adds to the histogram only when the bucket
  // changes (any order stays correct: every change flushes)
  int run_b = -1;
  float run_s = 0.f;
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_kq, b, attn_tiles_per_seq(a.N));
  const int map_voff = ((w * 16 + lr) * 16 + lg) * 4;
  const __amdgpu_buffer_rsrc_t rq = seq_rsrc(a.q, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rdo = seq_rsrc(a.dout, a.ld_dout, s0, h * a.dv, L, a.dv);
  const int last_qt = (L - 1) / TT;

  // tile pairs only with LDS-staged fragments (TT = 64); the wide-head instances keep one
  // tile per workgroup (a runtime pass loop there spilled ~1.6 KB/lane at d = 256)
  for (int pass = 0; pass < (TT == 64 ? 2 : 1); ++pass) {
  const int kt = pass == 0 ? kt_a : kt_b;
  const int k0 = kt * 64;
  if (pass == 1) {
    if (kt < 0 || k0 >= L) break;
    lds_barrier();  // the first pass's epilogue reads of Qs / Ds
  }
  // this lane's key (as the column of S and dP) and its K^T / V^T fragments
  const int kj = k0 + w * 16 + lr;
  const bool k_ok = kj < L;
  // TT = 64: the workgroup's 64 key rows are staged through LDS as coalesced tiles
  // (below); scattered per-lane row loads cost ~12K cycles of address processing when
  // every workgroup of the launch starts together
  constexpr bool STAGED = TT == 64;
  float kreg[KSTEPS], vreg[KSTEPS];
  if constexpr (!STAGED) {
    const int64_t row = s0 + (k_ok ? kj : L - 1);
    gptr<float> krow = as_global(a.k) + row * a.ld_qk + h * a.dqk;
    gptr<float> vrow = as_global(a.v) + row * a.ld_v + h * a.dv;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      const float x = krow[d < a.dqk ? d : a.dqk - 1];
      kreg[st] = d < a.dqk ? x : 0.f;
      if (DO_K) {
        const float y = vrow[d < a.dv ? d : a.dv - 1];
        vreg[st] = d < a.dv ? y : 0.f;
      }
    }
  }
  f4 dV[VTILES], dK[C::KT];
#pragma unroll
  for (int t = 0; t < VTILES; ++t) dV[t] = f4_zero();
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dK[t] = f4_zero();

  BufTile<C::KPT, TT> qst;
  BufTile<C::VP, TT> dst;
  uint32_t mw[C::TB], mwn[C::TB];
  auto load_tile = [&](int qt, uint32_t (&m)[C::TB]) {
    qst.load(rq, a.ld_qk, qt * TT, a.dqk, v2);
    dst.load(rdo, a.ld_dout, qt * TT, a.dv, v2);
#pragma unroll
    for (int qb = 0; qb < C::TB; ++qb)
      m[qb] = buf_ld_u32(rmap, map_voff, map_soff(qt * TT + qb * 16, k0, false));
  };

  const int wk_lo = k0 + w * 16;
  // the epilogue's silu'(h) inputs.  STAGED: coalesced tiles loaded into the stage
  // registers during the last query tile (a load at the end put one more HBM round trip
  // on every workgroup's tail: +16 us per launch at C2).  Wide heads: read in the
  // epilogue (128 prefetched values per lane spilled; their workgroups run for ms)
  if constexpr (STAGED) {
    // K / V rows k0 .. k0 + 63 (rows past L and columns past dqk / dv read as 0) in their
    // own staging registers, issued together with the first query tile's loads: one HBM
    // round trip for the prologue instead of two (the K / V stores wait only for their
    // own loads, which were issued first)
    BufTile<C::KPT, TT> kst0;
    BufTile<C::VP, TT> vst0;
    kst0.load(seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk), a.ld_qk, k0, a.dqk, v2);
    vst0.load(seq_rsrc(a.v, a.ld_v, s0, h * a.dv, L, a.dv), a.ld_v, k0, a.dv, v2);
    load_tile(k0 / TT, mw);
    kst0.store(Qs, C::LDQ, v2);
    vst0.store(Ds, C::LDV, v2);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      kreg[st] = Qs[(w * 16 + lr) * C::LDQ + 4 * st + lg];
      vreg[st] = Ds[(w * 16 + lr) * C::LDV + 4 * st + lg];
    }
    lds_barrier();
  } else {
    load_tile(k0 / TT, mw);
  }
  qst.store(Qs, C::LDQ, v2);
  dst.store(Ds, C::LDV, v2);
  __syncthreads();
#ifdef GR_STAMP
  unsigned long long st_t0 = gr_stamp(), st_ld = 0, st_mm1 = 0, st_ew = 0, st_bias = 0,
                     st_mm2 = 0, st_sync = 0;
  const unsigned long long st_begin = st_t0;
#endif
  // The first tile's map words were loaded just before the loop: consume them here.  A
  // load still pending at the loop entry is merged into the loop-header state by the
  // waitcnt pass, which then makes block qb of EVERY tile wait for all but the last
  // (3 - qb) loads issued so far -- the whole next-tile prefetch.
#pragma unroll
  for (int qb = 0; qb < C::TB; ++qb) asm volatile("" ::"v"(mw[qb]));
  for (int qt = k0 / TT; qt <= last_qt; ++qt) {
    const int q0 = qt * TT;
    const bool more = qt < last_qt;
    if (more) {
      load_tile(qt + 1, mwn);
    } else if (STAGED && a.hv) {  // the epilogue's silu'(h) rows of this workgroup's keys
      qst.load(seq_rsrc(a.hk, a.ld_h, s0, h * a.dqk, L, a.dqk), a.ld_h, k0, a.dqk, v2h);
      dst.load(seq_rsrc(a.hv, a.ld_h, s0, h * a.dv, L, a.dv), a.ld_h, k0, a.dv, v2h);
    }
    GR_ST(st_ld, 0);
#pragma unroll
    for (int qb = 0; qb < C::TB; ++qb) {
      const int qb0 = q0 + qb * 16;
      if (qb0 < L && qb0 + 15 >= wk_lo) {  // wave-uniform: inside the sequence, causal
        // S[query 4lg + r][key lr] and dP alike
        f4 s = f4_zero(), dp = f4_zero();
        const float* qrow = Qs + (qb * 16 + lr) * C::LDQ + lg;
        const float* drow = Ds + (qb * 16 + lr) * C::LDV + lg;
        // the block's LDS operands are requested before the first MFMA (the chain then
        // waits on in-order completions instead of one round trip per k-step), PW
        // k-steps ahead; the bias terms are gathered in the same burst
        float qa[PW], da[PW], bias[4];
        int bk[4];
#pragma unroll
        for (int st = 0; st < PW; ++st) {
          qa[st] = qrow[4 * st];
          if (DO_K) da[st] = drow[4 * st];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = qb0 + 4 * lg + r;
          int pi = a.N - 1 + kj - qi;
          pi = pi < 0 ? 0 : (pi > npos - 1 ? npos - 1 : pi);
          bk[r] = (mw[qb] >> (8 * r)) & 0xFF;
          bias[r] = bias_in_s ? posw[pi] + tsw[bk[r]] : 0.f;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int st = 0; st < KSTEPS; ++st) {
          const float q0v = qa[st % PW];
          const float d0v = DO_K ? da[st % PW] : 0.f;
          if (PW < KSTEPS && st + PW < KSTEPS) {
            qa[st % PW] = qrow[4 * (st + PW)];
            if (DO_K) da[st % PW] = drow[4 * (st + PW)];
          }
          s = mfma16x16x4(q0v, kreg[st], s);
          if (DO_K) dp = mfma16x16x4(d0v, vreg[st], dp);
        }
        GR_ST(st_mm1, s[0] + dp[0]);
        float p[4], ds[4];
        bool okr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = qb0 + 4 * lg + r;
          const bool ok = k_ok && qi < L && kj <= qi;
          okr[r] = ok;
          float x = s[r];
          if (bias_in_s) x = x + bias[r];
          const float sg = sigmoidf_(x);
          p[r] = DO_V && ok ? x * sg * a.inv_n : 0.f;
          ds[r] = DO_K && ok ? dp[r] * (sg * (1.0f + x * (1.0f - sg))) * a.inv_n : 0.f;
#ifdef GR_STAMP
          if (r == 3) GR_ST(st_ew, ds[0] + ds[1] + ds[2] + ds[3] + p[0] + p[1] + p[2] + p[3]);
#endif
        }
        if (DO_K && a.ds) {  // dS tile (query block, key block), row-major [query][key]
          const int qbi = qb0 >> 4, kbi = wk_lo >> 4;
          float* dt = a.ds + ((int64_t)bh * a.ds_tps + qbi * (qbi + 1) / 2 + kbi) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) dt[(4 * lg + r) * 16 + lr] = ds[r];
        }
        // Relative-bias gradients.  dpos_w: element (query 4lg + r, key lr) has diagonal
        // e = lr - (4lg + r); rotating row 4lg + r left by its index inside the 16-lane
        // group puts the diagonals e = lr (main) and e = lr - 16 (wrapped) in lane lr;
        // they are summed over r and the 4 lane groups, and the main part plus the
        // previous block's wrapped part (same bins: the next block sits 16 queries
        // later) is added to the wave's histogram.  dts_w: equal consecutive buckets of
        // a lane are merged, then added.  The histograms are private to the wave, so the
        // LDS adds land in program order (deterministic).
        const int db = wk_lo - qb0;
        float rot[4], dA = 0.f, dB = 0.f;
        auto bias_stage = [&](int stage) {
          if (!has_bias) return;
          if (stage == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              rot[r] = __shfl(ds[r], (lg << 4) | ((lr + 4 * lg + r) & 15), 64);
          } else if (stage == 1) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const bool main = lr + 4 * lg + r < 16;
              dA += main ? rot[r] : 0.f;
              dB += main ? 0.f : rot[r];
            }
            // sums over the lane groups: rows xor 1 (permlane16 swap), halves (permlane32)
            auto ta = __builtin_amdgcn_permlane16_swap(__float_as_uint(dA), __float_as_uint(dA), false, false);
            auto tb = __builtin_amdgcn_permlane16_swap(__float_as_uint(dB), __float_as_uint(dB), false, false);
            dA = __uint_as_float(ta[0]) + __uint_as_float(ta[1]);
            dB = __uint_as_float(tb[0]) + __uint_as_float(tb[1]);
            auto ua = __builtin_amdgcn_permlane32_swap(__float_as_uint(dA), __float_as_uint(dA), false, false);
            auto ub = __builtin_amdgcn_permlane32_swap(__float_as_uint(dB), __float_as_uint(dB), false, false);
            dA = __uint_as_float(ua[0]) + __uint_as_float(ua[1]);
            dB = __uint_as_float(ub[0]) + __uint_as_float(ub[1]);
          } else if (stage == 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (okr[r] && bk[r] != run_b) {  // rare: the bucket changed
                if (run_b >= 0) atomicAdd(&wts[run_b], run_s);
                run_b = bk[r];
                run_s = 0.f;
              }
              run_s += ds[r];
            }
          } else {
            int bin = a.N - 1 + db + lr;
            bin = bin > npos - 1 ? npos - 1 : bin;
            if (lg == 0) atomicAdd(&whist[bin], dA + carry);
            carry = dB;
            last_db = db;
          }
        };
        // dV[key][c] += P^T dO ; dK[key][d] += dS^T Q   (k-step r: queries 4g + r)
        const float* dcol = Ds + (qb * 16 + 4 * lg) * C::LDV + lr;
        const float* qcol = Qs + (qb * 16 + 4 * lg) * C::LDQ + lr;
        if constexpr (VTILES + C::KT > 8) {  // wide heads: no registers to spare
#pragma unroll
          for (int stage = 0; stage < 4; ++stage) bias_stage(stage);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (DO_V) {
#pragma unroll
              for (int t = 0; t < VTILES; ++t)
                dV[t] = mfma16x16x4(p[r], dcol[r * C::LDV + t * 16], dV[t]);
            }
            if (DO_K) {
#pragma unroll
              for (int t = 0; t < C::KT; ++t)
                dK[t] = mfma16x16x4(ds[r], qcol[r * C::LDQ + t * 16], dK[t]);
            }
          }
        } else {
        // B operands of k-step r+1 are read from LDS while the MFMAs of step r run, and
        // bias stage r (shuffles / LDS adds: latency, little issue) is issued between
        // the MFMA groups so it runs under them
        float bvv[2][VTILES], bvk[2][C::KT];
#pragma unroll
        for (int t = 0; t < VTILES; ++t) bvv[0][t] = dcol[t * 16];
#pragma unroll
        for (int t = 0; t < C::KT; ++t) bvk[0][t] = qcol[t * 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r + 1 < 4) {
#pragma unroll
            for (int t = 0; t < VTILES; ++t) bvv[(r + 1) & 1][t] = dcol[(r + 1) * C::LDV + t * 16];
#pragma unroll
            for (int t = 0; t < C::KT; ++t) bvk[(r + 1) & 1][t] = qcol[(r + 1) * C::LDQ + t * 16];
          }
          bias_stage(r);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int t = 0; t < VTILES; ++t) dV[t] = mfma16x16x4(p[r], bvv[r & 1][t], dV[t]);
#pragma unroll
          for (int t = 0; t < C::KT; ++t) dK[t] = mfma16x16x4(ds[r], bvk[r & 1][t], dK[t]);
          __builtin_amdgcn_sched_barrier(0);
        }
        }
        GR_ST(st_mm2, dV[0][0] + dK[0][0] + dV[VTILES - 1][3] + dK[C::KT - 1][3]);
#ifdef GR_STAMP
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GR_ST(st_bias, 0);
#endif
      }
    }
    if (more) {
      lds_barrier();
      qst.store(Qs, C::LDQ, v2);
      dst.store(Ds, C::LDV, v2);
#pragma unroll
      for (int qb = 0; qb < C::TB; ++qb) mw[qb] = mwn[qb];
      lds_barrier();
    }
    GR_ST(st_sync, 0);
  }
#ifdef GR_STAMP
  if (lane == 0) {
    const int slot = (id * 4 + w) * 12;
    if (slot + 12 <= (1 << 16)) {
      gr_stamp_buf[slot + 0] = st_ld;
      gr_stamp_buf[slot + 1] = st_mm1;
      gr_stamp_buf[slot + 2] = st_ew;
      gr_stamp_buf[slot + 3] = st_bias;
      gr_stamp_buf[slot + 4] = st_mm2;
      gr_stamp_buf[slot + 5] = st_sync;
      gr_stamp_buf[slot + 6] = (unsigned long long)kt;
      gr_stamp_buf[slot + 7] = gr_stamp() - st_begin;
      gr_stamp_buf[slot + 8] = st_begin - st_entry;
    }
  }
#endif
  if (a.ds_flags) {
    // publish this key tile's dS tiles (plain stores, one agent-scope release, flag by an
    // atomic store): every wave drains its stores before the barrier, the releasing lane
    // waits again after the fence (cdna_hip_programming.md Guideline 16)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.ds_flags + (int64_t)bh * a.n_tiles + kt, 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (STAGED && a.hv) {
    lds_barrier();
    qst.store(Qs, C::LDQ, v2h);
    dst.store(Ds, C::LDV, v2h);
    lds_barrier();
  }
  if (has_bias && lg == 0) {  // the last block's wrapped diagonals
    const int bin = a.N - 1 + last_db - 16 + lr;
    if (bin >= 0 && bin < npos) whist[bin] += carry;
  }
  carry = 0.f;
  // the workgroup's bias slab is written before its dK / dV rows, behind an LDS-only
  // barrier (a __syncthreads() also drained the dS tile stores still in flight)
  if (pass == 1 || !(TT == 64 && kt_b >= 0 && kt_b * 64 < L)) {
    if (has_bias && run_b >= 0) atomicAdd(&wts[run_b], run_s);  // the open dts run
    if (has_bias && slab) {
      lds_barrier();
      for (int i = tid; i < npos; i += 256)
        slab[i] = ((hist[i] + hist[wbins + i]) + hist[2 * wbins + i]) + hist[3 * wbins + i];
      for (int i = tid; i <= a.nb; i += 256) {
        float acc = 0.f;
        for (int ww = 0; ww < 4; ++ww)
          for (int c = 0; c < GR_DTS_COPIES; ++c) acc += hist[ww * wbins + npos + c * tss + i];
        slab[npos + i] = acc;
      }
    }
  }
  // ---- epilogue: rows = keys wk_lo + 4lg + r, cols = lr + 16 t
  if constexpr (!STAGED) {  // silu'(h) from global: every load issued before any store
    if (DO_V)
      store_scaled<4, VTILES>([&](int i, int t) { return dV[t][i]; }, L, a.dv, s0, a.dvv, a.ld_d, a.hv,
                              a.ld_h, h * a.dv, [&](int i) { return wk_lo + 4 * lg + i; },
                              [&](int t) { return 16 * t + lr; });
    if (DO_K)
      store_scaled<4, C::KT>([&](int i, int t) { return dK[t][i]; }, L, a.dqk, s0, a.dk, a.ld_d, a.hk,
                             a.ld_h, h * a.dqk, [&](int i) { return wk_lo + 4 * lg + i; },
                             [&](int t) { return 16 * t + lr; });
  } else
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = wk_lo + 4 * lg + r;
    const bool row_ok = key < L;
    const int64_t row = s0 + (row_ok ? key : L - 1);
#pragma unroll
    for (int t = 0; t < VTILES; ++t) {
      const int c = t * 16 + lr;
      const bool ok = row_ok && c < a.dv;
      float g = dV[t][r];
      if (a.hv) {
        const float hp = STAGED ? Ds[(w * 16 + 4 * lg + r) * C::LDV + c]
                                : as_global(a.hv)[row * a.ld_h + h * a.dv + (c < a.dv ? c : a.dv - 1)];
        g *= ok ? silu_grad_(hp) : 0.f;
      }
      if (ok) a.dvv[row * a.ld_d + h * a.dv + c] = g;
    }
#pragma unroll
    for (int t = 0; t < C::KT; ++t) {
      const int c = t * 16 + lr;
      const bool ok = row_ok && c < a.dqk;
      float g = dK[t][r];
      if (a.hk) {
        const float hp = STAGED ? Qs[(w * 16 + 4 * lg + r) * C::LDQ + c]
                                : as_global(a.hk)[row * a.ld_h + h * a.dqk + (c < a.dqk ? c : a.dqk - 1)];
        g *= ok ? silu_grad_(hp) : 0.f;
      }
      if (ok) a.dk[row * a.ld_d + h * a.dqk + c] = g;
    }
  }
  }  // pass
#ifdef GR_STAMP
  if (lane == 0) {
    const int slot = (id * 4 + w) * 12;
    if (slot + 12 <= (1 << 16)) gr_stamp_buf[slot + 9] = gr_stamp() - st_entry;
  }
#endif
}

// ------------------------------------------------------------------ query-major: dQ
template <int KSTEPS, int VTILES, int TT, bool HB, bool V2>
__device__ __forceinline__ void attn_bwd_dq_body(const AttnBwdArgs& a, const int id) {
  const bool v2 = V2 || a.vec2, v2h = V2 || a.vec2h;
  using C = AttnBwdCfg<KSTEPS, VTILES, TT>;
  constexpr int LDK = C::LDQ;
  constexpr int LDV = 32 * ((C::VP - 2 + 31) / 32) + 2;  // A-operand reads only
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);  // [TT][LDK]
  float* Vs = Ks + TT * LDK;                   // [TT][LDV]
  float* tsw = Vs + TT * LDV;
  float* posw = tsw + (a.nb + 1);

  const int BH = a.B * a.H;
  int qt_a, qt_b = -1, bh;  // paired: query tiles p and T-1-p (see the dK/dV body)
  if (a.paired) {
    qt_a = id / BH;
    bh = id % BH;
    qt_b = a.n_tiles - 1 - qt_a;
    if (qt_b == qt_a) qt_b = -1;
  } else {
    const int rank = snake_rank(id, a.cus);
    qt_a = a.n_tiles - 1 - rank / BH;
    bh = rank % BH;
  }
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  if (qt_a * 64 >= L && (qt_b < 0 || qt_b * 64 >= L)) return;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr bool has_bias = HB;
  if (has_bias) {
    for (int i = tid; i <= a.nb; i += 256) tsw[i] = a.ts_w[i];
    for (int i = tid; i < 2 * a.N - 1; i += 256) posw[i] = a.pos_w[i];
  }
  const __amdgpu_buffer_rsrc_t rmap = map_rsrc(a.map_qk, b, attn_tiles_per_seq(a.N));
  const int map_voff = ((w * 16 + lr) * 16 + lg) * 4;
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const __amdgpu_buffer_rsrc_t rv = seq_rsrc(a.v, a.ld_v, s0, h * a.dv, L, a.dv);
  for (int pass = 0; pass < (TT == 64 ? 2 : 1); ++pass) {
  const int qt = pass == 0 ? qt_a : qt_b;
  const int q0 = qt * 64;
  if (pass == 1) {
    if (qt < 0 || q0 >= L) break;
    lds_barrier();  // the first pass's epilogue reads of Ks
  }
  const int qi = q0 + w * 16 + lr;
  const bool q_ok = qi < L;
  constexpr bool STAGED = TT == 64;  // Q / dO fragments and silu'(h) through LDS (see dK/dV)
  float qreg[KSTEPS], doreg[KSTEPS];
  if constexpr (!STAGED) {
    const int64_t row = s0 + (q_ok ? qi : L - 1);
    gptr<float> qrow = as_global(a.q) + row * a.ld_qk + h * a.dqk;
    gptr<float> drow = as_global(a.dout) + row * a.ld_dout + h * a.dv;
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      const int d = 4 * st + lg;
      const float x = qrow[d < a.dqk ? d : a.dqk - 1];
      qreg[st] = d < a.dqk ? x : 0.f;
      const float y = drow[d < a.dv ? d : a.dv - 1];
      doreg[st] = d < a.dv ? y : 0.f;
    }
  }
  f4 dQ[C::KT];
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dQ[t] = f4_zero();
  const int wq_lo = q0 + w * 16;
  float hq_pre[4][STAGED ? 1 : C::KT];  // the epilogue's silu'(h) inputs (see the dK/dV body)
  if (!STAGED && a.hq) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qo = wq_lo + 4 * lg + r;
      gptr<float> hqr = as_global(a.hq) + (s0 + (qo < L ? qo : L - 1)) * a.ld_h + h * a.dqk;
#pragma unroll
      for (int t = 0; t < (STAGED ? 1 : C::KT); ++t) {
        const int c = t * 16 + lr;
        hq_pre[r][t] = hqr[c < a.dqk ? c : a.dqk - 1];
      }
    }
  }

  BufTile<C::KPT, TT> kst;
  BufTile<C::VP, TT> vst;
  uint32_t mw[C::TB], mwn[C::TB];
  auto load_tile = [&](int kt, uint32_t (&m)[C::TB]) {
    kst.load(rk, a.ld_qk, kt * TT, a.dqk, v2);
    vst.load(rv, a.ld_v, kt * TT, a.dv, v2);
#pragma unroll
    for (int kb = 0; kb < C::TB; ++kb)
      m[kb] = buf_ld_u32(rmap, map_voff, map_soff(q0, kt * TT + kb * 16, true));
  };
  if constexpr (STAGED) {
    // the workgroup's Q / dO rows and the first key tile in one round trip (see dK/dV)
    BufTile<C::KPT, TT> qst0;
    BufTile<C::VP, TT> dst0;
    qst0.load(seq_rsrc(a.q, a.ld_qk, s0, h * a.dqk, L, a.dqk), a.ld_qk, q0, a.dqk, v2);
    dst0.load(seq_rsrc(a.dout, a.ld_dout, s0, h * a.dv, L, a.dv), a.ld_dout, q0, a.dv, v2);
    load_tile(0, mw);
    qst0.store(Ks, LDK, v2);
    dst0.store(Vs, LDV, v2);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < KSTEPS; ++st) {
      qreg[st] = Ks[(w * 16 + lr) * LDK + 4 * st + lg];
      doreg[st] = Vs[(w * 16 + lr) * LDV + 4 * st + lg];
    }
    lds_barrier();
  } else {
    load_tile(0, mw);
  }
  kst.store(Ks, LDK, v2);
  vst.store(Vs, LDV, v2);
  __syncthreads();

  const int last_kt = min(q0 + 63, L - 1) / TT;
#pragma unroll
  for (int kb = 0; kb < C::TB; ++kb) asm volatile("" ::"v"(mw[kb]));  // see the dK/dV body
  for (int kt = 0; kt <= last_kt; ++kt) {
    const int k0 = kt * TT;
    const bool more = kt < last_kt;
    if (more) {
      load_tile(kt + 1, mwn);
    } else if (STAGED && a.hq) {
      kst.load(seq_rsrc(a.hq, a.ld_h, s0, h * a.dqk, L, a.dqk), a.ld_h, q0, a.dqk, v2h);
    }
#pragma unroll
    for (int kb = 0; kb < C::TB; ++kb) {
      const int kb0 = k0 + kb * 16;
      if (kb0 <= wq_lo + 15 && kb0 < L) {  // wave-uniform causal / length skip
        f4 s = f4_zero(), dpt = f4_zero();
        const float* krow = Ks + (kb * 16 + lr) * LDK + lg;
        const float* vrow = Vs + (kb * 16 + lr) * LDV + lg;
#pragma unroll
        for (int st = 0; st < KSTEPS; ++st) {
          s = mfma16x16x4(krow[4 * st], qreg[st], s);
          dpt = mfma16x16x4(vrow[4 * st], doreg[st], dpt);
        }
        // s[r] = S^T[key kb0 + 4lg + r][query qi]
        float ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = kb0 + 4 * lg + r;
          const bool ok = q_ok && kj <= qi;
          float x = s[r];
          if (has_bias) {
            const int bucket = (mw[kb] >> (8 * r)) & 0xFF;
            int pi = a.N - 1 + kj - qi;
            pi = pi < 0 ? 0 : (pi > 2 * a.N - 2 ? 2 * a.N - 2 : pi);
            x = x + (posw[pi] + tsw[bucket]);
          }
          ds[r] = ok ? dpt[r] * silu_grad_(x) * a.inv_n : 0.f;
        }
        const float* kcol = Ks + (kb * 16 + 4 * lg) * LDK + lr;
        if constexpr (C::KT > 8) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < C::KT; ++t)
              dQ[t] = mfma16x16x4(ds[r], kcol[r * LDK + t * 16], dQ[t]);
        } else {
        float bk[2][C::KT];
#pragma unroll
        for (int t = 0; t < C::KT; ++t) bk[0][t] = kcol[t * 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r + 1 < 4) {
#pragma unroll
            for (int t = 0; t < C::KT; ++t) bk[(r + 1) & 1][t] = kcol[(r + 1) * LDK + t * 16];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int t = 0; t < C::KT; ++t) dQ[t] = mfma16x16x4(ds[r], bk[r & 1][t], dQ[t]);
          __builtin_amdgcn_sched_barrier(0);
        }
        }
      }
    }
    if (more) {
      lds_barrier();
      kst.store(Ks, LDK, v2);
      vst.store(Vs, LDV, v2);
#pragma unroll
      for (int kb = 0; kb < C::TB; ++kb) mw[kb] = mwn[kb];
      lds_barrier();
    }
  }
  if (STAGED && a.hq) {
    lds_barrier();
    kst.store(Ks, LDK, v2h);
    lds_barrier();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qo = wq_lo + 4 * lg + r;
    const bool row_ok = qo < L;
    const int64_t row = s0 + (row_ok ? qo : L - 1);
#pragma unroll
    for (int t = 0; t < C::KT; ++t) {
      const int c = t * 16 + lr;
      const bool ok = row_ok && c < a.dqk;
      float g = dQ[t][r];
      if (a.hq) {
        const float hp = STAGED ? Ks[(w * 16 + 4 * lg + r) * LDK + c] : hq_pre[r][STAGED ? 0 : t];
        g *= ok ? silu_grad_(hp) : 0.f;
      }
      if (ok) a.dq[row * a.ld_d + h * a.dqk + c] = g;
    }
  }
  }  // pass
}

// ------------------------------------------------------------------ query-major from dS
// dQ = dS K from the dS tiles the key-major pass stored (no recompute of S, dP, the
// bias or the SiLU terms): per 16 x 16 block a lane's A fragment is one float4 of the
// row-major tile (query lr, keys 4lg .. 4lg + 3 = k-steps 0..3, the order the
// recomputing query-major pass uses), B = the K tile staged in LDS.  Sums run in the
// same key order as the recomputing pass, so dQ is unchanged.
// WAIT (one-launch form): the key tiles are taken in DESCENDING order, each after its
// producer workgroup's flag (one lane polls relaxed with s_sleep, then one agent-scope
// acquire and a barrier); a spin that exceeds its bound returns false before anything
// is written and the caller recomputes the tile instead, so no schedule can hang it.
template <int KSTEPS, int VTILES, int TT, bool V2, bool WAIT = false>
__device__ __forceinline__ bool attn_bwd_dq_ds_body(const AttnBwdArgs& a, const int id) {
  const bool v2 = V2 || a.vec2, v2h = V2 || a.vec2h;
  using C = AttnBwdCfg<KSTEPS, VTILES, TT>;
  // TT = 64: 64-key K tiles (narrow heads); TT = 16: 16-key K tiles (wide heads, d > 128),
  // the epilogue's silu'(h) rows then come from global (the K stage holds 16 rows only)
  static_assert(TT == 64 || TT == 16, "dQ from dS: 64- or 16-row tiles");
  constexpr bool WIDE = TT == 16;
  constexpr int LDK = C::LDQ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);  // [TT][LDK]
  int* wstat = reinterpret_cast<int*>(Ks + TT * LDK);
  const int BH = a.B * a.H;
  const int rank = snake_rank(id, a.cus);
  const int qt = a.n_tiles - 1 - rank / BH;
  const int bh = rank % BH;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qt * 64;
  if (q0 >= L) return true;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int wq_lo = q0 + w * 16;
  const int qbi = wq_lo >> 4;
  // WAIT: tile j of the walk is key tile last_kt - j
  auto wait_tile = [&](int kt) -> bool {
    if (tid == 0) {
      const uint32_t* f = a.ds_flags + (int64_t)bh * a.n_tiles + kt;
      int ok = 1;
      for (uint32_t spins = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u;) {
        __builtin_amdgcn_s_sleep(4);
        if (++spins > (1u << 20)) {  // ~ms: give up, recompute instead
          ok = 0;
          break;
        }
      }
      if (ok) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      wstat[0] = ok;
    }
    __syncthreads();
    return wstat[0] != 0;
  };
  const bool w_ok = wq_lo < L;  // wave-uniform: no valid query row otherwise
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const float* dsq = a.ds + ((int64_t)bh * a.ds_tps + qbi * (qbi + 1) / 2) * 256 + lr * 16 + 4 * lg;
  f4 dQ[C::KT];
#pragma unroll
  for (int t = 0; t < C::KT; ++t) dQ[t] = f4_zero();
  BufTile<C::KPT, TT> kst;
  f4 dsv[C::TB], dsn[C::TB];
  auto load_tile = [&](int kt, f4 (&d)[C::TB]) {
    kst.load(rk, a.ld_qk, kt * TT, a.dqk, v2);
#pragma unroll
    for (int kb = 0; kb < C::TB; ++kb) {
      const int kbi = (kt * TT + kb * 16) >> 4;
      d[kb] = (w_ok && kbi <= qbi) ? *reinterpret_cast<const f4*>(dsq + kbi * 256) : f4_zero();
    }
  };
  const int last_kt = min(q0 + 63, L - 1) / TT;
  auto tile_of = [&](int j) { return WAIT ? last_kt - j : j; };
  if (WAIT && !wait_tile(tile_of(0))) return false;
  load_tile(tile_of(0), dsv);
  kst.store(Ks, LDK, v2);
  __syncthreads();
#pragma unroll
  for (int kb = 0; kb < C::TB; ++kb) asm volatile("" ::"v"(dsv[kb]));  // see the dK/dV body
  for (int j = 0; j <= last_kt; ++j) {
    const int kt = tile_of(j);
    const int k0 = kt * TT;
    const bool more = j < last_kt;
    if (more) {
      if (WAIT && !wait_tile(tile_of(j + 1))) return false;
      load_tile(tile_of(j + 1), dsn);
    } else if (!WIDE && a.hq) {  // the epilogue's silu'(h) rows of this workgroup's queries
      kst.load(seq_rsrc(a.hq, a.ld_h, s0, h * a.dqk, L, a.dqk), a.ld_h, q0, a.dqk, v2h);
    }
#pragma unroll
    for (int kb = 0; kb < C::TB; ++kb) {
      const int kb0 = k0 + kb * 16;
      if (w_ok && kb0 <= wq_lo + 15 && kb0 < L) {
        const float* kcol = Ks + (kb * 16 + 4 * lg) * LDK + lr;
        float bk[2][C::KT];
#pragma unroll
        for (int t = 0; t < C::KT; ++t) bk[0][t] = kcol[t * 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (r + 1 < 4) {
#pragma unroll
            for (int t = 0; t < C::KT; ++t) bk[(r + 1) & 1][t] = kcol[(r + 1) * LDK + t * 16];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int t = 0; t < C::KT; ++t) dQ[t] = mfma16x16x4(dsv[kb][r], bk[r & 1][t], dQ[t]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if (more) {
      lds_barrier();
      kst.store(Ks, LDK, v2);
#pragma unroll
      for (int kb = 0; kb < C::TB; ++kb) dsv[kb] = dsn[kb];
      lds_barrier();
    }
  }
  if constexpr (WIDE) {
    if (!w_ok) return true;
    store_scaled<4, C::KT>([&](int i, int t) { return dQ[t][i]; }, L, a.dqk, s0, a.dq, a.ld_d, a.hq,
                           a.ld_h, h * a.dqk, [&](int i) { return wq_lo + 4 * lg + i; },
                           [&](int t) { return 16 * t + lr; });
    return true;
  }
  if (a.hq) {
    lds_barrier();
    kst.store(Ks, LDK, v2h);
    lds_barrier();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qo = wq_lo + 4 * lg + r;
    const bool row_ok = qo < L;
    const int64_t row = s0 + (row_ok ? qo : L - 1);
#pragma unroll
    for (int t = 0; t < C::KT; ++t) {
      const int c = t * 16 + lr;
      const bool ok = row_ok && c < a.dqk;
      float g = dQ[t][r];
      if (a.hq) g *= ok ? silu_grad_(Ks[(w * 16 + 4 * lg + r) * LDK + c]) : 0.f;
      if (ok) a.dq[row * a.ld_d + h * a.dqk + c] = g;
    }
  }
  return true;
}

// ------------------------------------------------------------------ entry points
// BWD_V2: every kernel body is instantiated twice, with the pair staging fixed at compile
// time when all rows qualify.  With a runtime flag the unused dword path's load
// destinations stayed live across the join, and the waitcnt pass made each tile's first
// block wait for the whole next-tile prefetch (vmcnt(3) of ~20) before writing them.
#define BWD_V2(a) ((a).vec2 && ((a).vec2h || !(a).hq))
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnBwdArgs a) {
  GR_TL_BEGIN();
  if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, true>(a, blockIdx.x);
  else attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, false>(a, blockIdx.x);
  GR_TL_END(blockIdx.x, 0);
}
// wide heads: dV workgroups (even blockIdx) and dK workgroups (odd), key tile j = blockIdx / 2
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_dkv_split_kernel(AttnBwdArgs a) {
  const int j = blockIdx.x >> 1;
  if (blockIdx.x & 1) {
    if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, true, 2>(a, j);
    else attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, false, 2>(a, j);
  } else {
    if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, true, 1>(a, j);
    else attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, false, 1>(a, j);
  }
}
// the same kinds as two launches: dV (235 VGPRs under a two-waves-per-SIMD bound, no
// histograms: two workgroups per CU) and dK (one wave per SIMD: the dpos histograms of
// N = 2059 take 76 KB of LDS per workgroup)
template <int KSTEPS, int VTILES, int TT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void attn_bwd_dv_kernel(AttnBwdArgs a) {
  if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, true, true, 1>(a, blockIdx.x);
  else attn_bwd_dkv_body<KSTEPS, VTILES, TT, true, false, 1>(a, blockIdx.x);
}
template <int KSTEPS, int VTILES, int TT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void attn_bwd_dv_nobias_kernel(AttnBwdArgs a) {
  if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, false, true, 1>(a, blockIdx.x);
  else attn_bwd_dkv_body<KSTEPS, VTILES, TT, false, false, 1>(a, blockIdx.x);
}
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_dk_kernel(AttnBwdArgs a) {
  if (BWD_V2(a)) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, true, 2>(a, blockIdx.x);
  else attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, false, 2>(a, blockIdx.x);
}
__device__ __forceinline__ void bias_grad_reduce_body(const float* slabs, int n_slabs, int n_pos,
                                                      int n_ts, float* dpos_w, float* dts_w, int blk);
// dQ = dS K at narrow heads, one wave per 16-query block (no LDS tile, no workgroup
// barrier): the lane's K elements (key row 4g + r of a block, column 16 t + lr) come from
// L2 through the range-checked sequence descriptor, PD key blocks in flight.  Blocks past
// the last one of the walk re-read it with a zero A operand (+0 to every sum), so the
// loads stay unconditional.  The MFMA sequence (key blocks ascending, k-step r = keys
// 4g + r) is the recomputing pass's: dQ is bit-identical to it.
// Returns false for an item past the sequence; otherwise the block's first query q0, the
// sequence's first row s0 and length L (the layer-boundary epilogue, hstu_attn_bwd_bnd).
template <int KSTEPS, int VTILES>
__device__ __forceinline__ bool attn_bwd_dq_wave_body(const AttnBwdArgs& a, const int item,
                                                      int* q0_out = nullptr, int* L_out = nullptr,
                                                      int64_t* s0_out = nullptr) {
  using C = AttnBwdCfg<KSTEPS, VTILES, 64>;
  constexpr int KT = C::KT, PD = 4;
  const int BH = a.B * a.H;
  const int qb = a.n_tiles * 4 - 1 - item / BH;  // heaviest blocks first
  const int bh = item % BH;
  if (qb < 0) return false;
  const int b = bh / a.H, h = bh % a.H;
  const int64_t s0 = a.offsets[b];
  const int L = (int)(a.offsets[b + 1] - s0);
  const int q0 = qb * 16;
  if (q0 >= L) return false;
  if (q0_out) {
    *q0_out = q0;
    *L_out = L;
    *s0_out = s0;
  }
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rk = seq_rsrc(a.k, a.ld_qk, s0, h * a.dqk, L, a.dqk);
  const float* dsq = a.ds + ((int64_t)bh * a.ds_tps + qb * (qb + 1) / 2) * 256 + lr * 16 + 4 * lg;
  const int rowb = (int)a.ld_qk * 4;  // bytes per K row
  int voff[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int c = 16 * t + lr;
    voff[t] = c < a.dqk ? (4 * lg * (int)a.ld_qk + c) * 4 : OOB_OFF;
  }
  f4 dQ[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) dQ[t] = f4_zero();
  f4 dsr[PD];
  float kr[PD][4][KT];
  auto load = [&](int u, int kb) {
    const int kc = kb < qb ? kb : qb;
    dsr[u] = *as_global(reinterpret_cast<const f4*>(dsq + kc * 256));
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < KT; ++t) kr[u][r][t] = buf_ld(rk, voff[t], (kc * 16 + r) * rowb);
  };
#pragma unroll
  for (int u = 0; u < PD; ++u) load(u, u);
  for (int kb0 = 0; kb0 <= qb; kb0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const bool live = kb0 + u <= qb;  // wave-uniform; a re-read block adds +0
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float av = live ? dsr[u][r] : 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t) dQ[t] = mfma16x16x4(av, kr[u][r][t], dQ[t]);
      }
      load(u, kb0 + PD + u);
    }
  }
  store_scaled<4, KT>([&](int i, int t) { return dQ[t][i]; }, L, a.dqk, s0, a.dq, a.ld_d, a.hq,
                      a.ld_h, h * a.dqk, [&](int i) { return q0 + 4 * lg + i; },
                      [&](int t) { return 16 * t + lr; });
  return true;
}

// dQ = dS K; the first n_bias workgroups reduce the bias slabs the dK/dV launch wrote (no
// launch of their own: they run beside the dQ workgroups).  TT = 64: four query blocks
// per workgroup, one per wave (attn_bwd_dq_wave_body).
template <int KSTEPS, int VTILES, int TT>
__global__ __launch_bounds__(256) void attn_bwd_dq_ds_kernel(AttnBwdArgs a, int n_bias, int n_slabs,
                                                             float* dpos_w, float* dts_w) {
  const int id = (int)blockIdx.x - n_bias;
  if (id < 0) {
    bias_grad_reduce_body(a.slabs, n_slabs, 2 * a.N - 1, a.nb + 1, dpos_w, dts_w, (int)blockIdx.x);
    return;
  }
  if constexpr (TT == 64) {
    attn_bwd_dq_wave_body<KSTEPS, VTILES>(a, id * 4 + wave_id());
  } else if constexpr (TT == 16) {
    if (BWD_V2(a)) attn_bwd_dq_ds_body<KSTEPS, VTILES, TT, true>(a, id);
    else attn_bwd_dq_ds_body<KSTEPS, VTILES, TT, false>(a, id);
  }
}
// dQ = dS K with the layer boundary as its epilogue (hstu_attn_bwd_bnd, H == 1): the
// workgroup stages the boundary's weight panels (ln_uvqk_bwd's W_uvqk^T, gate_o_bwd's W_o)
// in LDS, each wave computes and stores the dq rows of its 16-query block, then -- the
// rows' d_uvqk now complete -- runs the row-wave boundary unit of those 16 rows (rows past
// the sequence fall outside the ops' descriptors).  OP2 = false: the first layer, whose
// boundary is ln_uvqk_bwd alone.  The first n_bias workgroups reduce the bias slabs.
template <int KSTEPS, int VTILES, int KG1, int W, bool OP2>
__global__ __launch_bounds__(256) void attn_bwd_dq_bnd_kernel(AttnBwdArgs a, int n_bias, int n_slabs,
                                                              float* dpos_w, float* dts_w,
                                                              RwLnUvqkBwd<KG1, W, 2> op1,
                                                              RwGateOBwd<W, W, 2> op2) {
  using C1 = RowWaveCfg<KG1, W>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* W1 = reinterpret_cast<float*>(smem);
  float* W2 = W1 + C1::KP * C1::LDW;
  const int id = (int)blockIdx.x - n_bias;
  if (id < 0) {
    bias_grad_reduce_body(a.slabs, n_slabs, 2 * a.N - 1, a.nb + 1, dpos_w, dts_w, (int)blockIdx.x);
    return;
  }
  // the panels' loads land while dQ is computed; written to LDS after it
  RwStage<KG1, W, RwLnUvqkBwd<KG1, W, 2>> st1;
  RwStage<W, W, RwGateOBwd<W, W, 2>> st2;
  st1.load(op1);
  if constexpr (OP2) st2.load(op2);
  int q0 = 0, L = 0;
  int64_t s0 = 0;
  const bool live = attn_bwd_dq_wave_body<KSTEPS, VTILES>(a, id * 4 + wave_id(), &q0, &L, &s0);
  st1.store(W1);
  if constexpr (OP2) st2.store(W2);
  __syncthreads();  // the panels are staged (every wave reaches this, live or not)
  if (!live) return;
  // this wave's dq stores have landed before its unit reads the rows back (the rows' other
  // columns were written by earlier launches; no other wave writes these rows)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  op1.setup(s0 + L);
  op1.rd_aux = 16;  // d_uvqk rows: L2 (the dq columns were just stored by this wave)
  if constexpr (OP2) op2.setup(s0 + L);
  const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  const int64_t m = s0 + q0 + lr;
  const bool ok = q0 + lr < L;
  if constexpr (OP2) rw2_unit<KG1, W, W>(op1, op2, W1, W2, m, ok, lr, lg);
  else rw1_unit<KG1, W>(op1, W1, m, ok, lr, lg);
}

// the boundary of hstu_attn_bwd_bnd as the dQ launch's epilogue (see attn_bwd_dq_bnd_kernel)
struct BndCtx {
  RwArgsLnUvqkBwd a1;
  RwArgsGateOBwd a2;
  bool op2;
  int kg1;      // 13 | 16 (n_out in 16-column groups)
  bool fused;   // set by the launch that ran it
};

template <int KS, int VT, int KG1, bool OP2>
static int launch_dq_bnd_k(const AttnBwdArgs& aq, BndCtx& bc, int grid, int nbias, int n_slabs,
                           float* dpos_w, float* dts_w, hipStream_t st) {
  RwLnUvqkBwd<KG1, 4, 2> o1{};
  RwGateOBwd<4, 4, 2> o2{};
  bc.a1.fill(o1);
  if (OP2) bc.a2.fill(o2);
  const size_t lds = RowWaveCfg<KG1, 4>::LDS_BYTES + (OP2 ? RowWaveCfg<4, 4>::LDS_BYTES : 0);
  GR_TIMED(OP2 ? "attn_bwd_dq_bnd" : "attn_bwd_dq_bnd1", st, hipLaunchKernelGGL((attn_bwd_dq_bnd_kernel<KS, VT, KG1, 4, OP2>),
                                                 dim3(grid + nbias), dim3(256), lds, st, aq, nbias,
                                                 n_slabs, dpos_w, dts_w, o1, o2));
  GR_LAUNCH_CHECK("hstu_attn_bwd_bnd(dq + boundary)");
  bc.fused = true;
  return 0;
}
template <int KS, int VT>
static int launch_dq_bnd(const AttnBwdArgs& aq, BndCtx& bc, int grid, int nbias, int n_slabs,
                         float* dpos_w, float* dts_w, hipStream_t st) {
  if (bc.kg1 == 13) {
    return bc.op2 ? launch_dq_bnd_k<KS, VT, 13, true>(aq, bc, grid, nbias, n_slabs, dpos_w, dts_w, st)
                  : launch_dq_bnd_k<KS, VT, 13, false>(aq, bc, grid, nbias, n_slabs, dpos_w, dts_w, st);
  }
  return bc.op2 ? launch_dq_bnd_k<KS, VT, 16, true>(aq, bc, grid, nbias, n_slabs, dpos_w, dts_w, st)
                : launch_dq_bnd_k<KS, VT, 16, false>(aq, bc, grid, nbias, n_slabs, dpos_w, dts_w, st);
}

// One launch, dS handed over inside it: workgroups [0, grid_kv) are the key-major pass
// (publishing each key tile's dS), the rest compute dQ = dS K as the tiles appear (a
// workgroup that times out waiting recomputes its tile, attn_bwd_dq_body).  All key-major
// workgroups precede the dQ ones in dispatch order.
template <int KSTEPS, int VTILES, int TT, bool HB, bool V2>
__device__ __forceinline__ void attn_bwd_fused_ds_run(const AttnBwdArgs& a, int grid_kv) {
  const int id = blockIdx.x;
  if (id < grid_kv) {
    attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, V2>(a, id);
  } else if (!attn_bwd_dq_ds_body<KSTEPS, VTILES, TT, V2, true>(a, id - grid_kv)) {
    __syncthreads();
    AttnBwdArgs aq = a;
    aq.paired = 0;  // the dQ workgroups are single-tile whatever the key-major pairing
    attn_bwd_dq_body<KSTEPS, VTILES, TT, HB, V2>(aq, id - grid_kv);
  }
}
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_fused_ds_kernel(AttnBwdArgs a, int grid_kv) {
  if constexpr (TT == 64) {
    if (BWD_V2(a)) attn_bwd_fused_ds_run<KSTEPS, VTILES, TT, HB, true>(a, grid_kv);
    else attn_bwd_fused_ds_run<KSTEPS, VTILES, TT, HB, false>(a, grid_kv);
  }
}
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  GR_TL_BEGIN();
  if (BWD_V2(a)) attn_bwd_dq_body<KSTEPS, VTILES, TT, HB, true>(a, blockIdx.x);
  else attn_bwd_dq_body<KSTEPS, VTILES, TT, HB, false>(a, blockIdx.x);
  GR_TL_END(blockIdx.x + gridDim.x, 1);
}
// dK/dV and dQ in ONE launch: workgroups [0, grid) run the key-major pass (heaviest key
// tiles first), the next grid run the query-major pass.  At narrow heads both are bound
// by their heavy workgroups' chains of blocks with the CUs half idle, so the dQ
// workgroups fill the slots the light dK/dV workgroups free (a horizontal fusion: one
// dispatch, no stream fork/join).
// (Interleaving the two passes' workgroups measured slower: 72 vs 62 us at C2.)
template <int KSTEPS, int VTILES, int TT, bool HB>
__global__ __launch_bounds__(256) void attn_bwd_fused_kernel(AttnBwdArgs a, int grid_kv) {
  const int id = blockIdx.x;
  GR_TL_BEGIN();
  if (BWD_V2(a)) {
    if (id < grid_kv) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, true>(a, id);
    else attn_bwd_dq_body<KSTEPS, VTILES, TT, HB, true>(a, id - grid_kv);
  } else {
    if (id < grid_kv) attn_bwd_dkv_body<KSTEPS, VTILES, TT, HB, false>(a, id);
    else attn_bwd_dq_body<KSTEPS, VTILES, TT, HB, false>(a, id - grid_kv);
  }
  GR_TL_END(id, id < grid_kv ? 0 : 1);
}

// ------------------------------------------------------------------ slab reduce
// Deterministic: a workgroup owns 16 bins; thread (bin, g) sums slabs g, g+16, ... in
// order (loads 8-deep), then the 16 partials are added in g order.
__device__ __forceinline__ void bias_grad_reduce_body(const float* slabs, int n_slabs, int n_pos,
                                                      int n_ts, float* dpos_w, float* dts_w,
                                                      int blk) {
  __shared__ float part[16][17];
  const int nbins = n_pos + n_ts;
  const int bl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int i = blk * 16 + bl;
  const int ic = i < nbins ? i : nbins - 1;
  gptr<float> src = as_global(slabs);
  float acc = 0.f;
  int j = g;
  for (; j + 112 < n_slabs; j += 128) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(j + 16 * u) * nbins + ic];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; j < n_slabs; j += 16) acc += src[(int64_t)j * nbins + ic];
  part[g][bl] = acc;
  __syncthreads();
  if (g == 0 && i < nbins) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += part[k][bl];
    if (i < n_pos) dpos_w[i] = s;
    else dts_w[i - n_pos] = s;
  }
}
__global__ __launch_bounds__(256) void bias_grad_reduce_kernel(const float* slabs, int n_slabs,
                                                               int n_pos, int n_ts,
                                                               float* dpos_w, float* dts_w) {
  bias_grad_reduce_body(slabs, n_slabs, n_pos, n_ts, dpos_w, dts_w, blockIdx.x);
}

static size_t bwd_slab_bytes(int B, int N, int max_len, int H, int nb) {
  const int n_tiles = ceil_div(max_len, 64);
  return sizeof(float) * (size_t)n_tiles * B * H * (size_t)(2 * N - 1 + nb + 1);
}
// dS tiles of the two-pass backward (short sequences: N <= 512), after the slabs
constexpr int DS_MAX_N = 512;
static int ds_tiles_per_seq(int N) {
  const int nb = ceil_div(N, 16);
  return nb * (nb + 1) / 2;
}
static size_t bwd_ds_offset(int B, int N, int max_len, int H, int nb) {
  return (bwd_slab_bytes(B, N, max_len, H, nb) + 255) & ~(size_t)255;
}
static size_t bwd_ds_bytes(int B, int N, int H) {
  return N <= DS_MAX_N && option(GR_OPT_ATTN_BWD_DS) != 0
             ? sizeof(float) * 256 * (size_t)ds_tiles_per_seq(N) * B * H : 0;
}
// wide heads (d > 128: 16-row tiles): dS tiles for the dQ pass at any N (WIDE_DS option)
static bool wide_heads(int dqk, int dv) { return (dqk > dv ? dqk : dv) > 128; }
static size_t bwd_ds_bytes_d(int B, int N, int H, int dqk, int dv) {
  if (wide_heads(dqk, dv))
    return option(GR_OPT_ATTN_BWD_WIDE_DS) != 0
               ? sizeof(float) * 256 * (size_t)ds_tiles_per_seq(N) * B * H : 0;
  return bwd_ds_bytes(B, N, H);
}
// one-launch form (GR_OPT_ATTN_BWD_DS = 2): a flag word per (sequence, head, key tile)
static size_t bwd_flag_bytes(int B, int max_len, int H) {
  return option(GR_OPT_ATTN_BWD_DS) == 2 ? 256 + sizeof(uint32_t) * (size_t)B * H * ceil_div(max_len, 64) : 0;
}

template <int KS, int VT, int TT = 64>
static int launch_bwd(const AttnBwdArgs& a, float* dpos_w, float* dts_w, hipStream_t st,
                      BndCtx* bnd = nullptr) {
  using C = AttnBwdCfg<KS, VT, TT>;
  const int grid = a.n_tiles * a.B * a.H;
  const int nbins = 2 * a.N - 1 + a.nb + 1;
  const size_t tail = sizeof(float) * (a.nb + 1 + 2 * a.N - 1);
  const size_t lds_kv = sizeof(float) * (TT * C::LDQ + TT * C::LDV) + tail +
                        (a.map_kq ? sizeof(float) * 4 * (2 * a.N - 1 + GR_DTS_COPIES * dts_stride(a.nb + 1)) : 0);
  constexpr int LDV_Q = 32 * ((C::VP - 2 + 31) / 32) + 2;
  const size_t lds_q = sizeof(float) * (TT * C::LDQ + TT * LDV_Q) + tail;
  GR_REQUIRE(lds_kv <= 160 * 1024 && lds_q <= 160 * 1024,
             "hstu_attn_bwd: LDS (%zu, %zu B) exceeds 160 KiB (N=%d)", lds_kv, lds_q, a.N);
  const bool split = option(GR_OPT_ATTN_BWD_SPLIT) != 0;
  // Tile pairs (p, T-1-p) per workgroup when the single-tile grid needs more than one
  // round and the paired grid is resident in one: every workgroup then carries the same
  // causal work and one prologue serves two tiles (C2: 66.8 -> 62.4 us).  Otherwise single
  // tiles, heaviest first (LPT order).
  const int pgrid = ceil_div(a.n_tiles, 2) * a.B * a.H;
  const bool pairs_on = option(GR_OPT_ATTN_BWD_PAIRS) != 0 && a.n_tiles > 1 && TT == 64;
  const bool pairs_force = option(GR_OPT_ATTN_BWD_PAIRS) == 2 && a.n_tiles > 1 && TT == 64;
  int n_slabs = grid;
  if (TT == 64 && a.ds && a.ds_flags && !split) {
    // one launch: the dQ workgroups consume each key tile's dS as soon as it is published
    auto kern = a.map_kq ? attn_bwd_fused_ds_kernel<KS, VT, TT, true> : attn_bwd_fused_ds_kernel<KS, VT, TT, false>;
    AttnBwdArgs af = a;
    const size_t lds = (lds_kv > lds_q ? lds_kv : lds_q) + 16;
    af.paired = pairs_force;  // key-major pairs only on request (PAIRS = 2)
    const int g = af.paired ? pgrid : grid;
    n_slabs = g;
    zero_words_async(a.ds_flags, (int64_t)a.B * a.H * a.n_tiles, st);
    GR_TIMED("attn_bwd", st, hipLaunchKernelGGL(kern, dim3(g + grid), dim3(256), lds, st, af, g));
    GR_LAUNCH_CHECK("hstu_attn_bwd(fused dS)");
  } else if (a.ds && !split) {
    // two passes: dK/dV (+ dS tiles), then dQ = dS K with nothing recomputed (narrow heads
    // with GR_OPT_ATTN_BWD_DS = 1; wide heads by default, GR_OPT_ATTN_BWD_WIDE_DS)
    AttnBwdArgs akv = a, aq = a;
    if (TT == 16 && option(GR_OPT_ATTN_BWD_WIDE_SPLIT) == 2) {
      // wide heads: a dV launch (no histograms in LDS) then a dK launch
      auto kv = a.map_kq ? attn_bwd_dv_kernel<KS, VT, TT> : attn_bwd_dv_nobias_kernel<KS, VT, TT>;
      auto kk = a.map_kq ? attn_bwd_dk_kernel<KS, VT, TT, true> : attn_bwd_dk_kernel<KS, VT, TT, false>;
      akv.paired = 0;
      n_slabs = grid;
      const size_t lds_v = sizeof(float) * (TT * C::LDQ + TT * C::LDV) + tail;
      GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kv, dim3(grid), dim3(256), lds_v, st, akv));
      GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kk, dim3(grid), dim3(256), lds_kv, st, akv));
    } else if (TT == 16 && option(GR_OPT_ATTN_BWD_WIDE_SPLIT) != 0) {
      // wide heads: dV and dK workgroups (single tiles, heaviest first)
      auto ksp = a.map_kq ? attn_bwd_dkv_split_kernel<KS, VT, TT, true> : attn_bwd_dkv_split_kernel<KS, VT, TT, false>;
      akv.paired = 0;
      n_slabs = grid;
      GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(ksp, dim3(2 * grid), dim3(256), lds_kv, st, akv));
    } else {
      auto kkv = a.map_kq ? attn_bwd_dkv_kernel<KS, VT, TT, true> : attn_bwd_dkv_kernel<KS, VT, TT, false>;
      const int s_kv = device_cus() * resident_wgs(kkv, lds_kv);
      akv.paired = pairs_force || (pairs_on && grid > s_kv && pgrid <= s_kv);
      n_slabs = akv.paired ? pgrid : grid;
      GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kkv, dim3(n_slabs), dim3(256), lds_kv, st, akv));
    }
    GR_LAUNCH_CHECK("hstu_attn_bwd(dkv)");
    aq.paired = 0;
    // narrow heads: one wave per 16-query block, no LDS
    const size_t lds_dq = TT == 64 ? 0 : sizeof(float) * TT * C::LDQ + 16;
    const int grid_dq = grid;  // TT = 64: 4 query blocks per workgroup (one 64-row tile)
    const int nbias = a.map_kq ? ceil_div(nbins, 16) : 0;  // the slab reduce rides along
    if constexpr (TT == 64 && VT == 4 && (KS == 13 || KS == 16)) {
      if (bnd && a.H == 1)
        return launch_dq_bnd<KS, VT>(aq, *bnd, grid_dq, nbias, n_slabs, dpos_w, dts_w, st);
    }
    GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL((attn_bwd_dq_ds_kernel<KS, VT, TT>), dim3(grid_dq + nbias), dim3(256),
                                                   lds_dq, st, aq, nbias, n_slabs, dpos_w, dts_w));
    GR_LAUNCH_CHECK("hstu_attn_bwd(dq from dS)");
    return 0;
  } else if (!split && C::KT <= 8) {
    const size_t lds = lds_kv > lds_q ? lds_kv : lds_q;
    auto kern = a.map_kq ? attn_bwd_fused_kernel<KS, VT, TT, true> : attn_bwd_fused_kernel<KS, VT, TT, false>;
    AttnBwdArgs af = a;
    const int slots = device_cus() * resident_wgs(kern, lds);
    af.paired = pairs_force || (pairs_on && 2 * grid > slots && 2 * pgrid <= slots);
    const int g = af.paired ? pgrid : grid;
    n_slabs = g;
    GR_TIMED("attn_bwd", st, hipLaunchKernelGGL(kern, dim3(2 * g), dim3(256), lds, st, af, g));
    GR_LAUNCH_CHECK("hstu_attn_bwd(fused)");
  } else {
    auto kkv = a.map_kq ? attn_bwd_dkv_kernel<KS, VT, TT, true> : attn_bwd_dkv_kernel<KS, VT, TT, false>;
    auto kq = a.map_qk ? attn_bwd_dq_kernel<KS, VT, TT, true> : attn_bwd_dq_kernel<KS, VT, TT, false>;
    AttnBwdArgs akv = a, aq = a;
    const int s_kv = device_cus() * resident_wgs(kkv, lds_kv), s_q = device_cus() * resident_wgs(kq, lds_q);
    akv.paired = pairs_force || (pairs_on && grid > s_kv && pgrid <= s_kv);
    aq.paired = pairs_force || (pairs_on && grid > s_q && pgrid <= s_q);
    n_slabs = akv.paired ? pgrid : grid;
    GR_TIMED("attn_bwd_dkv", st, hipLaunchKernelGGL(kkv, dim3(n_slabs), dim3(256), lds_kv, st, akv));
    GR_LAUNCH_CHECK("hstu_attn_bwd(dkv)");
    GR_TIMED("attn_bwd_dq", st, hipLaunchKernelGGL(kq, dim3(aq.paired ? pgrid : grid), dim3(256), lds_q, st, aq));
    GR_LAUNCH_CHECK("hstu_attn_bwd(dq)");
  }
  if (a.map_kq) {
    GR_TIMED("attn_bias_reduce", st, hipLaunchKernelGGL(bias_grad_reduce_kernel, dim3(ceil_div(nbins, 16)), dim3(256), 0, st,
                       a.slabs, n_slabs, 2 * a.N - 1, a.nb + 1, dpos_w, dts_w));
    GR_LAUNCH_CHECK("hstu_attn_bwd(bias reduce)");
  }
  return 0;
}

}  // namespace gr

#ifdef GR_STAMP
extern "C" __attribute__((visibility("default"))) int gr_stamp_read(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gr::gr_stamp_buf), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
extern "C" __attribute__((visibility("default"))) int gr_timeline_read(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gr::gr_tl_buf), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#endif

extern "C" size_t hstu_attn_bwd_workspace_size(int B, int N, int max_len, int H,
                                               int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0) return 0;
  const size_t ds = gr::bwd_ds_bytes(B, N, H);
  return ds ? gr::bwd_ds_offset(B, N, max_len, H, num_buckets) + ds + gr::bwd_flag_bytes(B, max_len, H)
            : gr::bwd_slab_bytes(B, N, max_len, H, num_buckets);
}

extern "C" size_t hstu_attn_bwd_workspace_size_d(int B, int N, int max_len, int H, int dqk,
                                                 int dv, int num_buckets) {
  if (B <= 0 || N <= 0 || H <= 0 || max_len <= 0 || dqk <= 0 || dv <= 0) return 0;
  if (!gr::wide_heads(dqk, dv)) return hstu_attn_bwd_workspace_size(B, N, max_len, H, num_buckets);
  const size_t ds = gr::bwd_ds_bytes_d(B, N, H, dqk, dv);
  return ds ? gr::bwd_ds_offset(B, N, max_len, H, num_buckets) + ds
            : gr::bwd_slab_bytes(B, N, max_len, H, num_buckets);
}

namespace gr {
static int attn_bwd_impl(const float* q, const float* k, const float* v, int64_t ld_qk,
                         int64_t ld_v, const float* dout, int64_t ld_dout,
                         const int64_t* offsets, int B, int N, int max_len, int H, int dqk,
                         int dv, const uint8_t* bucket_map, const float* pos_w,
                         const float* ts_w, int num_buckets, const float* hq,
                         const float* hk, const float* hv, int64_t ld_h, float* dq,
                         float* dk, float* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                         void* workspace, size_t ws_bytes, void* stream, BndCtx* bnd) {
  GR_REQUIRE(q && k && v && dout && offsets && dq && dk && dvv, "hstu_attn_bwd: null pointer");
  GR_REQUIRE(B >= 0 && N > 0 && H > 0 && dqk > 0 && dv > 0, "hstu_attn_bwd: bad sizes");
  GR_REQUIRE(max_len >= 0 && max_len <= N, "hstu_attn_bwd: max_len %d not in [0, N=%d]", max_len, N);
  GR_REQUIRE(dqk <= 256 && dv <= 256, "hstu_attn_bwd: dqk/dv > 256 unsupported (%d, %d)", dqk, dv);
  GR_REQUIRE((hq == nullptr) == (hk == nullptr) && (hk == nullptr) == (hv == nullptr),
             "hstu_attn_bwd: hq/hk/hv must be all given or all NULL");
  if (bucket_map) {
    GR_REQUIRE(pos_w && ts_w && dpos_w && dts_w && num_buckets > 0 && num_buckets < 256,
               "hstu_attn_bwd: bucket_map given without pos_w/ts_w/dpos_w/dts_w");
    const size_t need = bwd_slab_bytes(B, N, max_len, H, num_buckets);
    GR_REQUIRE(workspace && ws_bytes >= need, "hstu_attn_bwd: workspace %zu B < %zu B", ws_bytes, need);
  }
  hipStream_t st = (hipStream_t)stream;
  if (B == 0 || max_len == 0) {
    if (bucket_map) {
      zero_words_async(dpos_w, 2 * N - 1, st);
      zero_words_async(dts_w, num_buckets + 1, st);
    }
    return 0;
  }
  const uint8_t* map_kq =
      bucket_map ? bucket_map + (size_t)B * attn_tiles_per_seq(N) * 4096 : nullptr;
  AttnBwdArgs a{q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, H, dqk, dv,
                ceil_div(max_len, 64), bucket_map, map_kq, pos_w, ts_w,
                bucket_map ? num_buckets : 0, hq, hk, hv, ld_h, dq, dk, dvv, ld_d,
                bucket_map ? (float*)workspace : nullptr, 1.0f / (float)N, 0};
  // snake pairing only when the grid is resident in <= 2 rounds; otherwise plain
  // heaviest-first (dynamic dispatch = longest-processing-time order)
  a.cus = (int64_t)a.n_tiles * B * H <= 2 * device_cus() ? device_cus() : (1 << 30);
  a.vec2 = pair_aligned({q, k, v, dout}, {ld_qk, ld_v, ld_dout, dqk, dv});
  a.vec2h = hq ? pair_aligned({hq, hk, hv}, {ld_h, dqk, dv}) : 0;
  // a workspace large enough for the dS tiles: two-pass backward (short sequences with
  // GR_OPT_ATTN_BWD_DS and a bucket map; wide heads at any N, GR_OPT_ATTN_BWD_WIDE_DS)
  const bool wide = wide_heads(dqk, dv);
  const size_t ds_b = bwd_ds_bytes_d(B, N, H, dqk, dv);
  if (workspace && ds_b && (bucket_map || wide) &&
      ws_bytes >= bwd_ds_offset(B, N, max_len, H, num_buckets) + ds_b) {
    a.ds = (float*)((char*)workspace + bwd_ds_offset(B, N, max_len, H, num_buckets));
    a.ds_tps = ds_tiles_per_seq(N);
    const size_t fo = (bwd_ds_offset(B, N, max_len, H, num_buckets) + ds_b + 255) & ~(size_t)255;
    if (!wide && option(GR_OPT_ATTN_BWD_DS) == 2 && ws_bytes >= fo + bwd_flag_bytes(B, max_len, H) - 256)
      a.ds_flags = (uint32_t*)((char*)workspace + fo);
  }
  const int d = dqk > dv ? dqk : dv;
  if (d <= 8) return launch_bwd<2, 1>(a, dpos_w, dts_w, st, bnd);
  if (d <= 16) return launch_bwd<4, 1>(a, dpos_w, dts_w, st, bnd);
  if (d <= 32) return launch_bwd<8, 2>(a, dpos_w, dts_w, st, bnd);
  if (d <= 52) return launch_bwd<13, 4>(a, dpos_w, dts_w, st, bnd);
  if (d <= 64) return launch_bwd<16, 4>(a, dpos_w, dts_w, st, bnd);
  if (d <= 128) return launch_bwd<32, 8>(a, dpos_w, dts_w, st, bnd);
  return launch_bwd<64, 16, 16>(a, dpos_w, dts_w, st, bnd);
}
}  // namespace gr

extern "C" int hstu_attn_bwd(const float* q, const float* k, const float* v, int64_t ld_qk,
                             int64_t ld_v, const float* dout, int64_t ld_dout,
                             const int64_t* offsets, int B, int N, int max_len, int H, int dqk,
                             int dv, const uint8_t* bucket_map, const float* pos_w,
                             const float* ts_w, int num_buckets, const float* hq,
                             const float* hk, const float* hv, int64_t ld_h, float* dq,
                             float* dk, float* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                             void* workspace, size_t ws_bytes, void* stream) {
  return gr::attn_bwd_impl(q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, max_len, H, dqk, dv,
                           bucket_map, pos_w, ts_w, num_buckets, hq, hk, hv, ld_h, dq, dk, dvv, ld_d,
                           dpos_w, dts_w, workspace, ws_bytes, stream, nullptr);
}

extern "C" int hstu_attn_bwd_bnd(const float* q, const float* k, const float* v, int64_t ld_qk,
                                 int64_t ld_v, const float* dout, int64_t ld_dout,
                                 const int64_t* offsets, int B, int N, int max_len, int H, int dqk,
                                 int dv, const uint8_t* bucket_map, const float* pos_w,
                                 const float* ts_w, int num_buckets, const float* hq,
                                 const float* hk, const float* hv, int64_t ld_h, float* dq,
                                 float* dk, float* dvv, int64_t ld_d, float* dpos_w, float* dts_w,
                                 void* workspace, size_t ws_bytes, const GrBoundaryBwd* bnd,
                                 void* stream) {
  using namespace gr;
  GR_REQUIRE(bnd, "hstu_attn_bwd_bnd: null boundary");
  const GrBoundaryBwd& g = *bnd;
  GR_REQUIRE(g.dh && g.w_uvqk && g.x && g.x_stats && g.dx && g.D > 0 && g.n_out > 0,
             "hstu_attn_bwd_bnd: boundary null pointer or bad sizes");
  GR_REQUIRE(g.hdv == 0 || (g.w_o && g.u && g.attn && g.attn_stats && g.du && g.d_attn),
             "hstu_attn_bwd_bnd: gate_o backward null pointer");
  // the epilogue form: narrow single-head boundary shapes the row-wave ops instantiate
  BndCtx bc{};
  bc.a1 = RwArgsLnUvqkBwd{offsets, B, g.n_out, g.D, g.dh, g.ld_dh, g.w_uvqk, g.x, g.ld_x,
                          (const float2*)g.x_stats, g.dy_res, g.ld_dy, g.dx, g.ld_dx};
  bc.op2 = g.hdv > 0;
  if (bc.op2)
    bc.a2 = RwArgsGateOBwd{offsets, B, g.D, g.hdv, g.dx, g.ld_dx, g.w_o, g.u, g.ld_u, g.attn,
                           g.ld_attn, (const float2*)g.attn_stats, g.h_u, g.ld_h, g.dropout_p,
                           g.seed, g.seed_offset, g.du, g.ld_du, g.d_attn, g.ld_da};
  const int ng = ceil_div(g.n_out, 16);
  bc.kg1 = ng > 8 && ng <= 13 ? 13 : ng > 13 && ng <= 16 ? 16 : -1;
  auto in_w4 = [](int x) { return x > 32 && x <= 64; };  // the W = 4 (64-column) instantiation
  const bool aligned = pair_aligned({g.dh, g.x, g.dy_res, g.dx, g.u, g.attn, g.h_u, g.du, g.d_attn},
                                    {g.ld_dh, g.ld_x, g.ld_dy, g.ld_dx, g.ld_u, g.ld_attn, g.ld_h,
                                     g.ld_du, g.ld_da, g.n_out, g.D, g.hdv});
  // the epilogue reads the rows' d_uvqk from dh right after the dQ stores: only when dq,
  // dk and dv are column slices of dh (the layout ops.py uses); any other layout runs the
  // two calls, which are correct for every layout
  auto in_dh = [&](const float* p) {
    return p >= g.dh && p < g.dh + g.ld_dh && ld_d == g.ld_dh;
  };
  const bool alias_ok = in_dh(dq) && in_dh(dk) && in_dh(dvv);
  const bool fuse = option(GR_OPT_BOUNDARY_FUSE) != 0 && option(GR_OPT_ROWWAVE) != 0 && H == 1 &&
                    bc.kg1 > 0 && in_w4(g.D) && (!bc.op2 || in_w4(g.hdv)) && aligned && alias_ok &&
                    g.max_rows * 4 * 1024 <= 0x7fffffffLL;
  if (int rc = attn_bwd_impl(q, k, v, ld_qk, ld_v, dout, ld_dout, offsets, B, N, max_len, H, dqk, dv,
                             bucket_map, pos_w, ts_w, num_buckets, hq, hk, hv, ld_h, dq, dk, dvv,
                             ld_d, dpos_w, dts_w, workspace, ws_bytes, stream, fuse ? &bc : nullptr))
    return rc;
  if (bc.fused) return 0;
  if (g.hdv > 0)
    return hstu_boundary_bwd(g.dh, g.ld_dh, offsets, B, g.max_rows, g.D, g.n_out, g.w_uvqk, g.x,
                             g.ld_x, g.x_stats, g.dy_res, g.ld_dy, g.dx, g.ld_dx, g.hdv, g.w_o, g.u,
                             g.ld_u, g.attn, g.ld_attn, g.attn_stats, g.h_u, g.ld_h, g.dropout_p,
                             g.seed, g.seed_offset, g.du, g.ld_du, g.d_attn, g.ld_da, stream);
  return hstu_ln_uvqk_bwd(g.dh, g.ld_dh, offsets, B, g.max_rows, g.D, g.n_out, g.w_uvqk, g.x, g.ld_x,
                          g.x_stats, g.dy_res, g.ld_dy, g.dx, g.ld_dx, stream);
}
