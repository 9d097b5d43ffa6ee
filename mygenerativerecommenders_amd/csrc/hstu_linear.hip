// Fused projection GEMMs of the STU layer — gfx950, f32 MFMA (v_mfma_f32_16x16x4_f32).
//
// Reference: sequential_encoders/hstu.py:258-305 (LayerNorm -> mm(_uvqk) -> silu) and
// hstu.py:393-413 (u * LayerNorm(attn) -> dropout -> Linear _o -> + x), plus their
// autograd backward.  Each reference chain of 3-6 ATen kernels (and their backward)
// is one launch here:
//   hstu_ln_uvqk_fwd : row stats of x, (x-mu)*rstd staged on the fly, GEMM, silu epilogue
//   hstu_gate_o_fwd  : row stats of attn, u*LN(attn)*dropout staged on the fly, GEMM,
//                      bias + residual epilogue
//   hstu_gate_o_bwd  : dy @ W_o, epilogue = dropout bwd + gating bwd + LayerNorm bwd
//                      (row reductions in registers) + silu' of u
//   hstu_ln_uvqk_bwd : dh @ W_uvqk^T, epilogue = LayerNorm bwd + residual
//   gr_wgrad         : weight gradients A^T B (K = all rows) as split-M partial slabs
//                      reduced in a fixed order (deterministic, no atomics)
//
// Row-panel GEMM core: a 256-thread workgroup owns 64 rows (wave w: rows 16w..16w+15)
// and a panel of up to 256 output columns; K is streamed in chunks of 16 through LDS.
// A operand layout (row stride 18 == 18 mod 32) and B layout (stride == 16 mod 32) make
// the per-k-step ds_read_b32 of both operands bank-conflict-free.
#include <type_traits>

#include "common.h"
#include "attn_common.h"
#include "rowwave.h"

#include "../../include/gr_hstu.h"

namespace gr {

constexpr int BM = 64;
constexpr int BK = 16;
constexpr int LDA = BK + 2;

template <int NT>
struct PanelCfg {
  static constexpr int BN = NT * 16;
  static constexpr int LDB = (NT & 1) ? BN : BN + 16;  // == 16 mod 32
};

// Every global load below is UNCONDITIONAL (indices clamped into the valid range, the
// value masked afterwards): a guarded load makes hipcc branch around it and wait
// vmcnt(0) per element, serialising dozens of L2 round trips per tile.

// LayerNorm statistics of one row whose 16 lanes hold 16 values each (value j = column
// 16 j + sub, zero past K): a fixed summation order with fp contraction off, so the
// statistics pass below and gate_o's a16 epilogue (y_stats) give identical values.
__device__ __forceinline__ float2 ln_stats16(const float (&v)[16], int sub, int K, float eps) {
#pragma clang fp contract(off)
  const float invk = 1.f / (float)K;
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < 4; ++it) s += (v[4 * it] + v[4 * it + 1]) + (v[4 * it + 2] + v[4 * it + 3]);
  s = sum16(s);
  const float mean = s * invk;
  float q = 0.f;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    float d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = 4 * it + u;
      d[u] = 16 * j + sub < K ? v[j] - mean : 0.f;
    }
    q += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
  }
  q = sum16(q);
  return make_float2(mean, rsqrtf(q * invk + eps));
}

// Row statistics (mean, rstd) of rows [m0, m0+64) over K columns: wave w owns 16 rows,
// 4 at a time with 16 lanes per row; loads issued 4-deep before the reductions.
__device__ __forceinline__ void panel_row_stats(const float* base, int64_t ld, int64_t m0,
                                                int64_t total, int K, float eps,
                                                float2* st_lds, float2* st_glob) {
  gptr<float> src = as_global(base);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane & 15, rq = lane >> 4;
  const int64_t mlast = total - 1;
  const float invk = 1.f / (float)K;
  if (K <= 256) {
    // all 4 x 16 values of the lane's 4 rows issued before any reduction (the loop form
    // below is a chain of 2 x 4 x K/64 dependent round trips: ~30 us per workgroup at
    // K = 256); padding columns are 0, so the sums — in the same order — are unchanged
    float v[4][16];
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int64_t m = m0 + w * 16 + pass * 4 + rq;
      gptr<float> row = src + (m < mlast ? m : mlast) * ld;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = 16 * j + sub;
        v[pass][j] = row[k < K ? k : K - 1];
      }
    }
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int r = w * 16 + pass * 4 + rq;
      const int64_t m = m0 + r;
#pragma unroll
      for (int j = 0; j < 16; ++j) v[pass][j] = 16 * j + sub < K ? v[pass][j] : 0.f;
      const float2 mr = ln_stats16(v[pass], sub, K, eps);
      if (sub == 0) {
        st_lds[r] = mr;
        if (st_glob && m < total) st_glob[m] = mr;
      }
    }
    return;
  }
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = w * 16 + pass * 4 + rq;
    const int64_t m = m0 + r;
    const int64_t mc = m < mlast ? m : mlast;
    gptr<float> row = src + mc * ld;
    float s = 0.f;
    for (int k0 = 0; k0 < K; k0 += 64) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + 16 * u + sub;
        v[u] = row[k < K ? k : K - 1];
        v[u] = k < K ? v[u] : 0.f;
      }
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    s = sum16(s);
    const float mean = s * invk;
    float q = 0.f;
    for (int k0 = 0; k0 < K; k0 += 64) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + 16 * u + sub;
        v[u] = row[k < K ? k : K - 1] - mean;
        v[u] = k < K ? v[u] : 0.f;
      }
      q += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
    }
    q = sum16(q);
    const float rstd = rsqrtf(q * invk + eps);
    if (sub == 0) {
      st_lds[r] = make_float2(mean, rstd);
      if (st_glob && m < total) st_glob[m] = make_float2(mean, rstd);
    }
  }
}

// One A element of EB bytes (4: fp32, 2: bf16 -- the bf16-activation ops, Op::A0_BYTES)
template <int EB>
__device__ __forceinline__ float buf_ld_e(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (EB == 2)
    return __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0) << 16);
  else
    return buf_ld(r, voff, soff);
}

// Generic row-panel GEMM: C[m, n] = sum_k A'(m, k) * W'(k, n), epilogue by Op.
// K streams through LDS in chunks of 16 with the next chunk prefetched into registers
// (LDS-only barriers keep the prefetch in flight across the MFMA phase).  All operand
// loads go through buffer descriptors: A rows from m0 (rows past the end read 0), one
// voffset VGPR per thread with the row / k steps in SGPR soffsets; the raw values are
// transformed (LayerNorm, gating, dropout) when they are written to LDS.
//   Op: a_rsrc0/1(m0, total), a_ld0/1(), NSRC, a_xform(v0, v1, m, k, stats, valid),
//       w, bks(), bns()  (W'(k, n) = w[k * bks + n * bns]), prologue, epilogue.
template <int NT, int BKT, class Op>
__global__ __launch_bounds__(256) void rowpanel_kernel(Op op) {
  // BKT = K chunk per LDS stage: 16, or 64 when K is small enough for one or a few
  // chunks (ml-1m: K = 50 in one stage, K = 200 in 4) so the next chunk's global loads
  // are not exposed once per 16 columns of K
  using P = PanelCfg<NT>;
  constexpr int LDAT = BKT == 16 ? LDA : BKT + 4;  // 64-bank LDS: BKT + 4 == 4 mod 64
  constexpr int NP2 = P::BN <= 16 ? 16 : P::BN <= 32 ? 32 : P::BN <= 64 ? 64 : P::BN <= 128 ? 128 : 256;
  // B staging walks the memory-contiguous index fastest: n for row-major W' (RPB k-rows
  // per pass), k for transposed W' (BKT k per column, CPP columns per pass)
  constexpr int RPB = 256 / NP2;
  constexpr int CPP = 256 / BKT;
  constexpr int NB = Op::B_N_CONTIG ? (BKT + RPB - 1) / RPB : (P::BN + CPP - 1) / CPP;
  constexpr int RPA = 256 / BKT;  // A rows per pass
  constexpr int NA = BM / RPA;
  __shared__ __attribute__((aligned(16))) float As[BM * LDAT];
  __shared__ __attribute__((aligned(16))) float Bs[BKT * P::LDB];
  __shared__ float2 stats[BM];
  const int64_t total = op.offsets[op.B];
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  if (m0 >= total) return;
  const int n0 = blockIdx.y * P::BN;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;

  op.prologue(m0, total, stats);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t ra0 = op.a_rsrc0(m0, total);
  const __amdgpu_buffer_rsrc_t ra1 = op.a_rsrc1(m0, total);
  const int ld0 = (int)op.a_ld0(), ld1 = (int)op.a_ld1();
  const int a_c = tid % BKT, a_r = tid / BKT;  // A: column k0 + a_c of rows a_r + RPA i
  const int va0 = (a_r * ld0 + a_c) * 4, va1 = (a_r * ld1 + a_c) * 4;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)op.w, 0, op.K * op.N * 4, 0x00020000);
  const int bks = op.bks(), bns = op.bns();
  const int b_c = Op::B_N_CONTIG ? tid % NP2 : tid / BKT;  // B: column n0 + b_c (+CPP i)
  const int b_r = Op::B_N_CONTIG ? tid / NP2 : tid % BKT;  // of k-row b_r (+RPB i)
  const bool b_col = Op::B_N_CONTIG ? (b_c < P::BN && n0 + b_c < op.N) : true;
  const int vb = b_col ? (b_r * bks + (n0 + b_c) * bns) * 4 : OOB_OFF;

  float ra[NA], ra2[Op::NSRC == 2 ? NA : 1], rb[NB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      ra[i] = buf_ld(ra0, va0 + k0 * 4, i * RPA * ld0 * 4);
      if constexpr (Op::NSRC == 2) ra2[i] = buf_ld(ra1, va1 + k0 * 4, i * RPA * ld1 * 4);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (Op::B_N_CONTIG)
        rb[i] = buf_ld(rw, vb, (k0 + RPB * i) * bks * 4);
      else
        rb[i] = buf_ld(rw, vb, (k0 * bks + CPP * i * bns) * 4);
    }
  };
  auto store = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = a_r + RPA * i, k = k0 + a_c;
      const bool ok = m0 + r < total && k < op.K;
      const float v = op.a_xform(ra[i], Op::NSRC == 2 ? ra2[Op::NSRC == 2 ? i : 0] : 0.f, m0 + r, k,
                                 stats[r], ok);
      As[r * LDAT + a_c] = ok ? v : 0.f;
    }
    if constexpr (Op::B_N_CONTIG) {
      if (b_c < P::BN) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int kk = b_r + RPB * i;
          if (RPB * NB == BKT || kk < BKT)
            Bs[kk * P::LDB + b_c] = (b_col && k0 + kk < op.K) ? rb[i] : 0.f;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = b_c + CPP * i;
        if (CPP * NB == P::BN || c < P::BN)
          Bs[b_r * P::LDB + c] = (n0 + c < op.N && k0 + b_r < op.K) ? rb[i] : 0.f;
      }
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  // the epilogue's own row inputs (LayerNorm-backward rows, residuals), issued before the
  // K loop so they land during it instead of adding a round trip at the workgroup's end;
  // when they are many (more than 64 per lane: the C3 LayerNorm-backward panel holds 136,
  // ~300 registers with the accumulators, one wave per SIMD) the epilogue streams them
  // row by row after the loop instead
  constexpr bool STREAM_EPI = sizeof(typename Op::template Epi<NT>) > 64 * sizeof(float);
  typename Op::template Epi<NT> es;
  if constexpr (!STREAM_EPI) op.epi_load(es, m0 + w * 16 + 4 * lg, n0 + lr, total);

  auto chunk = [&](int k0, bool more) {
    if (more) load(k0 + BKT);
    const float* arow = As + (w * 16 + lr) * LDAT + lg;
    // operands of k-step ks+1 read from LDS while the MFMAs of step ks run; steps past
    // K (zero padding) are skipped when the whole K fits one stage
    const int ksn = more || BKT == 16 ? BKT / 4 : (op.K - k0 + 3) / 4;
    float av[2], bv[2][NT];
    av[0] = arow[0];
#pragma unroll
    for (int t = 0; t < NT; ++t) bv[0][t] = Bs[lg * P::LDB + lr + t * 16];
#pragma unroll
    for (int ks = 0; ks < BKT / 4; ++ks) {
      if (ks < ksn) {
        if (ks + 1 < BKT / 4) {
          av[(ks + 1) & 1] = arow[4 * (ks + 1)];
          const float* brow = Bs + (4 * (ks + 1) + lg) * P::LDB + lr;
#pragma unroll
          for (int t = 0; t < NT; ++t) bv[(ks + 1) & 1][t] = brow[t * 16];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(av[ks & 1], bv[ks & 1][t], acc[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    lds_barrier();
    if (more) {
      store(k0 + BKT);
      lds_barrier();
    }
  };

  load(0);
  store(0);
  lds_barrier();
  int k0 = 0;
  for (; k0 + BKT < op.K; k0 += BKT) chunk(k0, true);
  chunk(k0, false);
  // acc[t][r] = C[m0 + 16w + 4lg + r][n0 + 16t + lr]
  if constexpr (STREAM_EPI)
    op.epilogue_stream(acc, m0 + w * 16 + 4 * lg, n0 + lr, total);
  else
    op.epilogue(acc, es, m0 + w * 16 + 4 * lg, n0 + lr, total);
}

// bf16-operand row panel (autocast_dtype = bfloat16: the projections' matmuls in bf16
// as torch.autocast runs them, accumulation, LN, activations and epilogues in fp32).
// Same Op interface and output layout as rowpanel_kernel; K streams in chunks of 32
// (one v_mfma_f32_16x16x32_bf16 k-step): the transformed A values and the weight tile
// are rounded to bf16 when written to LDS, both as [row][k] images (A rows, weight
// columns) so each lane's 8 k-values are one 16-byte LDS read; row stride 40 bf16 (80 B:
// the 16 lanes of a read phase hit 16 distinct 16-byte bank groups).  Two LDS buffers:
// chunk k+1 is written into the other buffer right after chunk k's MFMAs, so one
// barrier per chunk.
template <int NT, class Op>
__global__ __launch_bounds__(256) void rowpanel_bf16_kernel(Op op) {
  using P = PanelCfg<NT>;
  constexpr int BKT = 32;
  constexpr int LDK = BKT + 8;  // bf16 elements per LDS row
  constexpr int NP2 = P::BN <= 16 ? 16 : P::BN <= 32 ? 32 : P::BN <= 64 ? 64 : P::BN <= 128 ? 128 : 256;
  constexpr int RPB = 256 / NP2;
  constexpr int CPP = 256 / BKT;
  constexpr int NB = Op::B_N_CONTIG ? (BKT + RPB - 1) / RPB : (P::BN + CPP - 1) / CPP;
  constexpr int RPA = 256 / BKT;
  constexpr int NA = BM / RPA;
  __shared__ __attribute__((aligned(16))) __bf16 As2[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) __bf16 Bs2[2][P::BN * LDK];
  __shared__ float2 stats[BM];
  const int64_t total = op.offsets[op.B];
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  if (m0 >= total) return;
  const int n0 = blockIdx.y * P::BN;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;

  op.prologue(m0, total, stats);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t ra0 = op.a_rsrc0(m0, total);
  const __amdgpu_buffer_rsrc_t ra1 = op.a_rsrc1(m0, total);
  const int ld0 = (int)op.a_ld0(), ld1 = (int)op.a_ld1();
  const int a_c = tid % BKT, a_r = tid / BKT;
  constexpr int E0 = Op::A0_BYTES;  // bytes per element of the first A source
  const int va0 = (a_r * ld0 + a_c) * E0, va1 = (a_r * ld1 + a_c) * 4;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)op.w, 0, op.K * op.N * 4, 0x00020000);
  const int bks = op.bks(), bns = op.bns();
  const int b_c = Op::B_N_CONTIG ? tid % NP2 : tid / BKT;
  const int b_r = Op::B_N_CONTIG ? tid / NP2 : tid % BKT;
  const bool b_col = Op::B_N_CONTIG ? (b_c < P::BN && n0 + b_c < op.N) : true;
  const int vb = b_col ? (b_r * bks + (n0 + b_c) * bns) * 4 : OOB_OFF;
  // B16 (the a16 ops): the weight as a bf16 [N][K] image (op.w16, K % 8 == 0); thread t
  // moves the 16-byte pieces p = t + 256 i (column p / 4, k-octet p % 4) of a chunk, which
  // land in the [column][k] LDS image unchanged
  constexpr bool B16 = Op::B16;
  constexpr int NB16 = B16 ? (P::BN * 4 + 255) / 256 : 1;
  const __amdgpu_buffer_rsrc_t rw16 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)op.w16, 0, B16 ? op.K * op.N * 2 : 0, 0x00020000);

  float ra[NA], ra2[Op::NSRC == 2 ? NA : 1], rb[B16 ? 1 : NB];
  u32x4_t rb16[NB16];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      ra[i] = buf_ld_e<E0>(ra0, va0 + k0 * E0, i * RPA * ld0 * E0);
      if constexpr (Op::NSRC == 2) ra2[i] = buf_ld(ra1, va1 + k0 * 4, i * RPA * ld1 * 4);
    }
    if constexpr (B16) {
#pragma unroll
      for (int i = 0; i < NB16; ++i) {
        const int p = tid + 256 * i, c = p >> 2, o = p & 3;
        const bool ok = p < P::BN * 4 && n0 + c < op.N && k0 + 8 * o < op.K;
        rb16[i] = __builtin_amdgcn_raw_buffer_load_b128(rw16, ok ? ((n0 + c) * op.K + k0 + 8 * o) * 2 : OOB_OFF, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (Op::B_N_CONTIG)
        rb[B16 ? 0 : i] = buf_ld(rw, vb, (k0 + RPB * i) * bks * 4);
      else
        rb[B16 ? 0 : i] = buf_ld(rw, vb, (k0 * bks + CPP * i * bns) * 4);
    }
  };
  auto store = [&](int k0, int buf) {
    __bf16* As = As2[buf];
    __bf16* Bs = Bs2[buf];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = a_r + RPA * i, k = k0 + a_c;
      const bool ok = m0 + r < total && k < op.K;
      const float v = op.a_xform(ra[i], Op::NSRC == 2 ? ra2[Op::NSRC == 2 ? i : 0] : 0.f, m0 + r, k,
                                 stats[r], ok);
      As[r * LDK + a_c] = (__bf16)(ok ? v : 0.f);
    }
    if constexpr (B16) {
#pragma unroll
      for (int i = 0; i < NB16; ++i) {
        const int p = tid + 256 * i;
        if ((P::BN * 4) % 256 == 0 || p < P::BN * 4)
          *reinterpret_cast<u32x4_t*>(Bs + (p >> 2) * LDK + 8 * (p & 3)) = rb16[i];
      }
    } else if constexpr (Op::B_N_CONTIG && RPB == 1) {
      // a thread owns one weight column's 32 k-values: 16 packed pair stores
      if (b_c < P::BN) {
#pragma unroll
        for (int i = 0; i < NB; i += 2) {
          const float lo = (b_col && k0 + i < op.K) ? rb[i] : 0.f;
          const float hi = (b_col && k0 + i + 1 < op.K) ? rb[i + 1] : 0.f;
          *reinterpret_cast<uint32_t*>(Bs + b_c * LDK + i) = pack_bf16(lo, hi);
        }
      }
    } else if constexpr (Op::B_N_CONTIG) {
      if (b_c < P::BN) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int kk = b_r + RPB * i;
          if (RPB * NB == BKT || kk < BKT)
            Bs[b_c * LDK + kk] = (__bf16)((b_col && k0 + kk < op.K) ? rb[i] : 0.f);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = b_c + CPP * i;
        if (CPP * NB == P::BN || c < P::BN)
          Bs[c * LDK + b_r] = (__bf16)((n0 + c < op.N && k0 + b_r < op.K) ? rb[i] : 0.f);
      }
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  typename Op::template Epi<NT> es;
  op.epi_load(es, m0 + w * 16 + 4 * lg, n0 + lr, total);

  load(0);
  store(0, 0);
  lds_barrier();
  int buf = 0;
  for (int k0 = 0; k0 < op.K; k0 += BKT) {
    const bool more = k0 + BKT < op.K;
    if (more) load(k0 + BKT);
    const __bf16* As = As2[buf];
    const __bf16* Bs = Bs2[buf];
    const u32x4_t av = *reinterpret_cast<const u32x4_t*>(As + (w * 16 + lr) * LDK + 8 * lg);
    u32x4_t bv[2];
    bv[0] = *reinterpret_cast<const u32x4_t*>(Bs + lr * LDK + 8 * lg);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t + 1 < NT)
        bv[(t + 1) & 1] = *reinterpret_cast<const u32x4_t*>(Bs + (16 * (t + 1) + lr) * LDK + 8 * lg);
      acc[t] = mfma_bf16(av, bv[t & 1], acc[t]);
    }
    if (more) store(k0 + BKT, buf ^ 1);  // the other buffer: last read before the barrier below
    lds_barrier();
    buf ^= 1;
  }
  op.epilogue(acc, es, m0 + w * 16 + 4 * lg, n0 + lr, total);
}

// Wide-shape bf16 row panel (K % 32 == 0, 16-byte aligned rows, 256-column panels: the
// C3 backward projections).  Same tile, LDS images and epilogue as rowpanel_bf16_kernel, with
//  * float4 operand loads: 10 vector-memory instructions per thread per 32-wide chunk
//    instead of 40 (the scalar staging, not the MFMAs, set the chunk time at D = 256);
//  * the epilogue's row inputs issued under the last chunk's MFMAs instead of before the
//    loop, so their registers are not live across it (the LayerNorm-backward panel held
//    128 of them: 256 VGPRs, one workgroup per CU).
// Staging maps (t = thread):
//  A        : k-quad t & 7 of rows t >> 3 and + 32            -> 8-byte LDS stores
//  B k-contig (W'(k, n) = w[k + n bns]): k-quad t & 7 of columns t >> 3 + 32 i, i < 8
//  B n-contig (W'(k, n) = w[k bks + n]): n-quad (lane >> 2) + 16 w of k-rows
//             8 i + 2 (lane & 3) + {0, 1}, i < 4              -> packed (k, k+1) stores
template <class Op>
__global__ __launch_bounds__(256) void rowpanel_bf16v_kernel(Op op) {
  constexpr int NT = 16, BN = 256, BKT = 32, LDK = BKT + 8;
  __shared__ __attribute__((aligned(16))) __bf16 As2[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) __bf16 Bs2[2][BN * LDK];
  __shared__ float2 stats[BM];
  const int64_t total = op.offsets[op.B];
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  if (m0 >= total) return;
  const int n0 = blockIdx.y * BN;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;

  op.prologue(m0, total, stats);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t ra0 = op.a_rsrc0(m0, total);
  const __amdgpu_buffer_rsrc_t ra1 = op.a_rsrc1(m0, total);
  const int ld0 = (int)op.a_ld0(), ld1 = (int)op.a_ld1();
  const int aq = tid & 7, ar = tid >> 3;
  // A0 in bf16 (Op::A0_BYTES == 2, an identity a_xform): the 4 k-values are one 8-byte load
  // whose bits go to LDS unchanged
  constexpr bool A0H = Op::A0_BYTES == 2;
  static_assert(!A0H || Op::A0_RAW, "bf16 A0 rows go to LDS untransformed");
  const int va0 = (ar * ld0 + 4 * aq) * Op::A0_BYTES, va1 = (ar * ld1 + 4 * aq) * 4;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)op.w, 0, op.K * op.N * 4, 0x00020000);
  const int bks = op.bks(), bns = op.bns();
  // k-contiguous: column bc + 32 i, k-quad bq; n-contiguous: n-quad bn, k-pair bp
  const int bq = tid & 7, bc = tid >> 3;
  const int bp = lane & 3, bn = (lane >> 2) + 16 * w;
  int vb;
  if constexpr (Op::B_N_CONTIG)
    vb = n0 + 4 * bn < op.N ? (2 * bp * bks + n0 + 4 * bn) * 4 : OOB_OFF;
  else
    vb = (4 * bq + (n0 + bc) * bns) * 4;

  // B16: the bf16 [N][K] weight image, 16-byte pieces as in rowpanel_bf16_kernel
  constexpr bool B16 = Op::B16;
  const __amdgpu_buffer_rsrc_t rw16 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)op.w16, 0, B16 ? op.K * op.N * 2 : 0, 0x00020000);
  f4 ra[2], ra2[Op::NSRC == 2 ? 2 : 1], rb[B16 ? 1 : 8];
  u32x2_t rh[A0H ? 2 : 1];
  u32x4_t rb16[B16 ? 4 : 1];
  auto ld4 = [](__amdgpu_buffer_rsrc_t r, int v, int s) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, v, s, 0));
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (A0H)
        rh[A0H ? i : 0] = __builtin_amdgcn_raw_buffer_load_b64(ra0, va0 + k0 * 2, i * 32 * ld0 * 2, 0);
      else
        ra[i] = ld4(ra0, va0 + k0 * 4, i * 32 * ld0 * 4);
      if constexpr (Op::NSRC == 2) ra2[Op::NSRC == 2 ? i : 0] = ld4(ra1, va1 + k0 * 4, i * 32 * ld1 * 4);
    }
    if constexpr (B16) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = tid + 256 * i, c = p >> 2, o = p & 3;
        const bool ok = n0 + c < op.N && k0 + 8 * o < op.K;
        rb16[B16 ? i : 0] = __builtin_amdgcn_raw_buffer_load_b128(rw16, ok ? ((n0 + c) * op.K + k0 + 8 * o) * 2 : OOB_OFF, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (Op::B_N_CONTIG)
        rb[B16 ? 0 : i] = ld4(rw, vb, (k0 + 8 * (i >> 1) + (i & 1)) * bks * 4);
      else
        rb[B16 ? 0 : i] = ld4(rw, vb, (k0 + 32 * i * bns) * 4);  // columns >= N: past the range, 0
    }
  };
  auto store = [&](int k0, int buf) {
    __bf16* As = As2[buf];
    __bf16* Bs = Bs2[buf];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = ar + 32 * i;
      const bool rok = m0 + r < total;
      if constexpr (A0H) {  // rows >= total read 0 (descriptor range)
        *reinterpret_cast<u32x2_t*>(As + r * LDK + 4 * aq) = rh[A0H ? i : 0];
        continue;
      }
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 4 * aq + j;
        const float x = op.a_xform(ra[i][j], Op::NSRC == 2 ? ra2[Op::NSRC == 2 ? i : 0][j] : 0.f,
                                   m0 + r, k, stats[r], rok);
        v[j] = rok ? x : 0.f;
      }
      *reinterpret_cast<u32x2_t*>(As + r * LDK + 4 * aq) =
          u32x2_t{pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3])};
    }
    if constexpr (B16) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = tid + 256 * i;
        *reinterpret_cast<u32x4_t*>(Bs + (p >> 2) * LDK + 8 * (p & 3)) = rb16[B16 ? i : 0];
      }
    } else if constexpr (Op::B_N_CONTIG) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<uint32_t*>(Bs + (4 * bn + j) * LDK + 8 * i + 2 * bp) =
              pack_bf16(rb[2 * i][j], rb[2 * i + 1][j]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        *reinterpret_cast<u32x2_t*>(Bs + (bc + 32 * i) * LDK + 4 * bq) =
            u32x2_t{pack_bf16(rb[i][0], rb[i][1]), pack_bf16(rb[i][2], rb[i][3])};
    }
  };

  f4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  auto mfmas = [&](int buf) {
    const __bf16* As = As2[buf];
    const __bf16* Bs = Bs2[buf];
    const u32x4_t av = *reinterpret_cast<const u32x4_t*>(As + (w * 16 + lr) * LDK + 8 * lg);
    u32x4_t bv[2];
    bv[0] = *reinterpret_cast<const u32x4_t*>(Bs + lr * LDK + 8 * lg);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (t + 1 < NT)
        bv[(t + 1) & 1] = *reinterpret_cast<const u32x4_t*>(Bs + (16 * (t + 1) + lr) * LDK + 8 * lg);
      acc[t] = mfma_bf16(av, bv[t & 1], acc[t]);
    }
  };

  load(0);
  store(0, 0);
  lds_barrier();
  int buf = 0;
  const int klast = op.K - BKT;
  for (int k0 = 0; k0 < klast; k0 += BKT) {
    load(k0 + BKT);
    mfmas(buf);
    store(k0 + BKT, buf ^ 1);
    lds_barrier();
    buf ^= 1;
  }
  typename Op::template Epi<NT> es;
  op.epi_load(es, m0 + w * 16 + 4 * lg, n0 + lr, total);
  mfmas(buf);
  op.epilogue(acc, es, m0 + w * 16 + 4 * lg, n0 + lr, total);
}

// descriptor over rows [m0, total) of a (rows, ld) matrix (column offset folded in base)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* base, int64_t ld,
                                                           int64_t m0, int64_t total) {
  int64_t bytes = (total - m0) * ld * 4;
  if (bytes > 0x7fffffff) bytes = 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + m0 * ld), 0, (int)bytes, 0x00020000);
}

// the same over bf16 rows (the bf16-activation ops)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const __bf16* base, int64_t ld,
                                                           int64_t m0, int64_t total) {
  int64_t bytes = (total - m0) * ld * 2;
  if (bytes > 0x7fffffff) bytes = 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + m0 * ld), 0, (int)bytes, 0x00020000);
}

// Op templates: A16 = the bf16-activation layout (autocast_dtype = bfloat16 at wide heads,
// hstu_*_a16): uvqk, h_pre, o_in and d_uvqk live in HBM as bf16, read with 2-byte loads
// and written rounded from the fp32 epilogue values; everything else is unchanged.
template <bool A16>
using act_t = typename std::conditional<A16, __bf16, float>::type;

// ------------------------------------------------------------------ ops
struct NoStats {
  __device__ void prologue(int64_t, int64_t, float2* st) const {
    if (threadIdx.x < BM) st[threadIdx.x] = make_float2(0.f, 1.f);
  }
};

__device__ __forceinline__ int64_t clamp_row(int64_t m, int64_t total) {
  return m < total ? m : total - 1;
}

// F1: uvqk = act(LN(x) @ W), W row-major (D, n_out)
template <bool A16>
struct OpLnUvqkT {
  static constexpr bool B_N_CONTIG = true;
  static constexpr int A0_BYTES = 4;
  static constexpr bool B16 = A16;  // the weight as a bf16 [N][K] image (w16)
  static constexpr bool A0_RAW = false;  // a_xform is the identity on A0 (bf16v's raw bf16 path)
  const int64_t* offsets;
  int B, K, N;
  const float* x;
  int64_t ldx;
  const float* w;
  float eps;
  int act;
  float2* x_stats;
  act_t<A16>* h_pre;
  act_t<A16>* out;
  int64_t ld_out;
  __bf16* xn;  // A16: optional bf16 LN(x) rows (ld K), the weight gradient's A operand
  int stats_given;
  const __bf16* w16;  // A16: W_uvqk^T as bf16, (n_out, D)  // A16: x_stats already holds the rows' (mean, rstd) (the previous
                    // layer's gate_o epilogue computed them): no statistics pass
  __device__ void prologue(int64_t m0, int64_t total, float2* st) const {
    if (A16 && stats_given) {
      if (threadIdx.x < BM) st[threadIdx.x] = ld_f2(x_stats, clamp_row(m0 + threadIdx.x, total));
      return;
    }
    panel_row_stats(x, ldx, m0, total, K, eps, st, blockIdx.y == 0 ? x_stats : nullptr);
  }
  static constexpr int NSRC = 1;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(x, ldx, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(x, ldx, m0, t); }
  __device__ int64_t a_ld0() const { return ldx; }
  __device__ int64_t a_ld1() const { return ldx; }
  __device__ float a_xform(float v, float, int64_t m, int k, float2 st, bool valid) const {
    const float y = (v - st.x) * st.y;
    if constexpr (A16)
      if (xn && valid && blockIdx.y == 0) xn[m * K + k] = (__bf16)y;
    return y;
  }
  __device__ int bks() const { return N; }
  __device__ int bns() const { return 1; }
  template <int NT>
  struct Epi {};
  template <int NT>
  __device__ void epi_load(Epi<NT>&, int64_t, int, int64_t) const {}
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>&, int64_t mrow, int ncol, int64_t total) const {
    if constexpr (A16) {
      // bf16 pairs: lanes lr, lr ^ 1 hold adjacent columns; the even lane stores rows 0, 1
      // and the odd lane rows 2, 3 of both columns as packed 4-byte stores (N, ld_out even)
      const bool odd = (threadIdx.x & 1) != 0;
      const int cb = ncol - (odd ? 1 : 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float sx = odd ? acc[t][0] : acc[t][2], sy = odd ? acc[t][1] : acc[t][3];
        const float rx = dpp_mov<0xB1>(sx), ry = dpp_mov<0xB1>(sy);
        const int n = cb + 16 * t;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int64_t m = mrow + (odd ? 2 : 0) + j;
          const float lo = odd ? (j ? ry : rx) : acc[t][j];
          const float hi = odd ? acc[t][2 + j] : (j ? ry : rx);
          if (m < total && n < N) {
            if (h_pre) *reinterpret_cast<uint32_t*>(h_pre + m * ld_out + n) = pack_bf16(lo, hi);
            *reinterpret_cast<uint32_t*>(out + m * ld_out + n) =
                act ? pack_bf16(siluf_(lo), siluf_(hi)) : pack_bf16(lo, hi);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      if (m >= total) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        if (n >= N) continue;
        const float v = acc[t][r];
        if (h_pre) h_pre[m * ld_out + n] = v;
        out[m * ld_out + n] = act ? siluf_(v) : v;
      }
    }
  }
};
using OpLnUvqk = OpLnUvqkT<false>;

__device__ __forceinline__ float dropout_keep(uint64_t seed, int64_t m, int k, int K, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t hsh = hash_u32(seed, (uint64_t)m * (uint64_t)K + (uint64_t)k);
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  return hsh >= thr ? 1.f / (1.f - p) : 0.f;
}

// F3: y = dropout(u * LN(attn)) @ W_o^T + b_o + x,  W_o row-major (D, hdv)
template <bool A16>
struct OpGateOT {
  static constexpr bool B_N_CONTIG = false;
  static constexpr int A0_BYTES = A16 ? 2 : 4;  // u
  static constexpr bool B16 = A16;  // the weight as a bf16 [N][K] image (w16)
  static constexpr bool A0_RAW = false;  // a_xform is the identity on A0 (bf16v's raw bf16 path)
  const int64_t* offsets;
  int B, K, N;  // K = hdv, N = D
  const act_t<A16>* u;
  int64_t ldu;
  const float* attn;
  int64_t lda;
  const float* w;
  const float* bias;
  const float* xres;
  int64_t ldx;
  float eps, p;
  uint64_t seed;
  const int64_t* seed_off;
  float2* a_stats;
  act_t<A16>* o_in;
  float* y;
  int64_t ldy;
  float2* y_stats;  // A16, N <= 256 (one panel): the LayerNorm (mean, rstd) of each y row
                    // with eps -- the next layer's x_stats, in panel_row_stats's order
  const __bf16* w16;  // A16: W_o as bf16, (D, hdv)
  __device__ void prologue(int64_t m0, int64_t total, float2* st) const {
    panel_row_stats(attn, lda, m0, total, K, eps, st, blockIdx.y == 0 ? a_stats : nullptr);
  }
  static constexpr int NSRC = 2;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(u, ldu, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(attn, lda, m0, t); }
  __device__ int64_t a_ld0() const { return ldu; }
  __device__ int64_t a_ld1() const { return lda; }
  __device__ float a_xform(float uv, float av, int64_t m, int k, float2 st, bool valid) const {
    float v = uv * ((av - st.x) * st.y);
    if (p > 0.f) v *= dropout_keep(seed + (seed_off ? (uint64_t)*seed_off : 0ull), m, k, K, p);
    if (valid && o_in && blockIdx.y == 0) o_in[m * K + k] = (act_t<A16>)v;
    return v;
  }
  __device__ int bks() const { return 1; }
  __device__ int bns() const { return K; }
  template <int NT>
  struct Epi {};
  template <int NT>
  __device__ void epi_load(Epi<NT>&, int64_t, int, int64_t) const {}
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>&, int64_t mrow, int ncol, int64_t total) const {
    float bv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = ncol + 16 * t;
      bv[t] = bias ? as_global(bias)[n < N ? n : N - 1] : 0.f;
    }
    if constexpr (A16 && NT == 16) {  // y_stats: the host requires the one-panel width
      if (y_stats) {
        epilogue_stats(acc, mrow, ncol, total);
        return;
      }
    }
    // every residual load issued before the first store (y may alias xres for hipcc,
    // which otherwise waits for each row's loads after the previous row's stores)
    float xv[4][NT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t mc = clamp_row(mrow + r, total);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        xv[r][t] = xres ? as_global(xres)[mc * ldx + (n < N ? n : N - 1)] : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      if (m >= total) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        if (n < N) y[m * ldy + n] = (acc[t][r] + bv[t]) + xv[r][t];
      }
    }
  }
  // y rows plus their LayerNorm statistics: a lane holds column 16 t + lr of its rows, the
  // layout panel_row_stats reduces (value j = column 16 j + sub), so the same sums in the
  // same order give the statistics the next layer's LN + UVQK would compute from y
  template <int NT>
  __device__ void epilogue_stats(f4 (&acc)[NT], int64_t mrow, int ncol, int64_t total) const {
    float bv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = ncol + 16 * t;
      bv[t] = bias ? as_global(bias)[n < N ? n : N - 1] : 0.f;
    }
    float xv[4][NT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t mc = clamp_row(mrow + r, total);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        xv[r][t] = xres ? as_global(xres)[mc * ldx + (n < N ? n : N - 1)] : 0.f;
      }
    }
    const int sub = ncol & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      float v[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) v[t] = 16 * t + sub < N ? (acc[t][r] + bv[t]) + xv[r][t] : 0.f;
      const float2 mr = ln_stats16(v, sub, N, eps);
      if (m < total) {
        if (sub == 0) y_stats[m] = mr;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n = ncol + 16 * t;
          if (n < N) y[m * ldy + n] = v[t];
        }
      }
    }
  }
};
using OpGateO = OpGateOT<false>;

// LayerNorm backward of one element: rstd * (dln - mean(dln) - ln * mean(dln * ln)), with
// the contraction spelled out so every epilogue rounds it the same way
__device__ __forceinline__ float ln_bwd_val(float rstd, float dln, float mean1, float ln, float mean2) {
  return rstd * __builtin_fmaf(-ln, mean2, dln - mean1);
}

// B1: g = dy @ W_o (rows, hdv); epilogue: dropout bwd, du = g*LN(a) (*silu'(h_u)),
//     d_attn = LayerNorm_bwd(g * u).  Needs the whole hdv row in one panel.
template <bool A16>
struct OpGateOBwdT : NoStats {
  static constexpr bool B_N_CONTIG = true;
  static constexpr int A0_BYTES = 4;  // dy
  static constexpr bool B16 = A16;  // the weight as a bf16 [N][K] image (w16)
  static constexpr bool A0_RAW = false;  // a_xform is the identity on A0 (bf16v's raw bf16 path)
  const int64_t* offsets;
  int B, K, N;  // K = D, N = hdv
  const float* dy;
  int64_t lddy;
  const float* w;
  const act_t<A16>* u;
  int64_t ldu;
  const float* attn;
  int64_t lda;
  const float2* a_stats;
  const act_t<A16>* h_u;
  int64_t ldh;
  float p;
  uint64_t seed;
  const int64_t* seed_off;
  act_t<A16>* du;
  int64_t lddu;
  act_t<A16>* da;  // A16: d_attn in bf16 -- the attention backward's dO, DMA-staged as is
  int64_t ldda;
  const __bf16* w16 = nullptr;  // A16: W_o^T as bf16, (hdv, D)
  static constexpr int NSRC = 1;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(dy, lddy, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(dy, lddy, m0, t); }
  __device__ int64_t a_ld0() const { return lddy; }
  __device__ int64_t a_ld1() const { return lddy; }
  __device__ float a_xform(float v, float, int64_t, int, float2, bool) const { return v; }
  __device__ int bks() const { return N; }
  __device__ int bns() const { return 1; }
  template <int NT>
  struct Epi {};
  template <int NT>
  __device__ void epi_load(Epi<NT>&, int64_t, int, int64_t) const {}
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>& es, int64_t mrow, int ncol, int64_t total) const {
    if constexpr (A16) {
      epilogue16(acc, mrow, ncol, total);
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      const bool row_ok = m < total;
      const int64_t mc = clamp_row(m, total);
      const float2 st = ld_f2(a_stats, mc);
      float av[NT], uv[NT], hv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        const int nc = n < N ? n : N - 1;
        av[t] = as_global(attn)[mc * lda + nc];
        uv[t] = (float)as_global(u)[mc * ldu + nc];
        hv[t] = h_u ? (float)as_global(h_u)[mc * ldh + nc] : 0.f;
      }
      float s1 = 0.f, s2 = 0.f;
      float lnv[NT], dln[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        const bool ok = row_ok && n < N;
        const float g = p > 0.f ? acc[t][r] * dropout_keep(seed + (seed_off ? (uint64_t)*seed_off : 0ull), m, n, N, p) : acc[t][r];
        const float ln = (av[t] - st.x) * st.y;
        float dd = g * ln;
        if (h_u) dd *= silu_grad_(hv[t]);
        if (ok) du[m * lddu + n] = (act_t<A16>)dd;
        lnv[t] = ok ? ln : 0.f;
        dln[t] = ok ? g * uv[t] : 0.f;
        s1 += dln[t];
        s2 += dln[t] * lnv[t];
      }
      s1 = sum16(s1);
      s2 = sum16(s2);
      const float inv = 1.f / (float)N;
      const float mean1 = s1 * inv, mean2 = s2 * inv;
      if (!row_ok) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        if (n < N) da[m * ldda + n] = ln_bwd_val(st.y, dln[t], mean1, lnv[t], mean2);
      }
    }
  }
  // bf16 layout: u / h_u read as the 4-byte bf16 pair holding the lane's column (a lane
  // pair reads the same word); du and d_attn written as packed pairs per row: the even
  // lane of a pair takes its partner's value by one DPP swap and stores both columns (no
  // values held across rows: two waves per SIMD).  Same values as the fp32 layout,
  // rounded to bf16 (d_attn through ln_bwd_val, the fp32 epilogue's formula).
  template <int NT>
  __device__ void epilogue16(f4 (&acc)[NT], int64_t mrow, int ncol, int64_t total) const {
    const bool odd = (threadIdx.x & 1) != 0;
    const int cb = ncol - (odd ? 1 : 0);
    // restrict-qualified views: the du / d_attn stores of one row do not order the next
    // row's loads (same-typed stores otherwise made hipcc wait vmcnt(0) between rows)
    const uint32_t* __restrict__ u32 = reinterpret_cast<const uint32_t*>(u);
    const uint32_t* __restrict__ h32 = reinterpret_cast<const uint32_t*>(h_u);
    const float* __restrict__ ap = attn;
    uint32_t* __restrict__ du32 = reinterpret_cast<uint32_t*>(du);
    uint32_t* __restrict__ da32 = reinterpret_cast<uint32_t*>(da);
    const uint64_t sd = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      const bool row_ok = m < total;
      const int64_t mc = clamp_row(m, total);
      const float2 st = ld_f2(a_stats, mc);
      float av[NT], uv[NT], hv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        const int nc = n < N ? n : N - 1;
        const int pc = (n < N ? cb + 16 * t : N - 2) >> 1;  // the pair's word (N even)
        av[t] = as_global(ap)[mc * lda + nc];
        const uint32_t wu = as_global(u32)[(mc * ldu >> 1) + pc];
        uv[t] = __uint_as_float(odd ? wu & 0xffff0000u : wu << 16);
        if (h_u) {
          const uint32_t wh = as_global(h32)[(mc * ldh >> 1) + pc];
          hv[t] = __uint_as_float(odd ? wh & 0xffff0000u : wh << 16);
        } else {
          hv[t] = 0.f;
        }
      }
      float s1 = 0.f, s2 = 0.f;
      float lnv[NT], dln[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        const bool ok = row_ok && n < N;
        const float g = p > 0.f ? acc[t][r] * dropout_keep(sd, m, n, N, p) : acc[t][r];
        const float ln = (av[t] - st.x) * st.y;
        float dd = g * ln;
        if (h_u) dd *= silu_grad_(hv[t]);
        const float other = dpp_mov<0xB1>(dd);  // the partner's column
        if (!odd && ok) du32[(m * lddu + cb + 16 * t) >> 1] = pack_bf16(dd, other);
        lnv[t] = ok ? ln : 0.f;
        dln[t] = ok ? g * uv[t] : 0.f;
        s1 += dln[t];
        s2 += dln[t] * lnv[t];
      }
      s1 = sum16(s1);
      s2 = sum16(s2);
      const float inv = 1.f / (float)N;
      const float mean1 = s1 * inv, mean2 = s2 * inv;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float dav = ln_bwd_val(st.y, dln[t], mean1, lnv[t], mean2);
        const float other = dpp_mov<0xB1>(dav);
        if (!odd && row_ok && cb + 16 * t < N) da32[(m * ldda + cb + 16 * t) >> 1] = pack_bf16(dav, other);
      }
    }
  }
};
using OpGateOBwd = OpGateOBwdT<false>;

// B3: dn = dh @ W_uvqk^T (rows, D); epilogue: dx = dy + LayerNorm_bwd(x; dn).
template <bool A16>
struct OpLnUvqkBwdT : NoStats {
  static constexpr bool B_N_CONTIG = false;
  static constexpr int A0_BYTES = A16 ? 2 : 4;  // dh
  static constexpr bool B16 = A16;  // the weight as a bf16 [N][K] image (w16)
  static constexpr bool A0_RAW = A16;  // a_xform is the identity on A0 (bf16v's raw bf16 path)
  const int64_t* offsets;
  int B, K, N;  // K = n_out (4hd), N = D
  const act_t<A16>* dh;
  int64_t lddh;
  const float* w;  // (D, n_out) row-major -> b(k, n) = w[n][k]
  const float* x;
  int64_t ldx;
  const float2* x_stats;
  const float* dy;
  int64_t lddy;
  float* dx;
  int64_t lddx;
  const __bf16* w16 = nullptr;  // A16: W_uvqk as bf16, (D, n_out)
  static constexpr int NSRC = 1;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(dh, lddh, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(dh, lddh, m0, t); }
  __device__ int64_t a_ld0() const { return lddh; }
  __device__ int64_t a_ld1() const { return lddh; }
  __device__ float a_xform(float v, float, int64_t, int, float2, bool) const { return v; }
  __device__ int bks() const { return 1; }
  __device__ int bns() const { return K; }
  template <int NT>
  struct Epi {
    float2 st[4];
    float xv[4][NT], dyv[4][NT];
  };
  template <int NT>
  __device__ void epi_load(Epi<NT>& es, int64_t mrow, int ncol, int64_t total) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t mc = clamp_row(mrow + r, total);
      es.st[r] = ld_f2(x_stats, mc);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        const int nc = n < N ? n : N - 1;
        es.xv[r][t] = as_global(x)[mc * ldx + nc];
        es.dyv[r][t] = dy ? as_global(dy)[mc * lddy + nc] : 0.f;
      }
    }
  }
  template <int NT>
  __device__ void row_in(float2& st, float (&xv)[NT], float (&dyv)[NT], int64_t m, int ncol,
                         int64_t total) const {
    const int64_t mc = clamp_row(m, total);
    st = ld_f2(x_stats, mc);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = ncol + 16 * t;
      const int nc = n < N ? n : N - 1;
      xv[t] = as_global(x)[mc * ldx + nc];
      dyv[t] = dy ? as_global(dy)[mc * lddy + nc] : 0.f;
    }
  }
  template <int NT>
  __device__ void row_out(const f4 (&acc)[NT], int r, float2 st, const float* xv, const float* dyv,
                          int64_t m, int ncol, int64_t total) const {
    const bool row_ok = m < total;
    float s1 = 0.f, s2 = 0.f;
    float xh[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = ncol + 16 * t;
      const bool ok = row_ok && n < N;
      xh[t] = ok ? (xv[t] - st.x) * st.y : 0.f;
      const float dn = ok ? acc[t][r] : 0.f;
      s1 += dn;
      s2 += dn * xh[t];
    }
    s1 = sum16(s1);
    s2 = sum16(s2);
    const float inv = 1.f / (float)N;
    const float mean1 = s1 * inv, mean2 = s2 * inv;
    if (!row_ok) return;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = ncol + 16 * t;
      if (n < N) dx[m * lddx + n] = dyv[t] + st.y * (acc[t][r] - mean1 - xh[t] * mean2);
    }
  }
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>& es, int64_t mrow, int ncol, int64_t total) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) row_out(acc, r, es.st[r], es.xv[r], es.dyv[r], mrow + r, ncol, total);
  }
  // streamed form (f32 row panel at 256 columns): row r + 1's inputs in flight while row r
  // is reduced and stored, two rows of registers instead of four
  template <int NT>
  __device__ void epilogue_stream(f4 (&acc)[NT], int64_t mrow, int ncol, int64_t total) const {
    float2 st[2];
    float xv[2][NT], dyv[2][NT];
    row_in(st[0], xv[0], dyv[0], mrow, ncol, total);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r + 1 < 4) row_in(st[(r + 1) & 1], xv[(r + 1) & 1], dyv[(r + 1) & 1], mrow + r + 1, ncol, total);
      row_out(acc, r, st[r & 1], xv[r & 1], dyv[r & 1], mrow + r, ncol, total);
    }
  }
};
using OpLnUvqkBwd = OpLnUvqkBwdT<false>;

template <class Op>
static int launch_rowpanel(const Op& op, int64_t max_rows, bool full_row, const char* name,
                           hipStream_t st) {
  const int nt_needed = ceil_div(op.N, 16);
  GR_REQUIRE(!full_row || nt_needed <= 16,
             "%s: %d output columns exceed one 256-column panel (row-reduction epilogue)", name,
             op.N);
  const int nt = nt_needed > 16 ? 16 : nt_needed;
  const int panels = ceil_div(op.N, nt * 16);
  dim3 grid((unsigned)((max_rows + BM - 1) / BM), (unsigned)panels);
  if (grid.x == 0) return 0;
  const char* tname = name + 5;  // "hstu_ln_uvqk_fwd" -> "ln_uvqk_fwd"
  // one 64-wide K stage when all of K fits it (ml-1m forward, K = 50: no K streaming,
  // padding k-steps skipped); measured slower for streamed K (the backward's K = 200:
  // 18.6 -> 27 us), so longer K keeps the 16-wide stages
  const bool wide_k = op.K > 16 && op.K <= 64 && nt <= 13;
#define GR_NT_CASE(NT_, BKT_)                                                                \
  case NT_:                                                                                  \
    GR_TIMED(tname, st, hipLaunchKernelGGL((rowpanel_kernel<NT_, BKT_, Op>), grid, dim3(256), 0, \
                                           st, op));                                         \
    break;
  if (wide_k) {
    switch (nt) {
      GR_NT_CASE(1, 64) GR_NT_CASE(2, 64) GR_NT_CASE(3, 64) GR_NT_CASE(4, 64) GR_NT_CASE(5, 64)
      GR_NT_CASE(6, 64) GR_NT_CASE(7, 64) GR_NT_CASE(8, 64) GR_NT_CASE(9, 64) GR_NT_CASE(10, 64)
      GR_NT_CASE(11, 64) GR_NT_CASE(12, 64) GR_NT_CASE(13, 64)
      default: GR_REQUIRE(false, "%s: bad panel width", name);
    }
  } else {
    switch (nt) {
      GR_NT_CASE(1, 16) GR_NT_CASE(2, 16) GR_NT_CASE(3, 16) GR_NT_CASE(4, 16) GR_NT_CASE(5, 16)
      GR_NT_CASE(6, 16) GR_NT_CASE(7, 16) GR_NT_CASE(8, 16) GR_NT_CASE(9, 16) GR_NT_CASE(10, 16)
      GR_NT_CASE(11, 16) GR_NT_CASE(12, 16) GR_NT_CASE(13, 16) GR_NT_CASE(14, 16)
      GR_NT_CASE(15, 16) GR_NT_CASE(16, 16)
      default: GR_REQUIRE(false, "%s: bad panel width", name);
    }
  }
#undef GR_NT_CASE
  GR_LAUNCH_CHECK(name);
  return 0;
}

// vec: operand rows 16-byte aligned (caller-checked); the float4 form also needs K a
// multiple of the 32-wide chunk, full 256-column panels and, for n-contiguous weights,
// N a multiple of 4 (a float4 never straddles the end of the weight)
template <class Op>
static int launch_rowpanel_bf16(const Op& op, int64_t max_rows, bool full_row, const char* name,
                                hipStream_t st, bool vec = false) {
  const int nt_needed = ceil_div(op.N, 16);
  GR_REQUIRE(!full_row || nt_needed <= 16,
             "%s: %d output columns exceed one 256-column panel (row-reduction epilogue)", name,
             op.N);
  const int nt = nt_needed > 16 ? 16 : nt_needed;
  const int panels = ceil_div(op.N, nt * 16);
  dim3 grid((unsigned)((max_rows + BM - 1) / BM), (unsigned)panels);
  if (grid.x == 0) return 0;
  const char* tname = name + 5;
  if constexpr (Op::A0_BYTES == 4 || Op::A0_RAW) {  // bf16 A0 rows with a transform: scalar panel
    if (vec && option(GR_OPT_PANEL_VEC) != 0 && nt == 16 && op.K % 32 == 0 &&
        (!Op::B_N_CONTIG || op.N % 4 == 0) && (int64_t)op.K * op.N * 4 <= 0x7fffffffLL) {
      GR_TIMED(tname, st, hipLaunchKernelGGL((rowpanel_bf16v_kernel<Op>), grid, dim3(256), 0, st, op));
      GR_LAUNCH_CHECK(name);
      return 0;
    }
  }
#define GR_NT_CASE(NT_)                                                                      \
  case NT_:                                                                                  \
    GR_TIMED(tname, st, hipLaunchKernelGGL((rowpanel_bf16_kernel<NT_, Op>), grid, dim3(256), 0, \
                                           st, op));                                         \
    break;
  switch (nt) {
    GR_NT_CASE(1) GR_NT_CASE(2) GR_NT_CASE(3) GR_NT_CASE(4) GR_NT_CASE(5) GR_NT_CASE(6)
    GR_NT_CASE(7) GR_NT_CASE(8) GR_NT_CASE(9) GR_NT_CASE(10) GR_NT_CASE(11) GR_NT_CASE(12)
    GR_NT_CASE(13) GR_NT_CASE(14) GR_NT_CASE(15) GR_NT_CASE(16)
    default: GR_REQUIRE(false, "%s: bad panel width", name);
  }
#undef GR_NT_CASE
  GR_LAUNCH_CHECK(name);
  return 0;
}

// ------------------------------------------------------------------ row-wave dispatch
// Narrow shapes (weight panel in LDS, <= 80 KiB) run the row-wave kernel (rowwave.h);
// everything else the row-panel kernel above.  Returns -1 when the shape / alignment
// is not covered (caller falls back), else the launch status.
constexpr size_t RW_LDS_MAX = 80 * 1024;

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

static int rw_bucket(int x) {  // 16-column groups, rounded up to an instantiated size
  const int g = ceil_div(x, 16);
  if (g <= 1) return 1;
  if (g <= 2) return 2;
  if (g <= 4) return 4;
  if (g <= 8) return 8;
  if (g <= 13) return 13;
  if (g <= 16) return 16;
  return -1;
}

template <int KG, int NT, int VEC, template <int, int, int> class OpT, class Args>
static int rw_launch(const Args& args, int64_t max_rows, const char* tname, hipStream_t st) {
  using C = RowWaveCfg<KG, NT>;
  if constexpr (C::LDS_BYTES > RW_LDS_MAX) {
    return -1;
  } else {
    OpT<KG, NT, VEC> op;
    args.fill(op);
    // grid-stride over 16-row units (persistent once the rows exceed 4 workgroups per CU)
    const int64_t units = (max_rows + 15) / 16;
    int grid = (int)((units + 3) / 4);
    const int cap = 4 * num_cus();
    if (grid > cap) grid = cap;
    if (grid < 1) return 0;
    GR_TIMED(tname, st, hipLaunchKernelGGL((rowwave_kernel<KG, NT, OpT<KG, NT, VEC>>), dim3(grid),
                                           dim3(256), C::LDS_BYTES, st, op));
    GR_LAUNCH_CHECK(tname);
    return 0;
  }
}

template <int KG, int VEC, template <int, int, int> class OpT, class Args>
static int rw_nt(const Args& a, int nt, int64_t max_rows, const char* tname, hipStream_t st) {
  switch (nt) {
    case 1: return rw_launch<KG, 1, VEC, OpT>(a, max_rows, tname, st);
    case 2: return rw_launch<KG, 2, VEC, OpT>(a, max_rows, tname, st);
    case 4: return rw_launch<KG, 4, VEC, OpT>(a, max_rows, tname, st);
    case 8: return rw_launch<KG, 8, VEC, OpT>(a, max_rows, tname, st);
    case 13: return rw_launch<KG, 13, VEC, OpT>(a, max_rows, tname, st);
    case 16: return rw_launch<KG, 16, VEC, OpT>(a, max_rows, tname, st);
  }
  return -1;
}

template <int VEC, template <int, int, int> class OpT, class Args>
static int rw_kg(const Args& a, int kg, int nt, int64_t max_rows, const char* tname, hipStream_t st) {
  switch (kg) {
    case 1: return rw_nt<1, VEC, OpT>(a, nt, max_rows, tname, st);
    case 2: return rw_nt<2, VEC, OpT>(a, nt, max_rows, tname, st);
    case 4: return rw_nt<4, VEC, OpT>(a, nt, max_rows, tname, st);
    case 8: return rw_nt<8, VEC, OpT>(a, nt, max_rows, tname, st);
    case 13: return rw_nt<13, VEC, OpT>(a, nt, max_rows, tname, st);
    case 16: return rw_nt<16, VEC, OpT>(a, nt, max_rows, tname, st);
  }
  return -1;
}

// vector width usable for every (pointer + column offset, leading dim, K, N) involved
static int rw_vec(std::initializer_list<const void*> ptrs, std::initializer_list<int64_t> lds) {
  for (int vec : {4, 2}) {
    bool ok = true;
    for (const void* p : ptrs)
      if (p && ((uintptr_t)p % (4 * vec)) != 0) ok = false;
    for (int64_t l : lds)
      if (l % vec != 0) ok = false;
    if (ok) return vec;
  }
  return 0;
}

template <template <int, int, int> class OpT, class Args>
static int rw_dispatch(const Args& a, int K, int N, int vec, int64_t max_rows, const char* tname,
                       hipStream_t st) {
  const int kg = rw_bucket(K), nt = rw_bucket(N);
  if (kg < 0 || nt < 0 || vec == 0) return -1;
  // measured (ml-1m, MI355X): the row-wave form wins for the square D x D projections
  // (gate/_o fwd+bwd, 26 -> 17 us, 20 -> 16 us); the row panel keeps the 4x-wide
  // UVQK projection (27 vs 33 us fwd) where one 16-row unit carries 13 column tiles
  if (kg > 8 || nt > 8) return -1;
  if (max_rows * 4 * 1024 > 0x7fffffffLL) return -1;  // 32-bit buffer offsets
  (void)vec;  // 4-aligned shapes run the 8-byte path too (one instantiation set)
  return rw_kg<2, OpT>(a, kg, nt, max_rows, tname, st);
}

// concat_ua row-wave launches (KG / NT = 3 segments of KGH 16-column groups)
template <class Op, int KG, int NT>
static int rw_launch_op(const Op& op, int64_t max_rows, const char* tname, hipStream_t st) {
  using C = RowWaveCfg<KG, NT>;
  if constexpr (C::LDS_BYTES > RW_LDS_MAX) {
    GR_REQUIRE(false, "%s: concat_ua weight panel (%d x %d groups) exceeds the LDS budget", tname,
               KG, NT);
  } else {
    const int64_t units = (max_rows + 15) / 16;
    int grid = (int)((units + 3) / 4);
    const int cap = 4 * num_cus();
    if (grid > cap) grid = cap;
    if (grid < 1) return 0;
    GR_TIMED(tname, st, hipLaunchKernelGGL((rowwave_kernel<KG, NT, Op>), dim3(grid), dim3(256),
                                           C::LDS_BYTES, st, op));
    GR_LAUNCH_CHECK(tname);
    return 0;
  }
}

static int cat_kgh(int hv) { return hv <= 16 ? 1 : hv <= 32 ? 2 : hv <= 64 ? 4 : -1; }

template <int KGH, int NT>
static int cat_fwd_nt(const RwArgsGateO& a, int hv, int64_t max_rows, hipStream_t st) {
  using Op = typename RwGateOCatT<KGH, NT, 2>::template Op<3 * KGH, NT, 2>;
  Op op;
  a.fill(op);
  op.hv = hv;
  return rw_launch_op<Op, 3 * KGH, NT>(op, max_rows, "gate_o_fwd", st);
}
template <int KGH>
static int cat_fwd_kgh(const RwArgsGateO& a, int hv, int nt, int64_t max_rows, hipStream_t st) {
  switch (nt) {
    case 1: return cat_fwd_nt<KGH, 1>(a, hv, max_rows, st);
    case 2: return cat_fwd_nt<KGH, 2>(a, hv, max_rows, st);
    case 4: return cat_fwd_nt<KGH, 4>(a, hv, max_rows, st);
    case 8: return cat_fwd_nt<KGH, 8>(a, hv, max_rows, st);
  }
  return -1;
}
template <int KGH, int KG>
static int cat_bwd_kg(const RwArgsGateOBwd& a, int hv, int64_t max_rows, hipStream_t st) {
  using Op = typename RwGateOCatBwdT<KGH, KG, 2>::template Op<KG, 3 * KGH, 2>;
  Op op;
  a.fill(op);
  op.hv = hv;
  return rw_launch_op<Op, KG, 3 * KGH>(op, max_rows, "gate_o_bwd", st);
}
template <int KGH>
static int cat_bwd_kgh(const RwArgsGateOBwd& a, int hv, int kg, int64_t max_rows, hipStream_t st) {
  switch (kg) {
    case 1: return cat_bwd_kg<KGH, 1>(a, hv, max_rows, st);
    case 2: return cat_bwd_kg<KGH, 2>(a, hv, max_rows, st);
    case 4: return cat_bwd_kg<KGH, 4>(a, hv, max_rows, st);
    case 8: return cat_bwd_kg<KGH, 8>(a, hv, max_rows, st);
  }
  return -1;
}

static bool rw_enabled() { return option(GR_OPT_ROWWAVE) != 0; }

}  // namespace gr

#ifndef GR_LINEAR_LIB_ONLY  // hstu_linear_a16.hip takes the kernels above, not the entries
// ====================================================================== C-ABI
using namespace gr;

static int hstu_ln_uvqk_fwd_impl(bool bf16, const float* x, int64_t ld_x, const int64_t* offsets, int B,
                                int64_t max_rows, int D, const float* w_uvqk, int n_out,
                                float eps, int activation, float* x_stats, float* h_pre,
                                float* uvqk, int64_t ld_out, void* stream) {
  GR_REQUIRE(x && offsets && w_uvqk && uvqk && x_stats, "hstu_ln_uvqk_fwd: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0 && max_rows >= 0, "hstu_ln_uvqk_fwd: bad sizes");
  GR_REQUIRE(activation == 0 || activation == 1, "hstu_ln_uvqk_fwd: activation must be 0|1");
  if (!bf16 && rw_enabled()) {
    RwArgsLnUvqk ra{offsets, B, D, n_out, x, ld_x, w_uvqk, eps, activation, (float2*)x_stats,
                    h_pre, uvqk, ld_out};
    const int vec = rw_vec({x, h_pre, uvqk}, {ld_x, ld_out, D, n_out});
    const int rc = rw_dispatch<RwLnUvqk>(ra, D, n_out, vec, max_rows, "ln_uvqk_fwd", (hipStream_t)stream);
    if (rc >= 0) return rc;
  }
  OpLnUvqk op{offsets, B, D, n_out, x, ld_x, w_uvqk, eps, activation, (float2*)x_stats,
              h_pre, uvqk, ld_out};
  // forward panels keep the scalar staging: measured faster at C3 (210 vs 219 us; gate_o
  // 132 vs 139 us, scripts/gemm_micro.py --bf16-panels); the float4 form pays off in the
  // backward panels, whose epilogue inputs otherwise hold the registers
  return bf16 ? launch_rowpanel_bf16(op, max_rows, false, "hstu_ln_uvqk_fwd", (hipStream_t)stream)
              : launch_rowpanel(op, max_rows, false, "hstu_ln_uvqk_fwd", (hipStream_t)stream);
}
#ifdef GR_STAMP
extern "C" __attribute__((visibility("default"))) int gr_rw_stamp_read(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(gr::gr_rw_buf), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int hstu_ln_uvqk_fwd(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                                int64_t max_rows, int D, const float* w_uvqk, int n_out,
                                float eps, int activation, float* x_stats, float* h_pre,
                                float* uvqk, int64_t ld_out, void* stream) {
  return hstu_ln_uvqk_fwd_impl(false, x, ld_x, offsets, B, max_rows, D, w_uvqk, n_out, eps, activation, x_stats, h_pre, uvqk, ld_out, stream);
}
extern "C" int hstu_ln_uvqk_fwd_bf16(const float* x, int64_t ld_x, const int64_t* offsets, int B,
                                int64_t max_rows, int D, const float* w_uvqk, int n_out,
                                float eps, int activation, float* x_stats, float* h_pre,
                                float* uvqk, int64_t ld_out, void* stream) {
  return hstu_ln_uvqk_fwd_impl(true, x, ld_x, offsets, B, max_rows, D, w_uvqk, n_out, eps, activation, x_stats, h_pre, uvqk, ld_out, stream);
}

static int hstu_gate_o_fwd_impl(bool bf16, const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                               const float* w_o, const float* b_o, const float* x_res,
                               int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                               const int64_t* seed_offset, float* attn_stats, float* o_in,
                               float* y, int64_t ld_y, void* stream) {
  GR_REQUIRE(u && attn && offsets && w_o && y && attn_stats, "hstu_gate_o_fwd: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_fwd: bad sizes");
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_gate_o_fwd: dropout_p %f", dropout_p);
  if (!bf16 && rw_enabled()) {
    RwArgsGateO ra{offsets, B, hdv, D, u, ld_u, attn, ld_attn, w_o, b_o, x_res, ld_x, eps,
                   dropout_p, seed, seed_offset, (float2*)attn_stats, o_in, y, ld_y};
    const int vec = rw_vec({u, attn, x_res, o_in, y}, {ld_u, ld_attn, ld_x, ld_y, hdv, D});
    const int rc = rw_dispatch<RwGateO>(ra, hdv, D, vec, max_rows, "gate_o_fwd", (hipStream_t)stream);
    if (rc >= 0) return rc;
  }
  OpGateO op{offsets, B, hdv, D, u, ld_u, attn, ld_attn, w_o, b_o, x_res, ld_x, eps, dropout_p,
             seed, seed_offset, (float2*)attn_stats, o_in, y, ld_y};
  return bf16 ? launch_rowpanel_bf16(op, max_rows, false, "hstu_gate_o_fwd", (hipStream_t)stream)
              : launch_rowpanel(op, max_rows, false, "hstu_gate_o_fwd", (hipStream_t)stream);
}
extern "C" int hstu_gate_o_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                               const float* w_o, const float* b_o, const float* x_res,
                               int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                               const int64_t* seed_offset, float* attn_stats, float* o_in,
                               float* y, int64_t ld_y, void* stream) {
  return hstu_gate_o_fwd_impl(false, u, ld_u, attn, ld_attn, offsets, B, max_rows, hdv, D, w_o, b_o, x_res, ld_x, eps, dropout_p, seed, seed_offset, attn_stats, o_in, y, ld_y, stream);
}
extern "C" int hstu_gate_o_fwd_bf16(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                               const float* w_o, const float* b_o, const float* x_res,
                               int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                               const int64_t* seed_offset, float* attn_stats, float* o_in,
                               float* y, int64_t ld_y, void* stream) {
  return hstu_gate_o_fwd_impl(true, u, ld_u, attn, ld_attn, offsets, B, max_rows, hdv, D, w_o, b_o, x_res, ld_x, eps, dropout_p, seed, seed_offset, attn_stats, o_in, y, ld_y, stream);
}

static int hstu_gate_o_bwd_impl(bool bf16, const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                               int64_t max_rows, int hdv, int D, const float* w_o,
                               const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const float* attn_stats, const float* h_u, int64_t ld_h,
                               float dropout_p, uint64_t seed, const int64_t* seed_offset,
                               float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                               void* stream) {
  GR_REQUIRE(dy && offsets && w_o && u && attn && attn_stats && du && d_attn,
             "hstu_gate_o_bwd: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0, "hstu_gate_o_bwd: bad sizes");
  if (!bf16 && rw_enabled()) {
    RwArgsGateOBwd ra{offsets, B, D, hdv, dy, ld_dy, w_o, u, ld_u, attn, ld_attn,
                      (const float2*)attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du,
                      d_attn, ld_da};
    const int vec = rw_vec({dy, u, attn, h_u, du, d_attn}, {ld_dy, ld_u, ld_attn, ld_h, ld_du, ld_da, hdv, D});
    const int rc = rw_dispatch<RwGateOBwd>(ra, D, hdv, vec, max_rows, "gate_o_bwd", (hipStream_t)stream);
    if (rc >= 0) return rc;
  }
  OpGateOBwd op;
  op.offsets = offsets; op.B = B; op.K = D; op.N = hdv; op.dy = dy; op.lddy = ld_dy;
  op.w = w_o; op.u = u; op.ldu = ld_u; op.attn = attn; op.lda = ld_attn;
  op.a_stats = (const float2*)attn_stats; op.h_u = h_u; op.ldh = ld_h; op.p = dropout_p;
  op.seed = seed; op.seed_off = seed_offset; op.du = du; op.lddu = ld_du; op.da = d_attn; op.ldda = ld_da;
  return bf16 ? launch_rowpanel_bf16(op, max_rows, true, "hstu_gate_o_bwd", (hipStream_t)stream,
                                     rw_vec({dy, w_o}, {ld_dy, hdv}) == 4)
              : launch_rowpanel(op, max_rows, true, "hstu_gate_o_bwd", (hipStream_t)stream);
}
extern "C" int hstu_gate_o_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                               int64_t max_rows, int hdv, int D, const float* w_o,
                               const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const float* attn_stats, const float* h_u, int64_t ld_h,
                               float dropout_p, uint64_t seed, const int64_t* seed_offset,
                               float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                               void* stream) {
  return hstu_gate_o_bwd_impl(false, dy, ld_dy, offsets, B, max_rows, hdv, D, w_o, u, ld_u, attn, ld_attn, attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du, d_attn, ld_da, stream);
}
extern "C" int hstu_gate_o_bwd_bf16(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                               int64_t max_rows, int hdv, int D, const float* w_o,
                               const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                               const float* attn_stats, const float* h_u, int64_t ld_h,
                               float dropout_p, uint64_t seed, const int64_t* seed_offset,
                               float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                               void* stream) {
  return hstu_gate_o_bwd_impl(true, dy, ld_dy, offsets, B, max_rows, hdv, D, w_o, u, ld_u, attn, ld_attn, attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du, d_attn, ld_da, stream);
}

static int hstu_ln_uvqk_bwd_impl(bool bf16, const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                int64_t max_rows, int D, int n_out, const float* w_uvqk,
                                const float* x, int64_t ld_x, const float* x_stats,
                                const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                void* stream) {
  GR_REQUIRE(dh && offsets && w_uvqk && x && x_stats && dx, "hstu_ln_uvqk_bwd: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && B >= 0, "hstu_ln_uvqk_bwd: bad sizes");
  if (!bf16 && rw_enabled()) {
    RwArgsLnUvqkBwd ra{offsets, B, n_out, D, dh, ld_dh, w_uvqk, x, ld_x, (const float2*)x_stats,
                       dy_res, ld_dy, dx, ld_dx};
    const int vec = rw_vec({dh, x, dy_res, dx}, {ld_dh, ld_x, ld_dy, ld_dx, n_out, D});
    const int rc = rw_dispatch<RwLnUvqkBwd>(ra, n_out, D, vec, max_rows, "ln_uvqk_bwd", (hipStream_t)stream);
    if (rc >= 0) return rc;
  }
  OpLnUvqkBwd op;
  op.offsets = offsets; op.B = B; op.K = n_out; op.N = D; op.dh = dh; op.lddh = ld_dh;
  op.w = w_uvqk; op.x = x; op.ldx = ld_x; op.x_stats = (const float2*)x_stats;
  op.dy = dy_res; op.lddy = ld_dy; op.dx = dx; op.lddx = ld_dx;
  return bf16 ? launch_rowpanel_bf16(op, max_rows, true, "hstu_ln_uvqk_bwd", (hipStream_t)stream,
                                     rw_vec({dh, w_uvqk}, {ld_dh, D}) == 4)
              : launch_rowpanel(op, max_rows, true, "hstu_ln_uvqk_bwd", (hipStream_t)stream);
}
extern "C" int hstu_ln_uvqk_bwd(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                int64_t max_rows, int D, int n_out, const float* w_uvqk,
                                const float* x, int64_t ld_x, const float* x_stats,
                                const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                void* stream) {
  return hstu_ln_uvqk_bwd_impl(false, dh, ld_dh, offsets, B, max_rows, D, n_out, w_uvqk, x, ld_x, x_stats, dy_res, ld_dy, dx, ld_dx, stream);
}
extern "C" int hstu_ln_uvqk_bwd_bf16(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                int64_t max_rows, int D, int n_out, const float* w_uvqk,
                                const float* x, int64_t ld_x, const float* x_stats,
                                const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                void* stream) {
  return hstu_ln_uvqk_bwd_impl(true, dh, ld_dh, offsets, B, max_rows, D, n_out, w_uvqk, x, ld_x, x_stats, dy_res, ld_dy, dx, ld_dx, stream);
}

extern "C" int hstu_gate_o_cat_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const int64_t* offsets, int B, int64_t max_rows, int hdv, int hvp,
                                   int D, const float* w_pad, const float* b_o, const float* x_res,
                                   int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                   const int64_t* seed_offset, float* attn_stats, float* o_in,
                                   float* y, int64_t ld_y, void* stream) {
  GR_REQUIRE(u && attn && offsets && w_pad && y && attn_stats, "hstu_gate_o_cat_fwd: null pointer");
  const int kgh = cat_kgh(hdv), nt = rw_bucket(D);
  GR_REQUIRE(kgh > 0 && hvp == 16 * kgh && nt > 0 && nt <= 8 && B >= 0,
             "hstu_gate_o_cat_fwd: hdv %d (hvp %d) / D %d unsupported (hdv <= 64, hvp = %d, D <= 128)",
             hdv, hvp, D, 16 * kgh);
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_gate_o_cat_fwd: dropout_p %f", dropout_p);
  GR_REQUIRE(rw_vec({u, attn, x_res, o_in, y}, {ld_u, ld_attn, ld_x, ld_y, hdv, D}) > 0,
             "hstu_gate_o_cat_fwd: rows and widths must be 8-byte aligned (even)");
  RwArgsGateO ra{offsets, B, 3 * hvp, D, u, ld_u, attn, ld_attn, w_pad, b_o, x_res, ld_x, eps,
                 dropout_p, seed, seed_offset, (float2*)attn_stats, o_in, y, ld_y};
  const hipStream_t st = (hipStream_t)stream;
  switch (kgh) {
    case 1: return cat_fwd_kgh<1>(ra, hdv, nt, max_rows, st);
    case 2: return cat_fwd_kgh<2>(ra, hdv, nt, max_rows, st);
    default: return cat_fwd_kgh<4>(ra, hdv, nt, max_rows, st);
  }
}

extern "C" int hstu_gate_o_cat_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                                   int64_t max_rows, int hdv, int hvp, int D, const float* w_pad,
                                   const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                   const float* attn_stats, const float* h_u, int64_t ld_h,
                                   float dropout_p, uint64_t seed, const int64_t* seed_offset,
                                   float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                                   void* stream) {
  GR_REQUIRE(dy && offsets && w_pad && u && attn && attn_stats && du && d_attn,
             "hstu_gate_o_cat_bwd: null pointer");
  const int kgh = cat_kgh(hdv), kg = rw_bucket(D);
  GR_REQUIRE(kgh > 0 && hvp == 16 * kgh && kg > 0 && kg <= 8 && B >= 0,
             "hstu_gate_o_cat_bwd: hdv %d (hvp %d) / D %d unsupported", hdv, hvp, D);
  GR_REQUIRE(rw_vec({dy, u, attn, h_u, du, d_attn}, {ld_dy, ld_u, ld_attn, ld_h, ld_du, ld_da, hdv, D}) > 0,
             "hstu_gate_o_cat_bwd: rows and widths must be 8-byte aligned (even)");
  RwArgsGateOBwd ra{offsets, B, D, 3 * hvp, dy, ld_dy, w_pad, u, ld_u, attn, ld_attn,
                    (const float2*)attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du,
                    d_attn, ld_da};
  const hipStream_t st = (hipStream_t)stream;
  switch (kgh) {
    case 1: return cat_bwd_kgh<1>(ra, hdv, kg, max_rows, st);
    case 2: return cat_bwd_kgh<2>(ra, hdv, kg, max_rows, st);
    default: return cat_bwd_kgh<4>(ra, hdv, kg, max_rows, st);
  }
}

// ------------------------------------------------------------------ concat_ua, any width
// hstu.py:398-400 at widths the LDS-resident row-wave form cannot hold (h dv > 64 or
// D > 128, e.g. C3): o_in = dropout([u, LN(attn), u * LN(attn)]) is materialised by an
// elementwise pass (one wave per row), and the projection runs through the row-panel GEMM
// with W_o streamed through LDS in k-chunks (no resident weight).  Backward: g = dy @ W_o
// (dropout applied as it is stored) into a (rows, 3 hdv) scratch, then one wave per row
// forms du and the LayerNorm backward of the attention branch.
namespace gr {

__global__ __launch_bounds__(256) void cat_oin_kernel(const float* u, int64_t ldu, const float* attn,
                                                      int64_t lda, const int64_t* offsets, int B,
                                                      int hv, float eps, float p, uint64_t seed,
                                                      const int64_t* seed_off, float2* a_stats,
                                                      float* o_in) {
  const int64_t total = offsets[B];
  const int64_t m = (int64_t)blockIdx.x * 4 + wave_id();
  if (m >= total) return;
  const int lane = threadIdx.x & 63;
  gptr<float> arow = as_global(attn) + m * lda;
  gptr<float> urow = as_global(u) + m * ldu;
  float s = 0.f;
  for (int c = lane; c < hv; c += 64) s += arow[c];
  const float mean = wave_sum(s) / (float)hv;
  float q = 0.f;
  for (int c = lane; c < hv; c += 64) {
    const float d = arow[c] - mean;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)hv + eps);
  if (lane == 0) a_stats[m] = make_float2(mean, rstd);
  const uint64_t se = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  float* orow = o_in + m * 3 * hv;
  for (int c = lane; c < hv; c += 64) {
    const float uv = urow[c], ln = (arow[c] - mean) * rstd;
    float v0 = uv, v1 = ln, v2 = uv * ln;
    if (p > 0.f) {
      v0 *= dropout_keep(se, m, c, 3 * hv, p);
      v1 *= dropout_keep(se, m, hv + c, 3 * hv, p);
      v2 *= dropout_keep(se, m, 2 * hv + c, 3 * hv, p);
    }
    orow[c] = v0;
    orow[hv + c] = v1;
    orow[2 * hv + c] = v2;
  }
}

// y = o_in @ W_o^T + b_o + x_res   (K = 3 hdv, N = D; W_o row-major (D, K))
struct OpLinRes : NoStats {
  static constexpr bool B_N_CONTIG = false;
  const int64_t* offsets;
  int B, K, N;
  const float* a;
  int64_t lda;
  const float* w;
  const float* bias;
  const float* xres;
  int64_t ldx;
  float* y;
  int64_t ldy;
  static constexpr int NSRC = 1;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(a, lda, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(a, lda, m0, t); }
  __device__ int64_t a_ld0() const { return lda; }
  __device__ int64_t a_ld1() const { return lda; }
  __device__ float a_xform(float v, float, int64_t, int, float2, bool) const { return v; }
  __device__ int bks() const { return 1; }
  __device__ int bns() const { return K; }
  template <int NT>
  struct Epi {};
  template <int NT>
  __device__ void epi_load(Epi<NT>&, int64_t, int, int64_t) const {}
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>&, int64_t mrow, int ncol, int64_t total) const {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      if (m >= total) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        if (n >= N) continue;
        const float bv = bias ? as_global(bias)[n] : 0.f;
        const float xv = xres ? as_global(xres)[m * ldx + n] : 0.f;
        y[m * ldy + n] = (acc[t][r] + bv) + xv;
      }
    }
  }
};

// g = (dy @ W_o) * dropout mask   (K = D, N = 3 hdv; W_o row-major (D, N))
struct OpCatG : NoStats {
  static constexpr bool B_N_CONTIG = true;
  const int64_t* offsets;
  int B, K, N;
  const float* dy;
  int64_t lddy;
  const float* w;
  float p;
  uint64_t seed;
  const int64_t* seed_off;
  float* g;
  static constexpr int NSRC = 1;
  __device__ __amdgpu_buffer_rsrc_t a_rsrc0(int64_t m0, int64_t t) const { return rows_rsrc(dy, lddy, m0, t); }
  __device__ __amdgpu_buffer_rsrc_t a_rsrc1(int64_t m0, int64_t t) const { return rows_rsrc(dy, lddy, m0, t); }
  __device__ int64_t a_ld0() const { return lddy; }
  __device__ int64_t a_ld1() const { return lddy; }
  __device__ float a_xform(float v, float, int64_t, int, float2, bool) const { return v; }
  __device__ int bks() const { return N; }
  __device__ int bns() const { return 1; }
  template <int NT>
  struct Epi {};
  template <int NT>
  __device__ void epi_load(Epi<NT>&, int64_t, int, int64_t) const {}
  template <int NT>
  __device__ void epilogue(f4 (&acc)[NT], const Epi<NT>&, int64_t mrow, int ncol, int64_t total) const {
    const uint64_t se = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = mrow + r;
      if (m >= total) continue;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = ncol + 16 * t;
        if (n >= N) continue;
        g[m * N + n] = p > 0.f ? acc[t][r] * dropout_keep(se, m, n, N, p) : acc[t][r];
      }
    }
  }
};

// du = (g0 + g2 LN(a)) (* silu'(h_u)),  d_attn = LayerNorm_bwd(a; g1 + g2 u)
__global__ __launch_bounds__(256) void cat_bwd_rows_kernel(const float* g, const float* u, int64_t ldu,
                                                           const float* attn, int64_t lda,
                                                           const float2* a_stats, const float* h_u,
                                                           int64_t ldh, const int64_t* offsets, int B,
                                                           int hv, float* du, int64_t lddu, float* da,
                                                           int64_t ldda) {
  const int64_t total = offsets[B];
  const int64_t m = (int64_t)blockIdx.x * 4 + wave_id();
  if (m >= total) return;
  const int lane = threadIdx.x & 63;
  const float2 st = ld_f2(a_stats, m);
  gptr<float> grow = as_global(g) + m * 3 * hv;
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < hv; c += 64) {
    const float ln = (as_global(attn)[m * lda + c] - st.x) * st.y;
    const float uv = as_global(u)[m * ldu + c];
    const float g0 = grow[c], g1 = grow[hv + c], g2 = grow[2 * hv + c];
    float d = g0 + g2 * ln;
    if (h_u) d *= silu_grad_(as_global(h_u)[m * ldh + c]);
    du[m * lddu + c] = d;
    const float dln = g1 + g2 * uv;
    s1 += dln;
    s2 += dln * ln;
  }
  const float mean1 = wave_sum(s1) / (float)hv, mean2 = wave_sum(s2) / (float)hv;
  for (int c = lane; c < hv; c += 64) {
    const float ln = (as_global(attn)[m * lda + c] - st.x) * st.y;
    const float uv = as_global(u)[m * ldu + c];
    const float dln = grow[hv + c] + grow[2 * hv + c] * uv;
    da[m * ldda + c] = st.y * (dln - mean1 - ln * mean2);
  }
}

}  // namespace gr

extern "C" int hstu_gate_o_cat_wide_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                        const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                                        const float* w_o, const float* b_o, const float* x_res,
                                        int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                        const int64_t* seed_offset, float* attn_stats, float* o_in,
                                        float* y, int64_t ld_y, void* stream) {
  using namespace gr;
  GR_REQUIRE(u && attn && offsets && w_o && o_in && y && attn_stats,
             "hstu_gate_o_cat_wide_fwd: null pointer (o_in is required: the GEMM operand)");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0 && max_rows >= 0, "hstu_gate_o_cat_wide_fwd: bad sizes");
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_gate_o_cat_wide_fwd: dropout_p %f", dropout_p);
  if (max_rows == 0 || B == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  GR_TIMED("gate_o_fwd", st, hipLaunchKernelGGL(cat_oin_kernel, dim3((unsigned)((max_rows + 3) / 4)), dim3(256), 0, st,
                                                u, ld_u, attn, ld_attn, offsets, B, hdv, eps, dropout_p, seed,
                                                seed_offset, (float2*)attn_stats, o_in));
  GR_LAUNCH_CHECK("hstu_gate_o_cat_wide_fwd(o_in)");
  OpLinRes op{};
  op.offsets = offsets; op.B = B; op.K = 3 * hdv; op.N = D;
  op.a = o_in; op.lda = 3 * hdv; op.w = w_o; op.bias = b_o; op.xres = x_res; op.ldx = ld_x;
  op.y = y; op.ldy = ld_y;
  return launch_rowpanel(op, max_rows, false, "hstu_gate_o_fwd", st);
}

extern "C" int hstu_gate_o_cat_wide_bwd(const float* dy, int64_t ld_dy, const int64_t* offsets, int B,
                                        int64_t max_rows, int hdv, int D, const float* w_o,
                                        const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                        const float* attn_stats, const float* h_u, int64_t ld_h,
                                        float dropout_p, uint64_t seed, const int64_t* seed_offset,
                                        float* g, float* du, int64_t ld_du, float* d_attn, int64_t ld_da,
                                        void* stream) {
  using namespace gr;
  GR_REQUIRE(dy && offsets && w_o && u && attn && attn_stats && g && du && d_attn,
             "hstu_gate_o_cat_wide_bwd: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && B >= 0 && max_rows >= 0, "hstu_gate_o_cat_wide_bwd: bad sizes");
  if (max_rows == 0 || B == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  OpCatG op{};
  op.offsets = offsets; op.B = B; op.K = D; op.N = 3 * hdv;
  op.dy = dy; op.lddy = ld_dy; op.w = w_o; op.p = dropout_p; op.seed = seed; op.seed_off = seed_offset;
  op.g = g;
  const int rc = launch_rowpanel(op, max_rows, false, "hstu_gate_o_bwd", st);
  if (rc) return rc;
  GR_TIMED("gate_o_bwd", st, hipLaunchKernelGGL(cat_bwd_rows_kernel, dim3((unsigned)((max_rows + 3) / 4)), dim3(256), 0, st,
                                                g, u, ld_u, attn, ld_attn, (const float2*)attn_stats, h_u, ld_h,
                                                offsets, B, hdv, du, ld_du, d_attn, ld_da));
  GR_LAUNCH_CHECK("hstu_gate_o_cat_wide_bwd(rows)");
  return 0;
}

// ------------------------------------------------------------------ layer boundaries
// gate_o(l) + ln_uvqk(l + 1) and ln_uvqk_bwd(l) + gate_o_bwd(l - 1) as ONE row-wave launch
// each (rowwave2_kernel): at ml-1m every projection launch is latency-bound (a 16-row
// unit per wave and ~1.6 units per SIMD), so the boundary's two launches cost about twice
// one, and the boundary rows (y, dx) are handed over in registers.  Shapes outside the
// instantiated set (D, h dv <= 64, n_out <= 256) fall back to the two separate launches,
// results agreeing to fp32 summation order (the fused UVQK product is a row-wave chain
// where the separate launch may take the row panel; bit-identical on the fallback shapes).
namespace gr {

static int rw2_bucket_small(int x) {  // the boundary's shared width (D and h dv) in 16-col groups
  const int g = ceil_div(x, 16);
  return g <= 1 ? 1 : g <= 2 ? 2 : g <= 4 ? 4 : -1;
}

template <int KG1, int NT1, int NT2, class Op1, class Op2>
static int rw2_launch(const Op1& op1, const Op2& op2, int64_t max_rows, const char* tname,
                      hipStream_t st) {
  using C1 = RowWaveCfg<KG1, NT1>;
  using C2 = RowWaveCfg<NT1, NT2>;
  constexpr size_t lds = C1::LDS_BYTES + C2::LDS_BYTES;
  if constexpr (lds > 150 * 1024) {
    return -1;
  } else {
    const int64_t units = (max_rows + 15) / 16;
    int grid = (int)((units + 3) / 4);
    const int per_cu = (int)((160 * 1024) / lds);
    const int cap = (per_cu < 1 ? 1 : per_cu > 4 ? 4 : per_cu) * num_cus();
    if (grid > cap) grid = cap;
    if (grid < 1) return 0;
    GR_TIMED(tname, st, hipLaunchKernelGGL((rowwave2_kernel<KG1, NT1, NT2, Op1, Op2>), dim3(grid),
                                           dim3(256), lds, st, op1, op2));
    GR_LAUNCH_CHECK(tname);
    return 0;
  }
}

template <int W, int NT2>
static int bfwd_launch(const RwArgsGateO& a1, const RwArgsLnUvqk& a2, int64_t max_rows, hipStream_t st) {
  RwGateO<W, W, 2> o1;
  RwLnUvqk<W, NT2, 2> o2;
  a1.fill(o1);
  a2.fill(o2);
  return rw2_launch<W, W, NT2>(o1, o2, max_rows, "boundary_fwd", st);
}
template <int W>
static int bfwd_nt(const RwArgsGateO& a1, const RwArgsLnUvqk& a2, int nt2, int64_t max_rows, hipStream_t st) {
  switch (nt2) {
    case 4: return bfwd_launch<W, 4>(a1, a2, max_rows, st);
    case 8: return bfwd_launch<W, 8>(a1, a2, max_rows, st);
    case 13: return bfwd_launch<W, 13>(a1, a2, max_rows, st);
    case 16: return bfwd_launch<W, 16>(a1, a2, max_rows, st);
  }
  return -1;
}

template <int KG1, int W>
static int bbwd_launch(const RwArgsLnUvqkBwd& a1, const RwArgsGateOBwd& a2, int64_t max_rows, hipStream_t st) {
  RwLnUvqkBwd<KG1, W, 2> o1;
  RwGateOBwd<W, W, 2> o2;
  a1.fill(o1);
  a2.fill(o2);
  return rw2_launch<KG1, W, W>(o1, o2, max_rows, "boundary_bwd", st);
}
template <int W>
static int bbwd_kg(const RwArgsLnUvqkBwd& a1, const RwArgsGateOBwd& a2, int kg1, int64_t max_rows, hipStream_t st) {
  switch (kg1) {
    case 4: return bbwd_launch<4, W>(a1, a2, max_rows, st);
    case 8: return bbwd_launch<8, W>(a1, a2, max_rows, st);
    case 13: return bbwd_launch<13, W>(a1, a2, max_rows, st);
    case 16: return bbwd_launch<16, W>(a1, a2, max_rows, st);
  }
  return -1;
}

}  // namespace gr

extern "C" int hstu_boundary_fwd(const float* u, int64_t ld_u, const float* attn, int64_t ld_attn,
                                 const int64_t* offsets, int B, int64_t max_rows, int hdv, int D,
                                 const float* w_o, const float* b_o, const float* x_res,
                                 int64_t ld_x, float eps, float dropout_p, uint64_t seed,
                                 const int64_t* seed_offset, float* attn_stats, float* o_in,
                                 float* y, int64_t ld_y, const float* w_uvqk, int n_out,
                                 int activation, float* x_stats, float* h_pre, float* uvqk,
                                 int64_t ld_out, void* stream) {
  GR_REQUIRE(u && attn && offsets && w_o && y && attn_stats && w_uvqk && uvqk && x_stats,
             "hstu_boundary_fwd: null pointer");
  GR_REQUIRE(hdv > 0 && D > 0 && n_out > 0 && B >= 0, "hstu_boundary_fwd: bad sizes");
  GR_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "hstu_boundary_fwd: dropout_p %f", dropout_p);
  GR_REQUIRE(activation == 0 || activation == 1, "hstu_boundary_fwd: activation must be 0|1");
  const hipStream_t st = (hipStream_t)stream;
  if (rw_enabled()) {
    RwArgsGateO a1{offsets, B, hdv, D, u, ld_u, attn, ld_attn, w_o, b_o, x_res, ld_x, eps,
                   dropout_p, seed, seed_offset, (float2*)attn_stats, o_in, y, ld_y};
    RwArgsLnUvqk a2{offsets, B, D, n_out, y, ld_y, w_uvqk, eps, activation, (float2*)x_stats,
                    h_pre, uvqk, ld_out};
    const int w = std::max(rw2_bucket_small(hdv), rw2_bucket_small(D));
    const int nt2 = rw_bucket(n_out);
    const int vec = rw_vec({u, attn, x_res, o_in, y, h_pre, uvqk},
                           {ld_u, ld_attn, ld_x, ld_y, ld_out, hdv, D, n_out});
    const bool fits = rw2_bucket_small(hdv) > 0 && rw2_bucket_small(D) > 0 && nt2 >= 4 && vec &&
                      max_rows * 4 * 1024 <= 0x7fffffffLL;
    if (fits) {
      int rc = -1;
      if (w == 1) rc = bfwd_nt<1>(a1, a2, nt2, max_rows, st);
      else if (w == 2) rc = bfwd_nt<2>(a1, a2, nt2, max_rows, st);
      else rc = bfwd_nt<4>(a1, a2, nt2, max_rows, st);
      if (rc >= 0) return rc;
    }
  }
  if (int rc = hstu_gate_o_fwd(u, ld_u, attn, ld_attn, offsets, B, max_rows, hdv, D, w_o, b_o, x_res,
                               ld_x, eps, dropout_p, seed, seed_offset, attn_stats, o_in, y, ld_y,
                               stream))
    return rc;
  return hstu_ln_uvqk_fwd(y, ld_y, offsets, B, max_rows, D, w_uvqk, n_out, eps, activation, x_stats,
                          h_pre, uvqk, ld_out, stream);
}

extern "C" int hstu_boundary_bwd(const float* dh, int64_t ld_dh, const int64_t* offsets, int B,
                                 int64_t max_rows, int D, int n_out, const float* w_uvqk,
                                 const float* x, int64_t ld_x, const float* x_stats,
                                 const float* dy_res, int64_t ld_dy, float* dx, int64_t ld_dx,
                                 int hdv, const float* w_o, const float* u, int64_t ld_u,
                                 const float* attn, int64_t ld_attn, const float* attn_stats,
                                 const float* h_u, int64_t ld_h, float dropout_p, uint64_t seed,
                                 const int64_t* seed_offset, float* du, int64_t ld_du,
                                 float* d_attn, int64_t ld_da, void* stream) {
  GR_REQUIRE(dh && offsets && w_uvqk && x && x_stats && dx && w_o && u && attn && attn_stats && du &&
                 d_attn,
             "hstu_boundary_bwd: null pointer");
  GR_REQUIRE(D > 0 && n_out > 0 && hdv > 0 && B >= 0, "hstu_boundary_bwd: bad sizes");
  const hipStream_t st = (hipStream_t)stream;
  if (rw_enabled()) {
    RwArgsLnUvqkBwd a1{offsets, B, n_out, D, dh, ld_dh, w_uvqk, x, ld_x, (const float2*)x_stats,
                       dy_res, ld_dy, dx, ld_dx};
    RwArgsGateOBwd a2{offsets, B, D, hdv, dx, ld_dx, w_o, u, ld_u, attn, ld_attn,
                      (const float2*)attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du,
                      d_attn, ld_da};
    const int w = std::max(rw2_bucket_small(hdv), rw2_bucket_small(D));
    const int kg1 = rw_bucket(n_out);
    const int vec = rw_vec({dh, x, dy_res, dx, u, attn, h_u, du, d_attn},
                           {ld_dh, ld_x, ld_dy, ld_dx, ld_u, ld_attn, ld_h, ld_du, ld_da, n_out, D, hdv});
    const bool fits = rw2_bucket_small(hdv) > 0 && rw2_bucket_small(D) > 0 && kg1 >= 4 && vec &&
                      max_rows * 4 * 1024 <= 0x7fffffffLL;
    if (fits) {
      int rc = -1;
      if (w == 1) rc = bbwd_kg<1>(a1, a2, kg1, max_rows, st);
      else if (w == 2) rc = bbwd_kg<2>(a1, a2, kg1, max_rows, st);
      else rc = bbwd_kg<4>(a1, a2, kg1, max_rows, st);
      if (rc >= 0) return rc;
    }
  }
  if (int rc = hstu_ln_uvqk_bwd(dh, ld_dh, offsets, B, max_rows, D, n_out, w_uvqk, x, ld_x, x_stats,
                                dy_res, ld_dy, dx, ld_dx, stream))
    return rc;
  return hstu_gate_o_bwd(dx, ld_dx, offsets, B, max_rows, hdv, D, w_o, u, ld_u, attn, ld_attn,
                         attn_stats, h_u, ld_h, dropout_p, seed, seed_offset, du, ld_du, d_attn,
                         ld_da, stream);
}

#endif  // GR_LINEAR_LIB_ONLY
