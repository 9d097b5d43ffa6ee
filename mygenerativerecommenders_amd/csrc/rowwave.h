// Row-wave projection GEMM for the narrow STU shapes (K <= 256, K x N weight panel fits
// in LDS; ml-1m: D = 50, n_out = 200) — gfx950, f32 MFMA.
//
// Work unit = ONE WAVE x 16 rows.  A workgroup stages the whole weight panel W (K x N)
// in LDS once and its 4 waves then loop over 16-row units (grid-stride, persistent),
// with the next unit's rows prefetched into registers while the current one runs.
// Per unit a lane holds the 16 rows' A values in the MFMA B-operand layout with a
// permuted K order: lane (row lr, group lg) loads A[row][16g + 4lg .. 16g + 4lg + 3]
// (one 8/16-byte load per g), and k-step j of group g uses k = 16g + 4lg + j — the
// weight side reads W[16g + 4lg + j][n] from LDS accordingly.  The product is taken
// transposed, C^T = W^T A^T, so a lane ends with 4 CONSECUTIVE output columns of its
// row (acc[t][r] = C[row lr][16t + 4lg + r]) — vector stores and in-register row
// reductions (lanes lr, lr+16, lr+32, lr+48 hold one row).
#pragma once

#include "common.h"

namespace gr {

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// Buffer descriptor over rows [0, rows) of a (rows, ld) f32 matrix starting at column c0
// of `base`; loads past the last row return 0, stores there are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mat_rsrc(const float* base, int64_t ld,
                                                          int64_t rows, int c0) {
  int64_t bytes = rows > 0 ? (rows * ld - c0) * 4 : 0;
  if (bytes > 0x7fffffff) bytes = 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + c0), 0, (int)bytes, 0x00020000);
}

// Byte offset that fails the buffer range check: loads through it return 0 and stores
// are dropped — column / row masking without branches.
constexpr int OOB = OOB_OFF;

// A lane's "quad": 4 columns of a 16-column tile (base tb) owned by lane group lg.
//   VEC = 4 (16-byte aligned rows):  tb + 4lg + e                     (one 16-byte access)
//   VEC = 2 ( 8-byte aligned rows):  tb + 2lg + (e & 1) + 8 (e >> 1)  (two 8-byte accesses;
//                                     the 4 lane groups cover 32 contiguous bytes each)
// With N % VEC == 0 each access is entirely inside or outside [0, N).
template <int VEC>
__device__ __forceinline__ int qcol(int tb, int lg, int e) {
  return VEC == 4 ? tb + 4 * lg + e : tb + 2 * lg + (e & 1) + 8 * (e >> 1);
}
// aux: cache policy of the loads (16 = sc1: served by L2, not the CU's vector L1 -- rows
// this wave stored in the same launch, whose L1 lines another wave may have filled first)
template <int VEC>
__device__ __forceinline__ f4 ldq(__amdgpu_buffer_rsrc_t r, int64_t row_off, int tb, int lg,
                                  int N = 1 << 30, int aux = 0) {
  if constexpr (VEC == 4) {
    const int c = qcol<4>(tb, lg, 0);
    const u4v v = aux ? __builtin_amdgcn_raw_buffer_load_b128(r, c < N ? (int)((row_off + c) * 4) : OOB, 0, 16)
                      : __builtin_amdgcn_raw_buffer_load_b128(r, c < N ? (int)((row_off + c) * 4) : OOB, 0, 0);
    return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
  } else {
    const int c0 = qcol<2>(tb, lg, 0), c2 = qcol<2>(tb, lg, 2);
    const int o0 = c0 < N ? (int)((row_off + c0) * 4) : OOB, o2 = c2 < N ? (int)((row_off + c2) * 4) : OOB;
    const u2v a = aux ? __builtin_amdgcn_raw_buffer_load_b64(r, o0, 0, 16) : __builtin_amdgcn_raw_buffer_load_b64(r, o0, 0, 0);
    const u2v b = aux ? __builtin_amdgcn_raw_buffer_load_b64(r, o2, 0, 16) : __builtin_amdgcn_raw_buffer_load_b64(r, o2, 0, 0);
    return f4{__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(b.x), __uint_as_float(b.y)};
  }
}
template <int VEC>
__device__ __forceinline__ void stq(__amdgpu_buffer_rsrc_t r, int64_t row_off, int tb, int lg,
                                    int N, f4 v) {
  if constexpr (VEC == 4) {
    const int c = qcol<4>(tb, lg, 0);
    __builtin_amdgcn_raw_buffer_store_b128(
        u4v{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])},
        r, c < N ? (int)((row_off + c) * 4) : OOB, 0, 0);
  } else {
    const int c0 = qcol<2>(tb, lg, 0), c2 = qcol<2>(tb, lg, 2);
    __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(v[0]), __float_as_uint(v[1])}, r,
                                          c0 < N ? (int)((row_off + c0) * 4) : OOB, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(v[2]), __float_as_uint(v[3])}, r,
                                          c2 < N ? (int)((row_off + c2) * 4) : OOB, 0, 0);
  }
}

// sum over the 4 lanes holding one row (lanes lr, lr + 16, lr + 32, lr + 48)
__device__ __forceinline__ float row4_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

template <int KG, int NT>
struct RowWaveCfg {
  static constexpr int KP = KG * 16;
  static constexpr int NP = NT * 16;
  // == 4 mod 16: the 4 lane groups' k-rows of one step (2 or 4 rows apart) cover every
  // bank exactly twice (the minimum for 64 lanes)
  static constexpr int LDW = NP + 4;
  static constexpr size_t LDS_BYTES = sizeof(float) * KP * LDW;
};

// Op interface (VEC = quad access width, see qcol):
//   K, N, offsets/B (total rows = offsets[B]); weight W'(k, n) = w[k * bks() + n * bns()],
//   K_CONTIG: bks() == 1 (staging walks k fastest);
//   setup(total); load(src, m, lg) issues a unit's input loads; prep(src, a, m, row_ok, lg)
//   turns them into the A quads; epi_load(es, m, row_ok, lg) issues the epilogue's row
//   inputs before the MFMAs; epi(acc, es, m, row_ok, lg) consumes acc[t][e] =
//   C[m][qcol(16t, lg, e)].
// Stage an Op's weight panel W' (KG*16 x NT*16, LDS row stride LDW) into LDS once per
// workgroup (the same layout and load order as rowwave_kernel's staging below).
template <int KG, int NT, class Op>
__device__ __forceinline__ void rw_stage_w(const Op& op, float* Wl) {
  using C = RowWaveCfg<KG, NT>;
  constexpr int VEC = Op::VEC;
  const int tid = threadIdx.x;
  constexpr int FP = Op::K_CONTIG ? C::KP : C::NP;
  constexpr int SP = Op::K_CONTIG ? C::NP : C::KP;
  constexpr int FP2 = FP <= 16 ? 16 : FP <= 32 ? 32 : FP <= 64 ? 64 : FP <= 128 ? 128 : 256;
  constexpr int SSTEP = 256 / FP2;
  constexpr int ITER = SP / SSTEP;
  constexpr int BATCH = ITER < 64 ? ITER : 64;
  const int f = tid % FP2, s0 = tid / FP2;
  const int64_t wlast = (int64_t)(op.K - 1) * op.bks() + (int64_t)(op.N - 1) * op.bns() + 1;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)op.w, 0, (int)(wlast * 4 < 0x7fffffff ? wlast * 4 : 0x7fffffff), 0x00020000);
  if (f < FP) {
#pragma unroll 1
    for (int i0 = 0; i0 < ITER; i0 += BATCH) {
      float v[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int sl = s0 + (i0 + i) * SSTEP;
        const int k = Op::K_CONTIG ? f : sl;
        const int p = Op::K_CONTIG ? sl : f;
        const int n = (p & ~15) + qcol<VEC>(0, (p & 15) >> 2, p & 3);
        const bool ok = k < op.K && n < op.N;
        v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rw, ok ? (int)(((int64_t)k * op.bks() + (int64_t)n * op.bns()) * 4) : OOB, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int sl = s0 + (i0 + i) * SSTEP;
        if (i0 + i < ITER) Wl[(Op::K_CONTIG ? f : sl) * C::LDW + (Op::K_CONTIG ? sl : f)] = v[i];
      }
    }
  }
}

// rw_stage_w split in two: load() issues the panel's loads into registers (e.g. before other
// work of the kernel, so they land meanwhile), store() writes them to LDS later (the same
// layout and values as rw_stage_w).  ITER <= 64 loads per thread.
template <int KG, int NT, class Op>
struct RwStage {
  using C = RowWaveCfg<KG, NT>;
  static constexpr int VEC = Op::VEC;
  static constexpr int FP = Op::K_CONTIG ? C::KP : C::NP;
  static constexpr int SP = Op::K_CONTIG ? C::NP : C::KP;
  static constexpr int FP2 = FP <= 16 ? 16 : FP <= 32 ? 32 : FP <= 64 ? 64 : FP <= 128 ? 128 : 256;
  static constexpr int SSTEP = 256 / FP2;
  static constexpr int ITER = SP / SSTEP;
  static_assert(ITER <= 64, "one batch of loads");
  float v[ITER];
  __device__ __forceinline__ void load(const Op& op) {
    const int tid = threadIdx.x;
    const int f = tid % FP2, s0 = tid / FP2;
    const int64_t wlast = (int64_t)(op.K - 1) * op.bks() + (int64_t)(op.N - 1) * op.bns() + 1;
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)op.w, 0, (int)(wlast * 4 < 0x7fffffff ? wlast * 4 : 0x7fffffff), 0x00020000);
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int sl = s0 + i * SSTEP;
      const int k = Op::K_CONTIG ? f : sl;
      const int p = Op::K_CONTIG ? sl : f;
      const int n = (p & ~15) + qcol<VEC>(0, (p & 15) >> 2, p & 3);
      const bool ok = f < FP && k < op.K && n < op.N;
      v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rw, ok ? (int)(((int64_t)k * op.bks() + (int64_t)n * op.bns()) * 4) : OOB, 0, 0));
    }
  }
  __device__ __forceinline__ void store(float* Wl) const {
    const int tid = threadIdx.x;
    const int f = tid % FP2, s0 = tid / FP2;
    if (f < FP) {
#pragma unroll
      for (int i = 0; i < ITER; ++i) {
        const int sl = s0 + i * SSTEP;
        Wl[(Op::K_CONTIG ? f : sl) * C::LDW + (Op::K_CONTIG ? sl : f)] = v[i];
      }
    }
  }
};

// acc[t] = sum_k W'(k, 16 t + .) a(k): the row-wave k-step loop of rowwave_kernel
template <int KG, int NT, int VEC>
__device__ __forceinline__ void rw_mma(const float* Wl, const float (&a)[KG][4], f4 (&acc)[NT],
                                       int lr, int lg) {
  using C = RowWaveCfg<KG, NT>;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
  int wofs = 0;
  asm volatile("" : "+v"(wofs));
  const float* wbase = Wl + wofs + lr;
  float wv[2][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wv[0][t] = wbase[qcol<VEC>(0, lg, 0) * C::LDW + 16 * t];
#pragma unroll
  for (int s = 0; s < 4 * KG; ++s) {
    const int g = s >> 2, e = s & 3;
    if (s + 1 < 4 * KG) {
      const float* wrow = wbase + qcol<VEC>(16 * ((s + 1) >> 2), lg, (s + 1) & 3) * C::LDW;
#pragma unroll
      for (int t = 0; t < NT; ++t) wv[(s + 1) & 1][t] = wrow[16 * t];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(wv[s & 1][t], a[g][e], acc[t]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Two row-wave GEMMs chained per 16-row unit (a layer boundary of the encoder): Op1's
// epilogue stores its output rows AND hands the quads, still in registers, to Op2 as its
// A operand (Op1's NT == Op2's KG: one lane's 4 consecutive output columns are exactly
// its 4 k values of the next product).  Both weight panels stay in LDS.  The forward
// boundary is gate_o(l) -> ln_uvqk(l + 1) (y = x + o W_o^T + b, then silu(LN(y) W_uvqk)),
// the backward one ln_uvqk_bwd(l) -> gate_o_bwd(l - 1) (dx_l is the dy of layer l - 1):
// one launch and no re-read of the boundary rows instead of two launches.
#ifdef GR_STAMP
// Diagnostic build only (-DGR_STAMP): per-wave s_memrealtime stamps of rowwave2_kernel
// (entry, panels staged, product 1, epilogue 1, product 2, epilogue 2), gr_rw_stamp_read.
static __device__ unsigned long long gr_rw_buf[1 << 15];
#define GR_RW_T(i)                                                                  \
  do {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    rw_t[i] = __builtin_amdgcn_s_memrealtime();                                     \
    __builtin_amdgcn_sched_barrier(0);                                              \
  } while (0)
#else
#define GR_RW_T(i) do { } while (0)
#endif

template <int KG1, int NT1, int NT2, class Op1, class Op2>
__global__ __launch_bounds__(256) void rowwave2_kernel(Op1 op1, Op2 op2) {
#ifdef GR_STAMP
  unsigned long long rw_t[8] = {};
#endif
  GR_RW_T(0);
  using C1 = RowWaveCfg<KG1, NT1>;
  constexpr int VEC = Op1::VEC;
  static_assert(Op2::VEC == VEC, "one quad layout");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* W1 = reinterpret_cast<float*>(smem);
  float* W2 = W1 + C1::KP * C1::LDW;
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  (void)tid;
  const int64_t total = op1.offsets[op1.B];
  op1.setup(total);
  op2.setup(total);
  const int64_t n_units = (total + 15) / 16;
  int64_t u = (int64_t)blockIdx.x * 4 + w;
  const int64_t ustep = (int64_t)gridDim.x * 4;
  typename Op1::Src cur;
  if (u < n_units) op1.load(cur, u * 16 + lr, lg);
  rw_stage_w<KG1, NT1>(op1, W1);
  rw_stage_w<NT1, NT2>(op2, W2);
  __syncthreads();
  GR_RW_T(1);
  for (; u < n_units; u += ustep) {
    const int64_t m = u * 16 + lr;
    const bool ok = m < total;
    float a1[KG1][4];
    op1.prep(cur, a1, m, ok, lg);
    typename Op1::Epi es1;
    op1.epi_load(es1, m, ok, lg);
    typename Op2::Epi es2;
    op2.epi_load(es2, m, ok, lg);
    f4 acc1[NT1];
    rw_mma<KG1, NT1, VEC>(W1, a1, acc1, lr, lg);
#ifdef GR_STAMP
    asm volatile("" ::"v"(acc1[0][0]));
#endif
    GR_RW_T(2);
    typename Op2::Src s2;
    op1.epi(acc1, es1, m, ok, lg, s2.v);
    if (u + ustep < n_units) op1.load(cur, m + ustep * 16, lg);  // the next unit's rows
    float a2[NT1][4];
    op2.prep(s2, a2, m, ok, lg);
#ifdef GR_STAMP
    asm volatile("" ::"v"(a2[0][0]));
#endif
    GR_RW_T(3);
    f4 acc2[NT2];
    rw_mma<NT1, NT2, VEC>(W2, a2, acc2, lr, lg);
#ifdef GR_STAMP
    asm volatile("" ::"v"(acc2[0][0]));
#endif
    GR_RW_T(4);
    op2.epi(acc2, es2, m, ok, lg);
    GR_RW_T(5);
  }
#ifdef GR_STAMP
  const int slot = ((int)blockIdx.x * 4 + w) * 8;
  if (lane == 0 && slot + 8 <= (1 << 15))
    for (int i = 0; i < 8; ++i) gr_rw_buf[slot + i] = rw_t[i];
#endif
}

template <int KG, int NT, class Op>
__global__ __launch_bounds__(256) void rowwave_kernel(Op op) {
  using C = RowWaveCfg<KG, NT>;
  constexpr int VEC = Op::VEC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Wl = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, w = wave_id(), lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int64_t total = op.offsets[op.B];
  op.setup(total);
  const int64_t n_units = (total + 15) / 16;
  int64_t u = (int64_t)blockIdx.x * 4 + w;
  const int64_t ustep = (int64_t)gridDim.x * 4;
  typename Op::Src cur, nxt;
  if (u < n_units) op.load(cur, u * 16 + lr, lg);  // first unit's rows in flight during staging

#ifndef GR_RW_NOSTAGE
  // Stage W' once per workgroup.  LDS column 16t + i holds weight column 16t + pi(i),
  // pi(4g + e) = qcol(0, g, e): MFMA output row i of tile t is then exactly the column
  // the lane's quad stores.  Threads walk the memory-contiguous index fastest; batches
  // of 16 loads in flight.
  {
    constexpr int FP = Op::K_CONTIG ? C::KP : C::NP;  // fast extent
    constexpr int SP = Op::K_CONTIG ? C::NP : C::KP;  // slow extent
    constexpr int FP2 = FP <= 16 ? 16 : FP <= 32 ? 32 : FP <= 64 ? 64 : FP <= 128 ? 128 : 256;
    constexpr int SSTEP = 256 / FP2;
    constexpr int ITER = SP / SSTEP;
    // the whole panel's loads in flight at once (one L2 round trip per workgroup; batches
    // of 16 cost C2's 400 one-unit-per-wave workgroups three extra trips before any MFMA)
    constexpr int BATCH = ITER < 64 ? ITER : 64;
    const int f = tid % FP2, s0 = tid / FP2;
    // W through a buffer descriptor: entries outside K x N read as 0 from the range check
    // (a select after a plain load let hipcc sink each load into a branch and wait for it
    // there: ITER serial round trips per workgroup)
    const int64_t wlast = (int64_t)(op.K - 1) * op.bks() + (int64_t)(op.N - 1) * op.bns() + 1;
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)op.w, 0, (int)(wlast * 4 < 0x7fffffff ? wlast * 4 : 0x7fffffff), 0x00020000);
    if (f < FP) {
#pragma unroll 1
      for (int i0 = 0; i0 < ITER; i0 += BATCH) {
        float v[BATCH];
#pragma unroll
        for (int i = 0; i < BATCH; ++i) {
          const int sl = s0 + (i0 + i) * SSTEP;
          const int k = Op::K_CONTIG ? f : sl;
          const int p = Op::K_CONTIG ? sl : f;  // LDS column
          const int n = (p & ~15) + qcol<VEC>(0, (p & 15) >> 2, p & 3);
          const bool ok = k < op.K && n < op.N;
          v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rw, ok ? (int)(((int64_t)k * op.bks() + (int64_t)n * op.bns()) * 4) : OOB, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < BATCH; ++i) {
          const int sl = s0 + (i0 + i) * SSTEP;
          if (i0 + i < ITER) Wl[(Op::K_CONTIG ? f : sl) * C::LDW + (Op::K_CONTIG ? sl : f)] = v[i];
        }
      }
    }
  }
#endif
  __syncthreads();
  for (; u < n_units; u += ustep) {
    const int64_t m = u * 16 + lr;
    const bool more = u + ustep < n_units;
    if (more) op.load(nxt, m + ustep * 16, lg);
    float a[KG][4];
    op.prep(cur, a, m, m < total, lg);
    // the epilogue's own row inputs are issued now, so they land while the MFMAs run
    // (loaded inside epi they added one dependent round trip per unit)
    typename Op::Epi es;
    op.epi_load(es, m, m < total, lg);
    f4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4_zero();
    // opaque zero: keeps hipcc from hoisting the (loop-invariant) LDS weight reads out
    // of the unit loop into hundreds of registers
    int wofs = 0;
    asm volatile("" : "+v"(wofs));
    const float* wbase = Wl + wofs + lr;
    // k-step s = (g, e) uses k = qcol(16g, lg, e); software-pipelined: the NT weight
    // values of step s+1 are read from LDS while the NT MFMAs of step s run
    float wv[2][NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) wv[0][t] = wbase[qcol<VEC>(0, lg, 0) * C::LDW + 16 * t];
#pragma unroll
    for (int s = 0; s < 4 * KG; ++s) {
      const int g = s >> 2, e = s & 3;
      if (s + 1 < 4 * KG) {
        const float* wrow = wbase + qcol<VEC>(16 * ((s + 1) >> 2), lg, (s + 1) & 3) * C::LDW;
#pragma unroll
        for (int t = 0; t < NT; ++t) wv[(s + 1) & 1][t] = wrow[16 * t];
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this step's MFMAs
#ifndef GR_RW_NOMFMA
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16x16x4(wv[s & 1][t], a[g][e], acc[t]);
#else
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t][0] += wv[s & 1][t] * a[g][e];
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
#ifndef GR_RW_NOSTORE
    op.epi(acc, es, m, m < total, lg);
#else
    float sink = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) sink += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    if (sink == 1.2345f) op.epi(acc, es, m, m < total, lg);
#endif
    if (more) cur = nxt;
  }
}

// ------------------------------------------------------------------ ops
// F1: uvqk = silu(LN(x) @ W), W (D, n_out) row-major; h_pre = pre-activation.
template <int KG, int NT, int VEC_>
struct RwLnUvqk {
  static constexpr int VEC = VEC_;
  static constexpr bool K_CONTIG = false;
  const int64_t* offsets;
  int B, K, N;
  const float* x;
  int64_t ldx;
  const float* w;
  float eps;
  int act;
  float2* x_stats;
  float* h_pre;
  float* out;
  int64_t ld_out;
  __amdgpu_buffer_rsrc_t rx, rh, ro;
  struct Src { f4 v[KG]; };
  __device__ int bks() const { return N; }
  __device__ int bns() const { return 1; }
  __device__ void setup(int64_t total) {
    rx = mat_rsrc(x, ldx, total, 0);
    rh = mat_rsrc(h_pre ? h_pre : out, ld_out, h_pre ? total : 0, 0);
    ro = mat_rsrc(out, ld_out, total, 0);
  }
  __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
    for (int g = 0; g < KG; ++g) s.v[g] = ldq<VEC>(rx, m * ldx, 16 * g, lg, K);
  }
  __device__ void prep(const Src& s, float (&a)[KG][4], int64_t m, bool row_ok, int lg) const {
    // columns >= K load as 0 (masked accesses), so plain sums are exact
    float sum = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) sum += s.v[g][e];
    const float mean = row4_sum(sum) * (1.f / (float)K);
    float sq = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = qcol<VEC>(16 * g, lg, e) < K ? s.v[g][e] - mean : 0.f;
        sq += d * d;
      }
    const float rstd = rsqrtf(row4_sum(sq) * (1.f / (float)K) + eps);
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        a[g][e] = qcol<VEC>(16 * g, lg, e) < K ? (s.v[g][e] - mean) * rstd : 0.f;
    if (lg == 0 && row_ok) x_stats[m] = make_float2(mean, rstd);
  }
  struct Epi {};
  __device__ void epi_load(Epi&, int64_t, bool, int) const {}
  __device__ void epi(f4 (&acc)[NT], const Epi&, int64_t m, bool, int lg) const {
    // rows past the end fall outside the descriptors (stores dropped)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      stq<VEC>(rh, m * ld_out, 16 * t, lg, N, acc[t]);  // records = 0 when h_pre is NULL
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act ? siluf_(acc[t][e]) : acc[t][e];
      stq<VEC>(ro, m * ld_out, 16 * t, lg, N, o);
    }
  }
};

__device__ __forceinline__ float rw_dropout_keep(uint64_t seed, int64_t m, int k, int K, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t hsh = hash_u32(seed, (uint64_t)m * (uint64_t)K + (uint64_t)k);
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  return hsh >= thr ? 1.f / (1.f - p) : 0.f;
}

// F3: y = dropout(u * LN(attn)) @ W_o^T + b_o + x;  W_o (D, hdv) row-major -> W'(k, n) = W_o[n][k]
template <int KG, int NT, int VEC_>
struct RwGateO {
  static constexpr int VEC = VEC_;
  static constexpr bool K_CONTIG = true;
  const int64_t* offsets;
  int B, K, N;  // K = hdv, N = D
  const float* u;
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
  float* o_in;
  float* y;
  int64_t ldy;
  int rd_aux = 0;  // cache policy of the attn loads (16: rows stored earlier in the launch)
  __amdgpu_buffer_rsrc_t ru, ra, rx, ro, ry, rb;
  uint64_t seed_eff;
  struct Src { f4 v[KG]; f4 uu[KG]; };
  __device__ int bks() const { return 1; }
  __device__ int bns() const { return K; }
  __device__ void setup(int64_t total) {
    ru = mat_rsrc(u, ldu, total, 0);
    ra = mat_rsrc(attn, lda, total, 0);
    rx = mat_rsrc(xres ? xres : y, ldx, xres ? total : 0, 0);
    ro = mat_rsrc(o_in ? o_in : y, K, o_in ? total : 0, 0);
    ry = mat_rsrc(y, ldy, total, 0);
    rb = mat_rsrc(bias ? bias : y, N, bias ? 1 : 0, 0);
    seed_eff = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  }
  __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      s.v[g] = ldq<VEC>(ra, m * lda, 16 * g, lg, K, rd_aux);
      s.uu[g] = ldq<VEC>(ru, m * ldu, 16 * g, lg, K);
    }
  }
  __device__ void prep(const Src& s, float (&a)[KG][4], int64_t m, bool row_ok, int lg) const {
    float sum = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) sum += s.v[g][e];
    const float mean = row4_sum(sum) * (1.f / (float)K);
    float sq = 0.f;
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = qcol<VEC>(16 * g, lg, e) < K ? s.v[g][e] - mean : 0.f;
        sq += d * d;
      }
    const float rstd = rsqrtf(row4_sum(sq) * (1.f / (float)K) + eps);
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = qcol<VEC>(16 * g, lg, e);
        float v = s.uu[g][e] * ((s.v[g][e] - mean) * rstd);
        if (p > 0.f) v *= rw_dropout_keep(seed_eff, m, k, K, p);
        a[g][e] = k < K ? v : 0.f;
        o[e] = a[g][e];
      }
      stq<VEC>(ro, m * K, 16 * g, lg, K, o);  // records = 0 when o_in is NULL
    }
    if (lg == 0 && row_ok) a_stats[m] = make_float2(mean, rstd);
  }
  struct Epi { f4 xv[NT], bv[NT]; };
  __device__ void epi_load(Epi& es, int64_t m, bool, int lg) const {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      es.xv[t] = ldq<VEC>(rx, m * ldx, 16 * t, lg, N);  // 0 when xres is NULL
      es.bv[t] = ldq<VEC>(rb, 0, 16 * t, lg, N);        // 0 when bias is NULL
    }
  }
  // out (optional): the stored y quads, for a fused consumer (rowwave2_kernel)
  __device__ void epi(f4 (&acc)[NT], const Epi& es, int64_t m, bool, int lg, f4* out = nullptr) const {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f4 xv = es.xv[t], bv = es.bv[t];
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (acc[t][e] + bv[e]) + xv[e];
      stq<VEC>(ry, m * ldy, 16 * t, lg, N, o);
      if (out) out[t] = o;
    }
  }
};

// B1: g = dy @ W_o (rows, hdv), W'(k, n) = W_o[k][n]; epilogue: dropout bwd,
//     du = g * LN(attn) (* silu'(h_u)), d_attn = LayerNorm_bwd(g * u).
template <int KG, int NT, int VEC_>
struct RwGateOBwd {
  static constexpr int VEC = VEC_;
  static constexpr bool K_CONTIG = false;
  const int64_t* offsets;
  int B, K, N;  // K = D, N = hdv
  const float* dy;
  int64_t lddy;
  const float* w;
  const float* u;
  int64_t ldu;
  const float* attn;
  int64_t lda;
  const float2* a_stats;
  const float* h_u;
  int64_t ldh;
  float p;
  uint64_t seed;
  const int64_t* seed_off;
  float* du;
  int64_t lddu;
  float* da;
  int64_t ldda;
  __amdgpu_buffer_rsrc_t rdy, ru, ra, rh, rdu, rda;
  uint64_t seed_eff;
  struct Src { f4 v[KG]; };
  __device__ int bks() const { return N; }
  __device__ int bns() const { return 1; }
  __device__ void setup(int64_t total) {
    rdy = mat_rsrc(dy, lddy, total, 0);
    ru = mat_rsrc(u, ldu, total, 0);
    ra = mat_rsrc(attn, lda, total, 0);
    rh = mat_rsrc(h_u ? h_u : u, ldh, h_u ? total : 0, 0);
    rdu = mat_rsrc(du, lddu, total, 0);
    rda = mat_rsrc(da, ldda, total, 0);
    seed_eff = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
  }
  __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
    for (int g = 0; g < KG; ++g) s.v[g] = ldq<VEC>(rdy, m * lddy, 16 * g, lg, K);
  }
  __device__ void prep(const Src& s, float (&a)[KG][4], int64_t, bool, int) const {
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[g][e] = s.v[g][e];  // columns >= K loaded as 0
  }
  struct Epi { float2 st; f4 av[NT], uv[NT], hv[NT]; };
  __device__ void epi_load(Epi& es, int64_t m, bool row_ok, int lg) const {
    es.st = ld_f2(a_stats, row_ok ? m : 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      es.av[t] = ldq<VEC>(ra, m * lda, 16 * t, lg, N);
      es.uv[t] = ldq<VEC>(ru, m * ldu, 16 * t, lg, N);
      es.hv[t] = ldq<VEC>(rh, m * ldh, 16 * t, lg, N);  // 0 when h_u is NULL
    }
  }
  __device__ void epi(f4 (&acc)[NT], const Epi& es, int64_t m, bool row_ok, int lg) const {
    const float2 st = es.st;
    float s1 = 0.f, s2 = 0.f;
    f4 lnv[NT], dln[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f4 av = es.av[t], uv = es.uv[t], hv = es.hv[t];
      f4 duv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = qcol<VEC>(16 * t, lg, e);
        const bool ok = row_ok && n < N;
        const float gg = p > 0.f ? acc[t][e] * rw_dropout_keep(seed_eff, m, n, N, p) : acc[t][e];
        const float ln = (av[e] - st.x) * st.y;
        float dd = gg * ln;
        if (h_u) dd *= silu_grad_(hv[e]);
        duv[e] = dd;
        lnv[t][e] = ok ? ln : 0.f;
        dln[t][e] = ok ? gg * uv[e] : 0.f;
        s1 += dln[t][e];
        s2 += dln[t][e] * lnv[t][e];
      }
      stq<VEC>(rdu, m * lddu, 16 * t, lg, N, duv);
    }
    s1 = row4_sum(s1);
    s2 = row4_sum(s2);
    const float inv = 1.f / (float)N;
    const float mean1 = s1 * inv, mean2 = s2 * inv;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = st.y * (dln[t][e] - mean1 - lnv[t][e] * mean2);
      stq<VEC>(rda, m * ldda, 16 * t, lg, N, o);
    }
  }
};

// F3 with concat_ua (hstu.py:398-400): o_in = dropout([u, a, u * a]), a = LN(attn),
// y = o_in @ W_o^T + b_o + x.  The three hdv-wide segments sit at 16-aligned k offsets
// seg * hvp (hvp = 16 KGH >= hdv) of a zero-padded weight W' (D, 3 hvp) built by the
// caller; the stored o_in is unpadded (rows, 3 hdv) for the weight gradient; the
// dropout mask hashes (row, seg * hdv + c) over the 3 hdv-wide o_in.
template <int KGH, int NT, int VEC_>
struct RwGateOCatT {
  template <int KG, int NT_, int V_>
  struct Op {
    static_assert(KG == 3 * KGH, "KG = 3 segments of KGH groups");
    static constexpr int VEC = V_;
    static constexpr bool K_CONTIG = true;
    const int64_t* offsets;
    int B, K, N;  // K = 3 hvp (padded), N = D
    int hv;       // hdv
    const float* u;
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
    float* o_in;
    float* y;
    int64_t ldy;
    __amdgpu_buffer_rsrc_t ru, ra, rx, ro, ry, rb;
    uint64_t seed_eff;
    struct Src { f4 v[KGH]; f4 uu[KGH]; };
    __device__ int bks() const { return 1; }
    __device__ int bns() const { return K; }
    __device__ void setup(int64_t total) {
      ru = mat_rsrc(u, ldu, total, 0);
      ra = mat_rsrc(attn, lda, total, 0);
      rx = mat_rsrc(xres ? xres : y, ldx, xres ? total : 0, 0);
      ro = mat_rsrc(o_in ? o_in : y, 3 * hv, o_in ? total : 0, 0);
      ry = mat_rsrc(y, ldy, total, 0);
      rb = mat_rsrc(bias ? bias : y, N, bias ? 1 : 0, 0);
      seed_eff = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
    }
    __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
      for (int g = 0; g < KGH; ++g) {
        s.v[g] = ldq<VEC>(ra, m * lda, 16 * g, lg, hv);
        s.uu[g] = ldq<VEC>(ru, m * ldu, 16 * g, lg, hv);
      }
    }
    __device__ void prep(const Src& s, float (&a)[KG][4], int64_t m, bool row_ok, int lg) const {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < KGH; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) sum += s.v[g][e];
      const float mean = row4_sum(sum) * (1.f / (float)hv);
      float sq = 0.f;
#pragma unroll
      for (int g = 0; g < KGH; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = qcol<VEC>(16 * g, lg, e) < hv ? s.v[g][e] - mean : 0.f;
          sq += d * d;
        }
      const float rstd = rsqrtf(row4_sum(sq) * (1.f / (float)hv) + eps);
#pragma unroll
      for (int seg = 0; seg < 3; ++seg)
#pragma unroll
        for (int g = 0; g < KGH; ++g) {
          f4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = qcol<VEC>(16 * g, lg, e);
            const float ln = (s.v[g][e] - mean) * rstd;
            float v = seg == 0 ? s.uu[g][e] : (seg == 1 ? ln : s.uu[g][e] * ln);
            if (p > 0.f) v *= rw_dropout_keep(seed_eff, m, seg * hv + c, 3 * hv, p);
            a[seg * KGH + g][e] = c < hv ? v : 0.f;
            o[e] = a[seg * KGH + g][e];
          }
          stq<VEC>(ro, m * 3 * hv + seg * hv, 16 * g, lg, hv, o);  // records = 0 when o_in is NULL
        }
      if (lg == 0 && row_ok) a_stats[m] = make_float2(mean, rstd);
    }
    struct Epi { f4 xv[NT_], bv[NT_]; };
    __device__ void epi_load(Epi& es, int64_t m, bool, int lg) const {
#pragma unroll
      for (int t = 0; t < NT_; ++t) {
        es.xv[t] = ldq<VEC>(rx, m * ldx, 16 * t, lg, N);
        es.bv[t] = ldq<VEC>(rb, 0, 16 * t, lg, N);
      }
    }
    __device__ void epi(f4 (&acc)[NT_], const Epi& es, int64_t m, bool, int lg) const {
#pragma unroll
      for (int t = 0; t < NT_; ++t) {
        f4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (acc[t][e] + es.bv[t][e]) + es.xv[t][e];
        stq<VEC>(ry, m * ldy, 16 * t, lg, N, o);
      }
    }
  };
};

// B1 with concat_ua: g = dy @ W' (rows, 3 hvp); per column c of the hdv-wide segments
// g1, g2, g3 (dropout bwd), du = g1 + g3 * a (* silu'(h_u)), da = g2 + g3 * u,
// d_attn = LayerNorm_bwd(attn; da).
template <int KGH, int KG_, int VEC_>
struct RwGateOCatBwdT {
  template <int KG, int NT, int V_>
  struct Op {
    static_assert(NT == 3 * KGH, "NT = 3 segments of KGH tiles");
    static constexpr int VEC = V_;
    static constexpr bool K_CONTIG = false;
    const int64_t* offsets;
    int B, K, N;  // K = D, N = 3 hvp
    int hv;
    const float* dy;
    int64_t lddy;
    const float* w;
    const float* u;
    int64_t ldu;
    const float* attn;
    int64_t lda;
    const float2* a_stats;
    const float* h_u;
    int64_t ldh;
    float p;
    uint64_t seed;
    const int64_t* seed_off;
    float* du;
    int64_t lddu;
    float* da;
    int64_t ldda;
    __amdgpu_buffer_rsrc_t rdy, ru, ra, rh, rdu, rda;
    uint64_t seed_eff;
    struct Src { f4 v[KG]; };
    __device__ int bks() const { return N; }
    __device__ int bns() const { return 1; }
    __device__ void setup(int64_t total) {
      rdy = mat_rsrc(dy, lddy, total, 0);
      ru = mat_rsrc(u, ldu, total, 0);
      ra = mat_rsrc(attn, lda, total, 0);
      rh = mat_rsrc(h_u ? h_u : u, ldh, h_u ? total : 0, 0);
      rdu = mat_rsrc(du, lddu, total, 0);
      rda = mat_rsrc(da, ldda, total, 0);
      seed_eff = seed + (seed_off ? (uint64_t)*seed_off : 0ull);
    }
    __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
      for (int g = 0; g < KG; ++g) s.v[g] = ldq<VEC>(rdy, m * lddy, 16 * g, lg, K);
    }
    __device__ void prep(const Src& s, float (&a)[KG][4], int64_t, bool, int) const {
#pragma unroll
      for (int g = 0; g < KG; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[g][e] = s.v[g][e];
    }
    struct Epi { float2 st; f4 av[KGH], uv[KGH], hv_[KGH]; };
    __device__ void epi_load(Epi& es, int64_t m, bool row_ok, int lg) const {
      es.st = ld_f2(a_stats, row_ok ? m : 0);
#pragma unroll
      for (int t = 0; t < KGH; ++t) {
        es.av[t] = ldq<VEC>(ra, m * lda, 16 * t, lg, hv);
        es.uv[t] = ldq<VEC>(ru, m * ldu, 16 * t, lg, hv);
        es.hv_[t] = ldq<VEC>(rh, m * ldh, 16 * t, lg, hv);
      }
    }
    __device__ void epi(f4 (&acc)[NT], const Epi& es, int64_t m, bool row_ok, int lg) const {
      const float2 st = es.st;
      float s1 = 0.f, s2 = 0.f;
      f4 lnv[KGH], dln[KGH];
#pragma unroll
      for (int t = 0; t < KGH; ++t) {
        f4 duv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = qcol<VEC>(16 * t, lg, e);
          const bool ok = row_ok && c < hv;
          float g1 = acc[t][e], g2 = acc[KGH + t][e], g3 = acc[2 * KGH + t][e];
          if (p > 0.f) {
            g1 *= rw_dropout_keep(seed_eff, m, c, 3 * hv, p);
            g2 *= rw_dropout_keep(seed_eff, m, hv + c, 3 * hv, p);
            g3 *= rw_dropout_keep(seed_eff, m, 2 * hv + c, 3 * hv, p);
          }
          const float ln = (es.av[t][e] - st.x) * st.y;
          float dd = g1 + g3 * ln;
          if (h_u) dd *= silu_grad_(es.hv_[t][e]);
          duv[e] = dd;
          lnv[t][e] = ok ? ln : 0.f;
          dln[t][e] = ok ? g2 + g3 * es.uv[t][e] : 0.f;
          s1 += dln[t][e];
          s2 += dln[t][e] * lnv[t][e];
        }
        stq<VEC>(rdu, m * lddu, 16 * t, lg, hv, duv);
      }
      s1 = row4_sum(s1);
      s2 = row4_sum(s2);
      const float inv = 1.f / (float)hv;
      const float mean1 = s1 * inv, mean2 = s2 * inv;
#pragma unroll
      for (int t = 0; t < KGH; ++t) {
        f4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = st.y * (dln[t][e] - mean1 - lnv[t][e] * mean2);
        stq<VEC>(rda, m * ldda, 16 * t, lg, hv, o);
      }
    }
  };
};

// B3: dn = dh @ W_uvqk^T (rows, D), W'(k, n) = W_uvqk[n][k]; epilogue: dx = dy + LN_bwd(x; dn).
template <int KG, int NT, int VEC_>
struct RwLnUvqkBwd {
  static constexpr int VEC = VEC_;
  static constexpr bool K_CONTIG = true;
  const int64_t* offsets;
  int B, K, N;  // K = n_out, N = D
  const float* dh;
  int64_t lddh;
  const float* w;
  const float* x;
  int64_t ldx;
  const float2* x_stats;
  const float* dy;
  int64_t lddy;
  float* dx;
  int64_t lddx;
  int rd_aux = 0;  // cache policy of the dh loads (16: rows stored earlier in the launch)
  __amdgpu_buffer_rsrc_t rdh, rx, rdy, rdx;
  struct Src { f4 v[KG]; };
  __device__ int bks() const { return 1; }
  __device__ int bns() const { return K; }
  __device__ void setup(int64_t total) {
    rdh = mat_rsrc(dh, lddh, total, 0);
    rx = mat_rsrc(x, ldx, total, 0);
    rdy = mat_rsrc(dy ? dy : x, lddy, dy ? total : 0, 0);
    rdx = mat_rsrc(dx, lddx, total, 0);
  }
  __device__ void load(Src& s, int64_t m, int lg) const {
#pragma unroll
    for (int g = 0; g < KG; ++g) s.v[g] = ldq<VEC>(rdh, m * lddh, 16 * g, lg, K, rd_aux);
  }
  __device__ void prep(const Src& s, float (&a)[KG][4], int64_t, bool, int) const {
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[g][e] = s.v[g][e];
  }
  struct Epi { float2 st; f4 xv[NT], dyv[NT]; };
  __device__ void epi_load(Epi& es, int64_t m, bool row_ok, int lg) const {
    es.st = ld_f2(x_stats, row_ok ? m : 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      es.xv[t] = ldq<VEC>(rx, m * ldx, 16 * t, lg, N);
      es.dyv[t] = ldq<VEC>(rdy, m * lddy, 16 * t, lg, N);  // 0 when dy is NULL
    }
  }
  // out (optional): the stored dx quads, for a fused consumer (rowwave2_kernel)
  __device__ void epi(f4 (&acc)[NT], const Epi& es, int64_t m, bool row_ok, int lg,
                      f4* out = nullptr) const {
    const float2 st = es.st;
    float s1 = 0.f, s2 = 0.f;
    f4 xh[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f4 xv = es.xv[t];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = row_ok && qcol<VEC>(16 * t, lg, e) < N;
        xh[t][e] = ok ? (xv[e] - st.x) * st.y : 0.f;
        const float dn = ok ? acc[t][e] : 0.f;
        s1 += dn;
        s2 += dn * xh[t][e];
      }
    }
    s1 = row4_sum(s1);
    s2 = row4_sum(s2);
    const float inv = 1.f / (float)N;
    const float mean1 = s1 * inv, mean2 = s2 * inv;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f4 dyv = es.dyv[t];
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = dyv[e] + st.y * (acc[t][e] - mean1 - xh[t][e] * mean2);
      stq<VEC>(rdx, m * lddx, 16 * t, lg, N, o);
      if (out) {
#pragma unroll
        for (int e = 0; e < 4; ++e) out[t][e] = qcol<VEC>(16 * t, lg, e) < N ? o[e] : 0.f;
      }
    }
  }
};

// ------------------------------------------------------------------ one unit, callable
// One 16-row unit of rowwave2_kernel's loop (rows m = the lane's row, ok = its validity)
// for kernels that run a layer boundary as the epilogue of other work (the attention
// backward's dQ pass, hstu_attn_bwd_bnd): the panels W1 / W2 are staged (rw_stage_w) and
// the ops set up (setup(row_end): rows >= row_end read 0, their stores are dropped).  Same
// arithmetic as the rowwave2_kernel unit, so results are bit-identical to it.
template <int KG1, int NT1, int NT2, class Op1, class Op2>
__device__ __forceinline__ void rw2_unit(const Op1& op1, const Op2& op2, const float* W1,
                                         const float* W2, int64_t m, bool ok, int lr, int lg) {
  constexpr int VEC = Op1::VEC;
  typename Op1::Src cur;
  op1.load(cur, m, lg);
  float a1[KG1][4];
  op1.prep(cur, a1, m, ok, lg);
  typename Op1::Epi es1;
  op1.epi_load(es1, m, ok, lg);
  typename Op2::Epi es2;
  op2.epi_load(es2, m, ok, lg);
  f4 acc1[NT1];
  rw_mma<KG1, NT1, VEC>(W1, a1, acc1, lr, lg);
  typename Op2::Src s2;
  op1.epi(acc1, es1, m, ok, lg, s2.v);
  float a2[NT1][4];
  op2.prep(s2, a2, m, ok, lg);
  f4 acc2[NT2];
  rw_mma<NT1, NT2, VEC>(W2, a2, acc2, lr, lg);
  op2.epi(acc2, es2, m, ok, lg);
}
// the same for one op (rowwave_kernel's unit)
template <int KG, int NT, class Op>
__device__ __forceinline__ void rw1_unit(const Op& op, const float* Wl, int64_t m, bool ok, int lr,
                                         int lg) {
  constexpr int VEC = Op::VEC;
  typename Op::Src cur;
  op.load(cur, m, lg);
  float a[KG][4];
  op.prep(cur, a, m, ok, lg);
  typename Op::Epi es;
  op.epi_load(es, m, ok, lg);
  f4 acc[NT];
  rw_mma<KG, NT, VEC>(Wl, a, acc, lr, lg);
  op.epi(acc, es, m, ok, lg);
}

// ------------------------------------------------------------------ host-side op arguments
struct RwArgsLnUvqk {
  const int64_t* offsets; int B, K, N; const float* x; int64_t ldx; const float* w; float eps;
  int act; float2* x_stats; float* h_pre; float* out; int64_t ld_out;
  template <class Op> void fill(Op& o) const {
    o.offsets = offsets; o.B = B; o.K = K; o.N = N; o.x = x; o.ldx = ldx; o.w = w; o.eps = eps;
    o.act = act; o.x_stats = x_stats; o.h_pre = h_pre; o.out = out; o.ld_out = ld_out;
  }
};
struct RwArgsGateO {
  const int64_t* offsets; int B, K, N; const float* u; int64_t ldu; const float* attn; int64_t lda;
  const float* w; const float* bias; const float* xres; int64_t ldx; float eps, p; uint64_t seed;
  const int64_t* seed_off; float2* a_stats; float* o_in; float* y; int64_t ldy;
  template <class Op> void fill(Op& o) const {
    o.offsets = offsets; o.B = B; o.K = K; o.N = N; o.u = u; o.ldu = ldu; o.attn = attn; o.lda = lda;
    o.w = w; o.bias = bias; o.xres = xres; o.ldx = ldx; o.eps = eps; o.p = p; o.seed = seed;
    o.seed_off = seed_off; o.a_stats = a_stats; o.o_in = o_in; o.y = y; o.ldy = ldy;
  }
};
struct RwArgsGateOBwd {
  const int64_t* offsets; int B, K, N; const float* dy; int64_t lddy; const float* w; const float* u;
  int64_t ldu; const float* attn; int64_t lda; const float2* a_stats; const float* h_u; int64_t ldh;
  float p; uint64_t seed; const int64_t* seed_off; float* du; int64_t lddu; float* da; int64_t ldda;
  template <class Op> void fill(Op& o) const {
    o.offsets = offsets; o.B = B; o.K = K; o.N = N; o.dy = dy; o.lddy = lddy; o.w = w; o.u = u;
    o.ldu = ldu; o.attn = attn; o.lda = lda; o.a_stats = a_stats; o.h_u = h_u; o.ldh = ldh; o.p = p;
    o.seed = seed; o.seed_off = seed_off; o.du = du; o.lddu = lddu; o.da = da; o.ldda = ldda;
  }
};
struct RwArgsLnUvqkBwd {
  const int64_t* offsets; int B, K, N; const float* dh; int64_t lddh; const float* w; const float* x;
  int64_t ldx; const float2* x_stats; const float* dy; int64_t lddy; float* dx; int64_t lddx;
  template <class Op> void fill(Op& o) const {
    o.offsets = offsets; o.B = B; o.K = K; o.N = N; o.dh = dh; o.lddh = lddh; o.w = w; o.x = x;
    o.ldx = ldx; o.x_stats = x_stats; o.dy = dy; o.lddy = lddy; o.dx = dx; o.lddx = lddx;
  }
};

}  // namespace gr
