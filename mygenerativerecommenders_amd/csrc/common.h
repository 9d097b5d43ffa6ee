// Shared device/host helpers for the gfx950 HSTU + MIPS library.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdlib>
#include <initializer_list>
#include <cstdio>
#include <string>

#include "../../include/gr_hstu.h"

// Every hipLaunchKernelGGL in this library's sources goes through gr::launch_kernel (timed
// inside GR_TIMED regions when timing is on).
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernelName, ...) ::gr::launch_kernel((kernelName), __VA_ARGS__)

namespace gr {

// ---------------------------------------------------------------- error plumbing
void set_error(const char* fmt, ...);
const char* last_error();
// Launch option (gr_set_option; GR_OPT_* in gr_hstu.h).
int64_t option(int which);

#define GR_REQUIRE(cond, ...)                \
  do {                                       \
    if (!(cond)) {                           \
      ::gr::set_error(__VA_ARGS__);          \
      return 1;                              \
    }                                        \
  } while (0)

// ---------------------------------------------------------------- live kernel timing
// When enabled (gr_timing_enable), every kernel launched inside a GR_TIMED region is
// dispatched through hipExtLaunchKernel with a start / stop event pair that the dispatch
// packet itself timestamps (the same begin / end a rocprofv3 kernel trace reports; no
// separate event-record packets around the launch); gr_timing_query drains and sums
// them per kernel name.
bool timing_enabled();
void timing_push(const char* name, hipEvent_t start, hipEvent_t stop);
const char*& timing_region();  // name of the enclosing GR_TIMED region (thread-local)

template <typename F, typename... Args>
inline void launch_kernel(F kernel, const dim3& grid, const dim3& block, uint32_t shmem,
                          hipStream_t st, Args... args) {
  const char* name = timing_region();
  if (name && timing_enabled()) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, e0, e1, 0, args...);
    timing_push(name, e0, e1);
  } else {
    kernel<<<grid, block, shmem, st>>>(args...);
  }
}

#define GR_TIMED(name, stream, ...)                 \
  do {                                              \
    const char* prev_ = ::gr::timing_region();      \
    ::gr::timing_region() = (name);                 \
    (void)(stream);                                 \
    __VA_ARGS__;                                    \
    ::gr::timing_region() = prev_;                  \
  } while (0)

#define GR_LAUNCH_CHECK(what)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::gr::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));     \
      return 2;                                                                 \
    }                                                                           \
  } while (0)

// ---------------------------------------------------------------- MFMA (f32 in / f32 acc)
// v_mfma_f32_16x16x4_f32: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
// C/D: col = l&15, row = 4*(l>>4) + reg.  Bit-exact k-ordered fmaf chain.
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

// Two floats -> packed bf16 pair (round-to-nearest-even), lo in the low half.
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
// C += A B over k = 32: a = A[row lane%16][k 8(lane/16) .. +7], b = B[k ..][col lane%16]
__device__ __forceinline__ f4 mfma_bf16(u32x4_t a, u32x4_t b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ f4 mfma16x16x4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f4 f4_zero() { return f4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------- activations
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float siluf_(float x) { return x * sigmoidf_(x); }
// d silu / dx = s * (1 + x * (1 - s))
__device__ __forceinline__ float silu_grad_(float x) {
  float s = sigmoidf_(x);
  return s * (1.0f + x * (1.0f - s));
}

// ---------------------------------------------------------------- counter-based RNG
// Dropout masks are a pure function of (seed, element index): the backward pass
// regenerates them instead of storing them.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// DPP lane move within a 16-lane row (no LDS crossbar traffic, unlike __shfl*).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// reduce across the 16 lanes that share (lane >> 4): quad xor 1, quad xor 2, then the
// half-row and row mirrors (every lane of a quad / half-row already holds the same
// partial, so the mirrors equal xor 4 / xor 8 — the same sums as the xor butterfly).
__device__ __forceinline__ float sum16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// Buffer voffset of a masked lane: loads through it return 0 and stores are dropped.
// A descriptor's num_records is an int (< 2^31 bytes) and voffsets are unsigned, so 2^31
// — plus any row step below 2^31 — fails the range check for every buffer this library
// builds.  (Rounds 1-5 used 2^30, which a buffer over 1 GiB would have served from real
// data; tests/test_gpu_wgrad.py::test_wgrad_stream_operand_over_1gib covers that case.)
constexpr int OOB_OFF = (int)0x80000000u;

// Global-address-space view of a pointer: keeps hipcc on global_load (counted by
// vmcnt alone) where address-space inference fails (pointers through structs /
// lambdas), instead of flat_load (which forces vmcnt(0) + lgkmcnt(0) waits).
template <class T>
using gptr = const T __attribute__((address_space(1)))*;
template <class T>
__device__ __forceinline__ gptr<T> as_global(const T* p) {
  return (gptr<T>)p;
}

__device__ __forceinline__ float2 ld_f2(const float2* p, int64_t i) {
  typedef float fv2_ __attribute__((ext_vector_type(2)));
  const fv2_ v = as_global(reinterpret_cast<const fv2_*>(p))[i];
  return make_float2(v.x, v.y);
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations and
// meets the other waves, but leaves global loads in flight (a __syncthreads() lowers to
// s_waitcnt vmcnt(0) as well, which drains register prefetches).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave index as a scalar (threadIdx-derived values are otherwise divergent to hipcc,
// which turns wave-uniform loop exits into exec-mask branches).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// Zero n 32-bit words.  Used instead of hipMemsetAsync on every path a training step
// may capture into a HIP graph: a captured memset node left a counter un-zeroed on
// replay on MI355X (ROCm 7), which a kernel node does not.
static __global__ __launch_bounds__(256) void zero_words_kernel(uint32_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0u;
}
inline void zero_words_async(void* p, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, st,
                     (uint32_t*)p, n);
}

// CU count of the current device (cached; 256 on MI355X).
inline int device_cus() {
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

// Workgroups of `kernel` (256 threads, `lds` dynamic bytes) one CU holds at once.
template <typename K>
inline int resident_wgs(K kernel, size_t lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kernel), 256, lds) != hipSuccess || n < 1)
    n = 1;
  return n;
}

// One workgroup (256 threads): offsets[0] = 0, offsets[b + 1] = sum_{j <= b} lengths[j]
// (utils/ops.py:18-38).  Thread t owns lengths[t * per, (t + 1) * per); a 64-lane shuffle
// scan per wave, then the four wave totals meet in LDS (one barrier).
__device__ __forceinline__ void offsets_scan(const int64_t* lengths, int B, int64_t* offsets) {
  __shared__ int64_t wave_tot[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int per = (B + 255) / 256;
  const int lo = t * per, hi = min(B, lo + per);
  int64_t s = 0;
  for (int i = lo; i < hi; ++i) s += lengths[i];
  int64_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) wave_tot[wv] = inc;
  __syncthreads();
  int64_t run = inc - s;
  for (int w = 0; w < wv; ++w) run += wave_tot[w];
  if (t == 0) offsets[0] = 0;
  for (int i = lo; i < hi; ++i) {
    run += lengths[i];
    offsets[i + 1] = run;
  }
}

// relative-time bucket: max{b : thr[b] <= |dt|}, thr = integer threshold table of the
// reference bucket fn (hstu.py:579-581, clamped at hstu.py:117-123).
__device__ __forceinline__ int time_bucket(int64_t dt, const int64_t* thr_lds, int nb) {
  uint64_t ad = dt < 0 ? (uint64_t)(-dt) : (uint64_t)dt;
  int b = 0;
  if (ad > 1) {
    float f = (float)ad;
    b = (int)(__log2f(f) * 2.30283176f);  // log2(x) * ln(2) / 0.301
    b = b > nb ? nb : b;
  }
  // the estimate is the bucket or one off (every table threshold and 2e5 random |dt| up
  // to 2^40 checked on the host): both bracketing thresholds are read together, and the
  // walks below run only when it missed
  const uint64_t lo = (uint64_t)thr_lds[b], hi = (uint64_t)thr_lds[b < nb ? b + 1 : nb];
  if (ad >= lo && (b == nb || ad < hi)) return b;
  while (b < nb && ad >= (uint64_t)thr_lds[b + 1]) ++b;
  while (b > 0 && ad < (uint64_t)thr_lds[b]) --b;
  return b;
}

}  // namespace gr
