// Elementwise step of the Muon optimizer's bf16 Newton-Schulz chain (SURVEY §8 N4,
// reference optimizers/muon.py:3-29):  out = bf16(bf16(s * x) + y)  over bf16 tensors.
// The chain's two combines per iteration, B = b*A + (c*A)@A and X = a*X + B@X, each cost
// the reference two elementwise launches (the scaled operand, then the sum) with a
// rounding to bf16 after each; this kernel is one launch with the same two roundings,
// so the chain's result is bit-identical (tests/test_gpu_next_rows.py).  Any other
// rounding (a GEMM epilogue with beta, a single-rounding axpy) moves the orthogonalised
// update by ~5 % of its largest entry: the bf16 chain amplifies it.
#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

__device__ __forceinline__ float bf16_bits_to_float(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t float_to_bf16_bits(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// 8 elements (one 16-byte load per operand) per thread, grid-stride
__global__ __launch_bounds__(256) void bf16_scale_add_kernel(const uint4* x, float s, const uint4* y,
                                                             uint4* out, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const uint4 xv = x[i], yv = y[i];
    const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w}, ys[4] = {yv.x, yv.y, yv.z, yv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t w = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float sx = bf16_bits_to_float(float_to_bf16_bits(s * bf16_bits_to_float((uint16_t)(xs[j] >> (16 * h)))));
        const float r = sx + bf16_bits_to_float((uint16_t)(ys[j] >> (16 * h)));
        w |= (uint32_t)float_to_bf16_bits(r) << (16 * h);
      }
      o[j] = w;
    }
    out[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

__global__ __launch_bounds__(256) void bf16_scale_add_tail_kernel(const uint16_t* x, float s, const uint16_t* y,
                                                                  uint16_t* out, int64_t i0, int64_t n) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const float sx = bf16_bits_to_float(float_to_bf16_bits(s * bf16_bits_to_float(x[i])));
    out[i] = float_to_bf16_bits(sx + bf16_bits_to_float(y[i]));
  }
}

}  // namespace gr

extern "C" int gr_bf16_scale_add(const uint16_t* x, float s, const uint16_t* y, uint16_t* out,
                                 int64_t n, void* stream) {
  GR_REQUIRE(n >= 0 && (n == 0 || (x && y && out)), "gr_bf16_scale_add: bad args");
  if (n == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                     reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  const int64_t n8 = vec ? n / 8 : 0;
  if (n8 > 0) {
    const int64_t want = (n8 + 255) / 256;
    const unsigned grid = (unsigned)(want < 8 * 256 ? want : 8 * 256);
    GR_TIMED("bf16_scale_add", st, hipLaunchKernelGGL(gr::bf16_scale_add_kernel, dim3(grid), dim3(256), 0, st,
                                                      (const uint4*)x, s, (const uint4*)y, (uint4*)out, n8));
  }
  const int64_t rest = n - n8 * 8;  // unaligned operands, or the last n % 8 elements
  if (rest > 0)
    GR_TIMED("bf16_scale_add", st, hipLaunchKernelGGL(gr::bf16_scale_add_tail_kernel, dim3((unsigned)((rest + 255) / 256)),
                                                      dim3(256), 0, st, x, s, y, out, n8 * 8, n));
  GR_LAUNCH_CHECK("gr_bf16_scale_add");
  return 0;
}
