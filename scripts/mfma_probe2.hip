// Probe: 32x32x16 bf16 layouts, ds_read_tr16_b64, accumulator-as-A-operand (X^T . D)
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pk(float a, float b) {
  __bf16 x = (__bf16)a, y = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
// A: [32][16] bf16 row-major, B: [16][32] row-major, D: [32][32] bf16 row-major (k rows)
// out: X (32x32 f32 as [lane][16]) then Z = X^T D as [lane][16]
__global__ void probe(const uint16_t* A, const uint16_t* B, const uint16_t* D, float* out) {
  __shared__ __attribute__((aligned(16))) uint16_t Dl[32 * 32];
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  for (int i = l; i < 1024; i += 64) Dl[i] = D[i];
  __syncthreads();
  uint16_t a[8], b[8];
  for (int j = 0; j < 8; ++j) { a[j] = A[r * 16 + 8 * h + j]; b[j] = B[(8 * h + j) * 32 + r]; }
  f16v x = {};
  x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), x, 0, 0, 0);
  for (int i = 0; i < 16; ++i) out[l * 16 + i] = x[i];
  // Z = X^T D : A = X regs 8s..8s+7 as bf16; B = D[k][col] with k = 16s + 8(j>>2) + 4h + (j&3)
  f16v z = {};
  for (int s = 0; s < 2; ++s) {
    u32x4 af = {pk(x[8 * s], x[8 * s + 1]), pk(x[8 * s + 2], x[8 * s + 3]), pk(x[8 * s + 4], x[8 * s + 5]), pk(x[8 * s + 6], x[8 * s + 7])};
    // tr reads: 16-lane group g = l >> 4: rows r0 = 16s + 4h (+8), cols c0 = 16 (g & 1)
    const int g = l >> 4, q = (l & 15) >> 2, p = l & 3;
    s16x4 t0, t1;
    {
      const int row = 16 * s + 4 * h + q, col = 16 * (g & 1) + 4 * p;
      t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(Dl + row * 32 + col));
    }
    {
      const int row = 16 * s + 8 + 4 * h + q, col = 16 * (g & 1) + 4 * p;
      t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(Dl + row * 32 + col));
    }
    const u32x2 lo = __builtin_bit_cast(u32x2, t0), hi = __builtin_bit_cast(u32x2, t1);
    const u32x4 bf = {lo.x, lo.y, hi.x, hi.y};
    z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af), __builtin_bit_cast(bf16x8, bf), z, 0, 0, 0);
  }
  for (int i = 0; i < 16; ++i) out[1024 + l * 16 + i] = z[i];
}
extern "C" int run_probe(const void* A, const void* B, const void* D, float* out) {
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, (const uint16_t*)A, (const uint16_t*)B, (const uint16_t*)D, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
