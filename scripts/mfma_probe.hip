#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// a32/b32: per lane 8 bf16 (u32x4); a16/b16: per lane 4 bf16 (u32x2); out: [2][64][4]
__global__ void probe(const u32x4* a32, const u32x4* b32, const u32x2* a16, const u32x2* b16, float* out) {
  const int l = threadIdx.x;
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a32[l]), __builtin_bit_cast(bf16x8, b32[l]), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
  f4 d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a16[l]), __builtin_bit_cast(s16x4, b16[l]), d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[256 + l * 4 + r] = d[r];
}
extern "C" int run_probe(const void* a32, const void* b32, const void* a16, const void* b16, float* out) {
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, (const u32x4*)a32, (const u32x4*)b32, (const u32x2*)a16, (const u32x2*)b16, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
