// 32 x 32 x 16 bf16 MFMA helpers (gfx950): operand layouts, transposed LDS reads and the
// accumulator-as-operand form, shared by the wide attention kernels and the bf16 weight
// gradients.  Layouts verified on the GPU by scripts/mfma_probe2.py.
#pragma once

#include "common.h"

namespace gr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 f16_zero() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// C += A B over k = 16: a = A[row lane%32][k 8(lane/32) .. +7], b = B[k ..][col lane%32];
// C[row (reg & 3) + 8 (reg >> 2) + 4 (lane / 32)][col lane % 32]
__device__ __forceinline__ f32x16 mfma32(u32x4_t a, u32x4_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                  __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
// ds_read_b64_tr_b16: per 16-lane group, lane 4q + p gives the address of row q, columns
// 4p .. 4p + 3 of a 4 x 16 block of bf16; lane i receives column i of the 4 rows.
__device__ __forceinline__ u32x2_t tr16(const __bf16* p) {
  const s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_t*)(p));
  return __builtin_bit_cast(u32x2_t, v);
}
// B operand (8 bf16) for k-step s of a product whose A operand is a 32 x 32 accumulator in
// registers: element j of lane half h is k = 16 s + 8 (j >> 2) + 4 h + (j & 3), column =
// c0 + lane % 32, from a row-major [k][col] LDS tile with row stride rs (bf16 units).
__device__ __forceinline__ u32x4_t trB_acc(const __bf16* tile, int rs, int s, int c0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const __bf16* base = tile + (16 * s + 4 * h + q) * rs + c0 + 16 * (g & 1) + 4 * p;
  const u32x2_t lo = tr16(base), hi = tr16(base + 8 * rs);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
// The same in natural k order: element j of lane half h is k = 16 s + 8 h + j.
__device__ __forceinline__ u32x4_t trB_nat(const __bf16* tile, int rs, int s, int c0, int lane) {
  const int g = lane >> 4, h = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const __bf16* base = tile + (16 * s + 8 * h + q) * rs + c0 + 16 * (g & 1) + 4 * p;
  const u32x2_t lo = tr16(base), hi = tr16(base + 4 * rs);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}
}  // namespace gr
