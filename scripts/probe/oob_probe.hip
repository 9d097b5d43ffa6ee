// Probe: raw buffer dwordx4 loads (to VGPRs and to LDS) straddling num_records.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* p, int nrec, float* out) {
  __shared__ float s[64 * 4];
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nrec, 0x00020000);
  const int l = threadIdx.x;
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, l * 16, 0, 0);
  out[l * 4 + 0] = __uint_as_float(v[0]); out[l * 4 + 1] = __uint_as_float(v[1]);
  out[l * 4 + 2] = __uint_as_float(v[2]); out[l * 4 + 3] = __uint_as_float(v[3]);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s, 16, l * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int e = 0; e < 4; ++e) out[256 + l * 4 + e] = s[l * 4 + e];
}
int main() {
  float h[256]; for (int i = 0; i < 256; ++i) h[i] = 1000 + i;
  float *d, *o; hipMalloc(&d, 1024); hipMalloc(&o, 2048);
  hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, 40, o);  // 40 bytes = 10 floats: piece 2 (bytes 32..47) straddles
  float r[512]; hipMemcpy(r, o, 2048, hipMemcpyDeviceToHost);
  printf("vgpr: "); for (int i = 0; i < 16; ++i) printf("%g ", r[i]); printf("\n");
  printf("lds:  "); for (int i = 0; i < 16; ++i) printf("%g ", r[256 + i]); printf("\n");
  return 0;
}
