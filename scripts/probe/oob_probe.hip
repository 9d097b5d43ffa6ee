// Probe: the buffer range check that the kernels' masking relies on (common.h OOB_OFF).
//  (1) raw buffer dwordx4 loads (to VGPRs and to LDS) straddling num_records: the in-range
//      dwords arrive, the rest read 0;
//  (2) masked lanes at voffset 2^31 (OOB_OFF), 2^31 + a row step, 2^32 - 16, and the old
//      2^30, against a small buffer and against one of 1.5 GiB (where 2^30 is IN range and
//      returns real data, which is why OOB_OFF moved to 2^31);
//  (3) a store at voffset 2^31 is dropped.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probe/oob_probe.hip -o scripts/probe/oob_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void straddle(const float* p, int nrec, float* out) {
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

// lane l loads at voffset offs[l % 4] (+ soffset sstep): out[l] = first dword
__global__ void masked(const float* p, int nrec, const int* offs, int sstep, float* out) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nrec, 0x00020000);
  const int l = threadIdx.x;
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, offs[l & 3], sstep, 0);
  out[l] = __uint_as_float(v[0]) + __uint_as_float(v[1]) + __uint_as_float(v[2]) + __uint_as_float(v[3]);
}

__global__ void masked_store(float* p, int nrec) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nrec, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(-1.f), r, (int)0x80000000u, 0, 0);
}

int main() {
  int bad = 0;
  float h[256];
  for (int i = 0; i < 256; ++i) h[i] = 1000 + i;
  float *d, *o;
  hipMalloc(&d, 1024);
  hipMalloc(&o, 2048);
  hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
  straddle<<<1, 64>>>(d, 40, o);  // 40 bytes = 10 floats: piece 2 (bytes 32..47) straddles
  float r[512];
  hipMemcpy(r, o, 2048, hipMemcpyDeviceToHost);
  printf("straddle vgpr: ");
  for (int i = 0; i < 16; ++i) printf("%g ", r[i]);
  printf("\nstraddle lds:  ");
  for (int i = 0; i < 16; ++i) printf("%g ", r[256 + i]);
  printf("\n");
  for (int i = 0; i < 12; ++i) bad += r[i] != (i < 10 ? 1000.f + i : 0.f);

  // a 1.5 GiB buffer of ones
  const size_t big = (size_t)3 << 29;
  float* g = nullptr;
  if (hipMalloc(&g, big) != hipSuccess) { printf("alloc failed\n"); return 2; }
  hipMemset(g, 0, big);
  const float one = 1.f;
  const size_t probe_at[] = {(size_t)1 << 30, ((size_t)1 << 30) + 4096};
  for (size_t a : probe_at)
    for (int e = 0; e < 4; ++e) hipMemcpy((char*)g + a + 4 * e, &one, 4, hipMemcpyHostToDevice);
  int* doffs;
  hipMalloc(&doffs, 16);
  const int offs[4] = {(int)0x80000000u, (int)0xC0000000u, (int)0xFFFFFFF0u, (int)0x40000000};
  hipMemcpy(doffs, offs, 16, hipMemcpyHostToDevice);
  const int nrecs[2] = {64, (int)(((size_t)3 << 29) - 1)};
  for (int n : nrecs)
    for (int ss : {0, 4096}) {
      masked<<<1, 64>>>(g, n, doffs, ss, o);
      float m[64];
      hipMemcpy(m, o, 256, hipMemcpyDeviceToHost);
      printf("nrec %d soff %d: 2^31 -> %g, 3*2^30 -> %g, 2^32-16 -> %g, 2^30 -> %g\n", n, ss, m[0], m[1],
             m[2], m[3]);
      bad += m[0] != 0.f || m[1] != 0.f || m[2] != 0.f;  // OOB_OFF must read 0 at every size
    }
  masked_store<<<1, 64>>>(g, 64);
  float z[4];
  hipMemcpy(z, g, 16, hipMemcpyDeviceToHost);
  bad += z[0] != 0.f;
  const hipError_t e = hipDeviceSynchronize();
  printf("status %s, %s\n", hipGetErrorString(e), bad ? "FAIL" : "OK");
  return bad || e != hipSuccess ? 1 : 0;
}
