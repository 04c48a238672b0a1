// Probe: does the immediate offset of global_load_lds_dwordx4 (SADDR form) move the
// LDS destination as well as the global source?  Prints where each 16-B lane chunk
// landed.  Build: hipcc --offload-arch=gfx950 -O2 tools/glds_offset_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__global__ void k(const float* src, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = -1.f;
  __syncthreads();
  uint64_t base = (uint64_t)src;
  uint32_t voff = threadIdx.x * 16;
  uint32_t l = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2 offset:1024\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(l)) : "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 64) out[i] = lds[i];
}
int main() {
  float h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = (float)i;
  float *d, *o;
  hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof h);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  // LDS float index of the first value written and the global float it came from
  int first = -1;
  for (int i = 0; i < 2048; ++i) if (h[i] >= 0.f) { first = i; break; }
  printf("first LDS float written: %d, value (global float index): %.0f\n", first, first >= 0 ? h[first] : -1.f);
  printf("=> LDS shift %s; global shift %s\n", first == 256 ? "YES (offset applies to LDS)" : (first == 0 ? "no" : "?"),
         first >= 0 && h[first] == 256.f ? "yes" : "?");
  return 0;
}
