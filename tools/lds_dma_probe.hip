// Probe: do LDS-DMA writes (global_load_lds_dwordx4, M0 = LDS byte offset) land inside
// the issuing workgroup's LDS allocation for every allocation size and every position
// of the workgroup in the CU's LDS?  Each workgroup fills its whole dynamic LDS region
// (1-KB pieces, M0 = piece offset) with 16-B chunks tagged (workgroup, round, piece,
// lane), waits, and checks every chunk; a second check after the other workgroups' next
// rounds catches writes that landed in a neighbour.  Prints error counts per size.
// Build: hipcc --offload-arch=gfx950 -O2 tools/lds_dma_probe.hip -o tools/lds_dma_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}

// src[(round * nwg + wg) * pieces * 64 + piece * 64 + lane] = tag
__global__ __launch_bounds__(256) void fill_src(uint4* src, int nwg, int pieces, int rounds) {
  const int64_t n = (int64_t)rounds * nwg * pieces * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const int64_t r = i >> 6;
    const int piece = (int)(r % pieces);
    const int64_t wr = r / pieces;
    const int wg = (int)(wr % nwg), round = (int)(wr / nwg);
    src[i] = make_uint4(0xA5000000u | (uint32_t)wg, (uint32_t)round, (uint32_t)piece, (uint32_t)lane);
  }
}

__global__ __launch_bounds__(256) void probe(const uint4* src, int pieces, int rounds,
                                             unsigned long long* errs) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = blockIdx.x, nwg = gridDim.x;
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  unsigned long long bad = 0, bad_late = 0;
  for (int round = 0; round < rounds; ++round) {
    const uint4* s = src + ((int64_t)round * nwg + wg) * pieces * 64;
    for (int pc = wave; pc < pieces; pc += 4) glds16(s + pc * 64 + lane, base + pc * 1024);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = tid; i < pieces * 64; i += 256) {
      const uint4 v = lds[i];
      const uint4 e = make_uint4(0xA5000000u | (uint32_t)wg, (uint32_t)round, (uint32_t)(i >> 6),
                                 (uint32_t)(i & 63));
      bad += (v.x != e.x || v.y != e.y || v.z != e.z || v.w != e.w);
    }
    // let the neighbours run a while, then look again (a write of theirs that landed here)
    for (int k = 0; k < 2000; ++k) __builtin_amdgcn_s_sleep(1);
    for (int i = tid; i < pieces * 64; i += 256) {
      const uint4 v = lds[i];
      const uint4 e = make_uint4(0xA5000000u | (uint32_t)wg, (uint32_t)round, (uint32_t)(i >> 6),
                                 (uint32_t)(i & 63));
      bad_late += (v.x != e.x || v.y != e.y || v.z != e.z || v.w != e.w);
    }
    __syncthreads();
  }
  if (bad) atomicAdd(errs, bad);
  if (bad_late) atomicAdd(errs + 1, bad_late);
}

// a co-resident victim: one workgroup per CU writes its own pattern with ds_write and
// re-checks it while the DMA writers run on another stream
__global__ __launch_bounds__(256) void victim(int chunks, int loops, unsigned long long* errs) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  const int tid = threadIdx.x;
  const uint32_t tag = 0x5A000000u | (uint32_t)blockIdx.x;
  for (int i = tid; i < chunks; i += 256) lds[i] = make_uint4(tag, (uint32_t)i, ~tag, ~(uint32_t)i);
  __syncthreads();
  unsigned long long bad = 0;
  for (int l = 0; l < loops; ++l) {
    for (int i = tid; i < chunks; i += 256) {
      const uint4 v = lds[i];
      bad += (v.x != tag || v.y != (uint32_t)i || v.z != ~tag || v.w != ~(uint32_t)i);
    }
    __builtin_amdgcn_s_sleep(8);
  }
  if (bad) atomicAdd(errs + 2, bad);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int kb_list[] = {24, 40, 50, 64, 66, 70, 74, 80, 96, 134, 146, 160};
  const int rounds = 6;
  unsigned long long* errs;
  hipMalloc(&errs, 3 * sizeof(unsigned long long));
  for (int kb : kb_list) {
    const int pieces = kb;             // 1 KB each
    const int per_cu = 160 / kb;       // workgroups the LDS allows per CU
    const int nwg = cus * (per_cu > 0 ? per_cu : 1) * 2;
    uint4* src;
    const size_t n = (size_t)rounds * nwg * pieces * 64;
    if (hipMalloc(&src, n * sizeof(uint4)) != hipSuccess) { printf("%3d KB: alloc failed\n", kb); continue; }
    hipLaunchKernelGGL(fill_src, dim3(4096), dim3(256), 0, 0, src, nwg, pieces, rounds);
    hipMemset(errs, 0, 2 * sizeof(unsigned long long));
    hipFuncSetAttribute(reinterpret_cast<const void*>(probe),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), kb * 1024, 0, src, pieces, rounds, errs);
    const hipError_t e = hipDeviceSynchronize();
    unsigned long long h[2] = {0, 0};
    hipMemcpy(h, errs, sizeof h, hipMemcpyDeviceToHost);
    printf("%3d KB x %d WG/CU (%d WGs): %s, wrong chunks %llu, wrong later %llu (of %llu)\n", kb,
           per_cu, nwg, hipGetErrorString(e), h[0], h[1],
           (unsigned long long)rounds * nwg * pieces * 64);
    hipFree(src);
  }
  // mixed residency: 66-KB DMA writers (two per CU, as skip_h) beside a 24-KB victim
  {
    hipStream_t a, b;
    hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    const int kb = 66, pieces = 66, nwg = cus * 2 * 8, vchunks = 24 * 64;
    uint4* src;
    const size_t n = (size_t)rounds * nwg * pieces * 64;
    hipMalloc(&src, n * sizeof(uint4));
    hipLaunchKernelGGL(fill_src, dim3(4096), dim3(256), 0, 0, src, nwg, pieces, rounds);
    hipMemset(errs, 0, 3 * sizeof(unsigned long long));
    hipDeviceSynchronize();
    hipFuncSetAttribute(reinterpret_cast<const void*>(probe),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
    hipLaunchKernelGGL(victim, dim3(cus), dim3(256), 24 * 1024, b, vchunks, 20000, errs);
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), kb * 1024, a, src, pieces, rounds, errs);
    const hipError_t e = hipDeviceSynchronize();
    unsigned long long h[3] = {0, 0, 0};
    hipMemcpy(h, errs, sizeof h, hipMemcpyDeviceToHost);
    printf("mixed: 66-KB writers + 24-KB victims: %s, writer wrong %llu / later %llu, victim wrong %llu\n",
           hipGetErrorString(e), h[0], h[1], h[2]);
    hipFree(src);
  }
  hipFree(errs);
  return 0;
}
