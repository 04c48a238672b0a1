// LDS-DMA throughput probe (gfx950): how many bytes per clock can a CU move by
// global_load_lds_dwordx4 into a ring of LDS slots, from an L2-resident image and from
// HBM, compared with plain 16-B loads into registers?  The inner-skip kernel streams a
// 16-KB weight slice (L2) and an 8-KB x piece (HBM) per slice step (mlp_fused_h.hip,
// skip_hp_kernel); this measures the copy engine without the MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 tools/dma_rate.hip -o tools/bin/dma_rate
// Run:   tools/bin/dma_rate   (prints one line per mode: GB/s chip-wide)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

__device__ __forceinline__ void glds16s(uint64_t sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  sbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sbase >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(sbase), "v"(voff), "s"(lds)
      : "memory");
}

constexpr int SLOT = 16384, NS = 4;

// MODE 0: every step each of the 4 waves DMAs 4 KB of a 16-KB slice of `img`
//         (256 KB, L2-resident: 16 slices); MODE 1: the same bytes from `big`
//         (streamed, HBM); MODE 2: 16 KB from img + 8 KB from big per step (skip_hp's mix)
template <int MODE>
__global__ __launch_bounds__(256) void dma_ring(const char* __restrict__ img,
                                                const char* __restrict__ big, int64_t big_bytes,
                                                int steps, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[NS * (SLOT + 8192)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t l0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int64_t per_wg = (int64_t)steps * (MODE == 2 ? 8192 : SLOT);
  const int64_t base = ((int64_t)blockIdx.x * per_wg) % (big_bytes - per_wg - 8 * SLOT);
  auto issue = [&](int n) {
    const uint32_t slot = l0 + (uint32_t)((n % NS) * (SLOT + 8192));
    if (MODE == 0 || MODE == 2) {
      const uint64_t src = (uint64_t)(img + (int64_t)(n & 15) * SLOT) + wave_u * 4096;
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16s(src + i * 1024, lane * 16, slot + wave_u * 4096 + i * 1024);
    }
    if (MODE == 1) {
      const uint64_t src = (uint64_t)(big + base + (int64_t)n * SLOT) + wave_u * 4096;
#pragma unroll
      for (int i = 0; i < 4; ++i) glds16s(src + i * 1024, lane * 16, slot + wave_u * 4096 + i * 1024);
    }
    if (MODE == 2) {
      const uint64_t src = (uint64_t)(big + base + (int64_t)n * 8192) + wave_u * 2048;
#pragma unroll
      for (int i = 0; i < 2; ++i) glds16s(src + i * 1024, lane * 16, slot + SLOT + wave_u * 2048 + i * 1024);
    }
  };
  constexpr int G = MODE == 2 ? 6 : 4;
  for (int n = 0; n < NS - 1; ++n) issue(n);
  int acc = 0;
  for (int n = 0; n < steps; ++n) {
    if (G == 6) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    acc += *reinterpret_cast<const int*>(lds + (n % NS) * (SLOT + 8192) + lane * 4);
    issue(n + NS - 1);  // beyond `steps` it re-reads valid memory (never used)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678) sink[0] = acc;
}

// plain 16-B loads of the L2 image into registers, 4 KB per wave per step, 3 steps ahead
__global__ __launch_bounds__(256) void ld_l2(const char* __restrict__ img, int steps, int* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint4 r[3][4];
  uint32_t acc = 0;
  auto ld = [&](int n, uint4 (&d)[4]) {
    const char* src = img + (int64_t)(n & 15) * SLOT + wave * 4096 + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<const uint4*>(src + i * 1024);
  };
  ld(0, r[0]);
  ld(1, r[1]);
  for (int n = 0; n < steps; n += 3) {
    ld(n + 2, r[2]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= r[0][i].x ^ r[0][i].w;
    ld(n + 3, r[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= r[1][i].x ^ r[1][i].w;
    ld(n + 4, r[1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= r[2][i].x ^ r[2][i].w;
  }
  if (acc == 0x12345678u) sink[0] = (int)acc;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t big_bytes = 2LL << 30;
  char *img, *big;
  int* sink;
  CHECK(hipMalloc(&img, 16 * SLOT));
  CHECK(hipMalloc(&big, big_bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(img, 1, 16 * SLOT));
  CHECK(hipMemset(big, 1, big_bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int steps = 512;
  for (int per_cu = 1; per_cu <= 2; ++per_cu) {
    const int grid = cus * per_cu;
    for (int mode = 0; mode < 4; ++mode) {
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(dma_ring<0>, grid, 256, 0, 0, img, big, big_bytes, steps, sink);
        if (mode == 1) hipLaunchKernelGGL(dma_ring<1>, grid, 256, 0, 0, img, big, big_bytes, steps, sink);
        if (mode == 2) hipLaunchKernelGGL(dma_ring<2>, grid, 256, 0, 0, img, big, big_bytes, steps, sink);
        if (mode == 3) hipLaunchKernelGGL(ld_l2, grid, 256, 0, 0, img, steps, sink);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      const double bytes = (double)grid * steps * (mode == 2 ? SLOT + 8192 : SLOT);
      const char* name[] = {"dma  L2 image 16KB/step", "dma  HBM stream 16KB/step",
                            "dma  L2 16KB + HBM 8KB/step", "load L2 image 16KB/step (regs)"};
      printf("wg/cu=%d %-32s %8.3f ms  %7.0f GB/s  %5.1f B/clk/CU @2.1GHz\n", per_cu, name[mode], ms,
             bytes / ms / 1e6, bytes / (ms * 1e-3) / cus / 2.1e9);
    }
  }
  return 0;
}
