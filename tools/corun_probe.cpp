// Co-residency probe: does skip_h_kernel, running on a second stream,
// change the results of a kernel that shares CUs with it?
//
// Victims (stream A), each compared bit for bit with its solo run:
//   fft240   the row rFFT of the 120 x 240 blocks (fft_r2c_dma_kernel, H = 120: a 24-KB
//            workgroup fits beside two 66-KB skip_h workgroups on one CU)
//   fft1440  the row rFFT at 721 x 1440 (a 150-KB workgroup: cannot share a CU with skip_h)
//   lds      a 24-KB, 12-wave kernel that fills its LDS with a tagged pattern (ds_write),
//            re-reads it for a while and reports every word that changed
// Aggressors (stream B, launched first): none | skip_h | x3 (gemm_x3, same product).
// Also: a masked LDS-DMA test (lanes 60..63 of a global_load_lds_dwordx4 inactive:
// does the DMA still write their 16-B chunks?).
//
// Build (needs libmsfno.so): see tools/build_tools.sh
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../modulated-spherical-fourier-neural-operator_amd/csrc/common.h"
#include "../modulated-spherical-fourier-neural-operator_amd/csrc/kernels.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define CM(x)                                                                       \
  do {                                                                              \
    int r_ = (x);                                                                   \
    if (r_ != 0) {                                                                  \
      fprintf(stderr, "msfno rc %d (%s) at %s:%d\n", r_, msfno_last_error(), __FILE__, \
              __LINE__);                                                            \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

__global__ void fill_rand(float* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = scale * ((float)(h & 0xFFFFFF) / 16777216.f - 0.5f);
  }
}
__global__ void fill_const(float* p, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// 12 waves, 24 KB of LDS: tag every word, re-read `loops` times, count words that changed
__global__ __launch_bounds__(768) void lds_victim(int loops, unsigned long long* errs,
                                                  uint32_t* first) {
  extern __shared__ uint32_t lds[];
  const int n = 6144;  // words
  const uint32_t tag = 0x5A000000u | (blockIdx.x << 13);
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = tag | i;
  __syncthreads();
  unsigned long long bad = 0;
  for (int it = 0; it < loops; ++it) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t v = lds[i];
      if (v != (tag | i)) {
        if (bad == 0) {
          const unsigned slot = atomicAdd(first, 1u);
          if (slot < 64) {
            first[1 + 3 * slot] = blockIdx.x;
            first[2 + 3 * slot] = i;
            first[3 + 3 * slot] = v;
          }
        }
        ++bad;
        lds[i] = tag | i;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (bad) atomicAdd(errs, bad);
}

// The instruction sequence hipcc emits for the rFFT's bin() in its remainder loop
// (fft_r2c_dma_kernel<FixedFFT<4,2,3,5>,12,false,2>, the lanes with one bin left):
//   v_mul_f32 o.lo = -0.5 d ; v_mul_f32 q.lo = 0.5 e
//   v_pk_mul_f32 p = o * t  op_sel:[0,1] op_sel_hi:[0,0]     p = (o.lo t.hi, o.lo t.lo)
//   v_pk_fma_f32 r = t * q - p                               r.lo = t.lo q.lo - p.lo
// VAR: 0 as emitted; 1 s_nop 0 between the packed pair; 2 s_nop 1; 3 s_nop 4;
// 4 the product as two v_mul_f32 (no packed producer).  MASK: run in lanes 57..63 only.
template <int VAR>
__device__ __forceinline__ float pk_seq(float c, float s, float d, float e) {
  float r;
#define PK_ASM(PROD, NOP)                                                           \
  asm volatile(                                                                     \
      "v_mov_b32 v100, %1\n\tv_mov_b32 v101, %2\n\tv_mov_b32 v102, %3\n\t"          \
      "v_mov_b32 v104, %4\n\ts_nop 4\n\t"                                            \
      "v_mul_f32 v102, -0.5, v102\n\t"                                               \
      "v_mul_f32 v104, 0.5, v104\n\t" PROD NOP                                       \
      "v_pk_fma_f32 v[108:109], v[100:101], v[104:105], v[106:107] neg_lo:[0,0,1] "  \
      "neg_hi:[0,0,1]\n\t"                                                           \
      "s_nop 4\n\tv_mov_b32 %0, v108"                                                \
      : "=v"(r)                                                                     \
      : "v"(c), "v"(s), "v"(d), "v"(e)                                              \
      : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", \
        "v110", "v111", "v112", "v113")
#define PK_MUL "v_pk_mul_f32 v[106:107], v[102:103], v[100:101] op_sel:[0,1] op_sel_hi:[0,0]\n\t"
  if constexpr (VAR == 0) PK_ASM(PK_MUL, "");
  else if constexpr (VAR == 8) PK_ASM("v_mov_b32 v103, 0\n\tv_mov_b32 v105, 0\n\ts_nop 1\n\t" PK_MUL, "");
  else if constexpr (VAR == 9) PK_ASM("v_mov_b32 v103, 0x7fc00000\n\tv_mov_b32 v105, 0x7fc00000\n\ts_nop 1\n\t" PK_MUL, "");
  else if constexpr (VAR == 10) PK_ASM("v_mov_b32 v103, 1.0\n\tv_mov_b32 v105, 1.0\n\ts_nop 1\n\t" PK_MUL, "");
  else if constexpr (VAR == 1) PK_ASM(PK_MUL, "s_nop 0\n\t");
  else if constexpr (VAR == 2) PK_ASM(PK_MUL, "s_nop 1\n\t");
  else if constexpr (VAR == 3) PK_ASM(PK_MUL, "s_nop 4\n\t");
  else if constexpr (VAR == 4) PK_ASM("v_mul_f32 v106, v102, v101\n\t", "");
  else if constexpr (VAR == 5) {  // packed producer, scalar consumer: r = c e/2 - p.lo
    asm volatile(
        "v_mov_b32 v100, %1\n\tv_mov_b32 v101, %2\n\tv_mov_b32 v102, %3\n\t"
        "v_mov_b32 v104, %4\n\ts_nop 4\n\t"
        "v_mul_f32 v102, -0.5, v102\n\t"
        "v_mul_f32 v104, 0.5, v104\n\t" PK_MUL
        "s_nop 4\n\tv_fma_f32 v108, v100, v104, -v106\n\t"
        "s_nop 4\n\tv_mov_b32 %0, v108"
        : "=v"(r)
        : "v"(c), "v"(s), "v"(d), "v"(e)
        : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109");
  } else if constexpr (VAR == 6) {  // p = (o.lo t.hi, o.hi t.lo) via a plain pk_mul of swapped pairs
    PK_ASM("v_mov_b32 v103, v102\n\tv_mov_b32 v110, v101\n\tv_mov_b32 v111, v100\n\ts_nop 1\n\t"
           "v_pk_mul_f32 v[106:107], v[102:103], v[110:111]\n\t", "");
  } else {  // VAR 7: the product by a packed add of (o.lo t.hi) computed scalar + 0
    PK_ASM("v_mul_f32 v110, v102, v101\n\tv_mov_b32 v111, 0\n\tv_mov_b32 v112, 0\n\t"
           "v_mov_b32 v113, 0\n\ts_nop 1\n\tv_pk_add_f32 v[106:107], v[110:111], v[112:113]\n\t", "");
  }
#undef PK_MUL
#undef PK_ASM
  return r;
}

template <int VAR, bool MASK>
__global__ __launch_bounds__(768) void pk_victim(int loops, unsigned long long* errs,
                                                 uint32_t* first) {
  extern __shared__ uint32_t lds_pad[];  // sized like the rFFT's workgroup (24 KB)
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) lds_pad[0] = 0;
  unsigned long long bad = 0;
  for (int it = 0; it < loops; ++it) {
    uint32_t h = (uint32_t)(it * 7919 + threadIdx.x * 104729 + blockIdx.x * 1299709);
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const float c = (float)(h & 0xFFFF) / 65536.f + 0.1f;
    const float s = -(float)((h >> 16) & 0xFFFF) / 65536.f - 0.2f;
    const float d = (float)(h & 0x3FF) / 256.f - 2.f;
    const float e = (float)((h >> 10) & 0x3FF) / 256.f - 2.f;
    if (!MASK || lane >= 57) {
      const float got = pk_seq<VAR>(c, s, d, e);
      const float want = fmaf(c, 0.5f * e, -((-0.5f * d) * s));
      if (__float_as_uint(got) != __float_as_uint(want)) {
        if (bad == 0) {
          const unsigned slot = atomicAdd(first, 1u);
          if (slot < 64) {
            first[1 + 3 * slot] = lane;
            first[2 + 3 * slot] = __float_as_uint(got);
            first[3 + 3 * slot] = __float_as_uint(want);
          }
        }
        ++bad;
      }
    }
  }
  if (bad) atomicAdd(errs, bad);
}

// one LDS-DMA with lanes >= act inactive into a tagged 1-KB region: which chunks changed?
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}
__global__ __launch_bounds__(64) void masked_dma(const uint4* src, int act, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[512];  // 2 KB: the piece + 1 KB after
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = 0xDEAD0000u | i;
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  if (threadIdx.x < act) glds16(src + threadIdx.x, base);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}


// synthetic aggressors: 256 threads, 66 KB of LDS (two workgroups per CU, like skip_h)
typedef _Float16 ph8 __attribute__((ext_vector_type(8)));
typedef float pf4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256, 2) void agg_mfma(int loops, float* out) {
  __shared__ char pad[67584];
  if (threadIdx.x == 1023) pad[threadIdx.x] = 0;
  ph8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.001f * (threadIdx.x + i)); b[i] = (_Float16)0.5f; }
  pf4 c[4] = {};
  for (int it = 0; it < loops; ++it)
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[k], 0, 0, 0);
  if (c[0][0] == 12345.f) out[threadIdx.x] = c[1][0] + c[2][0] + c[3][0];
}
__global__ __launch_bounds__(256, 2) void agg_dma(const uint4* src, int loops, float* out) {
  __shared__ __attribute__((aligned(16))) char ring[67584];
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)ring;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int it = 0; it < loops; ++it) {
    for (int q = 0; q < 16; ++q)
      glds16(src + (q * 4 + wave) * 64 + lane, base + (uint32_t)(((q * 4 + wave) % 64) * 1024));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (ring[threadIdx.x] == 123) out[threadIdx.x] = 1.f;
}
__global__ __launch_bounds__(256, 2) void agg_valu(int loops, float* out) {
  __shared__ char pad[67584];
  if (threadIdx.x == 1023) pad[threadIdx.x] = 0;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 v = {0.001f * threadIdx.x, 1.f}, w = {0.999f, 1.0001f};
  for (int it = 0; it < loops; ++it)
#pragma unroll
    for (int k = 0; k < 16; ++k) v = v * w + w;
  if (v[0] == 12345.f) out[threadIdx.x] = v[1];
}

struct Bufs {
  float *x240, *x1440, *xs, *W, *bias, *xk, *outk;
  float2 *X240, *X1440, *ref240, *ref1440, *st;
  void* ws;
  size_t ws_bytes;
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  const char* only = argc > 2 ? argv[2] : "";
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));

  // masked LDS-DMA
  {
    uint4* src;
    uint32_t* out;
    CK(hipMalloc(&src, 64 * 16));
    CK(hipMalloc(&out, 512 * 4));
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; ++i) h[i] = 0xC0DE0000u | i;
    CK(hipMemcpy(src, h.data(), 1024, hipMemcpyHostToDevice));
    for (int act : {64, 60, 32, 1}) {
      hipLaunchKernelGGL(masked_dma, dim3(1), dim3(64), 0, 0, src, act, out);
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> o(512);
      CK(hipMemcpy(o.data(), out, 2048, hipMemcpyDeviceToHost));
      int written = 0, stray = 0, wrong = 0;
      for (int lane = 0; lane < 64; ++lane)
        for (int w = 0; w < 4; ++w) {
          const int i = lane * 4 + w;
          const bool changed = o[i] != (0xDEAD0000u | i);
          if (lane < act) {
            written += changed;
            wrong += o[i] != (0xC0DE0000u | i);
          } else {
            stray += changed;
          }
        }
      int beyond = 0;
      for (int i = 256; i < 512; ++i) beyond += o[i] != (0xDEAD0000u | i);
      printf("masked_dma act=%2d: active words written %d/%d (wrong %d), inactive-lane words "
             "changed %d, words beyond the piece changed %d\n",
             act, written, act * 4, wrong, stray, beyond);
    }
    CK(hipFree(src));
    CK(hipFree(out));
  }

  const int C = 256, B = 8;
  const int64_t rows240 = (int64_t)16 * C * 120, rows1440 = (int64_t)2 * C * 721;
  const int64_t Pk = 120 * 240;  // skip_h: 8 fields of 120 x 240
  msfno::FFTPlan f240, f1440;
  CM(msfno::fft_plan_build(f240, 240));
  CM(msfno::fft_plan_build(f1440, 1440));
  Bufs b{};
  CK(hipMalloc(&b.x240, rows240 * 240 * 4));
  CK(hipMalloc(&b.x1440, rows1440 * 1440 * 4));
  CK(hipMalloc(&b.X240, rows240 * 121 * 8));
  CK(hipMalloc(&b.ref240, rows240 * 121 * 8));
  CK(hipMalloc(&b.X1440, rows1440 * 361 * 8));
  CK(hipMalloc(&b.ref1440, rows1440 * 361 * 8));
  CK(hipMalloc(&b.st, std::max(rows240, rows1440) * 8));
  CK(hipMalloc(&b.xs, B * C * 4));
  CK(hipMalloc(&b.W, C * C * 4));
  CK(hipMalloc(&b.bias, C * 4));
  CK(hipMalloc(&b.xk, (int64_t)B * C * Pk * 4));
  CK(hipMalloc(&b.outk, (int64_t)B * C * Pk * 4));
  b.ws_bytes = std::max(msfno::skip_h_workspace(B), msfno::gemm_x3_workspace(C, C, B));
  CK(hipMalloc(&b.ws, b.ws_bytes));
  unsigned long long* errs;
  uint32_t* first;
  CK(hipMalloc(&errs, 8));
  CK(hipMalloc(&first, 4 * 200));
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, b.x240, rows240 * 240, 1u, 2.f);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, b.x1440, rows1440 * 1440, 2u, 2.f);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, b.W, (int64_t)C * C, 3u, 0.1f);
  hipLaunchKernelGGL(fill_rand, dim3(1), dim3(256), 0, 0, b.bias, (int64_t)C, 4u, 0.1f);
  hipLaunchKernelGGL(fill_rand, dim3(1024), dim3(256), 0, 0, b.xk, (int64_t)B * C * Pk, 5u, 2.f);
  hipLaunchKernelGGL(fill_const, dim3(8), dim3(256), 0, 0, b.xs, (int64_t)B * C, 4096.f);
  CK(hipDeviceSynchronize());

  const float sc = 6.283185307179586f / 240.f, sc2 = 6.283185307179586f / 1440.f;
  CM(msfno::launch_fft_r2c_rows(f240, b.x240, b.ref240, b.st, rows240, 121, sc, sa));
  CM(msfno::launch_fft_r2c_rows(f1440, b.x1440, b.ref1440, b.st, rows1440, 361, sc2, sa));
  CK(hipStreamSynchronize(sa));

  auto aggressor = [&](const std::string& a) {
    if (a == "skip_h")
      CM(msfno::launch_skip_h(b.W, b.xs, b.xk, b.outk, b.bias, B, Pk, b.ws, b.ws_bytes, sb));
    else if (a == "mfma")
      hipLaunchKernelGGL(agg_mfma, dim3(2048), dim3(256), 0, sb, 20000, b.outk);
    else if (a == "dma")
      hipLaunchKernelGGL(agg_dma, dim3(2048), dim3(256), 0, sb, (const uint4*)b.xk, 300, b.outk);
    else if (a == "valu")
      hipLaunchKernelGGL(agg_valu, dim3(2048), dim3(256), 0, sb, 20000, b.outk);
    else if (a == "mlp")
      CM(msfno::launch_mlp_fused_h(b.xk, b.xs, b.bias, b.xs, nullptr, b.outk, (const unsigned short*)b.ws,
                                   b.W, b.bias, 1, Pk * 4, sb));
    else if (a == "x3") {
      msfno::GemmEpi e;
      e.bias = b.bias;
      CM(msfno::gemm_x3(b.W, C, b.xs, b.xk, b.outk, C, (int)Pk, C, (int)Pk, (int)Pk, C * Pk,
                        C * Pk, B, e, b.ws, b.ws_bytes, sb));
    }
  };
  std::vector<float2> h_got, h_ref;
  for (const char* victim : {"fft240", "lds", "fft1440"}) {
    if (only[0] && strcmp(only, victim) != 0) continue;
    for (const char* agg : {"none", "skip_h", "x3"}) {
      long long bad_total = 0;
      int bad_iters = 0;
      std::vector<int> bin_hist(361, 0), lane_hist(64, 0);
      int re_bad = 0, im_bad = 0;
      std::string examples;
      for (int it = 0; it < iters; ++it) {
        CK(hipMemsetAsync(errs, 0, 8, sa));
        CK(hipMemsetAsync(first, 0, 4 * 200, sa));
        CK(hipStreamSynchronize(sa));
        for (int rep = 0; rep < 3; ++rep) aggressor(agg);
        if (!strcmp(victim, "fft240")) {
          CM(msfno::launch_fft_r2c_rows(f240, b.x240, b.X240, b.st, rows240, 121, sc, sa));
        } else if (!strcmp(victim, "fft1440")) {
          CM(msfno::launch_fft_r2c_rows(f1440, b.x1440, b.X1440, b.st, rows1440, 361, sc2, sa));
        } else {
          hipLaunchKernelGGL(lds_victim, dim3(1024), dim3(768), 6144 * 4, sa, 400, errs, first);
          CK(hipGetLastError());
        }
        CK(hipDeviceSynchronize());
        if (!strcmp(victim, "lds")) {
          unsigned long long e = 0;
          uint32_t fh[200];
          CK(hipMemcpy(&e, errs, 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(fh, first, 800, hipMemcpyDeviceToHost));
          if (e) {
            ++bad_iters;
            bad_total += (long long)e;
            for (unsigned k = 0; k < std::min(fh[0], 4u); ++k) {
              char t[128];
              snprintf(t, sizeof t, " [wg %u word %u = %08x]", fh[1 + 3 * k], fh[2 + 3 * k],
                       fh[3 + 3 * k]);
              if (examples.size() < 600) examples += t;
            }
          }
          continue;
        }
        const bool big = !strcmp(victim, "fft1440");
        const int mm = big ? 361 : 121;
        const int64_t rows = big ? rows1440 : rows240;
        const int64_t n = rows * mm;
        h_got.resize(n);
        h_ref.resize(n);
        CK(hipMemcpy(h_got.data(), big ? b.X1440 : b.X240, n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_ref.data(), big ? b.ref1440 : b.ref240, n * 8, hipMemcpyDeviceToHost));
        long long bad = 0;
        for (int64_t i = 0; i < n; ++i) {
          const bool br = memcmp(&h_got[i].x, &h_ref[i].x, 4) != 0;
          const bool bi = memcmp(&h_got[i].y, &h_ref[i].y, 4) != 0;
          if (br || bi) {
            ++bad;
            re_bad += br;
            im_bad += bi;
            const int k = (int)(i % mm);
            bin_hist[k]++;
            lane_hist[k % 64]++;
            if (examples.size() < 900) {
              char t[200];
              snprintf(t, sizeof t, "\n    row %lld bin %d: got (%.9g, %.9g) want (%.9g, %.9g)",
                       (long long)(i / mm), k, h_got[i].x, h_got[i].y, h_ref[i].x, h_ref[i].y);
              examples += t;
            }
          }
        }
        if (bad) {
          ++bad_iters;
          bad_total += bad;
        }
      }
      printf("victim %-7s aggressor %-6s: %d of %d runs differ, %lld values", victim, agg,
             bad_iters, iters, bad_total);
      if (strcmp(victim, "lds") != 0 && bad_total) {
        printf(" (re %d, im %d); bins:", re_bad, im_bad);
        for (int k = 0; k < 361; ++k)
          if (bin_hist[k]) printf(" %d:%d", k, bin_hist[k]);
      }
      printf("%s\n", examples.c_str());
      fflush(stdout);
    }
  }
  // the packed-FP32 pair on its own, beside skip_h
  if (!only[0] || !strcmp(only, "pk")) {
    auto run_pk = [&](auto kern, const char* name) {
      for (const char* agg : {"none", "skip_h", "mfma", "dma", "valu", "mlp"}) {
        if (getenv("PK_AGG") && !strstr(getenv("PK_AGG"), agg)) continue;
        unsigned long long tot = 0;
        int bad_iters = 0;
        std::string ex;
        for (int it = 0; it < iters; ++it) {
          CK(hipMemsetAsync(errs, 0, 8, sa));
          CK(hipMemsetAsync(first, 0, 4 * 200, sa));
          CK(hipStreamSynchronize(sa));
          for (int rep = 0; rep < 3; ++rep) aggressor(agg);
          hipLaunchKernelGGL(kern, dim3(1024), dim3(768), 6144 * 4, sa, 3000, errs, first);
          CK(hipGetLastError());
          CK(hipDeviceSynchronize());
          unsigned long long e = 0;
          uint32_t fh[200];
          CK(hipMemcpy(&e, errs, 8, hipMemcpyDeviceToHost));
          CK(hipMemcpy(fh, first, 800, hipMemcpyDeviceToHost));
          if (e) {
            ++bad_iters;
            tot += e;
            for (unsigned k = 0; k < std::min(fh[0], 3u); ++k) {
              float g, w;
              memcpy(&g, &fh[2 + 3 * k], 4);
              memcpy(&w, &fh[3 + 3 * k], 4);
              char t[128];
              snprintf(t, sizeof t, " [lane %u got %.9g want %.9g]", fh[1 + 3 * k], g, w);
              if (ex.size() < 400) ex += t;
            }
          }
        }
        printf("victim %-12s aggressor %-6s: %d of %d runs differ, %llu values%s\n", name, agg,
               bad_iters, iters, tot, ex.c_str());
        fflush(stdout);
      }
    };
    run_pk(pk_victim<0, false>, "pk0_full");
    run_pk(pk_victim<8, false>, "pk8hizero");
    run_pk(pk_victim<9, false>, "pk9hinan");
    run_pk(pk_victim<10, false>, "pk10hione");
  }
  return 0;
}
