// The bf16x3 ("plane") number format of the x6 GEMM engine: an fp32 value split
// exactly into three bf16 terms t0 + t1 + t2 (8 significant bits each, 24
// together = the fp32 significand; round-to-nearest cvt, exact residuals).
// Producers (GEMM epilogues, the inverse FFT) write the three terms as separate
// planes; the x6p GEMM stages them without conversion.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace msfno {

// (a, b) -> packed bf16x2 terms t0 + t1 + t2 == (a, b) exactly (24 significant
// bits = the fp32 significand; round-to-nearest cvt, exact residuals)
typedef float f32x2_pk __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_pk __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  const f32x2_pk v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_pk));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ void split2(float a, float b, uint32_t& t0, uint32_t& t1, uint32_t& t2) {
  t0 = cvt_pk_bf16(a, b);
  a -= bf_lo(t0);
  b -= bf_hi(t0);
  t1 = cvt_pk_bf16(a, b);
  a -= bf_lo(t1);
  b -= bf_hi(t1);
  t2 = cvt_pk_bf16(a, b);
}

}  // namespace msfno
