// LDS-DMA helpers (global_load_lds) as inline asm, for gfx950.
//
// hipcc counts a __builtin_amdgcn_global_load_lds as a pending write of the
// whole LDS array and drains it (vmcnt(0)) before later ds_reads it cannot
// prove disjoint; in a ring / double-buffered structure that serialises the
// prefetch.  As inline asm the DMA is invisible to hipcc's waitcnt pass, so the
// kernel owns its completion: a counted `s_waitcnt vmcnt(N)` (N = vector-memory
// instructions the wave issued after the DMA), plus a barrier when other waves
// read the data (cdna_hip_programming.md §5.7).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace msfno {

typedef __attribute__((address_space(3))) void lds_void_t;

// LDS byte address of a pointer into __shared__ memory
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(lds_void_t*)p;
}

// one wave-instruction: lane l copies 16 B from gsrc to LDS byte (lds + 16 l);
// lds must be wave-uniform
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}

// one wave-instruction, SADDR form: lane l copies 16 B from sbase + voff (lane's 32-bit
// byte offset) to LDS byte lds + 16 l (sbase, lds wave-uniform)
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

// raw buffer access (stride 0) with a 32-bit lane offset and a wave-uniform SGPR offset:
// a strided fp32 plane is then addressed with at most one VALU op per access, not a
// 64-bit multiply-add; lanes whose LANE offset is past `bytes` (< 2^31) read 0 and drop
// their stores (the range check does not include the SGPR offset).
// aux 2 = nt (the nontemporal policy of __builtin_nontemporal_load / _store)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_ld_nt(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 2));
}
__device__ __forceinline__ void buf_st_nt(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 2);
}

// six wave-instructions in one block (one m0 save / restore): lane l copies 16 B
// from sbase + voff[i] to LDS byte lds + i * lds_step + 16 l.  sbase and lds must be
// wave-uniform (SGPR operands); voff[i] are the lane's byte offsets (SADDR + VADDR
// form, instruction offset 0); m0 advances by lds_step between the pieces.
template <int LDS_STEP>
__device__ __forceinline__ void glds16x6(uint64_t sbase, const uint32_t (&voff)[6], uint32_t lds) {
  unsigned keep;
  // make the uniformity explicit (SGPR operands)
  sbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sbase >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %1\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %1\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %1\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, %1\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %6, %1\n\t"
      "s_add_u32 m0, m0, %9\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %7, %1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(sbase), "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]), "v"(voff[4]),
        "v"(voff[5]), "s"(lds), "i"(LDS_STEP)
      : "memory", "scc");  // s_add_u32 writes SCC
}

// s_waitcnt vmcnt(n) for a run-time n, rounded down to a supported immediate
// (waiting for more than needed is safe)
__device__ __forceinline__ void wait_vmcnt(int n) {
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace msfno
