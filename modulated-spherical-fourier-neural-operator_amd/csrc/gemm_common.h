// Shared device code of the MFMA GEMMs (gemm.hip: fp32 MFMA, gemm_x6.hip:
// fp32-accurate 6-term bf16 split): kernel parameters, the XCD-aware tile
// remap, GELU(erf) and the LDS-staged fused epilogue.
#pragma once
#include <cstdlib>
#include "bf16x3.h"
#include "common.h"

namespace msfno {
typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmParams {
  const float* A;
  const float* B;
  float* C;
  int M, N, K, lda, ldb, ldc;
  int64_t sA, sB, sC;
  int tiles_m, tiles_n;
  const GemmDesc* descs;
  int ndesc;
  int vecA, vecB;
  // epilogue
  const float* bias;
  const float* addend;
  int64_t sBias, sD;
  int ldd, act, relu_period, relu_rows;
  int vecC;  // C (and addend) rows 16-B aligned: float4 epilogue loads/stores
  const float* rowscale;
  int rs_C;
  // gemm_x6: A pre-split into 3 bf16 planes [batch][3][Mp][Kp] (k contiguous)
  const unsigned short* Ax;
  int64_t sAx, sAxp;  // batch stride, plane stride (elements)
  int ldax;           // Kp
  // bf16x3 "plane" operands (gemm_x6.hip): B given as 3 exact bf16 terms
  // [batch sB][plane sBxp][K][ldb] instead of fp32; C written as planes
  // [batch sC][plane sCxp][M][ldc] (EPI_PLANES) instead of fp32
  const unsigned short* Bx;
  int64_t sBxp;
  unsigned short* Cx;
  int64_t sCxp;
  int cx16;  // plane rows 16-B aligned (ldc, sC, sCxp % 8 == 0, Cx 16-B aligned): uint4 stores
  // segmented K of A / columns of C (GemmEpi::segA_w ...; 0 = contiguous)
  int segA_w, segC_w;
  int64_t segA_stride, segC_stride;
  // K-concatenated fp32 B (GemmEpi::b2): rows k >= kb2 at B2 + (k - kb2) * ldb2
  const float* B2;
  int kb2, ldb2;
  int64_t sB2;
  // gemm_x6 on the x3h engine (NP = 2; gemm_x3_skip): B row k of batch z multiplied by
  // x3_bscale[z * K + k] while staged, accumulator row m by x3_rowmul[z * x3_ldrm + m]
  // before the epilogue (both powers of two)
  const float* x3_bscale;
  const float* x3_rowmul;
  int x3_ldrm;
};

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  // bijective: blocks that share an XCD (orig % 8) get contiguous logical ids
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// erf with the coefficients of ROCm's ocml erff, evaluated branch-free (both
// polynomial regimes, then a select) with the hardware exp2; |err| < 2e-7.
__device__ __forceinline__ float erf_fast(float x) {
  const float t = fabsf(x);
  const float s = t * t;
  float p = fmaf(__uint_as_float(0xba1345e1u), s, __uint_as_float(0x3ba10414u));
  p = fmaf(s, p, __uint_as_float(0xbcdac9b8u));
  p = fmaf(s, p, __uint_as_float(0x3de703beu));
  p = fmaf(s, p, __uint_as_float(0xbec09330u));
  p = fmaf(s, p, __uint_as_float(0x3e0375d0u));
  const float small = fmaf(t, p, t);
  float q = fmaf(__uint_as_float(0x378e98abu), t, __uint_as_float(0xb9c68948u));
  q = fmaf(t, q, __uint_as_float(0x3b7cd369u));
  q = fmaf(t, q, __uint_as_float(0xbcc618b2u));
  q = fmaf(t, q, __uint_as_float(0x3dda74e4u));
  q = fmaf(t, q, __uint_as_float(0x3f228afdu));
  q = fmaf(t, q, __uint_as_float(0x3e03c728u));
  q = fmaf(t, q, t);
  const float large = 1.0f - __builtin_amdgcn_exp2f(-1.44269504088896341f * q);
  const float r = t < 1.0f ? small : large;
  return copysignf(r, x);
}

// Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7): one rational + one exp2, no
// regime select (fewer VALU slots than the two-regime ocml form)
__device__ __forceinline__ float erf_as(float x) {
  const float t0 = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, t0, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-1.44269504088896341f * t0 * t0);
  return copysignf(fmaf(-p, e, 1.0f), x);
}

// the same A&S GELU on two values with packed fp32 math (v_pk_fma/mul/add_f32:
// two lanes' worth per instruction; only rcp/exp2 stay scalar)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 v) {
  const f32x2 z = v * 0.70710678118654752440f;
  const f32x2 t0 = __builtin_elementwise_abs(z);
  const f32x2 den = t0 * 0.3275911f + 1.0f;
  f32x2 t;
  t.x = __builtin_amdgcn_rcpf(den.x);
  t.y = __builtin_amdgcn_rcpf(den.y);
  f32x2 p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 q = (t0 * t0) * -1.44269504088896341f;
  f32x2 e;
  e.x = __builtin_amdgcn_exp2f(q.x);
  e.y = __builtin_amdgcn_exp2f(q.y);
  const f32x2 erfa = 1.0f - p * e;  // erf(|z|)
  f32x2 erfz;
  erfz.x = copysignf(erfa.x, z.x);
  erfz.y = copysignf(erfa.y, z.y);
  return (v * 0.5f) * (erfz + 1.0f);
}

#ifndef MSFNO_GELU_IMPL
#define MSFNO_GELU_IMPL 1  // 1: A&S 7.1.26 (measured 0.05-0.1 ms cheaper on fc1/fc2), 0: ocml form
#endif
__device__ __forceinline__ float gelu_erf(float v) {
#if MSFNO_GELU_IMPL == 1
  return 0.5f * v * (1.0f + erf_as(v * 0.70710678118654752440f));
#else
  return 0.5f * v * (1.0f + erf_fast(v * 0.70710678118654752440f));
#endif
}

// 16-B plane stores in the epilogue (MSFNO_CX16=0: 8-B stores, for A/B)
inline bool cx16_enabled() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_CX16");
    return !(e && e[0] == '0');
  }();
  return on;
}

// epilogue flags (+ EPI_GELU_B: GELU applied to the B operand while it is staged)
enum : int {
  EPI_BIAS = 1, EPI_ADD = 2, EPI_GELU = 4, EPI_RELU = 8, EPI_ROWSCALE = 32, EPI_GELU_B = 64,
  EPI_PLANES = 128  // store C as three exact bf16 terms (the x6 operand format)
};



// C tile epilogue.  acc holds each wave's (BM/WGM)x(BN/WGN) part of the tile
// (waves WGM x WGN, wave w at (w / WGN, w % WGN)) as 32x32 MFMA blocks (row
// (r&3)+8(r>>2)+4(lane>>5), col lane&31).  lds: at least 32*WGM*(BN+8) floats,
// free (the caller's main loop ended with a barrier).
// RB = 32: accumulators in the 32x32 MFMA block layout (floatx16 per block);
// RB = 16: the 16x16 layout (floatx4: row 4 (lane >> 4) + r, col lane & 15)
template <int BM, int BN, int EPI, int WGM = 2, int WGN = 2, int MT, int NT, int RB = 32,
          class AccV = floatx16, bool PAIRS = true>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, AccV (&acc)[MT][NT],
                                              float* lds, const float* bias_s, float* C,
                                              const float* addend, int M, int N, int ldc,
                                              int m0, int n0, int dflags) {
  constexpr int NTHR = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  static_assert(MT == WM / RB && NT == WN / RB, "accumulator shape");
  constexpr int CS_LD = BN + 8;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int half = lane >> 5, l32 = lane & 31;
  (void)bias_s; (void)addend; (void)dflags; (void)half; (void)l32;
  // ---- epilogue through LDS ---------------------------------------------------
  // Per MFMA row-tile i the waves write their 32-row slices into a (32 WGM) x BN
  // row-major LDS image; then all threads walk it with 16-B vectors: bias,
  // addend (all loads of a thread issued before any use), activation, and
  // coalesced float4 stores.  Keeps the accumulators in AGPRs until here, the
  // epilogue VGPR-light, and the global traffic in full lines.
  float* Cs = lds;  // the main loop ended with a barrier: staging memory is free
  constexpr int QPT = (RB * WGM * BN / 4) / NTHR;  // float4 per thread per row-tile
  constexpr int QC = QPT <= 8 ? QPT : (QPT % 8 == 0 ? 8 : (QPT % 6 == 0 ? 6 : 4));
  static_assert(QPT * NTHR * 4 == RB * WGM * BN && QPT % QC == 0, "epilogue mapping");
  const bool vecC = p.vecC;
  // plane output: a thread takes two adjacent float4 (8 columns) so each plane is
  // stored as one 16-B vector (half the store instructions of 8-B stores): fc1 1-3 %
  // faster; the spectral x6c epilogues were 5 % slower with it (PAIRS = false there)
  constexpr bool PAIR = PAIRS && (EPI & EPI_PLANES) != 0;
  static_assert(!PAIR || QC % 2 == 0, "pairs of float4");
  auto eidx = [&](int qq) { return PAIR ? (tid + NTHR * (qq >> 1)) * 2 + (qq & 1) : tid + NTHR * qq; };
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if constexpr (RB == 32) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Cs[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * CS_LD + wn * WN + j * 32 + l32] =
              acc[i][j][r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wm * 16 + 4 * (lane >> 4) + r) * CS_LD + wn * WN + j * 16 + (lane & 15)] =
              acc[i][j][r];
      }
    }
    __syncthreads();
    // in chunks of QC float4 per thread (<= 8: bounds the epilogue's VGPRs)
    for (int qc = 0; qc < QPT; qc += QC) {
      float4 add4[QC];
      if constexpr ((EPI & EPI_ADD) != 0) {
#pragma unroll
        for (int q = 0; q < QC; ++q) {
          const int idx = eidx(qc + q);
          const int lr = idx / (BN / 4);
          const int row = min(m0 + (lr / RB) * WM + i * RB + (lr % RB), M - 1);
          const int col = n0 + 4 * (idx % (BN / 4));
          const float* src = addend + (int64_t)row * p.ldd;
          if (vecC) {
            add4[q] = *reinterpret_cast<const float4*>(src + min(col, (N - 1) & ~3));
          } else {
            add4[q] = make_float4(src[min(col, N - 1)], src[min(col + 1, N - 1)],
                                  src[min(col + 2, N - 1)], src[min(col + 3, N - 1)]);
          }
        }
      }
      // all LDS reads of the row-tile first (one lgkmcnt wait), then the math and
      // the stores: per-q read->use chains serialised ~100 cycles each behind the
      // stores of the previous q
      float4 cv[QC];
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int idx = eidx(qc + q);
        cv[q] = *reinterpret_cast<const float4*>(Cs + (idx / (BN / 4)) * CS_LD + 4 * (idx % (BN / 4)));
      }
      float bvq[QC];
      if constexpr ((EPI & EPI_BIAS) != 0) {
#pragma unroll
        for (int q = 0; q < QC; ++q) {
          const int lr = eidx(qc + q) / (BN / 4);
          const int row = m0 + (lr / RB) * WM + i * RB + (lr % RB);
          bvq[q] = bias_s[min(row, M - 1) - m0];
        }
      }
      uint2 held[3];  // PAIR: the planes of the even float4, stored with the odd one
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int idx = eidx(qc + q);
        const int lr = idx / (BN / 4);
        const int c4 = idx % (BN / 4);
        const int row = m0 + (lr / RB) * WM + i * RB + (lr % RB);
        const int col = n0 + 4 * c4;
        float4 v = cv[q];
        const int rr = min(row, M - 1);
        if constexpr ((EPI & EPI_ROWSCALE) != 0) {
          const int C2 = 2 * p.rs_C;
          const float sv = (dflags & 1) ? p.rowscale[(rr / C2) * p.rs_C + rr % p.rs_C] : 1.f;
          v.x *= sv; v.y *= sv; v.z *= sv; v.w *= sv;
        }
        if constexpr ((EPI & EPI_BIAS) != 0) {
          const float bv = bvq[q];
          v.x += bv; v.y += bv; v.z += bv; v.w += bv;
        }
        if constexpr ((EPI & EPI_ADD) != 0) {
          v.x += add4[q].x; v.y += add4[q].y; v.z += add4[q].z; v.w += add4[q].w;
        }
        if constexpr ((EPI & EPI_GELU) != 0) {
          f32x2 lo = {v.x, v.y}, hi = {v.z, v.w};
          lo = gelu_erf2(lo);
          hi = gelu_erf2(hi);
          v = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
        if constexpr ((EPI & EPI_RELU) != 0) {
          if ((unsigned)row % (unsigned)p.relu_period < (unsigned)p.relu_rows) {
            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
          }
        }
        if constexpr ((EPI & EPI_PLANES) != 0) {
          uint32_t a0, a1, a2, b0, b1, b2;
          split2(v.x, v.y, a0, a1, a2);
          split2(v.z, v.w, b0, b1, b2);
          const bool full8 = PAIR && p.cx16 && col - 4 * (q & 1) + 7 < N;  // the pair's 8 columns
          if ((q & 1) == 0 && full8) {
            held[0] = make_uint2(a0, b0);
            held[1] = make_uint2(a1, b1);
            held[2] = make_uint2(a2, b2);
          } else if (full8) {
            if (row < M) {
              unsigned short* dst = p.Cx + blockIdx.z * p.sC + (int64_t)row * ldc + col - 4;
              *reinterpret_cast<uint4*>(dst) = make_uint4(held[0].x, held[0].y, a0, b0);
              *reinterpret_cast<uint4*>(dst + p.sCxp) = make_uint4(held[1].x, held[1].y, a1, b1);
              *reinterpret_cast<uint4*>(dst + 2 * p.sCxp) = make_uint4(held[2].x, held[2].y, a2, b2);
            }
          } else if (row < M) {
            unsigned short* dst = p.Cx + blockIdx.z * p.sC + (int64_t)row * ldc + col;
            if (col + 3 < N) {  // ldc % 4 == 0 (checked on the host): 8-B aligned
              *reinterpret_cast<uint2*>(dst) = make_uint2(a0, b0);
              *reinterpret_cast<uint2*>(dst + p.sCxp) = make_uint2(a1, b1);
              *reinterpret_cast<uint2*>(dst + 2 * p.sCxp) = make_uint2(a2, b2);
            } else {
              const uint32_t t[3][2] = {{a0, b0}, {a1, b1}, {a2, b2}};
              for (int e = 0; e < 4 && col + e < N; ++e)
                for (int pl = 0; pl < 3; ++pl)
                  dst[pl * p.sCxp + e] = (unsigned short)(t[pl][e >> 1] >> (16 * (e & 1)));
            }
          }
        } else if (row < M) {
          float* dst = C + (int64_t)row * ldc + col;
          if (p.segC_w) {  // band exchange layout (seg_w % 4 == 0: a float4 stays in a block)
            const int q = col / p.segC_w;
            dst += q * (p.segC_stride - p.segC_w);
          }
          if (vecC && col + 3 < N) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            if (col < N) dst[0] = v.x;
            if (col + 1 < N) dst[1] = v.y;
            if (col + 2 < N) dst[2] = v.z;
            if (col + 3 < N) dst[3] = v.w;
          }
        }
      }
    }
    if (i + 1 < MT) __syncthreads();
  }
}

}  // namespace msfno
