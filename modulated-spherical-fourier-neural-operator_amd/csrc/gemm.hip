// fp32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact fp32 fma chain, the
// chip's fp32 matrix peak).  Used for every dense contraction of the block:
//   * per-m Legendre contractions of the forward / inverse SHT (descriptor mode),
//   * the non-linear spectral MLP layers (complex GEMMs real-ified),
//   * the 1x1 convolutions (inner skip, MLP fc1/fc2) with fused epilogues.
// C[M,N] = A[M,K]·B[K,N], all row-major fp32.  Block tile BM×BN×16, 4 waves in
// a 2×2 arrangement, each wave owning (BM/2)×(BN/2) as 32×32 MFMA tiles.
// LDS is double buffered with one barrier per K-tile; A is staged k-major
// (transposed) so both MFMA operands are read as conflict-free ds_read_b32.
#include <cstdlib>
#include <string>

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

// epilogue flags (+ EPI_GELU_B: GELU applied to the B operand while it is staged)
enum : int { EPI_BIAS = 1, EPI_ADD = 2, EPI_GELU = 4, EPI_RELU = 8, EPI_ROWSCALE = 32, EPI_GELU_B = 64 };

template <int BM, int BN, int BK, bool VEC, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int LDA_S = BM + 2;  // staging-write conflict-free (see header)
  constexpr int LDB_S = BN;
  constexpr int A_LD = BM * BK / 1024;  // float4 staging loads per thread
  constexpr int B_LD = BN * BK / 1024;
  // one LDS array: the double-buffered A/B staging, reused by the epilogue as a
  // 64-row x (BN + 8) row-major image of the accumulators
  constexpr int CS_LD = BN + 8;
  constexpr int STAGE = 2 * BK * LDA_S + 2 * BK * LDB_S;
  constexpr int LDS_FLOATS = STAGE > 64 * CS_LD ? STAGE : 64 * CS_LD;
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  auto As = [&](int buf) { return lds + buf * (BK * LDA_S); };
  auto Bs = [&](int buf) { return lds + 2 * BK * LDA_S + buf * (BK * LDB_S); };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile -> problem mapping ----------------------------------------------
  const float* A = p.A;
  const float* B = p.B;
  float* C = p.C;
  int M = p.M, N = p.N, K = p.K, lda = p.lda, ldb = p.ldb, ldc = p.ldc;
  int tm, tn;
  const float* bias = p.bias;
  const float* addend = p.addend;
  int dflags = 0;
  if (p.descs) {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    int lo = 0, hi = p.ndesc - 1;
    while (lo < hi) {  // last desc with tile_start <= lin
      const int mid = (lo + hi + 1) >> 1;
      if (p.descs[mid].tile_start <= lin) lo = mid; else hi = mid - 1;
    }
    const GemmDesc d = p.descs[lo];
    A += d.offA; B += d.offB; C += d.offC;
    M = d.M; N = d.N; K = d.K; lda = d.lda; ldb = d.ldb; ldc = d.ldc;
    dflags = d.flags;
    const int local = lin - d.tile_start;
    tm = local % d.tiles_m;
    tn = local / d.tiles_m;
  } else {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    tm = lin % p.tiles_m;
    tn = lin / p.tiles_m;
    const int z = blockIdx.z;
    A += z * p.sA; B += z * p.sB; C += z * p.sC;
    if (bias) bias += z * p.sBias;
    if (addend) addend += z * p.sD;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;


  float4 ra[A_LD], rb[B_LD];

  // Branch-free staging: loads use clamped (always in-bounds) addresses and the
  // out-of-range elements are zeroed only when the registers are written to LDS
  // (after the MFMAs of the current tile), so hipcc neither predicates the loads
  // nor waits for them before the compute.  With VEC, rows are padded to a
  // multiple of 4 floats (ld % 4 == 0), so a float4 at k < K stays in its row.
  const int Mc = M > 0 ? M - 1 : 0, Kc = K > 0 ? K - 1 : 0, Nc = N > 0 ? N - 1 : 0;
  auto load_A = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int idx = tid + 256 * q;
      const int row = min(m0 + idx / (BK / 4), Mc);
      const int k = k0 + (idx % (BK / 4)) * 4;
      const float* src = A + (int64_t)row * lda;
      if constexpr (VEC) {
        ra[q] = *reinterpret_cast<const float4*>(src + min(k, Kc & ~3));
      } else {
        ra[q] = make_float4(src[min(k, Kc)], src[min(k + 1, Kc)], src[min(k + 2, Kc)],
                            src[min(k + 3, Kc)]);
      }
    }
  };
  auto load_B = [&](int kt, float4* dst) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int idx = tid + 256 * q;
      const int kr = min(k0 + idx / (BN / 4), Kc);
      const int col = n0 + (idx % (BN / 4)) * 4;
      const float* src = B + (int64_t)kr * ldb;
      if constexpr (VEC) {
        dst[q] = *reinterpret_cast<const float4*>(src + min(col, Nc & ~3));
      } else {
        dst[q] = make_float4(src[min(col, Nc)], src[min(col + 1, Nc)], src[min(col + 2, Nc)],
                             src[min(col + 3, Nc)]);
      }
    }
  };
  auto store_A = [&](int buf, int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / (BK / 4);
      const int k = (idx % (BK / 4)) * 4;
      const bool rok = m0 + row < M;
      const int kg = k0 + k;
      float* dst = As(buf) + k * LDA_S + row;
      dst[0] = (rok && kg + 0 < K) ? ra[q].x : 0.f;
      dst[LDA_S] = (rok && kg + 1 < K) ? ra[q].y : 0.f;
      dst[2 * LDA_S] = (rok && kg + 2 < K) ? ra[q].z : 0.f;
      dst[3 * LDA_S] = (rok && kg + 3 < K) ? ra[q].w : 0.f;
    }
  };
  auto store_B = [&](int buf, int kt, const float4* src) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int idx = tid + 256 * q;
      const int kr = idx / (BN / 4);
      const int col = (idx % (BN / 4)) * 4;
      const bool kok = k0 + kr < K;
      const int cg = n0 + col;
      float4 v = src[q];
      v.x = (kok && cg + 0 < N) ? v.x : 0.f;
      v.y = (kok && cg + 1 < N) ? v.y : 0.f;
      v.z = (kok && cg + 2 < N) ? v.z : 0.f;
      v.w = (kok && cg + 3 < N) ? v.w : 0.f;
      *reinterpret_cast<float4*>(Bs(buf) + kr * LDB_S + col) = v;
    }
  };

  const int half = lane >> 5;
  floatx16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int l32 = lane & 31;
  // the MFMAs of one staged k-tile; per_kk(kk) runs after each MFMA group
  auto mfma_tile = [&](int buf, auto&& per_kk) {
    const float* as = As(buf);
    const float* bs = Bs(buf);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int k = 2 * kk + half;
      float a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = as[k * LDA_S + wm * WM + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = bs[k * LDB_S + wn * WN + j * 32 + l32];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      per_kk(kk);
    }
  };

  if constexpr ((EPI & EPI_GELU_B) == 0) {
    if (nk > 0) {
      load_A(0);
      load_B(0, rb);
      store_A(0, 0);
      store_B(0, 0, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        load_A(kt + 1);
        load_B(kt + 1, rb);
      }
      mfma_tile(cur, [](int) {});
      if (kt + 1 < nk) {
        store_A(cur ^ 1, kt + 1);
        store_B(cur ^ 1, kt + 1, rb);
      }
      __syncthreads();
    }
  } else {
    // GELU(erf) of B (the MLP hidden layer) while it is staged: the next tile's
    // registers are transformed after the first MFMA groups of the current tile
    // (measured: spreading the GELUs over all groups with B loaded two tiles
    // ahead was slower, 3.50 vs 2.91 ms on fc2).
    constexpr int NE = B_LD * 4;
    auto gelu_all = [&]() {
#pragma unroll
      for (int q = 0; q < B_LD; ++q) {
        rb[q].x = gelu_erf(rb[q].x); rb[q].y = gelu_erf(rb[q].y);
        rb[q].z = gelu_erf(rb[q].z); rb[q].w = gelu_erf(rb[q].w);
      }
    };
    (void)NE;
    if (nk > 0) {
      load_A(0);
      load_B(0, rb);
      gelu_all();
      store_A(0, 0);
      store_B(0, 0, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) {
        load_A(kt + 1);
        load_B(kt + 1, rb);
      }
      mfma_tile(cur, [&](int kk) {
        if (kk == BK / 2 - 3 && more) gelu_all();
      });
      if (more) {
        store_A(cur ^ 1, kt + 1);
        store_B(cur ^ 1, kt + 1, rb);
      }
      __syncthreads();
    }
  }

  // ---- epilogue through LDS ---------------------------------------------------
  // Per MFMA row-tile i the four waves write their 32-row slices into a 64 x BN
  // row-major LDS image; then all 256 threads walk it with 16-B vectors: bias,
  // addend (all loads of a thread issued before any use), activation, and
  // coalesced float4 stores.  Keeps the accumulators in AGPRs until here, the
  // epilogue VGPR-light, and the global traffic in full lines.
  float* Cs = lds;  // the main loop ended with a barrier: staging memory is free
  constexpr int QPT = (64 * BN / 4) / 256;  // float4 per thread per row-tile
  const bool vecC = p.vecC;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Cs[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * CS_LD + wn * WN + j * 32 + l32] =
            acc[i][j][r];
    __syncthreads();
    float4 add4[QPT];
    if constexpr ((EPI & EPI_ADD) != 0) {
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        const int idx = tid + 256 * q;
        const int lr = idx / (BN / 4);
        const int row = min(m0 + (lr >> 5) * WM + i * 32 + (lr & 31), M - 1);
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
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      const int idx = tid + 256 * q;
      const int lr = idx / (BN / 4);
      const int c4 = idx % (BN / 4);
      const int row = m0 + (lr >> 5) * WM + i * 32 + (lr & 31);
      const int col = n0 + 4 * c4;
      float4 v = *reinterpret_cast<const float4*>(Cs + lr * CS_LD + 4 * c4);
      const int rr = min(row, M - 1);
      if constexpr ((EPI & EPI_ROWSCALE) != 0) {
        const int C2 = 2 * p.rs_C;
        const float sv = (dflags & 1) ? p.rowscale[(rr / C2) * p.rs_C + rr % p.rs_C] : 1.f;
        v.x *= sv; v.y *= sv; v.z *= sv; v.w *= sv;
      }
      if constexpr ((EPI & EPI_BIAS) != 0) {
        const float bv = bias[rr];
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
      if (row < M) {
        float* dst = C + (int64_t)row * ldc + col;
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
    if (i + 1 < MT) __syncthreads();
  }
}

GemmTile role_tile(GemmRole r, GemmTile dflt) {
  static int table[ROLE_COUNT];
  static bool init = false;
  if (!init) {
    for (int& t : table) t = -1;
    if (const char* e = getenv("MSFNO_TILES")) {
      static const char* names[ROLE_COUNT] = {"skip", "fc1", "fc2", "spec", "leg", "legi"};
      std::string spec(e);
      size_t pos = 0;
      while (pos < spec.size()) {
        size_t end = spec.find(',', pos);
        if (end == std::string::npos) end = spec.size();
        const std::string kv = spec.substr(pos, end - pos);
        const size_t eq = kv.find('=');
        if (eq != std::string::npos)
          for (int i = 0; i < ROLE_COUNT; ++i)
            if (kv.substr(0, eq) == names[i]) table[i] = atoi(kv.c_str() + eq + 1);
        pos = end + 1;
      }
    }
    init = true;
  }
  const int t = table[r];
  return (t >= 0 && t <= TILE_128x256) ? (GemmTile)t : dflt;
}

void gemm_tile_dims(GemmTile tile, int* bm, int* bn) {
  switch (tile) {
    case TILE_128x128: *bm = 128; *bn = 128; break;
    case TILE_128x64: *bm = 128; *bn = 64; break;
    case TILE_256x64: *bm = 256; *bn = 64; break;
    case TILE_256x128: *bm = 256; *bn = 128; break;
    case TILE_128x256: *bm = 128; *bn = 256; break;
    default: *bm = 64; *bn = 64; break;
  }
}

static GemmParams make_params(const float* A, const float* B, float* C, const GemmEpi& e) {
  GemmParams p{};
  p.A = A; p.B = B; p.C = C;
  p.bias = e.bias; p.addend = e.addend;
  p.sBias = e.sBias; p.sD = e.sD;
  p.ldd = e.ldd; p.act = e.act; p.relu_period = e.relu_period; p.relu_rows = e.relu_rows;
  p.rowscale = e.rowscale;
  p.rs_C = e.rs_C;
  return p;
}

template <int BM, int BN, int BK, int EPI>
static void launch_e(const GemmParams& p, dim3 grid, hipStream_t s) {
  if (p.vecA && p.vecB)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, true, EPI>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, false, EPI>), grid, dim3(256), 0, s, p);
}

static int epi_code(const GemmParams& p) {
  return (p.bias ? EPI_BIAS : 0) | (p.addend ? EPI_ADD : 0) | (p.act == 1 ? EPI_GELU : 0) |
         (p.relu_period ? EPI_RELU : 0) |
         (p.rowscale ? EPI_ROWSCALE : 0) | (p.act == 2 ? EPI_GELU_B : 0);
}

// the epilogue combinations the block uses (anything else is rejected)
template <int BM, int BN, int BK>
static int launch(const GemmParams& p, dim3 grid, hipStream_t s) {
  switch (epi_code(p)) {
    case 0: launch_e<BM, BN, BK, 0>(p, grid, s); break;
    case EPI_RELU: launch_e<BM, BN, BK, EPI_RELU>(p, grid, s); break;
    case EPI_ROWSCALE: launch_e<BM, BN, BK, EPI_ROWSCALE>(p, grid, s); break;
    case EPI_BIAS: launch_e<BM, BN, BK, EPI_BIAS>(p, grid, s); break;
    case EPI_BIAS | EPI_GELU: launch_e<BM, BN, BK, EPI_BIAS | EPI_GELU>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD: launch_e<BM, BN, BK, EPI_BIAS | EPI_ADD>(p, grid, s); break;
    case EPI_GELU_B | EPI_BIAS: launch_e<BM, BN, BK, EPI_GELU_B | EPI_BIAS>(p, grid, s); break;
    case EPI_GELU_B | EPI_BIAS | EPI_ADD:
      launch_e<BM, BN, BK, EPI_GELU_B | EPI_BIAS | EPI_ADD>(p, grid, s); break;
    case EPI_ADD: launch_e<BM, BN, BK, EPI_ADD>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD | EPI_GELU:  // decoder fc1 over the big-skip concatenation
      launch_e<BM, BN, BK, EPI_BIAS | EPI_ADD | EPI_GELU>(p, grid, s); break;
    default:
      set_error("gemm: unsupported epilogue combination");
      return MSFNO_EUNSUPPORTED;
  }
  return MSFNO_OK;
}

#ifndef MSFNO_GEMM_BK
#define MSFNO_GEMM_BK 16
#endif

static int dispatch(GemmTile tile, const GemmParams& p, dim3 grid, hipStream_t s) {
  int rc;
  switch (tile) {
    case TILE_128x128: rc = launch<128, 128, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_128x64: rc = launch<128, 64, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_256x64: rc = launch<256, 64, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_256x128: rc = launch<256, 128, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_128x256: rc = launch<128, 256, MSFNO_GEMM_BK>(p, grid, s); break;
    default: rc = launch<64, 64, MSFNO_GEMM_BK>(p, grid, s); break;
  }
  if (rc != MSFNO_OK) return rc;
  return launch_check("gemm_f32");
}

static bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

int gemm_uniform(GemmTile tile, const float* A, const float* B, float* C, int M, int N, int K,
                 int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int batch,
                 const GemmEpi& epi, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return MSFNO_OK;
  int bm, bn;
  gemm_tile_dims(tile, &bm, &bn);
  GemmParams p = make_params(A, B, C, epi);
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC;
  p.tiles_m = (int)cdiv(M, bm);
  p.tiles_n = (int)cdiv(N, bn);
  p.vecA = (lda % 4 == 0) && (sA % 4 == 0) && aligned16(A);
  p.vecB = (ldb % 4 == 0) && (sB % 4 == 0) && aligned16(B);
  p.vecC = (ldc % 4 == 0) && (sC % 4 == 0) && aligned16(C) &&
           (!epi.addend || ((epi.ldd % 4 == 0) && (epi.sD % 4 == 0) && aligned16(epi.addend)));
  MSFNO_REQUIRE(batch <= 65535, MSFNO_EINVAL, "gemm: batch too large");
  dim3 grid(p.tiles_m * p.tiles_n, 1, batch);
  return dispatch(tile, p, grid, s);
}

int gemm_desc(GemmTile tile, const float* A, const float* B, float* C, const GemmDesc* descs,
              int ndesc, int total_tiles, const GemmEpi& epi, hipStream_t s) {
  if (total_tiles <= 0) return MSFNO_OK;
  GemmParams p = make_params(A, B, C, epi);
  p.descs = descs;
  p.ndesc = ndesc;
  // descriptor problems are laid out with lda/ldb/offsets that are multiples of 4
  p.vecA = aligned16(A);
  p.vecB = aligned16(B);
  p.vecC = aligned16(C) && !epi.addend;
  return dispatch(tile, p, dim3(total_tiles), s);
}

}  // namespace msfno
