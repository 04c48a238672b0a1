// fp32-accurate GEMM on the bf16 matrix cores ("x6" split) for gfx950.
//
// Every fp32 operand value is split exactly into three bf16 terms
//   x = x0 + x1 + x2,  x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (8 significant bits each, 24 together = the fp32 significand; the residual
// subtractions are exact).  A·B is then the sum of the six products whose term
// orders add to <= 2:  a2b0 + a1b1 + a0b2 + a1b0 + a0b1 + a0b0.  bf16 x bf16
// products are exact in fp32 and v_mfma_f32_32x32x16_bf16 accumulates in fp32;
// the dropped products (a1b2, a2b1, a2b2) are below 2^-24 relative, i.e. under
// the fp32 rounding of the result.  Measured against an fp64 reference the error
// is at or below the fp32 MFMA kernel's (tests/test_gpu_gemm_x6.py).  Six bf16
// MFMAs (32 cycles each) replace eight v_mfma_f32_32x32x2_f32 (64 cycles each)
// per 32x32x16 block: 2.67x fewer matrix-core cycles.
//
// C[M,N] = A[M,K]·B[K,N]; A is the small operand (weights) and is pre-split by
// launch_split_a into bf16 planes [batch][3][Mp][Kp] (zero padded), B is fp32
// row-major and split while it is staged.  Tile BM x BN x 16, 4 waves (2x2),
// each wave (BM/2)x(BN/2) as 32x32 blocks — the fp32 kernel's C layout, so the
// fused epilogue (gemm_common.h) is shared.
// LDS images (bf16):
//   A: [plane][m][16 k], 32-B rows; the two 16-B k-halves of row m are swapped
//      when (m>>3)&1 so ds_read_b128 fragment reads are bank-conflict free;
//   B: [plane][k][BN + 32] (row-major as in HBM; +64 B per row makes the
//      transposed fragment reads conflict free), read with ds_read_b64_tr_b16
//      (4 k x 16 n per 16-lane group, delivered k-contiguous per lane).
#include <cstdlib>
#include <type_traits>
#include <string>

#include "gemm_common.h"

namespace msfno {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
__global__ void split_a_kernel(const float* __restrict__ A, unsigned short* __restrict__ Ax, int M,
                               int K, int lda, int64_t sA, int Mp, int Kp) {
  const int z = blockIdx.y;
  const int64_t plane = (int64_t)Mp * Kp;
  const int64_t n = plane / 2;  // bf16 pairs per plane (Kp even)
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)((2 * e) / Kp), k = (int)((2 * e) % Kp);
    const float* a = A + z * sA + (int64_t)m * lda;
    const float v0 = (m < M && k < K) ? a[k] : 0.f;
    const float v1 = (m < M && k + 1 < K) ? a[k + 1] : 0.f;
    uint32_t t0, t1, t2;
    split2(v0, v1, t0, t1, t2);
    uint32_t* o = reinterpret_cast<uint32_t*>(Ax + z * 3 * plane) + e;
    o[0] = t0;
    o[n] = t1;
    o[2 * n] = t2;
  }
}

// NP planes per value: 3 = x6 (bf16 terms, six MFMAs per product), 2 = x3h (fp16
// terms h0 = fp16(v), h1 = fp16(v - h0); a1·b0 + a0·b1 + a0·b0, three MFMAs; the
// operands power-of-two scaled into fp16 range: p.x3_bscale per B row, the A image
// row-scaled by the host, p.x3_rowmul undoing that per C row)
template <int NP>
struct X6Eng;
template <>
struct X6Eng<3> {
  typedef bf16x8 frag;
  __device__ static void split(float a, float b, uint32_t (&t)[3]) { split2(a, b, t[0], t[1], t[2]); }
  __device__ static floatx16 prod(const frag (&a)[3], const frag (&b)[3], floatx16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
    return c;
  }
};
template <>
struct X6Eng<2> {
  typedef f16x8 frag;
  __device__ static void split(float a, float b, uint32_t (&t)[2]) {
    const f32x2 v = {a, b};
    const f16x2 h0 = __builtin_convertvector(v, f16x2);
    const f32x2 r = v - __builtin_convertvector(h0, f32x2);
    const f16x2 h1 = __builtin_convertvector(r, f16x2);
    t[0] = __builtin_bit_cast(uint32_t, h0);
    t[1] = __builtin_bit_cast(uint32_t, h1);
  }
  __device__ static floatx16 prod(const frag (&a)[2], const frag (&b)[2], floatx16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c, 0, 0, 0);
    return c;
  }
};

// BPL: B arrives pre-split as bf16 planes (p.Bx), staged without conversion
template <int BM, int BN, int WGM, int WGN, bool VEC, int EPI, bool BPL, int NP = 3>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_x6_kernel(GemmParams p) {
  static_assert(NP == 3 || !BPL, "x3h: fp32 B only");
  typedef typename X6Eng<NP>::frag Frag;
  constexpr int BK = 16;
  constexpr int NTHR = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int A_PLANE = BM * BK;  // bf16 elements
  constexpr int A_STAGE = NP * A_PLANE;
  constexpr int B_ROW = BN + 32;
  constexpr int B_PLANE = BK * B_ROW;
  constexpr int B_STAGE = NP * B_PLANE;
  constexpr int STAGE_BYTES = 2 * (A_STAGE + B_STAGE) * 2;
  constexpr int EPI_BYTES = 32 * WGM * (BN + 8) * 4;
  constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  constexpr bool HAS_BIAS = (EPI & EPI_BIAS) != 0;
  constexpr int A_LD = 2 * NP * BM / NTHR;  // 16-B chunks of split A per thread
  constexpr int B_LD = BK * BN / 4 / NTHR;  // float4 of B per thread
  static_assert(A_LD * NTHR == 2 * NP * BM && B_LD * NTHR * 4 == BK * BN, "tile shape");
  // pre-split B: chunks of BCH bf16 (16 or 8 bytes), BPQ per thread
  constexpr int BCH = ((3 * BK * BN / 8) % NTHR == 0) ? 8 : 4;
  constexpr int BPQ = 3 * BK * BN / BCH / NTHR;
  static_assert(BPQ * NTHR * BCH == 3 * BK * BN, "plane tile shape");
  typedef typename std::conditional<BCH == 8, uint4, uint2>::type bchunk_t;
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES + (HAS_BIAS ? BM * 4 : 0)];
  unsigned short* const As = reinterpret_cast<unsigned short*>(lds_raw);
  unsigned short* const Bs = As + 2 * A_STAGE;
  float* const bias_s = reinterpret_cast<float*>(lds_raw + LDS_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int half = lane >> 5, l32 = lane & 31;

  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin % p.tiles_m, tn = lin / p.tiles_m;
  const int z = blockIdx.z;
  const unsigned short* Ax = p.Ax + z * p.sAx;
  const float* B = p.B + z * p.sB;
  const float* B2 = p.B2 ? p.B2 + z * p.sB2 : nullptr;
  float* C = p.C + z * p.sC;
  const float* bias = p.bias ? p.bias + z * p.sBias : nullptr;
  const float* addend = p.addend ? p.addend + z * p.sD : nullptr;
  const int M = p.M, N = p.N, K = p.K, ldb = p.ldb, ldc = p.ldc, ldax = p.ldax;
  const int64_t sAxp = p.sAxp;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    for (int r = tid; r < BM; r += NTHR) bias_s[r] = bias[min(m0 + r, M - 1)];
  }

  uint4 ra[A_LD];
  float4 rb[BPL ? 1 : B_LD];
  bchunk_t rbp[BPL ? BPQ : 1];
  const unsigned short* Bx = BPL ? p.Bx + z * p.sB : nullptr;
  const int Kc = K - 1, Nc = N - 1;
  auto load_A = [&](int kt) {
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int c = tid + NTHR * q;
      const int pl = c / (2 * BM), rem = c % (2 * BM);
      const int m = rem >> 1, h = rem & 1;
      ra[q] = *reinterpret_cast<const uint4*>(Ax + pl * sAxp + (int64_t)(m0 + m) * ldax +
                                              kt * BK + 8 * h);
    }
  };
  auto store_A = [&](int buf) {
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int c = tid + NTHR * q;
      const int pl = c / (2 * BM), rem = c % (2 * BM);
      const int m = rem >> 1, h = rem & 1;
      *reinterpret_cast<uint4*>(As + buf * A_STAGE + pl * A_PLANE + m * BK +
                                8 * (h ^ ((m >> 3) & 1))) = ra[q];
    }
  };
  auto load_B = [&](int kt) {
    if constexpr (BPL) {
#pragma unroll
      for (int q = 0; q < BPQ; ++q) {
        const int c = tid + NTHR * q;
        const int pl = c / (BK * BN / BCH), rem = c % (BK * BN / BCH);
        const int kr = min(kt * BK + rem / (BN / BCH), Kc);
        const int col = min(n0 + BCH * (rem % (BN / BCH)), Nc & ~(BCH - 1));
        rbp[q] = *reinterpret_cast<const bchunk_t*>(Bx + pl * p.sBxp + (int64_t)kr * ldb + col);
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int f = tid + NTHR * q;
      const int kr = min(kt * BK + f / (BN / 4), Kc);
      const int col = n0 + 4 * (f % (BN / 4));
      const float* src = (B2 && kr >= p.kb2) ? B2 + (int64_t)(kr - p.kb2) * p.ldb2
                                             : B + (int64_t)kr * ldb;
      if constexpr (VEC) {
        rb[q] = *reinterpret_cast<const float4*>(src + min(col, Nc & ~3));
      } else {
        rb[q] = make_float4(src[min(col, Nc)], src[min(col + 1, Nc)], src[min(col + 2, Nc)],
                            src[min(col + 3, Nc)]);
      }
    }
  };
  auto store_B = [&](int buf, int kt) {
    if constexpr (BPL) {
#pragma unroll
      for (int q = 0; q < BPQ; ++q) {
        const int c = tid + NTHR * q;
        const int pl = c / (BK * BN / BCH), rem = c % (BK * BN / BCH);
        const int kr = rem / (BN / BCH), cl = BCH * (rem % (BN / BCH));
        bchunk_t v = rbp[q];
        const bool kok = kt * BK + kr < K;
        if (!kok || n0 + cl + BCH > N) {  // K tail / ragged N: zero what is out of range
          unsigned short e[BCH];
          __builtin_memcpy(e, &v, sizeof(v));
          // the load was clamped to the last aligned chunk: re-read exact elements
          const int kr_g = min(kt * BK + kr, Kc);
          for (int t = 0; t < BCH; ++t) {
            const int cg = n0 + cl + t;
            e[t] = (kok && cg < N) ? Bx[pl * p.sBxp + (int64_t)kr_g * ldb + cg] : 0;
          }
          __builtin_memcpy(&v, e, sizeof(v));
        }
        *reinterpret_cast<bchunk_t*>(Bs + buf * B_STAGE + pl * B_PLANE + kr * B_ROW + cl) = v;
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int f = tid + NTHR * q;
      const int kr = f / (BN / 4), c4 = 4 * (f % (BN / 4));
      const bool kok = kt * BK + kr < K;
      const int cg = n0 + c4;
      float4 v = rb[q];
      v.x = (kok && cg + 0 < N) ? v.x : 0.f;
      v.y = (kok && cg + 1 < N) ? v.y : 0.f;
      v.z = (kok && cg + 2 < N) ? v.z : 0.f;
      v.w = (kok && cg + 3 < N) ? v.w : 0.f;
      if constexpr (NP == 2) {  // the B row's power-of-two scale (|scaled| < 2^14)
        const float bs = kok ? p.x3_bscale[z * K + kt * BK + kr] : 0.f;
        v.x *= bs; v.y *= bs; v.z *= bs; v.w *= bs;
      }
      uint32_t ta[NP], tb[NP];
      X6Eng<NP>::split(v.x, v.y, ta);
      X6Eng<NP>::split(v.z, v.w, tb);
      unsigned short* dst = Bs + buf * B_STAGE + kr * B_ROW + c4;
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        *reinterpret_cast<uint2*>(dst + pl * B_PLANE) = make_uint2(ta[pl], tb[pl]);
    }
  };

  floatx16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-lane fragment addresses (bf16 element offsets within one stage)
  int a_off[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * WM + i * 32 + l32;
    a_off[i] = row * BK + 8 * (half ^ ((row >> 3) & 1));
  }
  const int li = lane & 15, g16 = (lane >> 4) & 1;
  const int b_off = (8 * half + (li >> 2)) * B_ROW + wn * WN + 16 * g16 + 4 * (li & 3);

  auto mfma_tile = [&](int buf) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const unsigned short* as = As + buf * A_STAGE;
    const unsigned short* bs = Bs + buf * B_STAGE;
    Frag a[MT][NP];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        a[i][pl] = *reinterpret_cast<const Frag*>(as + pl * A_PLANE + a_off[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      Frag b[NP];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl) {
        const unsigned short* q = bs + pl * B_PLANE + b_off + j * 32;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)q));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)(q + 4 * B_ROW)));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        b[pl] = __builtin_bit_cast(Frag, v);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i][j] = X6Eng<NP>::prod(a[i], b, acc[i][j]);
    }
  };

  if (nk > 0) {
    load_A(0);
    load_B(0);
    store_A(0);
    store_B(0, 0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      load_A(kt + 1);
      load_B(kt + 1);
    }
    mfma_tile(cur);
    if (kt + 1 < nk) {
      store_A(cur ^ 1);
      store_B(cur ^ 1, kt + 1);
    }
    __syncthreads();
  }
  if constexpr (NP == 2) {  // undo the A image's row scales (32x32 C layout)
    const float* rm = p.x3_rowmul + (int64_t)z * p.x3_ldrm + m0;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float f = rm[wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j][r] *= f;
      }
  }
  gemm_epilogue<BM, BN, EPI, WGM, WGN>(p, acc, reinterpret_cast<float*>(lds_raw), bias_s, C, addend, M, N,
                             ldc, m0, n0, 0);
}

// ---- host ---------------------------------------------------------------------

bool gemm_use_x6() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_GEMM");
    return !(e && std::string(e) == "f32");
  }();
  return on;
}

size_t gemm_dense_workspace(int M, int K, int batch_a) {
  return gemm_use_x6() ? gemm_x6_workspace(M, K, batch_a) : 0;
}

// 256x256 (8 waves) when the grid still fills the chip twice over, else 128x128;
// M <= 128 always takes 128x128 (a 256-row tile would pad the MFMA work: the
// decoder's 256 -> 73 fc2 runs 0.61-0.66 ms on 128x128 vs 0.93 ms on 256x256).
// MSFNO_X6_TILE=<GemmTile id> overrides for experiments
static GemmTile x6_tile(int M, int N, int batch) {
  static const int forced = [] {
    const char* e = getenv("MSFNO_X6_TILE");
    return e ? atoi(e) : -1;
  }();
  if (forced >= 0 && forced <= TILE_256x256) return (GemmTile)forced;
  if (M <= 128) return TILE_128x128;
  const int64_t big = cdiv(M, 256) * cdiv(N, 256) * (int64_t)batch;
  return big >= 512 ? TILE_256x256 : TILE_128x128;
}

size_t gemm_x6_workspace(int M, int K, int batch) {
  // k padded to 32: the same buffers also hold gemm_x6p's 32-deep x6q A image
  const int64_t Mp = round_up(M, 256), Kp = round_up(K, 32);
  return (size_t)round_up(3 * Mp * Kp * 2 * (int64_t)batch, 256);
}

template <int BM, int BN, int WGM, int WGN, int EPI>
static void launch_x6_e(const GemmParams& p, dim3 grid, hipStream_t s) {
  if (p.Bx)
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WGM, WGN, true, EPI, true>), grid,
                       dim3(64 * WGM * WGN), 0, s, p);
  else if (p.vecB)
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WGM, WGN, true, EPI, false>), grid,
                       dim3(64 * WGM * WGN), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WGM, WGN, false, EPI, false>), grid,
                       dim3(64 * WGM * WGN), 0, s, p);
}

template <int BM, int BN, int WGM, int WGN>
static int launch_x6(const GemmParams& p, dim3 grid, hipStream_t s) {
  const int code = (p.bias ? EPI_BIAS : 0) | (p.addend ? EPI_ADD : 0) | (p.act == 1 ? EPI_GELU : 0) |
                   (p.relu_period ? EPI_RELU : 0) | (p.Cx ? EPI_PLANES : 0);
  if (p.act == 2 || p.rowscale) {
    set_error("gemm_x6: unsupported epilogue");
    return MSFNO_EUNSUPPORTED;
  }
  switch (code) {
    case 0: launch_x6_e<BM, BN, WGM, WGN, 0>(p, grid, s); break;
    case EPI_RELU: launch_x6_e<BM, BN, WGM, WGN, EPI_RELU>(p, grid, s); break;
    case EPI_BIAS: launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS>(p, grid, s); break;
    case EPI_BIAS | EPI_GELU: launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS | EPI_GELU>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD: launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS | EPI_ADD>(p, grid, s); break;
    case EPI_ADD: launch_x6_e<BM, BN, WGM, WGN, EPI_ADD>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD | EPI_GELU:
      launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS | EPI_ADD | EPI_GELU>(p, grid, s); break;
    case EPI_PLANES: launch_x6_e<BM, BN, WGM, WGN, EPI_PLANES>(p, grid, s); break;
    case EPI_RELU | EPI_PLANES: launch_x6_e<BM, BN, WGM, WGN, EPI_RELU | EPI_PLANES>(p, grid, s); break;
    case EPI_BIAS | EPI_GELU | EPI_PLANES:
      launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS | EPI_GELU | EPI_PLANES>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD | EPI_GELU | EPI_PLANES:
      launch_x6_e<BM, BN, WGM, WGN, EPI_BIAS | EPI_ADD | EPI_GELU | EPI_PLANES>(p, grid, s); break;
    default:
      set_error("gemm_x6: unsupported epilogue combination");
      return MSFNO_EUNSUPPORTED;
  }
  return MSFNO_OK;
}

int launch_split_a(const float* A, unsigned short* Ax, int M, int K, int lda, int64_t sA,
                   int batch, hipStream_t s) {
  const int Mp = (int)round_up(M, 256), Kp = (int)round_up(K, 16);
  const int64_t pairs = (int64_t)Mp * Kp / 2;
  const int blocks = (int)std::min<int64_t>(cdiv(pairs, 256), 1024);
  hipLaunchKernelGGL(split_a_kernel, dim3(blocks, batch), dim3(256), 0, s, A, Ax, M, K, lda, sA,
                     Mp, Kp);
  return launch_check("split_a");
}

int gemm_x6(GemmTile tile, const float* A, const float* B, float* C, int M, int N, int K, int lda,
            int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int batch, const GemmEpi& epi,
            void* ws, size_t ws_bytes, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(ws && ws_bytes >= gemm_x6_workspace(M, K, sA == 0 ? 1 : batch), MSFNO_EINVAL,
                "gemm_x6: workspace too small");
  MSFNO_REQUIRE(batch <= 65535, MSFNO_EINVAL, "gemm_x6: batch too large");
  unsigned short* Ax = static_cast<unsigned short*>(ws);
  const int abatch = sA == 0 ? 1 : batch;  // one A for every batch entry: split once
  MSFNO_TRY(launch_split_a(A, Ax, M, K, lda, sA, abatch, s));
  const int Mp = (int)round_up(M, 256), Kp = (int)round_up(K, 16);
  GemmParams p{};
  p.B = B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.ldb = ldb; p.ldc = ldc;
  p.sB = sB; p.sC = sC;
  p.bias = epi.bias; p.addend = epi.addend; p.sBias = epi.sBias; p.sD = epi.sD;
  p.ldd = epi.ldd; p.act = epi.act; p.relu_period = epi.relu_period; p.relu_rows = epi.relu_rows;
  p.rowscale = epi.rowscale;
  p.Ax = Ax; p.sAxp = (int64_t)Mp * Kp; p.sAx = sA == 0 ? 0 : 3 * p.sAxp; p.ldax = Kp;
  p.vecB = (ldb % 4 == 0) && (sB % 4 == 0) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  p.B2 = epi.b2; p.kb2 = epi.b2_k; p.ldb2 = epi.b2_ld; p.sB2 = epi.b2_stride;
  if (p.B2) {
    MSFNO_REQUIRE(!epi.b_planes && epi.b2_k > 0 && epi.b2_k < K, MSFNO_EINVAL,
                  "gemm_x6: bad K concatenation");
    p.vecB = p.vecB && (p.ldb2 % 4 == 0) && (p.sB2 % 4 == 0) &&
             ((reinterpret_cast<uintptr_t>(p.B2) & 15) == 0);
  }
  p.Bx = epi.b_planes; p.sBxp = epi.b_plane_stride;
  p.Cx = epi.c_planes; p.sCxp = epi.c_plane_stride;
  p.cx16 = cx16_enabled() && p.Cx && ldc % 8 == 0 && sC % 8 == 0 && p.sCxp % 8 == 0 &&
           (reinterpret_cast<uintptr_t>(p.Cx) & 15) == 0;
  if (p.Bx)
    MSFNO_REQUIRE(ldb % 8 == 0 && sB % 8 == 0 && p.sBxp % 8 == 0 &&
                      (reinterpret_cast<uintptr_t>(p.Bx) & 15) == 0,
                  MSFNO_EINVAL, "gemm_x6: B planes need ld, strides % 8 == 0 and 16-B alignment");
  if (p.Cx)
    MSFNO_REQUIRE(ldc % 4 == 0 && sC % 4 == 0 && p.sCxp % 4 == 0 &&
                      (reinterpret_cast<uintptr_t>(p.Cx) & 7) == 0,
                  MSFNO_EINVAL, "gemm_x6: C planes need ld, strides % 4 == 0 and 8-B alignment");
  p.vecC = (ldc % 4 == 0) && (sC % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
           (!epi.addend || ((epi.ldd % 4 == 0) && (epi.sD % 4 == 0) &&
                            ((reinterpret_cast<uintptr_t>(epi.addend) & 15) == 0)));
  // tile -> (BM, BN, wave grid): 128x128 4 waves, 256x128 8 waves (4x2),
  // 128x256 4 waves, 256x256 8 waves (4x2)
  int bm, bn;
  gemm_tile_dims(tile, &bm, &bn);
  if (tile != TILE_256x128 && tile != TILE_128x256 && tile != TILE_256x256) {
    tile = TILE_128x128; bm = bn = 128;
  }
  p.tiles_m = (int)cdiv(M, bm);
  p.tiles_n = (int)cdiv(N, bn);
  const dim3 grid(p.tiles_m * p.tiles_n, 1, batch);
  int rc;
  switch (tile) {
    case TILE_256x128: rc = launch_x6<256, 128, 4, 2>(p, grid, s); break;
    case TILE_128x256: rc = launch_x6<128, 256, 2, 2>(p, grid, s); break;
    case TILE_256x256: rc = launch_x6<256, 256, 4, 2>(p, grid, s); break;
    default: rc = launch_x6<128, 128, 2, 2>(p, grid, s); break;
  }
  if (rc != MSFNO_OK) return rc;
  return launch_check("gemm_x6");
}

// ---- x3h engine (NP = 2): the inner-skip GEMM ----------------------------------

// A image per batch z: W (M x K, ld lda) · diag(1 / bscale[z]) with row m scaled by
// tau = 2^(15 - e) (the row's max = f 2^e, f in [0.5, 1): scaled entries < 2^15), split
// into two fp16 planes [z][2][Mp][Kp]; rowmul[z * Mp + m] = 1 / tau.  One workgroup
// per (row, batch)
__global__ __launch_bounds__(256) void x3_image_kernel(const float* __restrict__ W, int M, int K,
                                                       int lda, const float* __restrict__ bscale,
                                                       unsigned short* __restrict__ img,
                                                       float* __restrict__ rowmul, int Mp, int Kp) {
  __shared__ float red[256];
  const int m = blockIdx.x, z = blockIdx.y;
  const float* w = W + (int64_t)min(m, M - 1) * lda;
  const float* bs = bscale + (int64_t)z * K;
  float mx = 0.f;
  if (m < M)
    for (int k = threadIdx.x; k < K; k += 256) mx = fmaxf(mx, fabsf(w[k] / bs[k]));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  mx = red[0];
  float tau = 1.f;
  if (mx > 0.f && isfinite(mx)) {
    int e;
    frexpf(mx, &e);
    tau = ldexpf(1.f, 15 - e);
  }
  const int64_t plane = (int64_t)Mp * Kp;
  uint32_t* o = reinterpret_cast<uint32_t*>(img + (int64_t)z * 2 * plane + (int64_t)m * Kp);
  for (int kk = threadIdx.x; kk < Kp / 2; kk += 256) {
    const int k = 2 * kk;
    const float v0 = (m < M && k < K) ? w[k] / bs[k] * tau : 0.f;
    const float v1 = (m < M && k + 1 < K) ? w[k + 1] / bs[k + 1] * tau : 0.f;
    uint32_t t[2];
    X6Eng<2>::split(v0, v1, t);
    o[kk] = t[0];
    o[plane / 2 + kk] = t[1];
  }
  if (threadIdx.x == 0) rowmul[(int64_t)z * Mp + m] = 1.f / tau;
}

size_t gemm_x3_workspace(int M, int K, int batch) {
  const int64_t Mp = round_up(M, 256), Kp = round_up(K, 16);
  return (size_t)(round_up(2 * Mp * Kp * 2 * (int64_t)batch, 256) + round_up(Mp * 4 * (int64_t)batch, 256));
}

template <int BM, int BN, int WGM, int WGN, int EPI>
static void launch_x3_e(const GemmParams& p, dim3 grid, hipStream_t s) {
  if (p.vecB)
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WGM, WGN, true, EPI, false, 2>), grid,
                       dim3(64 * WGM * WGN), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_x6_kernel<BM, BN, WGM, WGN, false, EPI, false, 2>), grid,
                       dim3(64 * WGM * WGN), 0, s, p);
}

// C[z] = A · (B[z] rows scaled by bscale[z]) / bscale-corrected A = A · B[z] (+ bias),
// fp32 in and out, on the x3h engine.  bscale[z * K + k] are powers of two under which
// every element of B row k has magnitude < 2^14 (launch_chan_affine's xscale); A is
// re-imaged per batch (x3_image_kernel) into the workspace
int gemm_x3(const float* A, int lda, const float* bscale, const float* B, float* C, int M, int N,
            int K, int ldb, int ldc, int64_t sB, int64_t sC, int batch, const GemmEpi& epi,
            void* ws, size_t ws_bytes, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(ws && ws_bytes >= gemm_x3_workspace(M, K, batch), MSFNO_EINVAL,
                "gemm_x3: workspace too small");
  MSFNO_REQUIRE(bscale && batch <= 65535, MSFNO_EINVAL, "gemm_x3: bad arguments");
  MSFNO_REQUIRE(!epi.addend && !epi.act && !epi.relu_period && !epi.rowscale && !epi.b_planes &&
                    !epi.c_planes && !epi.b2,
                MSFNO_EUNSUPPORTED, "gemm_x3: bias-only epilogue");
  const int Mp = (int)round_up(M, 256), Kp = (int)round_up(K, 16);
  unsigned short* Ax = static_cast<unsigned short*>(ws);
  float* rowmul = reinterpret_cast<float*>(static_cast<char*>(ws) +
                                           round_up(2LL * Mp * Kp * 2 * batch, 256));
  hipLaunchKernelGGL(x3_image_kernel, dim3(Mp, batch), dim3(256), 0, s, A, M, K, lda, bscale, Ax,
                     rowmul, Mp, Kp);
  MSFNO_TRY(launch_check("x3_image"));
  GemmParams p{};
  p.B = B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.ldb = ldb; p.ldc = ldc;
  p.sB = sB; p.sC = sC;
  p.bias = epi.bias; p.sBias = epi.sBias;
  p.Ax = Ax; p.sAxp = (int64_t)Mp * Kp; p.sAx = 2 * p.sAxp; p.ldax = Kp;
  p.vecB = (ldb % 4 == 0) && (sB % 4 == 0) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  p.vecC = (ldc % 4 == 0) && (sC % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
  p.x3_bscale = bscale;
  p.x3_rowmul = rowmul;
  p.x3_ldrm = Mp;
  // tiles as x6_tile (MSFNO_X6_TILE overrides: 6 = 256x256, 4 = 256x128, 0 = 128x128)
  const GemmTile tile = x6_tile(M, N, batch);
  const int bm = (tile == TILE_256x256 || tile == TILE_256x128) ? 256 : 128;
  const int bn = tile == TILE_256x256 ? 256 : 128;
  p.tiles_m = (int)cdiv(M, bm);
  p.tiles_n = (int)cdiv(N, bn);
  const dim3 grid(p.tiles_m * p.tiles_n, 1, batch);
  if (tile == TILE_256x256) {
    if (p.bias) launch_x3_e<256, 256, 4, 2, EPI_BIAS>(p, grid, s);
    else launch_x3_e<256, 256, 4, 2, 0>(p, grid, s);
  } else if (tile == TILE_256x128) {
    if (p.bias) launch_x3_e<256, 128, 4, 2, EPI_BIAS>(p, grid, s);
    else launch_x3_e<256, 128, 4, 2, 0>(p, grid, s);
  } else {
    if (p.bias) launch_x3_e<128, 128, 2, 2, EPI_BIAS>(p, grid, s);
    else launch_x3_e<128, 128, 2, 2, 0>(p, grid, s);
  }
  return launch_check("gemm_x3");
}

int gemm_dense(GemmRole role, GemmTile f32_tile, const float* A, const float* B, float* C, int M,
               int N, int K, int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC,
               int batch, const GemmEpi& epi, void* ws, size_t ws_bytes, hipStream_t s) {
  MSFNO_REQUIRE(!(epi.b_planes || epi.c_planes) || (gemm_use_x6() && ws), MSFNO_EINVAL,
                "gemm_dense: plane operands need the x6 engine");
  if (gemm_use_x6() && ws && epi.act != 2 && !epi.rowscale)
    return gemm_x6(x6_tile(M, N, batch), A, B, C, M, N, K, lda, ldb, ldc, sA, sB, sC, batch, epi,
                   ws, ws_bytes, s);
  return gemm_uniform(role_tile(role, f32_tile), A, B, C, M, N, K, lda, ldb, ldc, sA, sB, sC,
                      batch, epi, s);
}

}  // namespace msfno
