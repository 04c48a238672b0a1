// Legendre contractions of the SHT on the "x3h" engine, for gfx950.
//
// The per-(m, parity) problems of the forward and inverse Legendre transform
// (the reference's einsum in RealSHT / InverseRealSHT, driven from
// sfnonet.py:537-555) as one descriptor launch, C[R x N] = A[R x K] · B[K x N]:
//   forward  A = the latitude slab of one m (rows r = (b, re/im, c), K latitudes),
//            B = the table (K latitudes x N degrees l), C = the coefficients S;
//   inverse  A = S (K degrees), B = the table (K degrees x N latitudes), C = the slab.
// fp32 is emulated by two fp16 terms per operand (v = v0 + v1, v0 = fp16(v),
// v1 = fp16(v - v0)) and three fp16 MFMAs per product (a1·b0 + a0·b1 + a0·b0,
// fp32 accumulation; Ootomo & Yokota 2022, as gemm_x6c.hip's x3h chain).  fp16's
// range is kept by exact power-of-two scales: every row of A by sigma_r,t per
// k-tile t (the row's max over the tile's 32 k maps into [2^14, 2^15), found while
// the tile is staged), every column of B by tau_n (its max maps into [2^14, 2^15):
// in the table image, built once per table load).  An entry below 2^-24 of its row's
// (column's) maximum loses its low term: an error under the fp32 rounding of the dot
// product it enters.  Each k-tile's products are scaled back by 1 / sigma_r,t as
// they are added to the accumulator, the epilogue by 1 / tau_n.
//
// Tile 128 (rows) x BN (n: 64 by default, 128, 192) x 32 (k), 4 waves as 2 x 2, each
// 64 x BN/2 as 32x32x16 MFMA tiles; both operands k-contiguous in LDS ([plane][k16][row][16], the two
// 16-B halves of a row swapped when (row >> 3) & 1, gemm_x6.hip's A layout), two
// stages.  The table image is B^T: [plane][n][Kp] per problem (Kp = K rounded up
// to 32, zero padded), so its staging is plain 16-B copies.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "dma.h"
#include "gemm_common.h"

namespace msfno {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void x3_split(float a, float b, uint32_t& t0, uint32_t& t1) {
  const f2v v = {a, b};
  const h2v h0 = __builtin_convertvector(v, h2v);
  const f2v r = v - __builtin_convertvector(h0, f2v);
  const h2v h1 = __builtin_convertvector(r, h2v);
  t0 = __builtin_bit_cast(uint32_t, h0);
  t1 = __builtin_bit_cast(uint32_t, h1);
}

// 2^(s - e) for m = f 2^e, f in [0.5, 1); 1 for m = 0 or non-finite; exponent clamped
__device__ __forceinline__ float pow2_scale(float m, int s) {
  if (!(m > 0.f) || !isfinite(m)) return 1.f;
  int e;
  frexpf(m, &e);
  return ldexpf(1.f, min(max(s - e, -100), 100));
}

// A column of a segmented (band exchange layout) operand: k -> k + block * (stride - w)
__device__ __forceinline__ int64_t seg_k(int k, int w, int64_t stride) {
  return w ? k + (int64_t)(k / w) * (stride - w) : k;
}

// One workgroup per problem: per column n the scale tau_n, then the image
// [plane][n][Kp] of B^T · tau (zero padded to Kp) and 1 / tau_n.
__global__ __launch_bounds__(256) void x3d_image_kernel(const float* __restrict__ table,
                                                        const GemmDesc* __restrict__ descs,
                                                        unsigned short* __restrict__ img,
                                                        float* __restrict__ invs) {
  const GemmDesc d = descs[blockIdx.x];
  const float* B = table + d.offB;
  const int K = d.K, N = d.N, ldb = d.ldb;
  const int Kp = (max(K, 1) + X3D_BK - 1) / X3D_BK * X3D_BK;
  unsigned short* o = img + d.offBx;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    float m = 0.f;
    for (int k = 0; k < K; ++k) m = fmaxf(m, fabsf(B[(int64_t)k * ldb + n]));
    const float tau = pow2_scale(m, 15);
    invs[d.offBs + n] = 1.f / tau;
    uint32_t* o0 = reinterpret_cast<uint32_t*>(o + (int64_t)n * Kp);
    uint32_t* o1 = reinterpret_cast<uint32_t*>(o + ((int64_t)N + n) * Kp);
    for (int k = 0; k < Kp; k += 2) {
      const float v0 = k < K ? B[(int64_t)k * ldb + n] * tau : 0.f;
      const float v1 = k + 1 < K ? B[(int64_t)(k + 1) * ldb + n] * tau : 0.f;
      uint32_t t0, t1;
      x3_split(v0, v1, t0, t1);
      o0[k >> 1] = t0;
      o1[k >> 1] = t1;
    }
  }
}

struct X3DParams {
  const float* A;
  const unsigned short* img;
  const float* invs;
  float* C;
  const GemmDesc* descs;
  const int* tile_desc;  // tile -> descriptor index (or null: binary search)
  int ndesc;
  int segA_w, segC_w;
  int64_t segA_stride, segC_stride;
  int vecC;
};

struct X3FParams {
  const unsigned short* Ap;  // slab planes, interleaved per 8 k (2 x the fp32 offsets)
  const float* isr;          // 1 / sigma per slab row
  const unsigned short* img;
  const float* invs;
  float* C;
  const GemmDesc* descs;
  const int* tile_desc;
  // segmented A (latitude-band plans: the all-to-all receive buffer, one block per
  // source rank): k -> k + (k / segA_w) (segA_stride - segA_w); segA_w % 8 == 0
  int segA_w;
  int64_t segA_stride;
};

constexpr int BM = X3D_BM, BK = X3D_BK;
constexpr int KS = BK / 16;                 // 32x32x16 k-steps per k-tile
constexpr int A_PL = KS * BM * 16;          // fp16 per A plane in a stage
constexpr int WGM = 2, WGN = 2, WM = BM / WGM, MT = WM / 32;

__device__ __forceinline__ int swz(int row) { return (row >> 3) & 1; }

// BN: 64 or 192 columns per tile (192: one tile spans a whole problem's N <= 184 — A
// is read once, not once per 64 columns); PF: k-tiles in flight in registers (1, 2)
// DBG (diagnostic timing builds, wrong results; MSFNO_LEG_X3_DBG): 1 no MFMAs, 4 no
// main-loop loads (stale registers)
//
// Row scales per k-tile: the 8 threads that stage one row's 32 k of a k-tile reduce
// their max by lane shuffles and split the row under sigma = 2^(15 - e) of it; the
// k-tile's products go to a zeroed accumulator that is added to the running one times
// 1 / sigma (per row, from LDS) — no separate pass over A (a whole-K row-max pass
// per workgroup cost 0.13 / 0.18 ms of the forward / inverse 0.39 / 0.57).
template <int BN, int PF, int DBG = 0>
__global__ __launch_bounds__(256) void legendre_x3_kernel(X3DParams p) {
  constexpr int B_PL = KS * BN * 16;
  constexpr int STAGE = 2 * A_PL + 2 * B_PL;  // fp16 per stage
  constexpr int WN = BN / WGN, NT = WN / 32;
  constexpr int NB = 2 * BN * BK / 8 / 256;  // 16-B B pieces per thread and k-tile
  constexpr int EPI_FLOATS = 32 * WGM * (BN + 8);
  constexpr int LDS_BYTES = (2 * STAGE * 2 > EPI_FLOATS * 4) ? 2 * STAGE * 2 : EPI_FLOATS * 4;
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];
  __shared__ __attribute__((aligned(16))) float isg_s[2][BM];  // 1 / sigma per stage and row
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int half = lane >> 5, l32 = lane & 31;

  // ---- tile -> problem ----------------------------------------------------------------
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  int lo = 0, hi = p.ndesc - 1;
  if (p.tile_desc) {
    lo = p.tile_desc[lin];
  } else {
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (p.descs[mid].tile_start <= lin) lo = mid; else hi = mid - 1;
    }
  }
  const GemmDesc d = p.descs[lo];
  const int local = lin - d.tile_start;
  const int tm = local % d.tiles_m, tn = local / d.tiles_m;
  const int M = d.M, N = d.N, K = d.K, lda = d.lda;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = p.A + d.offA;
  const int Kp = (max(K, 1) + BK - 1) / BK * BK;
  const unsigned short* Bimg = p.img + d.offBx;
  const int nk = (K + BK - 1) / BK;

  // ---- staging: A fp32 -> two fp16 planes (row-scaled per k-tile); B image copies -----
  // A: 128 rows x 32 k = 1024 float4, 4 per thread (thread -> row idx / 8, k 4 (idx % 8):
  // the 8 lanes of a row are adjacent); (rows padded to 4 floats and segments to 16: a
  // float4 at k % 4 == 0 stays in its row and block; elements past K are masked)
  float4 ra[PF][4];
  uint4 rb[PF][NB];
  const int Kc = K > 0 ? K - 1 : 0;
  auto load = [&](int kt, auto buf_c) {
    constexpr int BUF = decltype(buf_c)::value;
    if constexpr ((DBG & 4) != 0) {
      if (kt > 1) return;
    }
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;
      const int row = min(m0 + (idx >> 3), M - 1);
      const int k = k0 + 4 * (idx & 7);
      const float* a = A + (int64_t)row * lda;
      ra[BUF][q] = *reinterpret_cast<const float4*>(a + seg_k(min(k, Kc & ~3), p.segA_w, p.segA_stride));
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int idx = tid + 256 * q;
      const int pl = idx / (4 * BN), n = (idx >> 2) % BN, c = idx & 3;
      const int ng = min(n0 + n, N - 1);
      rb[BUF][q] = *reinterpret_cast<const uint4*>(Bimg + ((int64_t)pl * N + ng) * Kp + k0 + 8 * c);
    }
  };
  auto store = [&](int st, int kt, auto buf_c) {
    constexpr int BUF = decltype(buf_c)::value;
    unsigned short* base = ring + st * STAGE;
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;
      const int r = idx >> 3, kk = 4 * (idx & 7);  // k within the tile: 0..28
      const bool rok = m0 + r < M;
      float v[4] = {ra[BUF][q].x, ra[BUF][q].y, ra[BUF][q].z, ra[BUF][q].w};
      float mx = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (rok && k0 + kk + e < K) ? v[e] : 0.f;
        mx = fmaxf(mx, fabsf(v[e]));
      }
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      mx = fmaxf(mx, __shfl_xor(mx, 4));
      const float sg = pow2_scale(mx, 15);
      if ((idx & 7) == 0) isg_s[st][r] = 1.f / sg;
      uint32_t a0, a1, b0, b1;
      x3_split(v[0] * sg, v[1] * sg, a0, a1);
      x3_split(v[2] * sg, v[3] * sg, b0, b1);
      const int ks = kk >> 4, c = (kk >> 3) & 1, w = kk & 7;
      unsigned short* dst = base + (ks * BM + r) * 16 + 8 * (c ^ swz(r)) + w;
      *reinterpret_cast<uint2*>(dst) = make_uint2(a0, b0);
      *reinterpret_cast<uint2*>(dst + A_PL) = make_uint2(a1, b1);
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int idx = tid + 256 * q;
      const int pl = idx / (4 * BN), n = (idx >> 2) % BN, c = idx & 3;
      const int ks = c >> 1, hc = c & 1;
      uint4 v = rb[BUF][q];
      if (n0 + n >= N) v = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(base + 2 * A_PL + pl * B_PL + (ks * BN + n) * 16 + 8 * (hc ^ swz(n))) = v;
    }
  };

  floatx16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto mfma_tile = [&](int st) {
    const unsigned short* base = ring + st * STAGE;
    floatx16 t[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      h8 a[MT][2], b[NT][2];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int row = wm * WM + i * 32 + l32;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          a[i][pl] = *reinterpret_cast<const h8*>(base + pl * A_PL + (ks * BM + row) * 16 +
                                                  8 * (half ^ swz(row)));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = wn * WN + j * 32 + l32;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          b[j][pl] = *reinterpret_cast<const h8*>(base + 2 * A_PL + pl * B_PL + (ks * BN + n) * 16 +
                                                  8 * (half ^ swz(n)));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          if constexpr ((DBG & 1) != 0) {
            t[i][j][0] += (float)a[i][0][0] + (float)a[i][1][0] + (float)b[j][0][0] + (float)b[j][1][0];
            continue;
          }
          t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][1], b[j][0], t[i][j], 0, 0, 0);
          t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], b[j][1], t[i][j], 0, 0, 0);
          t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], b[j][0], t[i][j], 0, 0, 0);
        }
    }
    // acc += t / sigma (rows (r & 3) + 8 (r >> 2) + 4 half of the 32-row block)
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 is = *reinterpret_cast<const float4*>(&isg_s[st][wm * WM + i * 32 + 8 * g4 + 4 * half]);
        const float isv[4] = {is.x, is.y, is.z, is.w};
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * g4 + e] = fmaf(t[i][j][4 * g4 + e], isv[e], acc[i][j][4 * g4 + e]);
      }
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (nk > 0) load(0, I0{});
  if constexpr (PF == 2) {
    if (nk > 1) load(1, I1{});
  }
  if (nk > 0) store(0, 0, I0{});
  __syncthreads();
  if constexpr (PF == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load(kt + 1, I0{});
      mfma_tile(kt & 1);
      if (kt + 1 < nk) store((kt + 1) & 1, kt + 1, I0{});
      __syncthreads();
    }
  } else {
    // register buffer b holds k-tiles of parity b: tile kt + 1 was loaded an iteration
    // ago, tile kt + 2 goes into the buffer tile kt left
    auto iter = [&](int kt, auto buf_c) {
      constexpr int BUF = decltype(buf_c)::value;
      using Other = std::integral_constant<int, BUF ^ 1>;
      if (kt + 2 < nk) load(kt + 2, buf_c);
      mfma_tile(BUF);
      if (kt + 1 < nk) store(BUF ^ 1, kt + 1, Other{});
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      iter(kt, I0{});
      if (kt + 1 < nk) iter(kt + 1, I1{});
    }
  }

  // ---- 1 / tau_n, then the shared fp32 epilogue ---------------------------------------
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const float it = p.invs[d.offBs + min(n0 + wn * WN + j * 32 + l32, N - 1)];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= it;
  }
  GemmParams q{};
  q.vecC = p.vecC;
  q.segC_w = p.segC_w;
  q.segC_stride = p.segC_stride;
  gemm_epilogue<BM, BN, 0, WGM, WGN>(q, acc, reinterpret_cast<float*>(lds_raw), nullptr,
                                     p.C + d.offC, nullptr, M, N, d.ldc, m0, n0, 0);
}

// ---- register-resident A (the inverse problems, K <= X3R_KMAX) -------------------------
// Inverse problems have a short K (the degrees of one parity, <= 181 at lmax 360) and
// a wide N (the latitudes): the tiled kernel above spends most of its time on per-tile
// prologues and epilogues (K = 3 k-tiles, 17 k tiles at config 2).  Here one workgroup
// owns 128 rows of one problem for ALL its columns: every wave loads its 32 rows x Kp
// of A once, splits them under one power-of-two scale per row (its max over the whole
// K into [2^14, 2^15)) and keeps both fp16 planes in registers (16 VGPRs per 32 k);
// the table image streams through a three-stage LDS ring by LDS-DMA in chunks of 32
// columns ([plane][ks][n 32][16], 16-B halves swapped by (n >> 3) & 1), one barrier per
// chunk; each chunk's 32 x 32 block per wave is scaled back (1 / sigma_row,
// 1 / tau_n) and stored straight from the accumulator (a row's 32 columns are 128
// contiguous bytes).  A and the output are touched once; the table once per 128 rows.
constexpr int X3R_NSTG = 3;
constexpr int X3R_STAGE = 2 * (X3R_KMAX / 16) * 1024;  // bytes per stage (max Kp)

// masked lanes store here, so every wave issues exactly 16 stores per chunk (the
// DMA waits count them)
__device__ float x3r_sink[256];

__device__ __forceinline__ int x3r_swz(int n) { return (n >> 3) & 1; }

template <int NK>
__device__ __forceinline__ void x3r_body(const X3DParams& p, const GemmDesc& d, int m0,
                                         unsigned char* ring, float* tau_s) {
  constexpr int STG = X3R_STAGE;  // bytes per stage
  constexpr int NST = X3R_NSTG;
  constexpr int KS = 2 * NK;       // 16-deep k-steps
  constexpr int KP = 32 * NK;      // padded K of the image
  constexpr int NI = KP / 32;      // DMA wave-instructions per wave and stage (= NK)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int M = d.M, N = d.N, K = d.K;
  const int nch = (N + 31) / 32;
  const unsigned short* Bimg = p.img + d.offBx;
  const uint32_t ring_lds = lds_addr(ring);

  // stage s <- columns 32 j .. +31 of the image; wave w issues pieces i = w + 4 q
  // (piece (pl, ks) is one 1-KB block of the stage)
  auto issue = [&](int j, int s) {
    const int n = lane >> 1, hc = (lane & 1) ^ x3r_swz(lane >> 1);
    const int ng = min(32 * j + n, N - 1);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int i = wave + 4 * q;
      const int pl = i / KS, ks = i % KS;
      const unsigned short* src = Bimg + ((int64_t)pl * N + ng) * KP + 16 * ks + 8 * hc;
      glds16(src, ring_lds + s * STG + i * 1024);
    }
  };
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (j < nch) issue(j, j);
  // 1 / tau_n of every column into LDS (no global load inside the chunk loop: hipcc
  // would wait for it with a vmcnt that also drains the DMA in flight)
  for (int n = tid; n < N; n += 256) tau_s[n] = p.invs[d.offBs + n];

  // A: this lane's row, k = 16 ks + 8 half .. + 7 for every ks; one scale per row
  const int row = m0 + 32 * wave + l32;
  const float* Ar = p.A + d.offA + (int64_t)min(row, M - 1) * d.lda;
  float4 av[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = 16 * ks + 8 * half;
    if (k < K) {
      av[ks][0] = *reinterpret_cast<const float4*>(Ar + k);
      av[ks][1] = *reinterpret_cast<const float4*>(Ar + k + 4);
    } else {
      av[ks][0] = av[ks][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float mx = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    float v[8] = {av[ks][0].x, av[ks][0].y, av[ks][0].z, av[ks][0].w,
                  av[ks][1].x, av[ks][1].y, av[ks][1].z, av[ks][1].w};
    const int k = 16 * ks + 8 * half;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = (row < M && k + e < K) ? v[e] : 0.f;
      mx = fmaxf(mx, fabsf(v[e]));
    }
    av[ks][0] = make_float4(v[0], v[1], v[2], v[3]);
    av[ks][1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  const float sg = pow2_scale(mx, 15);
  h8 a[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    uint32_t t0[4], t1[4];
    x3_split(av[ks][0].x * sg, av[ks][0].y * sg, t0[0], t1[0]);
    x3_split(av[ks][0].z * sg, av[ks][0].w * sg, t0[1], t1[1]);
    x3_split(av[ks][1].x * sg, av[ks][1].y * sg, t0[2], t1[2]);
    x3_split(av[ks][1].z * sg, av[ks][1].w * sg, t0[3], t1[3]);
    a[ks][0] = __builtin_bit_cast(h8, make_uint4(t0[0], t0[1], t0[2], t0[3]));
    a[ks][1] = __builtin_bit_cast(h8, make_uint4(t1[0], t1[1], t1[2], t1[3]));
  }
  // 1 / sigma of the 16 rows this lane's accumulator holds: (r & 3) + 8 (r >> 2) + 4 half
  float isv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) isv[r] = __shfl(1.f / sg, (r & 3) + 8 * (r >> 2) + 4 * half);
  constexpr int NSTORE = 16;  // store instructions per chunk

  const int rbase = m0 + 32 * wave + 4 * half;
  float* Cb = p.C + d.offC;
  for (int j = 0; j < nch; ++j) {
    const int s = j % NST;
    // chunk j's DMA (j >= NST - 1; the first NST - 1 were drained with A) was followed
    // by the stores of chunks j - NST + 1 .. j - 1 and the NI pieces of each chunk
    // j + 1 .. j + NST - 2 that exists (wait_vmcnt caps the count: waiting longer is safe)
    int after = (NST - 1) * NSTORE;
#pragma unroll
    for (int k = 1; k <= NST - 2; ++k) after += (j + k < nch) ? NI : 0;
    wait_vmcnt(after);
    __syncthreads();
    if (j + NST - 1 < nch) issue(j + NST - 1, (j + NST - 1) % NST);
    const unsigned char* st = ring + s * STG;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int off = ks * 1024 + l32 * 32 + 16 * (half ^ x3r_swz(l32));
      const h8 b0 = *reinterpret_cast<const h8*>(st + off);
      const h8 b1 = *reinterpret_cast<const h8*>(st + KS * 1024 + off);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks][1], b0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks][0], b1, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[ks][0], b0, acc, 0, 0, 0);
    }
    const int col = 32 * j + l32;
    const float it = tau_s[min(col, N - 1)];
    const int64_t cc = seg_k(col, p.segC_w, p.segC_stride);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = rbase + (r & 3) + 8 * (r >> 2);
      float* dst = (rr < M && col < N) ? Cb + (int64_t)rr * d.ldc + cc : x3r_sink + lane;
      *dst = acc[r] * isv[r] * it;
    }
  }
}

// K = 0 problems (an odd parity without degrees): the output block is zero
__device__ __forceinline__ void x3r_zero(const X3DParams& p, const GemmDesc& d, int m0) {
  float* Cb = p.C + d.offC;
  for (int e = threadIdx.x; e < X3D_BM * d.N; e += blockDim.x) {
    const int r = m0 + e / d.N, c = e % d.N;
    if (r < d.M) Cb[(int64_t)r * d.ldc + seg_k(c, p.segC_w, p.segC_stride)] = 0.f;
  }
}

__global__ __launch_bounds__(256) void legendre_x3r_kernel(X3DParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[X3R_NSTG * X3R_STAGE];
  __shared__ __attribute__((aligned(16))) float tau_s[X3R_NMAX + 32];
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const GemmDesc d = p.descs[p.tile_desc[lin]];
  const int m0 = (lin - d.tile_start) * X3D_BM;
  switch ((d.K + 31) / 32) {
    case 0: x3r_zero(p, d, m0); break;
    case 1: x3r_body<1>(p, d, m0, ring, tau_s); break;
    case 2: x3r_body<2>(p, d, m0, ring, tau_s); break;
    case 3: x3r_body<3>(p, d, m0, ring, tau_s); break;
    case 4: x3r_body<4>(p, d, m0, ring, tau_s); break;
    case 5: x3r_body<5>(p, d, m0, ring, tau_s); break;
    default: x3r_body<6>(p, d, m0, ring, tau_s); break;
  }
}

// ---- register-resident B (the forward problems, Kp <= X3F_KMAX) ------------------------
// Forward problems have a long K (the latitudes of one hemisphere fold, 361 at 721)
// and a narrow N (the degrees of one parity, <= 181).  One workgroup owns 64 columns
// of one problem and X3F_RB rows: every wave keeps its 16 table columns x Kp as both
// fp16 planes in registers (the 16x16x32 B operand: 8 VGPRs per 32 k), the slab rows
// arrive already split (launch_transpose_fwd_sym_h: two fp16 terms interleaved per 8 k,
// one scale per channel) and stream through a three-stage LDS ring by LDS-DMA, 16 rows
// per chunk ([ks][plane][row 16][32 k], 16-B slots XOR-swizzled by (row >> 2) & 3: a fragment
// read covers all 64 banks once per 16 lanes); one barrier per chunk, the 16 x 16
// block per wave scaled back by 1 / sigma_row, 1 / tau_n and stored from the
// accumulator.  No conversion work in the kernel.
constexpr int X3F_STAGE = 2 * (X3F_KMAX / 32) * 1024;  // bytes per stage (max Kp)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int KS, int NST>
__device__ __forceinline__ void x3f_body(const X3FParams& p, const GemmDesc& d, int m0, int n0,
                                         unsigned char* ring, float* isr_s) {
  constexpr int KP = 32 * KS;
  constexpr int NP = 2 * KS;  // 1-KB pieces per stage
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = d.M, N = d.N, K = d.K;
  const int rows = min(X3F_RB, M - m0);
  const int nch = (rows + 15) / 16;
  const uint32_t ring_lds = lds_addr(ring);
  const int ni = (NP - wave + 3) / 4;  // pieces this wave issues per stage

  // stage s <- rows m0 + 16 j .. + 15, all Kp, both planes
  // piece i = (ks = i / 2, plane i % 2): both planes of a k-step from one wave, so the
  // second instruction finds the 128-B lines of the first in L2
  auto issue = [&](int j, int s) {
    const int r = lane >> 2, kg = (lane & 3) ^ ((r >> 2) & 3);
    const int row = min(m0 + 16 * j + r, M - 1);
    const unsigned short* rowp = p.Ap + 2 * (d.offA + (int64_t)row * d.lda);
#pragma unroll
    for (int q = 0; q < (NP + 3) / 4; ++q) {
      const int i = wave + 4 * q;
      if (i < NP) {
        const int pl = i & 1, ks = i >> 1;
        const int k = 32 * ks + 8 * kg;
        glds16(rowp + 2 * seg_k(k < K ? k : 0, p.segA_w, p.segA_stride) + 8 * pl,
               ring_lds + s * X3F_STAGE + i * 1024);
      }
    }
  };
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (j < nch) issue(j, j);

  // B: this wave's 16 columns, lane (n = lane & 15, k = 32 ks + 8 (lane >> 4) .. + 7)
  const int col = n0 + 16 * wave + (lane & 15);
  const unsigned short* bp = p.img + d.offBx + (int64_t)min(col, N - 1) * KP + 8 * (lane >> 4);
  h8 b[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      b[ks][pl] = *reinterpret_cast<const h8*>(bp + (int64_t)pl * N * KP + 32 * ks);
  const float it = p.invs[d.offBs + min(col, N - 1)];
  for (int r = tid; r < rows; r += 256) isr_s[r] = p.isr[m0 + r];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float* Cb = p.C + d.offC;
  const int ra = lane >> 4;  // the accumulator's rows 4 ra .. + 3
  for (int j = 0; j < nch; ++j) {
    const int s = j % NST;
    // chunk j's DMA (j >= NST - 1; the first NST - 1 were drained with B) was followed by
    // the 4 stores of each of chunks j - NST + 1 .. j - 1 and the ni pieces of each
    // chunk j + 1 .. j + NST - 2 that exists
    int after = 4 * (NST - 1);
#pragma unroll
    for (int k = 1; k <= NST - 2; ++k) after += (j + k < nch) ? ni : 0;
    wait_vmcnt(after);
    __syncthreads();
    if (j + NST - 1 < nch) issue(j + NST - 1, (j + NST - 1) % NST);
    const unsigned char* st = ring + s * X3F_STAGE;
    const int r16 = lane & 15, kq = lane >> 4;
    const int off = r16 * 64 + 16 * (kq ^ ((r16 >> 2) & 3));
    f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const h8 a0 = *reinterpret_cast<const h8*>(st + (2 * ks) * 1024 + off);
      const h8 a1 = *reinterpret_cast<const h8*>(st + (2 * ks + 1) * 1024 + off);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b[ks][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b[ks][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b[ks][0], acc, 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = 16 * j + 4 * ra + e;  // row within the workgroup's block
      const bool ok = rl < rows && col < N;
      float* dst = ok ? Cb + (int64_t)(m0 + rl) * d.ldc + col : x3r_sink + lane;
      *dst = acc[e] * isr_s[min(rl, X3F_RB - 1)] * it;
    }
  }
}

template <int NST>
__global__ __launch_bounds__(256) void legendre_x3f_kernel(X3FParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[NST * X3F_STAGE];
  __shared__ float isr_s[X3F_RB];
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const GemmDesc d = p.descs[p.tile_desc[lin]];
  const int local = lin - d.tile_start;
  // consecutive tiles share rows (the column blocks of one row block): A from L2
  const int tn = local % d.tiles_n, tm = local / d.tiles_n;
  const int m0 = tm * X3F_RB, n0 = tn * 64;
  switch ((d.K + 31) / 32) {
#define X3F_CASE(n) case n: x3f_body<n, NST>(p, d, m0, n0, ring, isr_s); break;
    X3F_CASE(1) X3F_CASE(2) X3F_CASE(3) X3F_CASE(4) X3F_CASE(5) X3F_CASE(6)
    X3F_CASE(7) X3F_CASE(8) X3F_CASE(9) X3F_CASE(10) X3F_CASE(11) X3F_CASE(12)
#undef X3F_CASE
    default: break;  // K = 0 never reaches here (the host requires 0 < K <= X3F_KMAX)
  }
}

}  // namespace

int legendre_x3f(const unsigned short* Ap, const float* isr,
                 const unsigned short* img, const float* invs, float* C, const GemmDesc* descs,
                 const int* tile_desc, int ndesc, int tiles, hipStream_t s, int segA_w,
                 int64_t segA_stride) {
  if (ndesc <= 0 || tiles <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(Ap && isr && img && invs && C && descs && tile_desc, MSFNO_EINVAL,
                "legendre_x3f: null operand");
  MSFNO_REQUIRE(segA_w % 8 == 0 && segA_w >= 0, MSFNO_EINVAL,
                "legendre_x3f: segments must hold whole 8-k groups");
  X3FParams p{};
  p.Ap = Ap; p.isr = isr;
  p.img = img; p.invs = invs; p.C = C;
  p.descs = descs; p.tile_desc = tile_desc;
  p.segA_w = segA_w; p.segA_stride = segA_stride;
  // MSFNO_X3F_NS=2: two LDS stages (49 KB, three workgroups per CU) instead of three
  static const int ns = [] {
    const char* e = getenv("MSFNO_X3F_NS");
    return (e && e[0] == '2') ? 2 : 3;
  }();
  if (ns == 2)
    hipLaunchKernelGGL(legendre_x3f_kernel<2>, dim3(tiles), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(legendre_x3f_kernel<3>, dim3(tiles), dim3(256), 0, s, p);
  return launch_check("legendre_x3f");
}

int legendre_x3r(const float* A, const unsigned short* img, const float* invs, float* C,
                 const GemmDesc* descs, const int* tile_desc, int ndesc, int tiles,
                 const GemmEpi& e, hipStream_t s) {
  if (ndesc <= 0 || tiles <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(A && img && invs && C && descs && tile_desc, MSFNO_EINVAL,
                "legendre_x3r: null operand");
  MSFNO_REQUIRE(!e.rowscale && !e.bias && !e.addend && !e.segA_w, MSFNO_EUNSUPPORTED,
                "legendre_x3r: plain epilogue, unsegmented A only");
  X3DParams p{};
  p.A = A; p.img = img; p.invs = invs; p.C = C;
  p.descs = descs; p.tile_desc = tile_desc; p.ndesc = ndesc;
  p.segC_w = e.segC_w; p.segC_stride = e.segC_stride;
  hipLaunchKernelGGL(legendre_x3r_kernel, dim3(tiles), dim3(256), 0, s, p);
  return launch_check("legendre_x3r");
}

int launch_legendre_x3_image(const float* table, const GemmDesc* descs, int ndesc,
                             unsigned short* img, float* invs, hipStream_t s) {
  if (ndesc <= 0) return MSFNO_OK;
  hipLaunchKernelGGL(x3d_image_kernel, dim3(ndesc), dim3(256), 0, s, table, descs, img, invs);
  return launch_check("legendre_x3_image");
}

// tile width of the x3h Legendre problems (MSFNO_LEG_X3_BN=64|128|192, per direction:
// MSFNO_LEG_X3_BN=<forward>,<inverse>)
int x3d_bn(int inverse) {
  static int bn[2] = {0, 0};
  if (!bn[0]) {
    bn[0] = bn[1] = 64;
    if (const char* e = getenv("MSFNO_LEG_X3_BN")) {
      int a = 0, b = 0;
      const int n = sscanf(e, "%d,%d", &a, &b);
      if (n >= 1) bn[0] = bn[1] = a;
      if (n == 2) bn[1] = b;
    }
    for (int& v : bn)
      if (v != 128 && v != 192) v = 64;
  }
  return bn[inverse ? 1 : 0];
}

int legendre_x3(const float* A, const unsigned short* img, const float* invs, float* C,
                const GemmDesc* descs, const int* tile_desc, int ndesc, int tiles, int bn,
                const GemmEpi& e, hipStream_t s) {
  if (ndesc <= 0 || tiles <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(A && img && invs && C && descs, MSFNO_EINVAL, "legendre_x3: null operand");
  MSFNO_REQUIRE(!e.rowscale && !e.bias && !e.addend, MSFNO_EUNSUPPORTED,
                "legendre_x3: plain epilogue only");
  X3DParams p{};
  p.A = A; p.img = img; p.invs = invs; p.C = C;
  p.descs = descs; p.tile_desc = tile_desc; p.ndesc = ndesc;
  p.segA_w = e.segA_w; p.segA_stride = e.segA_stride;
  p.segC_w = e.segC_w; p.segC_stride = e.segC_stride;
  p.vecC = (reinterpret_cast<uintptr_t>(C) & 15) == 0;  // every ldc / offC is a multiple of 4
  static const int pf = [] {  // k-tiles of register prefetch (2 measured no faster)
    const char* e = getenv("MSFNO_LEG_X3_PF");
    return (e && e[0] == '2') ? 2 : 1;
  }();
  static const int dbg = [] {
    const char* e = getenv("MSFNO_LEG_X3_DBG");
    return e ? atoi(e) & 7 : 0;
  }();
  static void (*const kd[8])(X3DParams) = {
      legendre_x3_kernel<64, 2, 0>, legendre_x3_kernel<64, 2, 1>, legendre_x3_kernel<64, 2, 0>,
      legendre_x3_kernel<64, 2, 1>, legendre_x3_kernel<64, 2, 4>, legendre_x3_kernel<64, 2, 5>,
      legendre_x3_kernel<64, 2, 4>, legendre_x3_kernel<64, 2, 5>};
  if (dbg)
    hipLaunchKernelGGL(kd[dbg], dim3(tiles), dim3(256), 0, s, p);
  else if (bn == 64)
    hipLaunchKernelGGL((pf == 1 ? legendre_x3_kernel<64, 1> : legendre_x3_kernel<64, 2>), dim3(tiles),
                       dim3(256), 0, s, p);
  else if (bn == 128)
    hipLaunchKernelGGL((pf == 1 ? legendre_x3_kernel<128, 1> : legendre_x3_kernel<128, 2>),
                       dim3(tiles), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((pf == 1 ? legendre_x3_kernel<192, 1> : legendre_x3_kernel<192, 2>),
                       dim3(tiles), dim3(256), 0, s, p);
  return launch_check("legendre_x3");
}

}  // namespace msfno
