// fp32-accurate GEMM on the bf16 matrix cores with BOTH operands in the
// bf16x3 plane format ("x6p"), for gfx950.
//
// Same arithmetic as gemm_x6.hip (C = sum of the six products a_i b_j with
// i + j <= 2 of the exact three-term bf16 splits, fp32 accumulation in the
// MFMA), but B is not converted in the kernel: its producer already wrote the
// three bf16 terms (EPI_PLANES epilogue, or launch_split_planes).  With no
// conversion work left, the operands go HBM/L2 -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging) into a ring of NSTAGE stages, so
// NSTAGE - 1 k-tiles are in flight while one is multiplied: one raw s_barrier and
// one counted vmcnt per k-tile (cdna_hip_programming.md §5, "Pipelining across
// barriers").  Two stages (one tile ahead) measured 1-3 % faster than three: the
// GEMM is clock (power) bound, not latency bound, at this size.
//
// Tile 256 x 256 x 16 (k), 8 waves as 4 (M) x 2 (N), each wave 64 x 128 as 2 x 4
// blocks of v_mfma_f32_32x32x16_bf16 (the C layout of the fp32 kernel, so the
// LDS epilogue of gemm_common.h is shared).
// LDS stage (48 KB): A [plane][256 m][16 k] with the two 16-B k-halves of row m
// swapped when (m >> 3) & 1 (conflict-free ds_read_b128); B [plane][16 k][256 n]
// with the 16-B column units of row r XORed by 4 (r & 3) (conflict-free
// ds_read_b64_tr_b16).  LDS-DMA writes lane-linear 1-KB pieces, so both
// swizzles are applied on the global source address.
// A (weights) is split once per call into [batch][plane][k-tile][Mp][16] so
// that every 1-KB piece is one contiguous run in memory.
#include <cstdlib>
#include <string>

#include "dma.h"
#include "gemm_common.h"

namespace msfno {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef lds_void_t lds_void;

constexpr int X6P_BM = 256, X6P_BN = 256, X6P_BK = 16;

// A (M x K fp32, row stride lda, batch stride sA) -> bf16x3 k-tiles
// Ax[z][plane][kt][Mp][16], zero padded to Mp x (KT * 16)
template <int TK>
__global__ void split_a_tiles_kernel(const float* __restrict__ A, unsigned short* __restrict__ Ax,
                                     int M, int K, int lda, int64_t sA, int Mp, int KT) {
  const int z = blockIdx.y;
  const int64_t plane = (int64_t)Mp * KT * TK;
  const int64_t n = plane / 2;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = 2 * e;
    const int kt = (int)(idx / ((int64_t)Mp * TK));
    const int rem = (int)(idx - (int64_t)kt * Mp * TK);
    const int m = rem / TK, k = kt * TK + (rem % TK);
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

// All spectral-MLP weights of a block in one launch: layer l's complex weight
// w (ci, co, 2) (SpectralAttentionS2 w.l / wout, layers.py:580-596) real-ified to
// [[Wr, -Wi], [Wi, Wr]] (2 co x 2 ci) and split straight into the x6p A image.
__global__ void spec_weights_x6p_kernel(SpecWeightsX6p a) {
  const int64_t total = a.start[a.nlayers];
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < a.nlayers && g >= a.start[l + 1]) ++l;
    const int ci = a.ci[l], co = a.co[l];
    const int M = 2 * co, K = 2 * ci;
    const int Mp = (M + X6P_BM - 1) / X6P_BM * X6P_BM, KT = (K + X6P_BK - 1) / X6P_BK;
    const int64_t n = (int64_t)Mp * KT * 8;  // pairs per plane
    const int64_t e = g - a.start[l];
    const int64_t idx = 2 * e;
    const int kt = (int)(idx / ((int64_t)Mp * 16));
    const int rem = (int)(idx - (int64_t)kt * Mp * 16);
    const int m = rem >> 4, k0 = kt * 16 + (rem & 15);
    float v[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = k0 + t;
      float x = 0.f;
      if (m < M && k < K) {
        const int ro = m / co, o = m - ro * co, ri = k / ci, i = k - ri * ci;
        const float wr = a.w[l][((int64_t)i * co + o) * 2], wi = a.w[l][((int64_t)i * co + o) * 2 + 1];
        x = ro == 0 ? (ri == 0 ? wr : -wi) : (ri == 0 ? wi : wr);
      }
      v[t] = x;
    }
    uint32_t t0, t1, t2;
    split2(v[0], v[1], t0, t1, t2);
    uint32_t* o = reinterpret_cast<uint32_t*>(a.out[l]) + e;
    o[0] = t0;
    o[n] = t1;
    o[2 * n] = t2;
  }
}

// fp32 rows -> bf16x3 planes: x[z][r][c] (ld ldx, batch stride sx) ->
// xp[z][plane][r][c] (ld ldp, plane stride pstride, batch stride sxp)
__global__ void split_planes_kernel(const float* __restrict__ x, unsigned short* __restrict__ xp,
                                    int rows, int cols, int ldx, int64_t sx, int ldp,
                                    int64_t pstride, int64_t sxp) {
  const int z = blockIdx.y;
  const int cp = (cols + 1) / 2;  // column pairs per row
  const int64_t n = (int64_t)rows * cp;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / cp), c = 2 * (int)(e - (int64_t)r * cp);
    const float* src = x + z * sx + (int64_t)r * ldx + c;
    const float v0 = src[0];
    const float v1 = (c + 1 < cols) ? src[1] : 0.f;
    uint32_t t0, t1, t2;
    split2(v0, v1, t0, t1, t2);
    unsigned short* d = xp + z * sxp + (int64_t)r * ldp + c;
    if (c + 1 < cols) {
      *reinterpret_cast<uint32_t*>(d) = t0;
      *reinterpret_cast<uint32_t*>(d + pstride) = t1;
      *reinterpret_cast<uint32_t*>(d + 2 * pstride) = t2;
    } else {
      d[0] = (unsigned short)t0;
      d[pstride] = (unsigned short)t1;
      d[2 * pstride] = (unsigned short)t2;
    }
  }
}

template <int EPI, int NSTAGE = 3, int WAVES = 8, int BNT = 256>
__global__ __launch_bounds__(64 * WAVES) void gemm_x6p_kernel(GemmParams p) {
  constexpr int BM = X6P_BM, BN = BNT, BK = X6P_BK;
  // 256 x 256 tiles: 8 waves as 4 x 2 (wave 64 x 128), or 4 waves as 2 x 2 (wave
  // 128 x 128, 256 accumulator registers: one wave per SIMD);
  // 256 x 128 tiles: 4 waves as 4 x 1 (wave 64 x 128), 72-KB ring: two workgroups per
  // CU, so one's epilogue stores overlap the other's main loop
  static_assert(BNT == 256 || (BNT == 128 && WAVES == 4), "tile / waves");
  constexpr int WGM = (BNT == 128 || WAVES == 8) ? 4 : 2, WGN = WAVES / WGM, NTHR = 64 * WAVES;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int A_PLANE = BM * BK;             // bf16 elements
  constexpr int B_PLANE = BK * BN;
  constexpr int STAGE = 3 * (A_PLANE + B_PLANE);
  constexpr int RING_BYTES = NSTAGE * STAGE * 2;
  constexpr int EPI_BYTES = 32 * WGM * (BN + 8) * 4;
  constexpr int LDS_BYTES = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  constexpr bool HAS_BIAS = (EPI & EPI_BIAS) != 0;
  constexpr int BPIECES = 3 * BK * BN * 2 / 1024;  // 1-KB B pieces per stage (24 or 12)
  constexpr int QA = 24 / WAVES;                    // A pieces per wave
  constexpr int QB = BPIECES / WAVES;               // B pieces per wave
  constexpr int LOADS = QA + QB;  // LDS-DMA wave-instructions per wave per k-tile
  constexpr int RPP = 1024 / (BN * 2);              // B rows per piece (2 or 4)
  static_assert(LOADS * WAVES * 1024 == STAGE * 2 && QB * WAVES == BPIECES, "stage pieces");
  // one LDS object only: a second __shared__ array makes hipcc drain the DMA
  // (vmcnt(0)) before the first ds_read of every k-tile
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES + (HAS_BIAS ? BM * 4 : 0)];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
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
  const unsigned short* Bx = p.Bx + z * p.sB;
  float* C = p.C + z * p.sC;
  const float* bias = p.bias ? p.bias + z * p.sBias : nullptr;
  const float* addend = p.addend ? p.addend + z * p.sD : nullptr;
  const int M = p.M, N = p.N, K = p.K, ldb = p.ldb, ldc = p.ldc;
  const int Mp = p.ldax;  // rows of the A tile image
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    for (int r = tid; r < BM; r += NTHR) bias_s[r] = bias[min(m0 + r, M - 1)];
  }

  // ---- LDS-DMA sources: per wave QA A pieces and QB B pieces of 1 KB per k-tile
  // A piece a = wave + WAVES q (q < QA): plane a / 8, rows 32 (a % 8) .. + 31
  // B piece b = wave + WAVES q (q < QB): plane b / (16 / RPP), k rows RPP (b % (16 / RPP)) ..
  const unsigned short* a_src[QA];
  int a_dst[QA], b_dst[QB];
  int64_t b_row_off[QB];
  int b_col[QB], b_row[QB];
#pragma unroll
  for (int q = 0; q < QA; ++q) {
    const int a = wave + WAVES * q;
    const int pl = a >> 3, mb = a & 7;
    const int m = 32 * mb + (lane >> 1);
    const int h = (lane & 1) ^ ((m >> 3) & 1);
    a_src[q] = Ax + (int64_t)pl * p.sAxp + (int64_t)(m0 + m) * 16 + 8 * h;
    a_dst[q] = pl * A_PLANE + mb * 32 * BK;
  }
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const int b = wave + WAVES * q;
    const int pl = b / (16 / RPP), rb = b % (16 / RPP);
    const int row = RPP * rb + lane / (64 / RPP);
    const int gu = (lane % (64 / RPP)) ^ (4 * (row & 3));
    b_row[q] = row;
    // clamp to the last full 16-B unit of the N columns (not of the row: B may start
    // mid-row, e.g. a pixel chunk of a wider plane)
    b_col[q] = min(n0 + 8 * gu, ((N + 7) & ~7) - 8);
    b_row_off[q] = (int64_t)pl * p.sBxp;
    b_dst[q] = 3 * A_PLANE + pl * B_PLANE + rb * RPP * BN;
  }
  const int64_t a_kstride = (int64_t)Mp * 16;  // elements per k-tile of one A plane
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(lds_void*)ring;
  auto issue = [&](int kt, int st) {
    const uint32_t base = ring_lds + (uint32_t)(st * STAGE * 2);
#pragma unroll
    for (int q = 0; q < QA; ++q)
      glds16(a_src[q] + kt * a_kstride,
             __builtin_amdgcn_readfirstlane(base + (uint32_t)(a_dst[q] * 2)));
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int kr = min(kt * BK + b_row[q], K - 1);
      glds16(Bx + b_row_off[q] + (int64_t)kr * ldb + b_col[q],
             __builtin_amdgcn_readfirstlane(base + (uint32_t)(b_dst[q] * 2)));
    }
  };

  floatx16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-lane fragment offsets within a stage (bf16 elements)
  int a_off[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * WM + i * 32 + l32;
    a_off[i] = row * BK + 8 * (half ^ ((row >> 3) & 1));
  }
  const int li = lane & 15, g16 = (lane >> 4) & 1;
  const int br = 8 * half + (li >> 2);  // k row of the first tr read (second: + 4)
  int b_off[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int c = wn * WN + j * 32 + 16 * g16 + 4 * (li & 3);
    b_off[j] = 3 * A_PLANE + br * BN + (((c >> 3) ^ (4 * (br & 3))) << 3) + (c & 7);
  }

  auto mfma_tile = [&](int st) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const unsigned short* base = ring + st * STAGE;
    bf16x8 a[MT][3];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = *reinterpret_cast<const bf16x8*>(base + pl * A_PLANE + a_off[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bf16x8 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const unsigned short* q = base + pl * B_PLANE + b_off[j];
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)q));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)(q + 4 * BN)));
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        b[pl] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        floatx16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][2], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][1], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][0], b[0], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  };

  if constexpr (HAS_BIAS) __syncthreads();  // bias_s visible; no DMA in flight yet
  issue(0, 0);
  if (NSTAGE == 3 && nk > 1) issue(1, 1);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // my DMA of k-tile kt has landed (k-tile kt + 1 may stay in flight) ...
    if (NSTAGE == 3 && kt + 1 < nk)
      wait_vmcnt(LOADS);
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ... and everyone's: after this barrier stage kt % 3 is complete and every
    // wave has finished reading stage (kt - 1) % 3, which the next issue refills
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (NSTAGE == 3) {
      if (kt + 2 < nk) issue(kt + 2, st == 0 ? 2 : st - 1);
    } else {
      if (kt + 1 < nk) issue(kt + 1, st ^ 1);
    }
    __builtin_amdgcn_s_setprio(1);
    mfma_tile(st);
    __builtin_amdgcn_s_setprio(0);
    st = NSTAGE == 3 ? (st == 2 ? 0 : st + 1) : (st ^ 1);
  }
  __syncthreads();  // all DMA retired (vmcnt(0) above); the ring is free for the epilogue
  gemm_epilogue<BM, BN, EPI, WGM, WGN>(p, acc, reinterpret_cast<float*>(lds_raw), bias_s, C,
                                       addend, M, N, ldc, m0, n0, 0);
}


// ---- 16x16x32 variant ("x6q") ---------------------------------------------------
// Same operands and arithmetic as gemm_x6p_kernel, on v_mfma_f32_16x16x32_bf16:
// at equal FLOPs the 16x16x32 stream holds a higher clock than the 32x32x16 one on
// random data (tools/mfma_shape_bench.hip: 1.26x; MI355X_MICROARCH.md "DVFS
// give-back" item 7).  Tile 256 x 128 x 32 (k), 8 waves as 4 x 2, each wave 64 x 64
// as 4 x 4 blocks of 16 x 16; two 72-KB stages (one k-tile in flight measured as
// fast as two for gemm_x6p).  A image [plane][k-tile of 32][Mp][32]; LDS: A rows of
// 64 B with the 16-B slots XORed by (m >> 2) & 3, B rows of 256 B with the 16-B
// units XORed by 2 (r & 3) + 8 ((r >> 3) & 1): both conflict-free for the
// ds_read_b128 / ds_read_b64_tr_b16 fragments of the 16x16x32 shape.
typedef float floatx4q __attribute__((ext_vector_type(4)));
constexpr int X6Q_BM = 256, X6Q_BN = 128, X6Q_BK = 32;

template <int EPI>
__global__ __launch_bounds__(512) void gemm_x6q_kernel(GemmParams p) {
  constexpr int BM = X6Q_BM, BN = X6Q_BN, BK = X6Q_BK;
  constexpr int WGM = 4, WGN = 2;
  constexpr int WM = BM / WGM, WN = BN / WGN;  // 64 x 64
  constexpr int MT = WM / 16, NT = WN / 16;
  constexpr int A_PLANE = BM * BK, B_PLANE = BK * BN;
  constexpr int STAGE = 3 * (A_PLANE + B_PLANE);  // 72 KB
  constexpr int NSTAGE = 2;
  constexpr int RING_BYTES = NSTAGE * STAGE * 2;
  constexpr int EPI_BYTES = 16 * WGM * (BN + 8) * 4;
  constexpr int LDS_BYTES = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  constexpr bool HAS_BIAS = (EPI & EPI_BIAS) != 0;
  static_assert(STAGE * 2 == 72 * 1024, "stage = 48 A + 24 B pieces of 1 KB");
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES + (HAS_BIAS ? BM * 4 : 0)];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const bias_s = reinterpret_cast<float*>(lds_raw + LDS_BYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin % p.tiles_m, tn = lin / p.tiles_m;
  const int z = blockIdx.z;
  const unsigned short* Ax = p.Ax + z * p.sAx;
  const unsigned short* Bx = p.Bx + z * p.sB;
  float* C = p.C + z * p.sC;
  const float* bias = p.bias ? p.bias + z * p.sBias : nullptr;
  const float* addend = p.addend ? p.addend + z * p.sD : nullptr;
  const int M = p.M, N = p.N, K = p.K, ldb = p.ldb, ldc = p.ldc;
  const int Mp = p.ldax;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    for (int r = tid; r < BM; r += 512) bias_s[r] = bias[min(m0 + r, M - 1)];
  }
  // LDS-DMA pieces c = wave + 8 q (q < 9): c < 48 -> A (plane c / 16, rows 16 (c % 16)),
  // else B (plane (c - 48) / 8, k rows 4 ((c - 48) % 8))
  const unsigned short* src[9];
  int dst[9], brow[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int c = wave + 8 * q;
    if (c < 48) {
      const int pl = c >> 4, rb = c & 15;
      const int m = 16 * rb + (lane >> 2);
      const int g = (lane & 3) ^ ((m >> 2) & 3);
      src[q] = Ax + (int64_t)pl * p.sAxp + (int64_t)(m0 + m) * BK + 8 * g;
      dst[q] = pl * A_PLANE + rb * 16 * BK;
      brow[q] = -1;
    } else {
      const int cb = c - 48;
      const int pl = cb >> 3, rq = cb & 7;
      const int row = 4 * rq + (lane >> 4);
      const int gu = (lane & 15) ^ (2 * (row & 3) + 8 * ((row >> 3) & 1));
      src[q] = Bx + (int64_t)pl * p.sBxp + min(n0 + 8 * gu, ldb - 8);
      dst[q] = 3 * A_PLANE + pl * B_PLANE + rq * 4 * BN;
      brow[q] = row;
    }
  }
  const int64_t a_kstride = (int64_t)Mp * BK;
  const uint32_t ring_lds = lds_addr(ring);
  auto issue = [&](int kt, int st) {
    const uint32_t base = ring_lds + (uint32_t)(st * STAGE * 2);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const unsigned short* gp = brow[q] < 0
                                     ? src[q] + kt * a_kstride
                                     : src[q] + (int64_t)min(kt * BK + brow[q], K - 1) * ldb;
      glds16(gp, base + (uint32_t)(dst[q] * 2));
    }
  };

  floatx4q acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  int a_off[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * WM + i * 16 + (lane & 15);
    a_off[i] = row * BK + 8 * ((lane >> 4) ^ ((row >> 2) & 3));
  }
  const int li = lane & 15, G = lane >> 4;
  const int r1 = 8 * G + (li >> 2);  // k row of the first tr read (second: + 4)
  const int fr = 2 * (r1 & 3) + 8 * ((r1 >> 3) & 1);
  int b_off[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int c = wn * WN + j * 16 + 4 * (li & 3);
    b_off[j] = 3 * A_PLANE + r1 * BN + (((c >> 3) ^ fr) << 3) + (c & 7);
  }
  auto mfma_tile = [&](int st) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const unsigned short* base = ring + st * STAGE;
    bf16x8 a[MT][3];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[i][pl] = *reinterpret_cast<const bf16x8*>(base + pl * A_PLANE + a_off[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bf16x8 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const unsigned short* qq = base + pl * B_PLANE + b_off[j];
        const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)qq));
        const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)(qq + 4 * BN)));
        const s16x8 v = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        b[pl] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        floatx4q c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[0], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  };

  if constexpr (HAS_BIAS) __syncthreads();
  issue(0, 0);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my DMA of k-tile kt landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's; the other stage is free
    if (kt + 1 < nk) issue(kt + 1, st ^ 1);
    __builtin_amdgcn_s_setprio(1);
    mfma_tile(st);
    __builtin_amdgcn_s_setprio(0);
    st ^= 1;
  }
  __syncthreads();
  gemm_epilogue<BM, BN, EPI, WGM, WGN, MT, NT, 16, floatx4q>(
      p, acc, reinterpret_cast<float*>(lds_raw), bias_s, C, addend, M, N, ldc, m0, n0, 0);
}

// ---- host ---------------------------------------------------------------------

size_t gemm_x6p_workspace(int M, int K, int batch_a) {
  // k padded to 32: covers the 16-deep (x6p) and 32-deep (x6q) A images
  const int64_t Mp = round_up(M, X6P_BM), Kp = round_up(K, 32);
  return (size_t)round_up(3 * Mp * Kp * 2 * (int64_t)batch_a, 256);
}

int gemm_x6p_split_a(const float* A, int M, int K, int lda, int64_t sA, int batch, void* ws,
                     size_t ws_bytes, hipStream_t s) {
  const int abatch = sA == 0 ? 1 : batch;
  const int Mp = (int)round_up(M, X6P_BM), KT = (int)cdiv(K, X6P_BK);
  MSFNO_REQUIRE(ws && ws_bytes >= gemm_x6p_workspace(M, K, abatch), MSFNO_EINVAL,
                "gemm_x6p_split_a: workspace too small");
  const int64_t pairs = (int64_t)Mp * KT * X6P_BK / 2;
  const int blocks = (int)std::min<int64_t>(cdiv(pairs, 256), 1024);
  hipLaunchKernelGGL(split_a_tiles_kernel<X6P_BK>, dim3(blocks, abatch), dim3(256), 0, s, A,
                     static_cast<unsigned short*>(ws), M, K, lda, sA, Mp, KT);
  return launch_check("split_a_tiles");
}

int launch_spec_weights_x6p(const SpecWeightsX6p& a, hipStream_t s) {
  if (a.nlayers <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(a.start[a.nlayers], 256), 4096);
  hipLaunchKernelGGL(spec_weights_x6p_kernel, dim3(blocks), dim3(256), 0, s, a);
  return launch_check("spec_weights_x6p");
}

size_t spec_weights_x6p_layout(SpecWeightsX6p& a) {
  size_t bytes = 0;
  a.start[0] = 0;
  for (int l = 0; l < a.nlayers; ++l) {
    const size_t b = gemm_x6p_workspace(2 * a.co[l], 2 * a.ci[l], 1);
    a.start[l + 1] = a.start[l] + (int64_t)round_up(2 * a.co[l], X6P_BM) *
                                      cdiv(2 * a.ci[l], X6P_BK) * 8;
    bytes += b;
  }
  return bytes;
}

int launch_split_planes(const float* x, unsigned short* xp, int rows, int cols, int ldx,
                        int64_t sx, int ldp, int64_t pstride, int64_t sxp, int batch,
                        hipStream_t s) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(ldp % 2 == 0 && pstride % 2 == 0 && sxp % 2 == 0, MSFNO_EINVAL,
                "split_planes: even plane strides required");
  const int64_t n = (int64_t)rows * ((cols + 1) / 2);
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 2048);
  hipLaunchKernelGGL(split_planes_kernel, dim3(blocks, batch), dim3(256), 0, s, x, xp, rows, cols,
                     ldx, sx, ldp, pstride, sxp);
  return launch_check("split_planes");
}

// MFMA shape of the plane GEMM: 32x32x16 (x6p) unless MSFNO_X6P_MFMA=16 (x6q,
// measured 2 % slower on the fc2 shape); ring depth MSFNO_X6P_STAGES=2|3 (x6p; 2
// k-tiles measured 1-3 % faster than 3 on fc1/fc2)
static bool use_x6q() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_X6P_MFMA");
    return e && std::string(e) == "16";
  }();
  return on;
}

// workgroup of the plane GEMM: 8 waves (default) or 4 (MSFNO_X6P_WAVES=4)
static int x6p_waves() {
  static const int w = [] {
    const char* e = getenv("MSFNO_X6P_WAVES");
    if (e && std::string(e) == "4x128") return 128;  // 256 x 128 tiles, 4 waves
    return (e && e[0] == '4') ? 4 : 8;
  }();
  return w;
}

template <int EPI>
static void launch_x6p_e(const GemmParams& p, dim3 grid, hipStream_t s, bool q) {
  static const int stages = [] {
    const char* e = getenv("MSFNO_X6P_STAGES");
    return (e && e[0] == '3') ? 3 : 2;
  }();
  if (q)
    hipLaunchKernelGGL((gemm_x6q_kernel<EPI>), grid, dim3(512), 0, s, p);
  else if (stages == 2 && x6p_waves() == 4)
    hipLaunchKernelGGL((gemm_x6p_kernel<EPI, 2, 4>), grid, dim3(256), 0, s, p);
  else if (stages == 2 && x6p_waves() == 128)
    hipLaunchKernelGGL((gemm_x6p_kernel<EPI, 2, 4, 128>), grid, dim3(256), 0, s, p);
  else if (stages == 2)
    hipLaunchKernelGGL((gemm_x6p_kernel<EPI, 2>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_x6p_kernel<EPI, 3>), grid, dim3(512), 0, s, p);
}

int gemm_x6p(const float* A, float* C, int M, int N, int K, int lda, int ldb, int ldc,
             int64_t sA, int64_t sB, int64_t sC, int batch, const GemmEpi& epi, void* ws,
             size_t ws_bytes, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return MSFNO_OK;
  const int abatch = sA == 0 ? 1 : batch;
  // the pre-split images of launch_spec_weights_x6p are 16-deep: x6p kernel for them
  const bool q = use_x6q() && !epi.a_planes;
  const int TKd = q ? X6Q_BK : X6P_BK;
  const size_t need = (size_t)round_up(3 * round_up(M, X6P_BM) * round_up(K, TKd) * 2 * (int64_t)abatch, 256);
  MSFNO_REQUIRE(epi.a_planes || (ws && ws_bytes >= need), MSFNO_EINVAL,
                "gemm_x6p: workspace too small");
  // a batched pre-split A (sA != 0) has gemm_x6p_split_a's layout: batch stride 3 planes
  MSFNO_REQUIRE(epi.b_planes, MSFNO_EINVAL, "gemm_x6p: B must be in the plane format");
  MSFNO_REQUIRE(batch <= 65535 && K > 0, MSFNO_EINVAL, "gemm_x6p: bad batch / K");
  MSFNO_REQUIRE(ldb % 8 == 0 && ldb >= 8 && sB % 8 == 0 && epi.b_plane_stride % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(epi.b_planes) & 15) == 0,
                MSFNO_EINVAL, "gemm_x6p: B planes need ld, strides % 8 == 0 and 16-B alignment");
  MSFNO_REQUIRE(epi.act != 2 && !epi.rowscale, MSFNO_EUNSUPPORTED,
                "gemm_x6p: unsupported epilogue");
  const int Mp = (int)round_up(M, X6P_BM), KT = (int)cdiv(K, TKd);
  unsigned short* Ax = static_cast<unsigned short*>(ws);
  if (epi.a_planes) {
    Ax = const_cast<unsigned short*>(epi.a_planes);  // already in the A image layout
  } else {
    const int64_t pairs = (int64_t)Mp * KT * TKd / 2;
    const int blocks = (int)std::min<int64_t>(cdiv(pairs, 256), 1024);
    if (q)
      hipLaunchKernelGGL(split_a_tiles_kernel<X6Q_BK>, dim3(blocks, abatch), dim3(256), 0, s, A,
                         Ax, M, K, lda, sA, Mp, KT);
    else
      hipLaunchKernelGGL(split_a_tiles_kernel<X6P_BK>, dim3(blocks, abatch), dim3(256), 0, s, A,
                         Ax, M, K, lda, sA, Mp, KT);
    MSFNO_TRY(launch_check("split_a_tiles"));
  }
  GemmParams p{};
  p.C = C;
  p.M = M; p.N = N; p.K = K; p.ldb = ldb; p.ldc = ldc;
  p.sB = sB; p.sC = sC;
  p.bias = epi.bias; p.addend = epi.addend; p.sBias = epi.sBias; p.sD = epi.sD;
  p.ldd = epi.ldd; p.act = epi.act; p.relu_period = epi.relu_period; p.relu_rows = epi.relu_rows;
  p.Ax = Ax; p.sAxp = (int64_t)Mp * KT * TKd; p.sAx = sA == 0 ? 0 : 3 * p.sAxp; p.ldax = Mp;
  p.Bx = epi.b_planes; p.sBxp = epi.b_plane_stride;
  p.Cx = epi.c_planes; p.sCxp = epi.c_plane_stride;
  p.cx16 = cx16_enabled() && p.Cx && ldc % 8 == 0 && sC % 8 == 0 && p.sCxp % 8 == 0 &&
           (reinterpret_cast<uintptr_t>(p.Cx) & 15) == 0;
  p.vecC = (ldc % 4 == 0) && (sC % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
           (!epi.addend || ((epi.ldd % 4 == 0) && (epi.sD % 4 == 0) &&
                            ((reinterpret_cast<uintptr_t>(epi.addend) & 15) == 0)));
  if (p.Cx)
    MSFNO_REQUIRE(ldc % 4 == 0 && sC % 4 == 0 && p.sCxp % 4 == 0 &&
                      (reinterpret_cast<uintptr_t>(p.Cx) & 7) == 0,
                  MSFNO_EINVAL, "gemm_x6p: C planes need ld, strides % 4 == 0 and 8-B alignment");
  p.tiles_m = Mp / X6P_BM;
  p.tiles_n = (int)cdiv(N, q ? X6Q_BN : (x6p_waves() == 128 ? 128 : X6P_BN));
  const dim3 grid(p.tiles_m * p.tiles_n, 1, batch);
  const int code = (p.bias ? EPI_BIAS : 0) | (p.addend ? EPI_ADD : 0) | (p.act == 1 ? EPI_GELU : 0) |
                   (p.relu_period ? EPI_RELU : 0) | (p.Cx ? EPI_PLANES : 0);
  switch (code) {
    case 0: launch_x6p_e<0>(p, grid, s, q); break;
    case EPI_RELU: launch_x6p_e<EPI_RELU>(p, grid, s, q); break;
    case EPI_RELU | EPI_PLANES: launch_x6p_e<EPI_RELU | EPI_PLANES>(p, grid, s, q); break;
    case EPI_PLANES: launch_x6p_e<EPI_PLANES>(p, grid, s, q); break;
    case EPI_BIAS: launch_x6p_e<EPI_BIAS>(p, grid, s, q); break;
    case EPI_BIAS | EPI_ADD: launch_x6p_e<EPI_BIAS | EPI_ADD>(p, grid, s, q); break;
    case EPI_ADD: launch_x6p_e<EPI_ADD>(p, grid, s, q); break;
    case EPI_BIAS | EPI_GELU | EPI_PLANES:
      launch_x6p_e<EPI_BIAS | EPI_GELU | EPI_PLANES>(p, grid, s, q); break;
    default:
      set_error("gemm_x6p: unsupported epilogue combination");
      return MSFNO_EUNSUPPORTED;
  }
  return launch_check("gemm_x6p");
}

}  // namespace msfno
