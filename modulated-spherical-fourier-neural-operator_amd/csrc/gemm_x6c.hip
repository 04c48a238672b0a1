// Spectral-MLP layer as a Gauss three-multiplication complex GEMM on the x6
// engine ("x6c"), for gfx950.
//
// One layer of SpectralAttentionS2.forward_mlp (layers.py:604-620; the
// contraction compl_mul2d_fwd_c, contractions.py:132-137) is Y = W · X over the
// channels of every (l, m) column, W (co x ci) and X (ci x T) complex.  With
//   P1 = Wr·Xr,  P2 = Wi·Xi,  P3 = (Wr + Wi)·(Xr + Xi)
// Re Y = P1 - P2 and Im Y = P3 - P1 - P2: three real products instead of the four
// of the real-ified [[Wr, -Wi], [Wi, Wr]] GEMM, 25 % fewer matrix-core cycles.
// Each product is an x6 product (gemm_x6p.hip) of bf16x3 planes, so both
// operands carry a third "matrix": Ws = Wr + Wi (weight prep) and Xs = Xr + Xi,
// which the producer of X writes next to Xr and Xi (the previous layer's
// epilogue, or split3m for layer 0).  ComplexReLU(real) (activations.py:42-46)
// is applied to Re in the epilogue, before Ys = Re + Im is formed.
//
// Activation layout ("3M planes"): X[b][mat][plane][c][ld], mat 0 = real,
// 1 = imaginary, 2 = real + imaginary.
// Tile 128 complex rows x 128 columns x 16 (k), 8 waves as 4 (M) x 2 (N), each
// wave 32 x 64 with three accumulator sets (P1, P2, P3).  Stage (72 KB) = A: 3
// matrices x 3 planes x [128][16] + B: 3 x 3 x [16][128]; two stages, one k-tile
// in flight (LDS-DMA, dma.h).  LDS swizzles as in gemm_x6p_kernel.
#include <cstdlib>

#include "dma.h"
#include "gemm_common.h"

namespace msfno {

typedef __bf16 bf16x8c __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8c __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2c __attribute__((ext_vector_type(2)));
typedef float f32x2c __attribute__((ext_vector_type(2)));
typedef short s16x4c __attribute__((ext_vector_type(4)));
typedef short s16x8c __attribute__((ext_vector_type(8)));

// NP planes per value: 3 = the x6 engine (bf16 terms, six MFMAs per product), 2 = the
// x3h engine (fp16 terms, three MFMAs; operands power-of-two scaled into fp16 range,
// see the scale arrays of X6CParams and spec_scales_x3h_kernel)
template <int NP>
struct X6CEng;
template <>
struct X6CEng<3> {
  typedef bf16x8c frag;
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
struct X6CEng<2> {
  typedef f16x8c frag;
  __device__ static void split(float a, float b, uint32_t (&t)[2]) {
    const f32x2c v = {a, b};
    const f16x2c h0 = __builtin_convertvector(v, f16x2c);
    const f32x2c r = v - __builtin_convertvector(h0, f32x2c);
    const f16x2c h1 = __builtin_convertvector(r, f16x2c);
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

constexpr int X6C_BM = 128, X6C_BN = 128, X6C_BK = 16;

struct X6CParams {
  const unsigned short* Aw;  // [mat][plane][kt][Mp][16]
  int64_t a_mat, a_plane;
  int Mp;
  const unsigned short* X;   // [b][mat][plane][ci][ldx]
  int64_t x_b, x_mat, x_plane;
  int ldx;
  unsigned short* Y;         // planes out [b][mat][plane][co][ldy] (hidden layers)
  int64_t y_b, y_mat, y_plane;
  int ldy;
  float* S;                  // fp32 out (output layer): Re rows at S + b*s_b, Im at + s_im
  int64_t s_b, s_im;
  int ldS;
  int co, ci, N;
  int tiles_m, tiles_n;
  int relu;
  // BF32 (layer 0): X given as fp32 rows instead of 3M planes: Re rows at
  // Xf + b*xf_b, Im rows at + xf_im, ld ldxf; split (and Re + Im formed) while staged
  const float* Xf;
  int64_t xf_b, xf_im;
  int ldxf;
  // LAY (tiled activations): k-tiles per column tile of the planes input / output
  // (round_up(rows, 128) / 16 of the producing layer)
  int kt_in, kt_out;
  // x3h (NP = 2) scaling, all powers of two: *lscale multiplies the accumulators
  // before the epilogue (layer constant: weight scale undone, output range set);
  // colscale[b * cs_b + column] multiplies the fp32 B values while staged (BF32 layer
  // 0: the per-column input scale) or the outputs in the epilogue (output layer)
  const float* lscale;
  const float* colscale;
  int64_t cs_b;
};

// Tiled 3M activations (LAY, MSFNO_X6C_TILED): the planes of a layer's activation
// stored as the LDS image of the next layer's B stages, [b][tn][kt][mat*3+plane][16
// rows][128 columns, 8-column chunks XOR-swizzled by 4 (row & 3)]: one k-tile stage of
// one column tile is a contiguous 36 KB, so the B DMA reads whole 1-KB pieces and the
// epilogue writes whole rows of 256 B (the row layout reads 4 rows of 256 B at a
// 130-KB stride per piece).  Pad rows (>= co) and columns (>= N) hold 0.
__device__ __forceinline__ int x6c_tile_swz(int r, int c) {
  return ((((c >> 3) ^ (4 * (r & 3)))) << 3) + (c & 7);
}

// x3h scales of the spectral MLP (one workgroup): per layer l a weight scale
// tau_l = 2^(15 - e) for the largest of |Wr|, |Wi|, |Wr + Wi| (= f 2^e, f in
// [0.5, 1)), and the row bound nu_l = max_o sum_i (|Wr| + |Wi|): a layer whose
// inputs are bounded by 2^14 in absolute value (re and im) has outputs bounded by
// nu_l 2^14, which sigma_l = 2^-ceil(log2 nu_l) brings back under 2^14 (so the next
// B operand Xr + Xi stays under 2^15 < 65504).  The hidden layers' epilogue
// multiplier is sigma_l / tau_l; the output layer's 1 / (tau_L prod sigma_l) (the
// per-column input scale of layer 0 is undone separately).  scl[2 l] = tau_l,
// scl[2 l + 1] = the multiplier.
__global__ void spec_scales_x3h_kernel(SpecWeightsX6p a) {
  __shared__ float red_m[256], red_n[256];
  float prod_sigma = 1.f;
  for (int l = 0; l < a.nlayers; ++l) {
    const int ci = a.ci[l], co = a.co[l];
    float m = 0.f, nu = 0.f;
    for (int o = threadIdx.x; o < co; o += blockDim.x) {
      float rsum = 0.f;
      for (int i = 0; i < ci; ++i) {
        const float wr = a.w[l][((int64_t)i * co + o) * 2], wi = a.w[l][((int64_t)i * co + o) * 2 + 1];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(wr), fabsf(wi)), fabsf(wr + wi)));
        rsum += fabsf(wr) + fabsf(wi);
      }
      nu = fmaxf(nu, rsum);
    }
    red_m[threadIdx.x] = m;
    red_n[threadIdx.x] = nu;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) {
        red_m[threadIdx.x] = fmaxf(red_m[threadIdx.x], red_m[threadIdx.x + s]);
        red_n[threadIdx.x] = fmaxf(red_n[threadIdx.x], red_n[threadIdx.x + s]);
      }
      __syncthreads();
    }
    m = red_m[0];
    nu = red_n[0];
    __syncthreads();
    int e = 0;
    float tau = 1.f;
    if (m > 0.f && isfinite(m)) {
      frexpf(m, &e);
      tau = ldexpf(1.f, 15 - e);
    }
    float sigma = 1.f;
    if (nu > 0.f && isfinite(nu)) sigma = ldexpf(1.f, -(int)ceilf(log2f(nu)));
    const bool last = l == a.nlayers - 1;
    if (threadIdx.x == 0) {
      a.scl[2 * l] = tau;
      a.scl[2 * l + 1] = last ? 1.f / (tau * prod_sigma) : sigma / tau;
    }
    prod_sigma *= sigma;
  }
}

// A image of one layer: Wr, Wi, Ws = Wr + Wi (co x ci each) from the reference
// weight w (ci, co, 2), each split into [plane][kt][Mp][16]; NP = 2: scaled by
// tau_l (a.scl) and split into two fp16 terms
template <int NP = 3>
__global__ void spec_weights_3m_kernel(SpecWeightsX6p a) {
  const int64_t total = a.start[a.nlayers];
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * blockDim.x) {
    int l = 0;
    while (l + 1 < a.nlayers && g >= a.start[l + 1]) ++l;
    const int ci = a.ci[l], co = a.co[l];
    const int Mp = (co + X6C_BM - 1) / X6C_BM * X6C_BM, KT = (ci + X6C_BK - 1) / X6C_BK;
    const int64_t n = (int64_t)Mp * KT * 8;  // pairs per plane
    const int64_t e = g - a.start[l];
    const int mat = (int)(e / n);
    const int64_t f = e - mat * n;
    const int64_t idx = 2 * f;
    const int kt = (int)(idx / ((int64_t)Mp * 16));
    const int rem = (int)(idx - (int64_t)kt * Mp * 16);
    const int o = rem >> 4, k0 = kt * 16 + (rem & 15);
    const float tau = NP == 2 ? a.scl[2 * l] : 1.f;
    float v[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int i = k0 + t;
      float x = 0.f;
      if (o < co && i < ci) {
        const float wr = a.w[l][((int64_t)i * co + o) * 2], wi = a.w[l][((int64_t)i * co + o) * 2 + 1];
        x = mat == 0 ? wr : (mat == 1 ? wi : wr + wi);
      }
      v[t] = x * tau;
    }
    uint32_t t[NP];
    X6CEng<NP>::split(v[0], v[1], t);
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out[l]) + mat * NP * n + f;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) out[pl * n] = t[pl];
  }
}

// S fp32 rows [b][ri][c] (ld ldS) -> 3M planes [b][mat][plane][c][ldx]
// 8 columns per thread: 16-B loads of re and im, 16-B stores of the 9 planes
// (ldS % 4 == 0, ldx % 8 == 0, 16-B aligned bases); the ragged row tail per column
__global__ void split3m_x8_kernel(const float* __restrict__ S, unsigned short* __restrict__ X,
                                  int C, int N, int ldS, int ldx, int64_t x_b, int64_t x_mat,
                                  int64_t x_plane) {
  const int b = blockIdx.y;
  const int c8 = (N + 7) / 8;
  const int64_t n = (int64_t)C * c8;
  const float* Sb = S + (int64_t)b * 2 * C * ldS;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e / c8), col = 8 * (int)(e - (int64_t)c * c8);
    const float* re = Sb + (int64_t)c * ldS + col;
    const float* im = Sb + (int64_t)(C + c) * ldS + col;
    float r[8], i[8];
    if (col + 8 <= N) {
      const float4 r0 = *reinterpret_cast<const float4*>(re), r1 = *reinterpret_cast<const float4*>(re + 4);
      const float4 i0 = *reinterpret_cast<const float4*>(im), i1 = *reinterpret_cast<const float4*>(im + 4);
      r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w; r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
      i[0] = i0.x; i[1] = i0.y; i[2] = i0.z; i[3] = i0.w; i[4] = i1.x; i[5] = i1.y; i[6] = i1.z; i[7] = i1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        r[q] = col + q < N ? re[q] : 0.f;
        i[q] = col + q < N ? im[q] : 0.f;
      }
    }
    unsigned short* d = X + b * x_b + (int64_t)c * ldx + col;
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      uint32_t t[3][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float a0 = mat == 0 ? r[2 * q] : (mat == 1 ? i[2 * q] : r[2 * q] + i[2 * q]);
        const float a1 = mat == 0 ? r[2 * q + 1] : (mat == 1 ? i[2 * q + 1] : r[2 * q + 1] + i[2 * q + 1]);
        split2(a0, a1, t[0][q], t[1][q], t[2][q]);
      }
      unsigned short* q0 = d + mat * x_mat;
      // columns past N are written as the split of 0 (the planes' pad columns)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        *reinterpret_cast<uint4*>(q0 + pl * x_plane) = make_uint4(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
    }
  }
}

__global__ void split3m_kernel(const float* __restrict__ S, unsigned short* __restrict__ X, int C,
                               int N, int ldS, int ldx, int64_t x_b, int64_t x_mat,
                               int64_t x_plane) {
  const int b = blockIdx.y;
  const int cp = (N + 1) / 2;
  const int64_t n = (int64_t)C * cp;
  const float* Sb = S + (int64_t)b * 2 * C * ldS;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e / cp), col = 2 * (int)(e - (int64_t)c * cp);
    const float* re = Sb + (int64_t)c * ldS + col;
    const float* im = Sb + (int64_t)(C + c) * ldS + col;
    const bool two = col + 1 < N;
    const float r0 = re[0], r1 = two ? re[1] : 0.f;
    const float i0 = im[0], i1 = two ? im[1] : 0.f;
    const float v[3][2] = {{r0, r1}, {i0, i1}, {r0 + i0, r1 + i1}};
    unsigned short* d = X + b * x_b + (int64_t)c * ldx + col;
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      uint32_t t0, t1, t2;
      split2(v[mat][0], v[mat][1], t0, t1, t2);
      unsigned short* q = d + mat * x_mat;
      if (two) {
        *reinterpret_cast<uint32_t*>(q) = t0;
        *reinterpret_cast<uint32_t*>(q + x_plane) = t1;
        *reinterpret_cast<uint32_t*>(q + 2 * x_plane) = t2;
      } else {
        q[0] = (unsigned short)t0;
        q[x_plane] = (unsigned short)t1;
        q[2 * x_plane] = (unsigned short)t2;
      }
    }
  }
}

// WGM x WGN waves: 4 x 2 (32 x 64 per wave, two waves per SIMD) or 2 x 2 (64 x 64
// per wave, one wave per SIMD: a third fewer LDS fragment reads per MFMA)
// BF32: the B operand arrives as fp32 Re / Im rows (layer 0, straight from the
// forward Legendre GEMM): each thread loads a float4 of Re and of Im for the next
// k-tile before the current one's MFMAs, and after them forms Re + Im, splits the
// three into bf16x3 and writes the nine B planes into the LDS stage; only A is DMA'd
// DBG (diagnostic timing builds only, wrong results; MSFNO_X6C_DBG): 1 no vmcnt wait
// for the k-tile DMA, 2 no DMA in the loop at all (stale stages), 4 no MFMAs
// LAY: bit 1 = B planes read in the tiled layout, bit 2 = planes written tiled
// NS: LDS stages (2; 3 for the x3h DMA-fed layers: two k-tiles in flight, 144 KB)
// BM_: tile rows (128, or 64 for grids that would not fill the chip: the 120 x 240
// blocks of the network, N = 7,260 modes, 57 column tiles)
template <bool PLANES_OUT, int WGM = 4, int WGN = 2, bool BF32 = false, int DBG = 0, int LAY = 0,
          int NP = 3, int NS = 2, int BM_ = X6C_BM>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_x6c_kernel(X6CParams p) {
  constexpr int BM = BM_, BN = X6C_BN, BK = X6C_BK;
  constexpr int NW = WGM * WGN;
  constexpr int NMP = 3 * NP;                 // matrix-planes per operand
  constexpr int APC = (BM / 32) * NMP;        // A pieces (1 KB: 32 rows x 16 k) per k-tile
  constexpr int BPC = 4 * NMP;                // B pieces (1 KB: 4 k rows x 128) per k-tile
  static_assert(BM % 32 == 0 && X6C_BM % BM == 0, "tile rows");
  static_assert(BF32 || (APC + BPC) % NW == 0, "DMA pieces per wave");
  constexpr int NPC = BF32 ? (APC + NW - 1) / NW : (APC + BPC) / NW;  // DMA pieces per wave and k-tile
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int A_PLANE = BM * BK, B_PLANE = BK * BN;  // 16-bit elements per matrix plane
  constexpr int A_ALL = NMP * A_PLANE;
  constexpr int STAGE = NMP * (A_PLANE + B_PLANE);      // 72 KB (x6) / 48 KB (x3h)
  constexpr int NSTAGE = NS;
  static_assert(NS == 2 || (NS == 3 && !BF32 && DBG == 0), "three stages: DMA-fed B only");
  constexpr int RING_BYTES = NSTAGE * STAGE * 2;
  constexpr int EPI_BYTES = 32 * WGM * (BN + 8) * 4;
  constexpr int LDS_BYTES = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  static_assert(STAGE * 2 == (APC + BPC) * 1024, "stage = A + B pieces of 1 KB");
  // the x3h engine writes hidden planes in the tiled layout only
  static_assert(NP == 3 || !PLANES_OUT || (LAY & 2) != 0, "x3h: tiled plane output only");
  typedef typename X6CEng<NP>::frag Frag;
  __shared__ __attribute__((aligned(16))) char lds_raw[LDS_BYTES];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int half = lane >> 5, l32 = lane & 31;

  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin % p.tiles_m, tn = lin / p.tiles_m;
  const int z = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const int K = p.ci, N = p.N, ldx = p.ldx;
  const int nk = (K + BK - 1) / BK;
  const unsigned short* X = p.X + z * p.x_b;

  // LDS-DMA pieces c = wave + NW q (q < NPC): c < APC -> A (matrix-plane c / 4, rows
  // 32 (c % 4) ..), else B (matrix-plane (c - APC) / 4, k rows 4 ((c - APC) % 4) ..)
  const unsigned short* src[NPC];
  int dst[NPC];
  int brow[NPC];  // B: k row of this lane within the k-tile (-1 for A pieces)
#pragma unroll
  for (int q = 0; q < NPC; ++q) {
    const int c = wave + NW * q;
    if (BF32 && c >= APC) {  // no B pieces; this slot idles
      src[q] = nullptr;
      dst[q] = 0;
      brow[q] = -2;
    } else if (c < APC) {
      const int mp = c / (BM / 32), mb = c % (BM / 32);
      const int mat = mp / NP, pl = mp - NP * mat;
      const int m = 32 * mb + (lane >> 1);
      const int h = (lane & 1) ^ ((m >> 3) & 1);
      src[q] = p.Aw + mat * p.a_mat + pl * p.a_plane + (int64_t)(m0 + m) * 16 + 8 * h;
      dst[q] = mp * A_PLANE + mb * 32 * BK;
      brow[q] = -1;
    } else {
      const int cb = c - APC;
      const int mp = cb >> 2, rq = cb & 3;
      const int mat = mp / NP, pl = mp - NP * mat;
      const int row = 4 * rq + (lane >> 4);
      const int gu = (lane & 15) ^ (4 * (row & 3));
      if constexpr ((LAY & 1) != 0)
        src[q] = X + ((int64_t)tn * p.kt_in * NMP + mp) * B_PLANE + rq * 4 * BN + 8 * (lane & 15) +
                 BN * (lane >> 4);
      else
        src[q] = X + mat * p.x_mat + pl * p.x_plane + min(n0 + 8 * gu, ldx - 8);
      dst[q] = A_ALL + mp * B_PLANE + rq * 4 * BN;
      brow[q] = row;
    }
  }
  const int64_t a_kstride = (int64_t)p.Mp * 16;
  const uint32_t ring_lds = lds_addr(ring);
  auto issue = [&](int kt, int st) {
    const uint32_t base = ring_lds + (uint32_t)(st * STAGE * 2);
#pragma unroll
    for (int q = 0; q < NPC; ++q) {
      if (BF32 && brow[q] == -2) continue;
      const unsigned short* g = brow[q] < 0
                                    ? src[q] + kt * a_kstride
                                    : ((LAY & 1) ? src[q] + (int64_t)kt * NMP * B_PLANE
                                                 : src[q] + (int64_t)min(kt * BK + brow[q], K - 1) * ldx);
      glds16(g, base + (uint32_t)(dst[q] * 2));
    }
  };
  // BF32 B staging: thread -> (k row, 4 columns); NW * 64 threads cover 16 x 128
  static_assert(!BF32 || NW * 64 * 4 == BK * BN, "BF32 staging: one float4 per thread");
  const int brow_f = tid / (BN / 4), bcol_f = 4 * (tid % (BN / 4));
  const float* Xf = BF32 ? p.Xf + z * p.xf_b : nullptr;
  float4 fre = make_float4(0.f, 0.f, 0.f, 0.f), fim = fre;
  float csb[4] = {1.f, 1.f, 1.f, 1.f};  // x3h BF32: per-column input scale of this thread's columns
  if constexpr (BF32 && NP == 2) {
    if (p.colscale) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        csb[e] = p.colscale[z * p.cs_b + min(n0 + bcol_f + e, N - 1)];
    }
  }
  static_assert(!BF32 || (LAY & 1) == 0, "BF32: fp32 rows in");
  auto load_bf = [&](int kt) {
    const int k = kt * BK + brow_f;
    const int kc = min(k, K - 1);
    const int col = min(n0 + bcol_f, (N - 1) & ~3);
    const float* r = Xf + (int64_t)kc * p.ldxf + col;
    fre = *reinterpret_cast<const float4*>(r);
    fim = *reinterpret_cast<const float4*>(r + p.xf_im);
  };
  auto store_bf = [&](int kt, int st) {
    const int k = kt * BK + brow_f;
    float re[4] = {fre.x, fre.y, fre.z, fre.w}, im[4] = {fim.x, fim.y, fim.z, fim.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // zero what is out of range (K tail, ragged N)
      const bool ok = k < K && n0 + bcol_f + e < N;
      re[e] = ok ? re[e] * csb[e] : 0.f;  // x3h: the column's input scale (else 1)
      im[e] = ok ? im[e] * csb[e] : 0.f;
    }
    const float sm[4] = {re[0] + im[0], re[1] + im[1], re[2] + im[2], re[3] + im[3]};
    const float* v[3] = {re, im, sm};
    unsigned short* base = ring + st * STAGE + A_ALL;
    const int u = bcol_f >> 3, h = (bcol_f >> 2) & 1;
    const int off = brow_f * BN + ((u ^ (4 * (brow_f & 3))) << 3) + 4 * h;
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      uint32_t ta[NP], tb[NP];
      X6CEng<NP>::split(v[mat][0], v[mat][1], ta);
      X6CEng<NP>::split(v[mat][2], v[mat][3], tb);
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
        *reinterpret_cast<uint2*>(base + (mat * NP + pl) * B_PLANE + off) = make_uint2(ta[pl], tb[pl]);
    }
  };

  floatx16 acc[3][MT][NT];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][i][j][r] = 0.f;
  int a_off[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * WM + i * 32 + l32;
    a_off[i] = row * BK + 8 * (half ^ ((row >> 3) & 1));
  }
  const int li = lane & 15, g16 = (lane >> 4) & 1;
  const int br = 8 * half + (li >> 2);
  int b_off[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int c = wn * WN + j * 32 + 16 * g16 + 4 * (li & 3);
    b_off[j] = A_ALL + br * BN + (((c >> 3) ^ (4 * (br & 3))) << 3) + (c & 7);
  }
  auto mfma_tile = [&](int st) {
    typedef __attribute__((address_space(3))) s16x4c lds_s16x4;
    const unsigned short* base = ring + st * STAGE;
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      Frag a[MT][NP];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
          a[i][pl] = *reinterpret_cast<const Frag*>(base + (mat * NP + pl) * A_PLANE + a_off[i]);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        Frag b[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
          const unsigned short* q = base + (mat * NP + pl) * B_PLANE + b_off[j];
          const s16x4c lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)q));
          const s16x4c hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)((__attribute__((address_space(3))) unsigned short*)(q + 4 * BN)));
          const s16x8c v = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
          b[pl] = __builtin_bit_cast(Frag, v);
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[mat][i][j] = X6CEng<NP>::prod(a[i], b, acc[mat][i][j]);
      }
    }
  };

  issue(0, 0);
  if constexpr (NS == 3) {
    if (nk > 1) issue(1, 1);
  }
  if constexpr (BF32) {
    load_bf(0);
    store_bf(0, 0);
  }
  if constexpr (NS == 3) {
    // k-tiles kt and kt + 1 in flight at the top of iteration kt: wait for kt only
    // (NPC DMA instructions per wave and k-tile), then refill the stage kt - 1 left
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPC) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) issue(kt + 2, (kt + 2) % 3);
      __builtin_amdgcn_s_setprio(1);
      mfma_tile(kt % 3);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr ((DBG & 1) == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my DMA of k-tile kt landed
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // everyone's landed; stage (kt + 1) & 1 is free
      if (kt + 1 < nk) {
        if constexpr ((DBG & 2) == 0) issue(kt + 1, (kt + 1) & 1);
        if constexpr (BF32) load_bf(kt + 1);  // after the DMA: in-order vmcnt
      }
      __builtin_amdgcn_s_setprio(1);
      if constexpr ((DBG & 4) == 0) mfma_tile(kt & 1);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (BF32) {
        if (kt + 1 < nk) store_bf(kt + 1, (kt + 1) & 1);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // x3h: the layer multiplier (weight scale undone, output range) and, for the fp32
  // output rows of the last layer, the per-column factor (layer 0's input scale undone)
  float mul[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) mul[j] = 1.f;
  if constexpr (NP == 2) {
    const float ls = *p.lscale;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      mul[j] = ls;
      if constexpr (!PLANES_OUT && (LAY & 2) == 0) {
        if (p.colscale) mul[j] *= p.colscale[z * p.cs_b + min(n0 + wn * WN + j * 32 + l32, N - 1)];
      }
    }
  }
  // Re = P1 - P2 (ComplexReLU on hidden layers), Im = P3 - P1 - P2, Ys = Re + Im
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p1 = acc[0][i][j][r] * mul[j], p2 = acc[1][i][j][r] * mul[j],
                    p3 = acc[2][i][j][r] * mul[j];
        float re = p1 - p2;
        const float im = p3 - p1 - p2;
        if (p.relu) re = fmaxf(re, 0.f);
        acc[0][i][j][r] = re;
        acc[1][i][j][r] = im;
        acc[2][i][j][r] = re + im;
      }
  float* lds = reinterpret_cast<float*>(lds_raw);
  GemmParams q{};
  q.vecC = 1;
  if constexpr (PLANES_OUT && (LAY & 2) != 0) {
    // tiled planes: every row and column of the tile (pad rows / columns are 0)
    constexpr int CS_LD = BN + 8;
    unsigned short* Yt = p.Y + z * p.y_b + (int64_t)tn * p.kt_out * NMP * B_PLANE;
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            lds[(wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * CS_LD + wn * WN + j * 32 +
                l32] = acc[mat][i][j][r];
      __syncthreads();
      constexpr int NQ = BM * BN / 4 / (64 * NW);
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int idx = tid + 64 * NW * qq;
        const int lr = idx / (BN / 4), c = 4 * (idx % (BN / 4));
        const float4 v = *reinterpret_cast<const float4*>(lds + lr * CS_LD + c);
        uint32_t ta[NP], tb[NP];
        X6CEng<NP>::split(v.x, v.y, ta);
        X6CEng<NP>::split(v.z, v.w, tb);
        const int m = m0 + lr, r = m & 15;
        unsigned short* d = Yt + ((int64_t)(m >> 4) * NMP + mat * NP) * B_PLANE + r * BN + x6c_tile_swz(r, c);
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
          *reinterpret_cast<uint2*>(d + pl * B_PLANE) = make_uint2(ta[pl], tb[pl]);
      }
      __syncthreads();
    }
  } else if constexpr (PLANES_OUT) {
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      q.Cx = p.Y + mat * p.y_mat;
      q.sC = p.y_b;
      q.sCxp = p.y_plane;
      gemm_epilogue<BM, BN, EPI_PLANES, WGM, WGN, MT, NT, 32, floatx16, false>(
          q, acc[mat], lds, nullptr, nullptr, nullptr, p.co, N, p.ldy, m0, n0, 0);
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int mat = 0; mat < 2; ++mat) {
      float* C = p.S + z * p.s_b + (mat ? p.s_im : 0);
      q.vecC = (p.ldS % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
      gemm_epilogue<BM, BN, 0, WGM, WGN>(q, acc[mat], lds, nullptr, C, nullptr, p.co, N, p.ldS,
                                         m0, n0, 0);
      __syncthreads();
    }
  }
}

// ---- host ---------------------------------------------------------------------

size_t gemm_x6c_weight_bytes(int co, int ci) {
  const int64_t Mp = round_up(co, X6C_BM), Kp = round_up(ci, X6C_BK);
  return (size_t)round_up(3 * 3 * Mp * Kp * 2, 256);
}

size_t spec_weights_3m_layout(SpecWeightsX6p& a) {
  size_t bytes = 0;
  a.start[0] = 0;
  for (int l = 0; l < a.nlayers; ++l) {
    a.start[l + 1] = a.start[l] + 3 * round_up(a.co[l], X6C_BM) * cdiv(a.ci[l], X6C_BK) * 8;
    bytes += gemm_x6c_weight_bytes(a.co[l], a.ci[l]);
  }
  return bytes;
}

int launch_spec_weights_3m(const SpecWeightsX6p& a, hipStream_t s) {
  if (a.nlayers <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(a.start[a.nlayers], 256), 4096);
  hipLaunchKernelGGL(spec_weights_3m_kernel<3>, dim3(blocks), dim3(256), 0, s, a);
  return launch_check("spec_weights_3m");
}

int launch_split3m(const float* S, unsigned short* X, int B, int C, int N, int ldS, int ldx,
                   hipStream_t s) {
  MSFNO_REQUIRE(ldx % 8 == 0, MSFNO_EINVAL, "split3m: ld must be a multiple of 8");
  const int64_t x_plane = (int64_t)C * ldx;
  if (ldS % 4 == 0 && ldx >= (N + 7) / 8 * 8 && ((reinterpret_cast<uintptr_t>(S) | reinterpret_cast<uintptr_t>(X)) & 15) == 0) {
    const int64_t n8 = (int64_t)C * ((N + 7) / 8);
    const int blocks = (int)std::min<int64_t>(cdiv(n8, 256), 4096);
    hipLaunchKernelGGL(split3m_x8_kernel, dim3(blocks, B), dim3(256), 0, s, S, X, C, N, ldS, ldx,
                       9 * x_plane, 3 * x_plane, x_plane);
    return launch_check("split3m");
  }
  const int64_t n = (int64_t)C * ((N + 1) / 2);
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 2048);
  hipLaunchKernelGGL(split3m_kernel, dim3(blocks, B), dim3(256), 0, s, S, X, C, N, ldS, ldx,
                     9 * x_plane, 3 * x_plane, x_plane);
  return launch_check("split3m");
}

// a layer on fp32 input rows (Re at Sin + b*2*ci*ldSin, Im ci rows later), split
// while staged: out 3M planes Y (ld ldy) or fp32 rows [b][re/im][co] of Sout (ld ldSout)
int gemm_x6c_f32b(const unsigned short* Aw, int co, int ci, const float* Sin, int ldSin, int N,
                  unsigned short* Y, int ldy, float* Sout, int ldSout, bool relu, int B,
                  hipStream_t s, bool tiled_out) {
  if (co <= 0 || N <= 0 || B <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(ldSin % 4 == 0 && (reinterpret_cast<uintptr_t>(Sin) & 15) == 0 && ldSin >= N,
                MSFNO_EINVAL, "gemm_x6c_f32b: fp32 rows need ld % 4 == 0 and 16-B alignment");
  MSFNO_REQUIRE((Y != nullptr) != (Sout != nullptr), MSFNO_EINVAL, "gemm_x6c_f32b: one output");
  MSFNO_REQUIRE(!Y || ldy % 8 == 0, MSFNO_EINVAL, "gemm_x6c_f32b: plane ld % 8 != 0");
  X6CParams p{};
  p.Mp = (int)round_up(co, X6C_BM);
  const int KT = (int)cdiv(ci, X6C_BK);
  p.Aw = Aw;
  p.a_plane = (int64_t)p.Mp * KT * 16;
  p.a_mat = 3 * p.a_plane;
  p.Xf = Sin;
  p.xf_b = 2LL * ci * ldSin;
  p.xf_im = (int64_t)ci * ldSin;
  p.ldxf = ldSin;
  p.ldx = 8;  // unused (no B planes)
  p.Y = Y;
  p.y_plane = (int64_t)co * ldy;
  p.y_mat = 3 * p.y_plane;
  p.y_b = 3 * p.y_mat;
  p.ldy = ldy;
  p.S = Sout;
  p.s_b = 2LL * co * ldSout;
  p.s_im = (int64_t)co * ldSout;
  p.ldS = ldSout;
  p.co = co; p.ci = ci; p.N = N;
  p.tiles_m = p.Mp / X6C_BM;
  p.tiles_n = (int)cdiv(N, X6C_BN);
  p.relu = relu ? 1 : 0;
  const dim3 grid(p.tiles_m * p.tiles_n, 1, B);
  if (Y && tiled_out) {
    p.kt_out = p.Mp / 16;
    p.y_b = x6c_tiled_elems(co, N);
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, true, 0, 2>), grid, dim3(512), 0, s, p);
  } else if (Y)
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, true>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_x6c_kernel<false, 4, 2, true>), grid, dim3(512), 0, s, p);
  return launch_check("gemm_x6c_f32b");
}

// elements of one field's tiled 3M activation with `rows` channel rows, N columns
int64_t x6c_tiled_elems(int rows, int N) {
  return cdiv(N, X6C_BN) * round_up(rows, X6C_BM) * 9 * X6C_BN;
}

// one spectral-MLP layer: X (3M planes, ci rows, ld ldx) -> Y (3M planes, co rows,
// ld ldx; relu) or, with S given, fp32 rows [b][re/im][co] of S (ld ldS)
int gemm_x6c(const unsigned short* Aw, int co, int ci, const unsigned short* X, int N, int ldx,
             unsigned short* Y, float* S, int ldS, bool relu, int B, hipStream_t s, int lay) {
  if (co <= 0 || N <= 0 || B <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(ldx % 8 == 0 && ldx >= 8 && (reinterpret_cast<uintptr_t>(X) & 15) == 0,
                MSFNO_EINVAL, "gemm_x6c: X planes need ld % 8 == 0 and 16-B alignment");
  MSFNO_REQUIRE((Y != nullptr) != (S != nullptr), MSFNO_EINVAL, "gemm_x6c: one output");
  X6CParams p{};
  p.Mp = (int)round_up(co, X6C_BM);
  const int KT = (int)cdiv(ci, X6C_BK);
  p.Aw = Aw;
  p.a_plane = (int64_t)p.Mp * KT * 16;
  p.a_mat = 3 * p.a_plane;
  p.X = X;
  p.x_plane = (int64_t)ci * ldx;
  p.x_mat = 3 * p.x_plane;
  p.x_b = 3 * p.x_mat;
  p.ldx = ldx;
  p.Y = Y;
  p.y_plane = (int64_t)co * ldx;
  p.y_mat = 3 * p.y_plane;
  p.y_b = 3 * p.y_mat;
  p.ldy = ldx;
  p.S = S;
  p.s_b = 2LL * co * ldS;
  p.s_im = (int64_t)co * ldS;
  p.ldS = ldS;
  p.co = co; p.ci = ci; p.N = N;
  p.tiles_m = p.Mp / X6C_BM;
  p.tiles_n = (int)cdiv(N, X6C_BN);
  p.relu = relu ? 1 : 0;
  const dim3 grid(p.tiles_m * p.tiles_n, 1, B);
  if (lay) {  // tiled activations (input must be tiled: the hidden layers / output layer)
    MSFNO_REQUIRE((lay & 1) != 0 && ((lay & 2) == 0 || Y), MSFNO_EINVAL, "gemm_x6c: tiled layout");
    p.x_b = x6c_tiled_elems(ci, N);
    p.kt_in = (int)round_up(ci, X6C_BM) / 16;
    p.kt_out = p.Mp / 16;
    if (Y) p.y_b = x6c_tiled_elems(co, N);
    if (Y)
      hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, false, 0, 3>), grid, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_x6c_kernel<false, 4, 2, false, 0, 1>), grid, dim3(512), 0, s, p);
    return launch_check("gemm_x6c");
  }
  // MSFNO_X6C_WAVES: 8 (4 x 2 waves of 32 x 64), 24 (2 x 4 waves of 64 x 32: the same
  // fragment bytes in 20 % fewer LDS read instructions), 4 (2 x 2 waves of 64 x 64)
  static const int waves = [] {
    const char* e = getenv("MSFNO_X6C_WAVES");
    const int v = e ? atoi(e) : 8;
    return (v == 4 || v == 24) ? v : 8;
  }();
  if (waves == 24) {
    if (Y)
      hipLaunchKernelGGL((gemm_x6c_kernel<true, 2, 4>), grid, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_x6c_kernel<false, 2, 4>), grid, dim3(512), 0, s, p);
  } else if (waves == 4) {
    if (Y)
      hipLaunchKernelGGL((gemm_x6c_kernel<true, 2, 2>), grid, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_x6c_kernel<false, 2, 2>), grid, dim3(256), 0, s, p);
  } else {
    static const int dbg = [] {
      const char* e = getenv("MSFNO_X6C_DBG");
      return e ? atoi(e) : 0;
    }();
    if (dbg > 0 && dbg < 8) {
      static void (*const kp[8])(X6CParams) = {
          nullptr, gemm_x6c_kernel<true, 4, 2, false, 1>, gemm_x6c_kernel<true, 4, 2, false, 2>,
          gemm_x6c_kernel<true, 4, 2, false, 3>, gemm_x6c_kernel<true, 4, 2, false, 4>,
          gemm_x6c_kernel<true, 4, 2, false, 5>, gemm_x6c_kernel<true, 4, 2, false, 6>,
          gemm_x6c_kernel<true, 4, 2, false, 7>};
      static void (*const kf[8])(X6CParams) = {
          nullptr, gemm_x6c_kernel<false, 4, 2, false, 1>, gemm_x6c_kernel<false, 4, 2, false, 2>,
          gemm_x6c_kernel<false, 4, 2, false, 3>, gemm_x6c_kernel<false, 4, 2, false, 4>,
          gemm_x6c_kernel<false, 4, 2, false, 5>, gemm_x6c_kernel<false, 4, 2, false, 6>,
          gemm_x6c_kernel<false, 4, 2, false, 7>};
      hipLaunchKernelGGL((Y ? kp[dbg] : kf[dbg]), grid, dim3(512), 0, s, p);
    } else if (Y) {
      hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2>), grid, dim3(512), 0, s, p);
    } else {
      hipLaunchKernelGGL((gemm_x6c_kernel<false, 4, 2>), grid, dim3(512), 0, s, p);
    }
  }
  return launch_check("gemm_x6c");
}

// ---- x3h spectral chain --------------------------------------------------------

int launch_spec_weights_3m_x3h(const SpecWeightsX6p& a, hipStream_t s) {
  if (a.nlayers <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(a.scl, MSFNO_EINVAL, "spec_weights_3m_x3h: no scale array");
  hipLaunchKernelGGL(spec_scales_x3h_kernel, dim3(1), dim3(256), 0, s, a);
  MSFNO_TRY(launch_check("spec_scales_x3h"));
  const int blocks = (int)std::min<int64_t>(cdiv(a.start[a.nlayers], 256), 4096);
  hipLaunchKernelGGL(spec_weights_3m_kernel<2>, dim3(blocks), dim3(256), 0, s, a);
  return launch_check("spec_weights_3m_x3h");
}

// per (b, column n): m = max over the C rows of |Re|, |Im| (S rows [b][re/im][c], ld
// ldS); alpha = 2^(14 - e) with m = f 2^e, f in [0.5, 1) (1 for an all-zero column).
// A workgroup = 64 columns x 16 row slices (a thread: 4 columns by float4, every 16th
// row), the slices combined through LDS: 16-B coalesced loads, 1024+ workgroups at
// the production shape instead of one latency-bound row walk per thread
__global__ __launch_bounds__(256) void spec_colscale_kernel(const float* __restrict__ S, int C, int N,
                                                            int ldS, float* __restrict__ cs,
                                                            int ldcs, int B) {
  __shared__ float4 red[16][16];
  const int b = blockIdx.y;
  const int cg = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + 4 * cg;
  const float* p = S + (int64_t)b * 2 * C * ldS;
  float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n + 3 < N && (ldS & 3) == 0) {
#pragma unroll 4
    for (int r = sl; r < 2 * C; r += 16) {
      const float4 v = *reinterpret_cast<const float4*>(p + (int64_t)r * ldS + n);
      m.x = fmaxf(m.x, fabsf(v.x)); m.y = fmaxf(m.y, fabsf(v.y));
      m.z = fmaxf(m.z, fabsf(v.z)); m.w = fmaxf(m.w, fabsf(v.w));
    }
  } else if (n < N) {
    for (int r = sl; r < 2 * C; r += 16) {
      const float* q = p + (int64_t)r * ldS + n;
      m.x = fmaxf(m.x, fabsf(q[0]));
      if (n + 1 < N) m.y = fmaxf(m.y, fabsf(q[1]));
      if (n + 2 < N) m.z = fmaxf(m.z, fabsf(q[2]));
      if (n + 3 < N) m.w = fmaxf(m.w, fabsf(q[3]));
    }
  }
  red[sl][cg] = m;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int c4 = threadIdx.x >> 2, e = threadIdx.x & 3;
  float mx = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const float4 v = red[t][c4];
    mx = fmaxf(mx, e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w)));
  }
  const int col = blockIdx.x * 64 + threadIdx.x;
  if (col >= ldcs) return;
  float a = 1.f;
  if (col < N && mx > 0.f && isfinite(mx)) {
    int ex;
    frexpf(mx, &ex);
    a = ldexpf(1.f, 14 - ex);
  }
  cs[(int64_t)b * ldcs + col] = a;
  cs[(int64_t)(B + b) * ldcs + col] = 1.f / a;
}

int launch_spec_colscale(const float* S, int B, int C, int N, int ldS, float* cs, int ldcs,
                         hipStream_t s) {
  if (B <= 0 || N <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(cs && ldcs >= N && B <= 65535, MSFNO_EINVAL, "spec_colscale: bad arguments");
  hipLaunchKernelGGL(spec_colscale_kernel, dim3((unsigned)cdiv(ldcs, 64), (unsigned)B), dim3(256),
                     0, s, S, C, N, ldS, cs, ldcs, B);
  return launch_check("spec_colscale");
}

int64_t x3c_tiled_elems(int rows, int N) {
  return cdiv(N, X6C_BN) * round_up(rows, X6C_BM) * 6 * X6C_BN;
}

int gemm_x3c(const unsigned short* Aw, int co, int ci, const float* Sin, int ldSin,
             const unsigned short* X, int N, unsigned short* Y, float* Sout, int ldSout,
             bool relu, const float* lscale, const float* colscale, int64_t cs_b, int B,
             hipStream_t s) {
  if (co <= 0 || N <= 0 || B <= 0) return MSFNO_OK;
  MSFNO_REQUIRE((Sin != nullptr) != (X != nullptr), MSFNO_EINVAL, "gemm_x3c: one input");
  MSFNO_REQUIRE((Y != nullptr) != (Sout != nullptr), MSFNO_EINVAL, "gemm_x3c: one output");
  MSFNO_REQUIRE(lscale, MSFNO_EINVAL, "gemm_x3c: no layer scale");
  MSFNO_REQUIRE(!Sin || (ldSin % 4 == 0 && ldSin >= N && (reinterpret_cast<uintptr_t>(Sin) & 15) == 0),
                MSFNO_EINVAL, "gemm_x3c: fp32 rows need ld % 4 == 0 and 16-B alignment");
  MSFNO_REQUIRE(!(Sin && Sout), MSFNO_EINVAL, "gemm_x3c: an fp32 layer writes planes");
  X6CParams p{};
  p.Mp = (int)round_up(co, X6C_BM);
  const int KT = (int)cdiv(ci, X6C_BK);
  p.Aw = Aw;
  p.a_plane = (int64_t)p.Mp * KT * 16;
  p.a_mat = 2 * p.a_plane;
  p.Xf = Sin;
  p.xf_b = 2LL * ci * ldSin;
  p.xf_im = (int64_t)ci * ldSin;
  p.ldxf = ldSin;
  p.X = X;
  p.x_b = x3c_tiled_elems(ci, N);
  p.ldx = 8;
  p.kt_in = (int)round_up(ci, X6C_BM) / 16;
  p.Y = Y;
  p.y_b = x3c_tiled_elems(co, N);
  p.kt_out = p.Mp / 16;
  p.S = Sout;
  p.s_b = 2LL * co * ldSout;
  p.s_im = (int64_t)co * ldSout;
  p.ldS = ldSout;
  p.co = co; p.ci = ci; p.N = N;
  p.tiles_m = p.Mp / X6C_BM;
  p.tiles_n = (int)cdiv(N, X6C_BN);
  p.relu = relu ? 1 : 0;
  p.lscale = lscale;
  p.colscale = colscale;
  p.cs_b = cs_b;
  const dim3 grid(p.tiles_m * p.tiles_n, 1, B);
  // three LDS stages for the DMA-fed layers (two k-tiles in flight): layers 1/2
  // 0.51 -> 0.49 ms, output 0.31 -> 0.29 ms (two interleaved pairs); MSFNO_X3C_NS=2
  // keeps two (A/B)
  static const int ns = [] {
    const char* e = getenv("MSFNO_X3C_NS");
    return (e && e[0] == '2') ? 2 : 3;
  }();
  // grids that would not fill the chip twice (the network's 120 x 240 blocks: 57 column
  // tiles) take 64-row tiles of four waves, two stages, two workgroups per CU
  // (MSFNO_X3C_BM64=0 keeps the 128-row tiles; 2 takes 64 rows for every DMA-fed layer:
  // hidden layers 0.65 vs 0.54 ms in-block, the output layer no faster once it is timed
  // beside the same side-stream skip: 0.293 ms with 64 rows in profiles/r06_v vs 0.292
  // with 128 in profiles/r06_t/ab_bm64.txt)
  static const int bm64_on = [] {
    const char* e = getenv("MSFNO_X3C_BM64");
    return e ? atoi(e) : 1;
  }();
  if (!Sin && bm64_on && ((int64_t)p.tiles_m * p.tiles_n * B < 2 * 256 || bm64_on == 2)) {
    p.tiles_m = p.Mp / 64;
    const dim3 g64(p.tiles_m * p.tiles_n, 1, B);
    if (Y)
      hipLaunchKernelGGL((gemm_x6c_kernel<true, 2, 2, false, 0, 3, 2, 2, 64>), g64, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_x6c_kernel<false, 2, 2, false, 0, 1, 2, 2, 64>), g64, dim3(256), 0, s, p);
    return launch_check("gemm_x3c");
  }
  // layer 0 (fp32 rows in) on the small grids too: 64-row tiles, 8 waves of 32 x 32 (the
  // fp32 staging needs 512 threads), two stages, two workgroups per CU: config 3 131.7 /
  // 132.3 / 132.1 vs 131.3 / 131.8 / 131.5 steps/s (three interleaved pairs,
  // profiles/r06_ac; MSFNO_X3C_L0_BM64=0 keeps the 128-row tiles)
  static const bool l0_bm64 = [] {
    const char* e = getenv("MSFNO_X3C_L0_BM64");
    return !(e && e[0] == '0');
  }();
  if (Sin && l0_bm64 && bm64_on && (int64_t)p.tiles_m * p.tiles_n * B < 2 * 256) {
    p.tiles_m = p.Mp / 64;
    const dim3 g64(p.tiles_m * p.tiles_n, 1, B);
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 2, 4, true, 0, 2, 2, 2, 64>), g64, dim3(512), 0, s, p);
    return launch_check("gemm_x3c");
  }
  if (Sin)
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, true, 0, 2, 2>), grid, dim3(512), 0, s, p);
  else if (Y && ns == 3)
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, false, 0, 3, 2, 3>), grid, dim3(512), 0, s, p);
  else if (Y)
    hipLaunchKernelGGL((gemm_x6c_kernel<true, 4, 2, false, 0, 3, 2>), grid, dim3(512), 0, s, p);
  else if (ns == 3)
    hipLaunchKernelGGL((gemm_x6c_kernel<false, 4, 2, false, 0, 1, 2, 3>), grid, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_x6c_kernel<false, 4, 2, false, 0, 1, 2>), grid, dim3(512), 0, s, p);
  return launch_check("gemm_x3c");
}

}  // namespace msfno
