// Fused block MLP on the "x3h" engine (gfx950): out = W2·GELU(W1·(a ⊙ x1 + t) + b1)
// + b2 + resid, C = 256, H = 512, hidden activation on-chip — the tiling of
// the round-2 MLP re-tiled (16x16x32 MFMAs, 16 pixels per wave, 64 per workgroup, two
// workgroups per CU, x1 straight from global memory into registers) with fp32
// emulated by TWO fp16 terms instead of three bf16 ones:
//
//   v = v0 + v1,  v0 = fp16(v) (RNE), v1 = fp16(v - v0)   (|v - v0 - v1| <= 2^-22 |v|)
//   a·b ~= a1·b0 + a0·b1 + a0·b0     (three fp16 MFMAs, fp32 accumulation; a1·b1 and
//                                     the representation residuals are O(2^-22))
//
// (the split of Ootomo & Yokota, "Recovering single precision accuracy from Tensor
// Cores while surpassing the FP32 theoretical peak performance", 2022).  Products of
// fp16 values are exact in fp32, so the only errors beyond an fp32 GEMM's own
// accumulation rounding are the O(2^-22) representation terms; measured against
// fp64 the GEMM error equals that of the fp32-MFMA and x6 engines (DESIGN.md §4,
// tests/test_gpu_x3h.py).  Half the MFMAs of x6 (the x6 kernels sit at the chip's
// sustained bf16 MFMA rate: MFMA-busy × clock is the same for every x6 kernel,
// DESIGN.md §8), two planes instead of three (a third less weight stream and
// register image).
//
// Range: fp16 holds |v| < 65504.  Every operand is scaled by exact powers of two chosen
// from a bound, so nothing overflows whatever the weights or the data:
//   - weights: every W1 row and every row of W2' = W2 · diag(1 / eta) (below) so that
//     its largest entry lies in [2^14, 2^15), undone in fp32 after the contraction;
//   - fc1 input x^ = a ⊙ x1 + t: per field by xi_b = 2^(14 - e), where
//     B_b = max_c abound[b][c] = f 2^e and abound = |a| sqrt(M2) + |a mu + t| >= |x^|
//     (chan_affine, from the norm1 statistics: |x1 - mu| <= sqrt(M2));
//   - hidden h_j = GELU(z_j), |h_j| <= |z_j| <= ||W1_j||_1 B_b + |b1_j|
//     <= L_j (B_b + 1), L_j = max(||W1_j||_1, |b1_j|): h is multiplied by
//     eta_j = 2^-ceil(log2 L_j) (from the weights, folded into W2's columns) and by
//     eta_b = 2^(14 - e'), B_b + 1 = f' 2^e' (per field), so |h'| < 2^14; the output
//     is unscaled by 1 / eta_b with W2's row scales.
// A term far below its bound keeps the bound's absolute precision (2^-38 of it), far
// under the fp32 rounding of the sums it enters.
//
// Slices (the 24-KB bf16x3 slices of mlp_fused.hip become 16 KB):
//   W1(j,kh): hidden rows 32j..+31, channels 128kh..+127: [pl 2][ks 4][t 2][r 16][32]
//   W2(j,oh): out rows 128oh..+127, hidden block j:       [pl 2][ot 8][r 16][32 (perm)]
// ring of four 16-KB slots; image = 64 slices, then the row scales (inverse) of W1
// (512) and W2' (256), then eta (512), as fp32.
#include "dma.h"
#include "gemm_common.h"
#include "kernels.h"

#include <cstdio>
#include <string>
#include <vector>
#include <type_traits>

namespace msfno {

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int MH_C = 256, MH_H = 512;
constexpr int MH_WAVES = 4;
constexpr int MH_HB = MH_H / 32;                    // hidden blocks
constexpr int MH_PLANE = 4096;                      // fp16 per plane within a slice
constexpr int MH_SLICE = 2 * MH_PLANE;              // fp16 per 16-KB slice
constexpr int MH_NS = 4;                            // ring slots
constexpr int MH_NSLICE = 4 * MH_HB;                // slices per tile
constexpr int64_t MH_IMG_ELEMS = (int64_t)MH_NSLICE * MH_SLICE;  // before the scales

struct MlpHParams {
  const float* x1;      // [B][C][P]
  const float* scale;   // [B][C]  x1 affine (norm1 + FiLM): a
  const float* shift;   // [B][C]  t
  const float* resid;   // [B][C][P] or null
  float* out;           // [B][C][P]
  const unsigned short* w1img;  // [HB][2 kh] slices
  const unsigned short* w2img;  // [HB][2 oh] slices
  const float* inv_s1;  // [H] 1 / (W1 row scale)
  const float* inv_s2;  // [C] 1 / (W2 row scale)
  const float* eta;     // [H] hidden-row scales eta_j (folded into W2's columns)
  const float* abound;  // [B][C] bound of |a ⊙ x1 + t| per channel
  const float* b1;      // [H]
  const float* b2;      // [C] or null
  int64_t P;
  int tiles_per_field;
  uint64_t* trace;      // MSFNO_MH_TRACE: 5 words per workgroup, or null
};

// 2^(t - e) for v = f 2^e (f in [0.5, 1)): maps v below 2^t; 1 for v = 0 / non-finite
__device__ __forceinline__ float pow2_below(float v, int t) {
  if (!(v > 0.f) || !isfinite(v)) return 1.f;
  int e;
  frexpf(v, &e);
  return ldexpf(1.f, min(max(t - e, -120), 120));
}

__host__ __device__ __forceinline__ int mh_swz(int r) { return ((r >> 2) & 1) << 1; }

__host__ __device__ __forceinline__ int mh_perm(int kappa) {
  const int g = kappa >> 3, e = kappa & 7;
  return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4);
}

// (a, b) -> packed fp16x2 terms h0 + h1 (RNE; v_cvt_pk_f16_f32)
__device__ __forceinline__ void split2h(float a, float b, uint32_t& t0, uint32_t& t1) {
  const f2v v = {a, b};
  const half2v h0 = __builtin_convertvector(v, half2v);
  const f2v r = v - __builtin_convertvector(h0, f2v);
  const half2v h1 = __builtin_convertvector(r, half2v);
  t0 = __builtin_bit_cast(uint32_t, h0);
  t1 = __builtin_bit_cast(uint32_t, h1);
}

__device__ __forceinline__ half8 mh_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(half8, make_uint4(a, b, c, d));
}

// eta_j = 2^-ceil(log2 L_j), L_j = max(||W1_j||_1, |b1_j|): L_j eta_j <= 1
__global__ void mh_eta_kernel(const float* __restrict__ W1, const float* __restrict__ b1,
                              float* __restrict__ eta) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= MH_H) return;
  const float* row = W1 + (int64_t)r * MH_C;
  double l1 = 0.0;
  for (int k = 0; k < MH_C; ++k) l1 += fabs((double)row[k]);
  const double L = fmax(l1, b1 ? fabs((double)b1[r]) : 0.0) * (1.0 + 1e-6);
  float e = 1.f;
  if (L > 0.0 && L < 1e30) {
    int x;
    frexp(L, &x);  // L = f 2^x, f in [0.5, 1): L 2^-x < 1
    e = (float)ldexp(1.0, min(max(-x, -120), 120));
  }
  eta[r] = e;
}

// row scales: 2^(15 - e) with max |row| = f 2^e, f in [0.5, 1) -> max scaled in [2^14, 2^15);
// the W2 rows taken as W2' = W2 diag(1 / eta)
__global__ void mh_scale_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                const float* __restrict__ eta, float* __restrict__ s1,
                                float* __restrict__ s2) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= MH_H + MH_C) return;
  const bool first = r < MH_H;
  const float* row = first ? W1 + (int64_t)r * MH_C : W2 + (int64_t)(r - MH_H) * MH_H;
  const int n = first ? MH_C : MH_H;
  float m = 0.f;
  for (int k = 0; k < n; ++k) m = fmaxf(m, fabsf(first ? row[k] : row[k] / eta[k]));
  float sc = 1.f;
  if (m > 0.f && isfinite(m)) {
    int e;
    frexpf(m, &e);
    sc = ldexpf(1.f, 15 - e);
  }
  if (first) s1[r] = sc; else s2[r - MH_H] = sc;
}

// W1 (H x C fp32) · diag(s1) -> [j][kh][pl][ks][t][r][32]
__global__ void mh_w1_image_kernel(const float* __restrict__ W1, const float* __restrict__ s1,
                                   unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)MH_HB * 2 * 4 * 2 * 16 * 16;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 15);
    const int r = (int)((e >> 4) & 15);
    const int t = (int)((e >> 8) & 1);
    const int ks = (int)((e >> 9) & 3);
    const int kh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;
    const int g = (kk >> 3) ^ mh_swz(r);
    const int k = 128 * kh + 32 * ks + 8 * g + (kk & 7);
    const int row = 32 * j + 16 * t + r;
    const float* src = W1 + (int64_t)row * MH_C + k;
    const float sc = s1[row];
    uint32_t t0, t1;
    split2h(src[0] * sc, src[1] * sc, t0, t1);
    uint32_t* o = reinterpret_cast<uint32_t*>(
        img + (int64_t)(j * 2 + kh) * MH_SLICE + ((ks * 2 + t) * 16 + r) * 32 + kk);
    o[0] = t0;
    o[MH_PLANE / 2] = t1;
  }
}

// W2' (C x H fp32, W2 diag(1 / eta)) · row scales -> [j][oh][pl][ot][r][32], hidden index
// permuted by mh_perm
__global__ void mh_w2_image_kernel(const float* __restrict__ W2, const float* __restrict__ eta,
                                   const float* __restrict__ s2, unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)MH_HB * 2 * 8 * 16 * 16;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 15);
    const int r = (int)((e >> 4) & 15);
    const int ot = (int)((e >> 8) & 7);
    const int oh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;
    const int kap = 8 * ((kk >> 3) ^ mh_swz(r)) + (kk & 7);
    const int orow = 128 * oh + 16 * ot + r;
    const float* row = W2 + (int64_t)orow * MH_H + 32 * j;
    const float* er = eta + 32 * j;
    const float sc = s2[orow];
    const int k0 = mh_perm(kap), k1 = mh_perm(kap + 1);
    uint32_t t0, t1;
    split2h(row[k0] / er[k0] * sc, row[k1] / er[k1] * sc, t0, t1);
    uint32_t* o = reinterpret_cast<uint32_t*>(
        img + (int64_t)(j * 2 + oh) * MH_SLICE + (ot * 16 + r) * 32 + kk);
    o[0] = t0;
    o[MH_PLANE / 2] = t1;
  }
}

// 1 / scale, in place
__global__ void mh_invert_kernel(float* __restrict__ s) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < MH_H + MH_C) s[r] = 1.f / s[r];
}

__device__ __forceinline__ const unsigned short* mh_slice_src(const MlpHParams& p, int q) {
  if (q < 2) return p.w1img + (int64_t)q * MH_SLICE;
  if (q >= MH_NSLICE - 2)
    return p.w2img + (int64_t)(2 * (MH_HB - 1) + (q - (MH_NSLICE - 2))) * MH_SLICE;
  const int j = 1 + ((q - 2) >> 2), r = (q - 2) & 3;
  return r < 2 ? p.w1img + (int64_t)(2 * j + r) * MH_SLICE
               : p.w2img + (int64_t)(2 * (j - 1) + (r - 2)) * MH_SLICE;
}

// four wave-instructions (one m0 save / restore): lane l copies 16 B from sbase +
// voff[i] to LDS byte lds + i * LDS_STEP + 16 l (dma.h glds16x6, four pieces)
template <int LDS_STEP>
__device__ __forceinline__ void glds16x4(uint64_t sbase, const uint32_t (&voff)[4], uint32_t lds) {
  unsigned keep;
  sbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sbase >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %1\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %1\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %1\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, %1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(sbase), "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]), "s"(lds),
        "i"(LDS_STEP)
      : "memory", "scc");
}



// The block MLP for one tile of 64 pixels (4 waves of 16; two workgroups per CU).
// Prologue: the weight slices 0..3 go in flight by LDS-DMA; the field's range scalars
// (xi_b from max_c abound, eta_b from B_b + 1) are reduced over the workgroup; x1 of the
// wave's 16 pixels is normalised (a ⊙ x1 + t, times xi_b) and split into fp16x2 B
// fragments kept in registers.  Then 64 slice steps: W1(j, 0..1) into the fc1
// accumulator of block j while block j - 1 is unscaled, + b1, GELU'd, scaled by
// eta_j eta_b and split into fc2's B fragment (in place: mf_perm orders W2's columns),
// W2(j - 1, 0..1) into the 256 x 16 output accumulators.  Epilogue: unscale + b2 +
// residual, one store per output.
constexpr int MH_LDS = MH_NS * MH_SLICE * 2 + (3 * MH_H + 2 * MH_C + 8) * 4;

// BUF: x1, residual and output addressed as raw buffers (32-bit lane offsets, SGPR row
// offsets; the host takes it when a field's C x P fp32 plane is below 2 GB)
template <int AHEAD, bool TRACE, bool BUF, bool ILV = false>
__device__ __forceinline__ void mlp_fused_h_tile(const MlpHParams& p, int lin, char* lds_raw) {
  constexpr int W = MH_WAVES, NS = MH_NS;
  constexpr int RING_BYTES = NS * MH_SLICE * 2;
  constexpr int TPX = 16 * W;  // pixels per workgroup tile
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const b1s = reinterpret_cast<float*>(lds_raw + RING_BYTES);
  float* const is1s = b1s + MH_H;
  float* const hss = is1s + MH_H;  // eta_j eta_b
  float* const b2s = hss + MH_H;   // the epilogue's vectors (no global loads there)
  float* const is2s = b2s + MH_C;
  float* const red = is2s + MH_C;  // per-wave maxima of abound

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int z = lin / p.tiles_per_field;
  uint64_t tr[3] = {0, 0, 0};
  if constexpr (TRACE) tr[0] = __builtin_amdgcn_s_memrealtime();
  const int64_t P = p.P;
  const int64_t px = (int64_t)(lin - z * p.tiles_per_field) * TPX + 16 * wave + r16;

  // ---- slices 0..NS-1 in flight --------------------------------------------------------
  const uint32_t ring_lds = lds_addr(ring);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  uint32_t piece_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) piece_off[i] = (uint32_t)(i * W * 1024 + lane * 16);
  auto issue = [&](int q) {
    const uint64_t src = reinterpret_cast<uint64_t>(mh_slice_src(p, q)) + (uint64_t)wave_u * 1024;
    glds16x4<W * 1024>(src, piece_off, ring_lds + (uint32_t)((q % NS) * MH_SLICE * 2 + wave_u * 1024));
  };
#pragma unroll
  for (int q = 0; q < NS; ++q) issue(q);

  // ---- x1 loads, the field's bound B_b = max_c abound (thread tid: channel tid) ------
  const int64_t pxc = px < P ? px : P - 1;
  const uint32_t P4 = (uint32_t)(P * 4);
  float xv[8][8];
  if constexpr (BUF) {
    const auto xr = buf_rsrc(p.x1 + (int64_t)z * MH_C * P, (int64_t)MH_C * P * 4);
    const uint32_t vo = (uint32_t)(((int64_t)(8 * g) * P + pxc) * 4);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[ks][e] = buf_ld_nt(xr, vo, (uint32_t)(32 * ks + e) * P4);
  } else {
    const float* xcol = p.x1 + (int64_t)z * MH_C * P + pxc;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xv[ks][e] = __builtin_nontemporal_load(xcol + (int64_t)(32 * ks + 8 * g + e) * P);
  }
  float bm = p.abound[(int64_t)z * MH_C + tid];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bm = fmaxf(bm, __shfl_xor(bm, o));
  if (lane == 0) red[wave] = bm;
  __syncthreads();  // (also: the first NS slices and the x1 loads landed)
  const float Bb = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float xi = pow2_below(Bb, 14);          // |x^ xi| < 2^14
  const float etab = pow2_below(Bb + 1.f, 14);  // |h eta_j eta_b| < 2^14

  // ---- normalised x1 -> fp16x2 B fragments (k-step ks: channels 32 ks + 8 g + 0..7) ----
  const float* sc = p.scale + (int64_t)z * MH_C;
  const float* sh = p.shift + (int64_t)z * MH_C;
  half8 xf[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int c0 = 32 * ks + 8 * g;
    const float4 sa = *reinterpret_cast<const float4*>(sc + c0);
    const float4 sb = *reinterpret_cast<const float4*>(sc + c0 + 4);
    const float4 ta = *reinterpret_cast<const float4*>(sh + c0);
    const float4 tb = *reinterpret_cast<const float4*>(sh + c0 + 4);
    const float sv[8] = {sa.x * xi, sa.y * xi, sa.z * xi, sa.w * xi,
                         sb.x * xi, sb.y * xi, sb.z * xi, sb.w * xi};
    const float tv[8] = {ta.x * xi, ta.y * xi, ta.z * xi, ta.w * xi,
                         tb.x * xi, tb.y * xi, tb.z * xi, tb.w * xi};
    uint32_t t[2][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      split2h(fmaf(sv[2 * e], xv[ks][2 * e], tv[2 * e]),
              fmaf(sv[2 * e + 1], xv[ks][2 * e + 1], tv[2 * e + 1]), t[0][e], t[1][e]);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) xf[ks][pl] = mh_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
  }
  floatx4 oacc[16];
#pragma unroll
  for (int ot = 0; ot < 16; ++ot) oacc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float ixi = 1.f / xi, ietab = 1.f / etab;
  for (int i = tid; i < MH_H; i += 64 * W) {
    b1s[i] = p.b1[i];
    is1s[i] = p.inv_s1[i] * ixi;
    hss[i] = p.eta[i] * etab;
  }
  for (int i = tid; i < MH_C; i += 64 * W) {
    b2s[i] = p.b2 ? p.b2[i] : 0.f;
    is2s[i] = p.inv_s2[i] * ietab;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (TRACE) tr[1] = __builtin_amdgcn_s_memrealtime();

  floatx4 hacc[2][2];  // [parity][tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int t = 0; t < 2; ++t) hacc[a][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  uint32_t hfu[2][4];  // fc2 B fragment of the converted block [plane][pair]

  const int a_lane = r16 * 32 + 8 * (g ^ mh_swz(r16));
  auto afrag = [&](const unsigned short* q) -> half8 {
    return *reinterpret_cast<const half8*>(q);
  };

  // step q: slice q landed for every wave (slices up to q + NS - 2 may stay in flight);
  // the slot of slice q - 1 is free and takes slice q + NS - 1
  auto step_begin = [&](int q) {
    const int after = min(NS - 2, MH_NSLICE - 1 - q);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    return ring + (q % NS) * MH_SLICE;
  };
  auto refill = [&](int q) {
    if (q >= 1 && q + NS - 1 < MH_NSLICE) issue(q + NS - 1);
  };

  // c += a (x) b, three fp16 MFMAs
  auto mfma3 = [](const half8 (&a)[2], const half8 (&b)[2], floatx4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
  };
  // two tiles' triples interleaved (no MFMA reads the accumulator its predecessor writes;
  // each accumulator sees the same three products in the same order as mfma3)
  auto mfma3x2 = [](const half8 (&a)[2], const half8 (&b)[2], floatx4& c,
                    const half8 (&a2)[2], const half8 (&b2)[2], floatx4& c2) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[1], b2[0], c2, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[0], b2[1], c2, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2[0], b2[0], c2, 0, 0, 0);
  };
  // ILV: the steps issue tile pairs through mfma3x2 (MLP 1.924 -> 1.905 ms in-block, three
  // interleaved pairs, profiles/r06_p/ab_mfma_pairs.txt; MSFNO_MH_ILV=0 restores the single-tile order)
  constexpr bool ilv = ILV;

  // pair e2 (0..3) of hidden block j in hacc[PAR]: unscale, + b1, GELU(erf), scale, split
  auto conv_pair = [&](int j, int e2, auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    const int t = e2 >> 1, i = 2 * (e2 & 1);
    const int row = 32 * j + 16 * t + 4 * g + i;
    const float2 b = *reinterpret_cast<const float2*>(b1s + row);
    const float2 is = *reinterpret_cast<const float2*>(is1s + row);
    const float2 hs = *reinterpret_cast<const float2*>(hss + row);
    f32x2 v = {fmaf(hacc[PAR][t][i], is.x, b.x), fmaf(hacc[PAR][t][i + 1], is.y, b.y)};
    v = gelu_erf2(v) * f32x2{hs.x, hs.y};
    split2h(v.x, v.y, hfu[0][e2], hfu[1][e2]);
  };

  auto fc1_step = [&](const unsigned short* slot, int q, auto kh_c, auto par_c, auto conv_c,
                      int jc) {
    constexpr int KH = decltype(kh_c)::value, PAR = decltype(par_c)::value;
    constexpr bool CONV = decltype(conv_c)::value;
    using PPrev = std::integral_constant<int, PAR ^ 1>;
    auto aoff = [&](int u, int pl) { return ((pl * 4 + (u >> 1)) * 2 + (u & 1)) * 512 + a_lane; };
    half8 a[AHEAD + 2][2];  // (the pair path rotates over AHEAD + 2)
#pragma unroll
    for (int k = 0; k < AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) a[k][pl] = afrag(slot + aoff(k, pl));
    if constexpr (ilv) {  // tile pairs (u, u + 1): A fragments AHEAD = 2 ahead cover both
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        mfma3x2(a[u % (AHEAD + 2)], xf[KH * 4 + (u >> 1)], hacc[PAR][0],
                a[(u + 1) % (AHEAD + 2)], xf[KH * 4 + (u >> 1)], hacc[PAR][1]);
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (u + k + AHEAD < 8) {
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
              a[(u + k + AHEAD) % (AHEAD + 2)][pl] = afrag(slot + aoff(u + k + AHEAD, pl));
          }
        if (u == 0) refill(q);
        if constexpr (CONV) {
          if (u == 2 || u == 6) conv_pair(jc, 2 * KH + (u >> 2), PPrev{});
        }
      }
    } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + AHEAD < 8) {
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          a[(u + AHEAD) % (AHEAD + 1)][pl] = afrag(slot + aoff(u + AHEAD, pl));
      }
      mfma3(a[u % (AHEAD + 1)], xf[KH * 4 + (u >> 1)], hacc[PAR][u & 1]);
      if (u == 0) refill(q);
      if constexpr (CONV) {
        if (u == 2 || u == 6) conv_pair(jc, 2 * KH + (u >> 2), PPrev{});
      }
    }
    }
    if constexpr (CONV && KH == 1) {
#pragma unroll
      for (int t = 0; t < 2; ++t) hacc[PAR ^ 1][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto fc2_step = [&](const unsigned short* slot, int q, auto oh_c) {
    constexpr int OH = decltype(oh_c)::value;
    auto aoff = [&](int u, int pl) { return (pl * 8 + u) * 512 + a_lane; };
    const half8 hb[2] = {mh_frag(hfu[0][0], hfu[0][1], hfu[0][2], hfu[0][3]),
                         mh_frag(hfu[1][0], hfu[1][1], hfu[1][2], hfu[1][3])};
    half8 a[AHEAD + 2][2];  // (the pair path rotates over AHEAD + 2)
#pragma unroll
    for (int k = 0; k < AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) a[k][pl] = afrag(slot + aoff(k, pl));
    if constexpr (ilv) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        mfma3x2(a[u % (AHEAD + 2)], hb, oacc[OH * 8 + u], a[(u + 1) % (AHEAD + 2)], hb, oacc[OH * 8 + u + 1]);
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (u + k + AHEAD < 8) {
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
              a[(u + k + AHEAD) % (AHEAD + 2)][pl] = afrag(slot + aoff(u + k + AHEAD, pl));
          }
        if (u == 0) refill(q);
      }
    } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + AHEAD < 8) {
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          a[(u + AHEAD) % (AHEAD + 1)][pl] = afrag(slot + aoff(u + AHEAD, pl));
      }
      mfma3(a[u % (AHEAD + 1)], hb, oacc[OH * 8 + u]);
      if (u == 0) refill(q);
    }
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  using T = std::true_type;
  auto do_round = [&](int j, auto par_c) {
    const int q = 2 + 4 * (j - 1);
    fc1_step(step_begin(q), q, I0{}, par_c, T{}, j - 1);
    fc1_step(step_begin(q + 1), q + 1, I1{}, par_c, T{}, j - 1);
    fc2_step(step_begin(q + 2), q + 2, I0{});
    fc2_step(step_begin(q + 3), q + 3, I1{});
  };
  fc1_step(step_begin(0), 0, I0{}, I0{}, F{}, 0);
  fc1_step(step_begin(1), 1, I1{}, I0{}, F{}, 0);
  for (int j = 1; j < MH_HB; j += 2) {
    do_round(j, I1{});
    if (j + 1 < MH_HB) do_round(j + 1, I0{});
  }
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) conv_pair(MH_HB - 1, e2, I1{});
  // the residual of every output row, all loads in flight at once and under the last
  // two steps' MFMAs (the x1 fragments are dead: their registers take it)
  float rv[16][4];
  if (p.resid && BUF) {
    const auto rr = buf_rsrc(p.resid + (int64_t)z * MH_C * P, (int64_t)MH_C * P * 4);
    const uint32_t vo = (uint32_t)(((int64_t)(4 * g) * P + pxc) * 4);
#pragma unroll
    for (int ot = 0; ot < 16; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i) rv[ot][i] = buf_ld_nt(rr, vo, (uint32_t)(16 * ot + i) * P4);
  } else if (p.resid) {
    const float* rs = p.resid + (int64_t)z * MH_C * P + pxc;
#pragma unroll
    for (int ot = 0; ot < 16; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        rv[ot][i] = __builtin_nontemporal_load(rs + (int64_t)(16 * ot + 4 * g + i) * P);
  } else {
#pragma unroll
    for (int ot = 0; ot < 16; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i) rv[ot][i] = 0.f;
  }
  fc2_step(step_begin(MH_NSLICE - 2), MH_NSLICE - 2, I0{});
  fc2_step(step_begin(MH_NSLICE - 1), MH_NSLICE - 1, I1{});
  if constexpr (TRACE) {
    // diagnostic (MSFNO_MH_TRACE): per workgroup the CU it ran on and the real-time
    // clock (100 MHz) at entry, after the prologue's loads, after the last MFMA step
    // and once its stores are issued
    tr[2] = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    if (tid == 0) {
      uint64_t* t = p.trace + 5 * (int64_t)blockIdx.x;
      t[0] = ((uint64_t)xcc << 32) | hw;
      t[1] = tr[0];
      t[2] = tr[1];
      t[3] = tr[2];
    }
  }

  // ---- epilogue: unscale + b2 + residual, store (rows 16 ot + 4 g + i) ----------------
  if (px >= P) return;
  float* o = p.out + (int64_t)z * MH_C * P + px;
  const auto orr = buf_rsrc(p.out + (int64_t)z * MH_C * P, (int64_t)MH_C * P * 4);
  const uint32_t vo = (uint32_t)(((int64_t)(4 * g) * P + px) * 4);
#pragma unroll
  for (int ot = 0; ot < 16; ++ot) {
    const int r0 = 16 * ot + 4 * g;
    const float4 is = *reinterpret_cast<const float4*>(is2s + r0);
    const float4 b = *reinterpret_cast<const float4*>(b2s + r0);
    const float isv[4] = {is.x, is.y, is.z, is.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = fmaf(oacc[ot][i], isv[i], bv[i]) + rv[ot][i];
      if constexpr (BUF) buf_st_nt(v, orr, vo, (uint32_t)(16 * ot + i) * P4);
      else o[(int64_t)(r0 + i) * P] = v;
    }
  }
  if constexpr (TRACE) {
    if (tid == 0) p.trace[5 * (int64_t)blockIdx.x + 4] = __builtin_amdgcn_s_memrealtime();
  }
}

// TRACE (MSFNO_MH_TRACE, diagnostic): per-workgroup CU id and phase timestamps
template <int AHEAD, bool TRACE, bool BUF, bool ILV = false>
__global__ __launch_bounds__(256, 2) void mlp_fused_h_kernel(MlpHParams p) {
  __shared__ __attribute__((aligned(16))) char lds_raw[MH_LDS];
  mlp_fused_h_tile<AHEAD, TRACE, BUF, ILV>(p, xcd_remap(blockIdx.x, gridDim.x), lds_raw);
}

// The fc1 half of mlp_fused_h_kernel with 256 output rows and no hidden layer:
// a wave's 16 pixels of x, scaled per channel by the power of two xs (chan_affine's
// norm0 bound, |xs x| < 2^14) and split into fp16x2 B fragments in registers; the
// per-batch weight image W'[c][k] = rs_c Ws[c][k] / xs_k (rs_c puts the row's maximum
// into [2^14, 2^15)) streams through the four-slot LDS ring as 16 slices of 16 KB
// (output block j of 32 rows, channel half kh: the W1 slice layout); all 256 x 16
// outputs stay in the accumulators and are stored once, unscaled by 1 / rs_c, + bs.
// (gemm_x3 with in-kernel split, 256 x 256 tiles: 0.83 ms at config 2.)
constexpr int SK_NSLICE = 16;

struct SkipHParams {
  const float* x;       // [B][C][P]
  const float* xs;      // [B][C] power-of-two channel scales
  float* out;           // [B][C][P]
  const unsigned short* img;  // [B][16 slices]
  const float* inv_rs;  // [B][C]
  const float* bias;    // [C] or null
  int64_t P;
  int tiles_per_field;
};

// The per-batch skip weight image in one launch (it was two: the row scales, then the
// image, 5.6 us each per block and batch at the network's 120 x 240 blocks): one
// 256-thread workgroup per (row c, batch b).  rs[b][c] = 2^(15 - e) for
// max_k |Ws[c][k] / xs[b][k]| = f 2^e, inv_rs = 1 / rs; then the row of
// W' = rs Ws / xs split into fp16x2 in mh_w1_image_kernel's slice layout
// [b][j][kh][pl][ks][t][r][32] (8 blocks j; thread k < 128 writes the pair 2k, 2k + 1)
__global__ __launch_bounds__(256) void sk_prep_kernel(const float* __restrict__ W,
                                                      const float* __restrict__ xs,
                                                      float* __restrict__ rs,
                                                      float* __restrict__ inv_rs,
                                                      unsigned short* __restrict__ img) {
  __shared__ float wmax[4];
  const int b = blockIdx.y, c = blockIdx.x, k = threadIdx.x;
  const float* row = W + (int64_t)c * MH_C;
  const float* xsb = xs ? xs + (int64_t)b * MH_C : nullptr;
  float m = fabsf(xsb ? row[k] / xsb[k] : row[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((k & 63) == 0) wmax[k >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  float sc = 1.f;
  if (m > 0.f && isfinite(m)) {
    int e;
    frexpf(m, &e);
    sc = ldexpf(1.f, 15 - e);
  }
  if (k == 0) {
    rs[(int64_t)b * MH_C + c] = sc;
    inv_rs[(int64_t)b * MH_C + c] = 1.f / sc;
  }
  if (k >= 128) return;
  const int k0 = 2 * k;  // the pair (k0, k0 + 1): one kh, ks, 8-channel group
  const int j = c >> 5, t = (c >> 4) & 1, r = c & 15;
  const int kh = k0 >> 7, ks = (k0 >> 5) & 3, gq = (k0 >> 3) & 3;
  const int kk = 8 * (gq ^ mh_swz(r)) + (k0 & 7);  // its stored position in the 32-wide row
  uint32_t t0, t1;
  if (xsb)
    split2h(row[k0] / xsb[k0] * sc, row[k0 + 1] / xsb[k0 + 1] * sc, t0, t1);
  else
    split2h(row[k0] * sc, row[k0 + 1] * sc, t0, t1);
  unsigned short* ib = img + (int64_t)b * SK_NSLICE * MH_SLICE;
  uint32_t* o = reinterpret_cast<uint32_t*>(ib + (int64_t)(j * 2 + kh) * MH_SLICE + ((ks * 2 + t) * 16 + r) * 32 + kk);
  o[0] = t0;
  o[MH_PLANE / 2] = t1;
}

template <int NS, int MINB>
__global__ __launch_bounds__(256, MINB) void skip_h_kernel(SkipHParams p) {
  constexpr int W = 4;
  constexpr int RING_BYTES = NS * MH_SLICE * 2;
  __shared__ __attribute__((aligned(16))) char lds_raw[RING_BYTES + 2 * MH_C * 4];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const irs = reinterpret_cast<float*>(lds_raw + RING_BYTES);
  float* const bs = irs + MH_C;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int z = lin / p.tiles_per_field;
  const int64_t P = p.P;
  const int64_t px = (int64_t)(lin - z * p.tiles_per_field) * 64 + 16 * wave + r16;
  const unsigned short* img = p.img + (int64_t)z * SK_NSLICE * MH_SLICE;

  const uint32_t ring_lds = lds_addr(ring);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  uint32_t piece_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) piece_off[i] = (uint32_t)(i * W * 1024 + lane * 16);
  auto issue = [&](int q) {
    const uint64_t src = reinterpret_cast<uint64_t>(img + (int64_t)q * MH_SLICE) + (uint64_t)wave_u * 1024;
    glds16x4<W * 1024>(src, piece_off, ring_lds + (uint32_t)((q % NS) * MH_SLICE * 2 + wave_u * 1024));
  };
#pragma unroll
  for (int q = 0; q < NS; ++q) issue(q);

  // x -> scaled fp16x2 B fragments (k-step ks: channels 32 ks + 8 g + 0..7)
  const float* xcol = p.x + (int64_t)z * MH_C * P + (px < P ? px : P - 1);
  half8 xf[8][2];
  {
    const float* xsb = p.xs + (int64_t)z * MH_C;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int c0 = 32 * ks + 8 * g;
      float xv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = __builtin_nontemporal_load(xcol + (int64_t)(c0 + e) * P);
      const float4 sa = *reinterpret_cast<const float4*>(xsb + c0);
      const float4 sb = *reinterpret_cast<const float4*>(xsb + c0 + 4);
      const float sv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
      uint32_t t[2][4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        split2h(sv[2 * e] * xv[2 * e], sv[2 * e + 1] * xv[2 * e + 1], t[0][e], t[1][e]);
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) xf[ks][pl] = mh_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
    }
  }
  for (int i = tid; i < MH_C; i += 256) {
    irs[i] = p.inv_rs[(int64_t)z * MH_C + i];
    bs[i] = p.bias ? p.bias[i] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  floatx4 oacc[16];
#pragma unroll
  for (int ot = 0; ot < 16; ++ot) oacc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int a_lane = r16 * 32 + 8 * (g ^ mh_swz(r16));

#pragma unroll
  for (int q = 0; q < SK_NSLICE; ++q) {
    // slice q landed (up to NS - 2 later slices may stay in flight); slot of q - 1 free
    const int after = min(NS - 2, SK_NSLICE - 1 - q);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned short* slot = ring + (q % NS) * MH_SLICE;
    const int j = q >> 1, kh = q & 1;
    auto aoff = [&](int u, int pl) { return ((pl * 4 + (u >> 1)) * 2 + (u & 1)) * 512 + a_lane; };
    half8 a[3][2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) a[k][pl] = *reinterpret_cast<const half8*>(slot + aoff(k, pl));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + 2 < 8) {
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          a[(u + 2) % 3][pl] = *reinterpret_cast<const half8*>(slot + aoff(u + 2, pl));
      }
      const half8* av = a[u % 3];
      const half8* xb = xf[kh * 4 + (u >> 1)];
      floatx4& c = oacc[2 * j + (u & 1)];
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[1], xb[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], xb[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], xb[0], c, 0, 0, 0);
      if (u == 0 && q >= 1 && q + NS - 1 < SK_NSLICE) issue(q + NS - 1);
    }
  }

  // epilogue: rows 16 ot + 4 g + i of pixel px
  if (px >= P) return;
  float* o = p.out + (int64_t)z * MH_C * P + px;
#pragma unroll
  for (int ot = 0; ot < 16; ++ot) {
    const int r0 = 16 * ot + 4 * g;
    const float4 is = *reinterpret_cast<const float4*>(irs + r0);
    const float4 b = *reinterpret_cast<const float4*>(bs + r0);
    const float isv[4] = {is.x, is.y, is.z, is.w};
    const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) o[(int64_t)(r0 + i) * P] = fmaf(oacc[ot][i], isv[i], bv[i]);
  }
}

// Persistent, pipelined form of skip_h_kernel (one workgroup of 4 waves per CU, one
// wave per SIMD with the whole register file: 32 pixels per wave as two 16-pixel
// groups, 128 per tile; a contiguous range of tiles per workgroup).  skip_h_kernel
// runs one tile per workgroup: its x loads, its 16 slice steps and its 64 four-byte
// stores per lane are three phases that every CU enters at the same time, so HBM idles
// while the MFMAs run and the MFMAs idle while x streams in.  Here one ring carries,
// per slice step, the weight slice of this tile AND one 16-channel piece of the NEXT
// tile's x (8 KB, LDS-DMA), which the step converts into the next tile's B fragments
// in registers; the outputs leave through a per-wave LDS transpose as 16-B stores
// (whole 128-B lines, 32 per lane instead of 128).  HBM then streams x and out under
// the MFMAs, and each A fragment read from LDS feeds both pixel groups.
//
// vmcnt accounting (each wave, in issue order): group n = 6 LDS-DMAs (four 1-KB weight
// pieces + two x-piece rows pairs), issued at step n - (NS - 1); a tile's 32 output
// stores come after its step 15.  The wait for group n at step n leaves NS - 2 younger
// groups in flight, plus the previous tile's stores when n is one of the first NS - 1
// steps of a tile (tile 0: those groups were drained in the prologue).  The tail
// issues dummy groups (the last tile again) so the counts stay exact, and the kernel
// drains every DMA before it exits.
constexpr int SP_NS = 5, SP_W = 4, SP_PX = 32 * SP_W;
constexpr int SP_XPAIR = 1024 + 32;                  // two 512-B x rows + bank pad
constexpr int SP_WBYTES = MH_SLICE * 2;              // 16 KB of weights
constexpr int SP_SLOT = SP_WBYTES + 8 * SP_XPAIR;    // 24,832 B
constexpr int SP_ERS = 36;                           // epilogue row stride (floats)
constexpr int SP_EPI = 32 * SP_ERS * 4;              // per wave: 32 channels x 32 pixels
constexpr int SP_LDS = SP_NS * SP_SLOT + SP_W * SP_EPI + 3 * MH_C * 4;
constexpr int SP_GROUP = 6;                          // DMAs per wave and step
static_assert(SP_LDS <= 160 * 1024, "skip_hp LDS");
static_assert(SP_SLOT % 16 == 0 && SP_EPI % 16 == 0, "skip_hp LDS alignment");
static_assert(SP_GROUP * (SP_NS - 2) + 32 <= 63, "skip_hp vmcnt range");

struct SkipHPParams {
  const float* x;
  const float* xs;
  float* out;
  const unsigned short* img;
  const float* inv_rs;
  const float* bias;
  int64_t P;
  int tiles_per_field;
  int tiles;
};

__global__ __launch_bounds__(64 * SP_W, 1) void skip_hp_kernel(SkipHPParams p) {
  constexpr int NS = SP_NS;
  __shared__ __attribute__((aligned(16))) char lds[SP_LDS];
  float* const epi_all = reinterpret_cast<float*>(lds + NS * SP_SLOT);
  float* const xsl = reinterpret_cast<float*>(lds + NS * SP_SLOT + SP_W * SP_EPI);
  float* const irsl = xsl + MH_C;
  float* const bl = irsl + MH_C;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t P = p.P;
  const int t0 = (int)((int64_t)blockIdx.x * p.tiles / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * p.tiles / gridDim.x);
  const int ntile = t1 - t0;  // >= 1: the host launches at most `tiles` workgroups
  const int tpf = p.tiles_per_field;
  const uint32_t ring_lds = lds_addr(lds);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  // x piece of step q: 16 channels 32 (q >> 1) + 8 g' + 4 (q & 1) + e (g' 0..3, e 0..3),
  // piece row i = 4 g' + e, rows (2k, 2k + 1) at k * SP_XPAIR.  This wave's two DMAs move
  // rows 4 wave + 2 h2 + (lane >> 5), pixels 4 (lane & 31) .. + 3 of the tile.
  const uint32_t w_voff = (uint32_t)lane * 16;
  uint32_t x_voff_row[2];
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    const int xrow = 4 * wave + 2 * h2 + (lane >> 5);
    x_voff_row[h2] = (uint32_t)(8 * (xrow >> 2) + (xrow & 3)) * (uint32_t)P * 4;
  }
  const int xcol = 4 * (lane & 31);

  // per-tile DMA sources (uniform): the tile's weight image, the x base of the tile
  // after it (or of itself at the end: never read) and that tile's pixel limit
  struct Src {
    uint64_t w, x;
    uint32_t xo[2];
  };
  auto src_of = [&](int tl) {
    if (tl >= ntile) tl = ntile - 1;  // tail: dummy groups
    const int t = t0 + tl;
    const int z = t / tpf;
    const int tn = tl + 1 < ntile ? t + 1 : t;
    const int zn = tn / tpf;
    const int64_t pxt = (int64_t)(tn - zn * tpf) * SP_PX;
    const int64_t room = P - 4 - pxt;  // >= 0: P % 4 == 0 and pxt < P
    const int lim = room < SP_PX - 4 ? (int)room : SP_PX - 4;
    Src r;
    r.w = reinterpret_cast<uint64_t>(p.img + (int64_t)z * SK_NSLICE * MH_SLICE) + (uint64_t)(wave_u * 1024);
    r.x = reinterpret_cast<uint64_t>(p.x + (int64_t)zn * MH_C * P + pxt);
    const uint32_t c4 = (uint32_t)min(xcol, lim) * 4;
    r.xo[0] = x_voff_row[0] + c4;
    r.xo[1] = x_voff_row[1] + c4;
    return r;
  };
  auto issue = [&](const Src& sr, int n, int q) {
    // opaque copies: keep the per-step address arithmetic at the step (hoisted to the
    // tile start, 16 steps of addresses overflow the SGPRs)
    uint64_t wb = sr.w, xb0 = sr.x, p4 = (uint64_t)P * 4;
    asm volatile("" : "+s"(wb), "+s"(xb0), "+s"(p4));
    const uint32_t slot = ring_lds + (uint32_t)((n % NS) * SP_SLOT);
    const uint64_t wq = wb + (uint64_t)q * MH_SLICE * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds16s(wq + (uint64_t)(i * 4096), w_voff, slot + (uint32_t)(i * 4096 + wave_u * 1024));
    const uint64_t xq = xb0 + (uint64_t)(32 * (q >> 1) + 4 * (q & 1)) * p4;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
      glds16s(xq, sr.xo[h2], slot + (uint32_t)(SP_WBYTES + (2 * wave_u + h2) * SP_XPAIR));
  };

  int zc = t0 / tpf, zx = (ntile > 1 ? t0 + 1 : t0) / tpf;
  for (int i = tid; i < MH_C; i += 64 * SP_W) {
    bl[i] = p.bias ? p.bias[i] : 0.f;
    irsl[i] = p.inv_rs[(int64_t)zc * MH_C + i];
    xsl[i] = p.xs[(int64_t)zx * MH_C + i];
  }
  {
    const Src s0 = src_of(0);
#pragma unroll
    for (int n = 0; n < NS - 1; ++n) issue(s0, n, n);
  }

  // the first tile's x -> B fragments (plain loads, once per workgroup)
  half8 xf[2][8][2];
  {
    const float* xsb = p.xs + (int64_t)zc * MH_C;
#pragma unroll
    for (int pg = 0; pg < 2; ++pg) {
      int64_t px = (int64_t)(t0 - zc * tpf) * SP_PX + 32 * wave + 16 * pg + r16;
      if (px > P - 1) px = P - 1;  // past the field's end (never stored)
      const float* xw = p.x + (int64_t)zc * MH_C * P;
      const uint32_t lo = (uint32_t)(8 * g) * (uint32_t)P + (uint32_t)px;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int c0 = 32 * ks + 8 * g;
        float xv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          xv[e] = __builtin_nontemporal_load(xw + (int64_t)(32 * ks + e) * P + lo);
        const float4 sa = *reinterpret_cast<const float4*>(xsb + c0);
        const float4 sb = *reinterpret_cast<const float4*>(xsb + c0 + 4);
        const float sv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
        uint32_t t[2][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          split2h(sv[2 * e] * xv[2 * e], sv[2 * e + 1] * xv[2 * e + 1], t[0][e], t[1][e]);
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) xf[pg][ks][pl] = mh_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int a_lane = r16 * 32 + 8 * (g ^ mh_swz(r16));
  float* const ep = epi_all + wave * 32 * SP_ERS;
  uint32_t xn[2][8][2][4];

  for (int tl = 0; tl < ntile; ++tl) {
    const int t = t0 + tl;
    if (tl > 0) {
      const int zc2 = t / tpf, zx2 = (tl + 1 < ntile ? t + 1 : t) / tpf;
      if (zc2 != zc || zx2 != zx) {  // a field boundary: new scale tables (drains the ring)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int i = tid; i < MH_C; i += 64 * SP_W) {
          irsl[i] = p.inv_rs[(int64_t)zc2 * MH_C + i];
          xsl[i] = p.xs[(int64_t)zx2 * MH_C + i];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        zc = zc2;
        zx = zx2;
      }
    }
    const Src s_cur = src_of(tl), s_nxt = src_of(tl + 1);
    floatx4 oacc[2][16];
#pragma unroll
    for (int pg = 0; pg < 2; ++pg)
#pragma unroll
      for (int ot = 0; ot < 16; ++ot) oacc[pg][ot] = floatx4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int q = 0; q < SK_NSLICE; ++q) {
      const int n = tl * SK_NSLICE + q;
      if (q < NS - 1) asm volatile("s_waitcnt vmcnt(50)" ::: "memory");  // 6 (NS-2) + 32
      else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");              // 6 (NS-2)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const char* slot = lds + (n % NS) * SP_SLOT;
      // the next tile's x piece -> its B fragments (channels 32 ks + 8 g + 4 h + 0..3)
      {
        const int ks = q >> 1, h = q & 1;
        const float4 sv = *reinterpret_cast<const float4*>(xsl + 32 * ks + 8 * g + 4 * h);
#pragma unroll
        for (int pg = 0; pg < 2; ++pg) {
          const char* xb = slot + SP_WBYTES + 4 * (32 * wave + 16 * pg + r16);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = *reinterpret_cast<const float*>(xb + (2 * g + (e >> 1)) * SP_XPAIR + (e & 1) * 512);
          split2h(sv.x * v[0], sv.y * v[1], xn[pg][ks][0][2 * h], xn[pg][ks][1][2 * h]);
          split2h(sv.z * v[2], sv.w * v[3], xn[pg][ks][0][2 * h + 1], xn[pg][ks][1][2 * h + 1]);
        }
      }
      const unsigned short* ws = reinterpret_cast<const unsigned short*>(slot);
      const int j = q >> 1, kh = q & 1;
      auto aoff = [&](int u, int pl) { return ((pl * 4 + (u >> 1)) * 2 + (u & 1)) * 512 + a_lane; };
      half8 a[3][2];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) a[k][pl] = *reinterpret_cast<const half8*>(ws + aoff(k, pl));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u + 2 < 8) {
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            a[(u + 2) % 3][pl] = *reinterpret_cast<const half8*>(ws + aoff(u + 2, pl));
        }
        const half8* av = a[u % 3];
#pragma unroll
        for (int pg = 0; pg < 2; ++pg) {
          const half8* xb = xf[pg][kh * 4 + (u >> 1)];
          floatx4& c = oacc[pg][2 * j + (u & 1)];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[1], xb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], xb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], xb[0], c, 0, 0, 0);
        }
        if (u == 0) {
          if (q + NS - 1 < SK_NSLICE) issue(s_cur, n + NS - 1, q + NS - 1);
          else issue(s_nxt, n + NS - 1, q + NS - 1 - SK_NSLICE);
        }
      }
    }

    // epilogue: row 16 ot + 4 g + i, pixel 32 wave + 16 pg + r16; 32 rows per round
    // through the wave's LDS patch, out as 16-B stores (a row's 32 pixels = one line)
    {
      const int64_t px0 = (int64_t)(t - zc * tpf) * SP_PX + 32 * wave;
      float* const ob = p.out + (int64_t)zc * MH_C * P + px0;
      const uint32_t so = (uint32_t)(lane >> 3) * (uint32_t)P + 4u * (uint32_t)(lane & 7);
      const bool in = px0 + 4 * (lane & 7) < P;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int o2 = 0; o2 < 2; ++o2) {
          const int r0 = 16 * (2 * c + o2) + 4 * g;
          const float4 is = *reinterpret_cast<const float4*>(irsl + r0);
          const float4 bb = *reinterpret_cast<const float4*>(bl + r0);
#pragma unroll
          for (int pg = 0; pg < 2; ++pg) {
            const floatx4 acc = oacc[pg][2 * c + o2];
            float* e0 = ep + (16 * o2 + 4 * g) * SP_ERS + 16 * pg + r16;
            e0[0] = fmaf(acc[0], is.x, bb.x);
            e0[SP_ERS] = fmaf(acc[1], is.y, bb.y);
            e0[2 * SP_ERS] = fmaf(acc[2], is.z, bb.z);
            e0[3 * SP_ERS] = fmaf(acc[3], is.w, bb.w);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int row = 8 * k + (lane >> 3), col = 4 * (lane & 7);
          const floatx4 v = *reinterpret_cast<const floatx4*>(ep + row * SP_ERS + col);
          if (in)
            __builtin_nontemporal_store(
                v, reinterpret_cast<floatx4*>(ob + (int64_t)(32 * c + 8 * k) * P + so));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
#pragma unroll
    for (int pg = 0; pg < 2; ++pg)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          xf[pg][ks][pl] = mh_frag(xn[pg][ks][pl][0], xn[pg][ks][pl][1], xn[pg][ks][pl][2], xn[pg][ks][pl][3]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's dummy DMAs land before exit
}

// xs[r] = 2^(14 - e), max_p |x[r][p]| = f 2^e (f in [0.5, 1)): every |xs x| < 2^14 (the
// x3h B-row scale of a standalone 1x1 conv, whose input has no norm statistics); one
// 256-thread workgroup per row r
__global__ __launch_bounds__(256) void chan_pow2_scale_kernel(const float* __restrict__ x,
                                                              int64_t P, float* __restrict__ xs) {
  __shared__ float wmax[4];
  const float* row = x + (int64_t)blockIdx.x * P;
  float m = 0.f;
  for (int64_t p = threadIdx.x; p < P; p += 256) m = fmaxf(m, fabsf(row[p]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    xs[blockIdx.x] = pow2_below(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])), 14);
}

}  // namespace

int launch_chan_pow2_scale(const float* x, int64_t rows, int64_t P, float* xs, hipStream_t s) {
  MSFNO_REQUIRE(x && xs && rows > 0 && rows < (1LL << 31) && P >= 1, MSFNO_EINVAL,
                "chan_pow2_scale: bad arguments");
  hipLaunchKernelGGL(chan_pow2_scale_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, P, xs);
  return launch_check("chan_pow2_scale");
}

size_t skip_h_workspace(int B) {
  return (size_t)B * SK_NSLICE * MH_SLICE * 2 + (size_t)B * MH_C * 4 * 2 + 256;
}

// MSFNO_SKIP_H=0 keeps gemm_x3 for the inner skip
bool skip_h_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SKIP_H");
    return !(e && e[0] == '0');
  }();
  return on;
}


int launch_skip_h(const float* W, const float* xs, const float* x, float* out, const float* bias,
                  int B, int64_t P, void* ws, size_t ws_bytes, hipStream_t s, bool side) {
  MSFNO_REQUIRE(W && xs && x && out && ws && B > 0 && P >= 1 && ws_bytes >= skip_h_workspace(B),
                MSFNO_EINVAL, "skip_h: bad arguments");
  unsigned short* img = static_cast<unsigned short*>(ws);
  float* rs = reinterpret_cast<float*>(img + (int64_t)B * SK_NSLICE * MH_SLICE);
  float* inv_rs = rs + (int64_t)B * MH_C;
  hipLaunchKernelGGL(sk_prep_kernel, dim3(MH_C, B), dim3(256), 0, s, W, xs, rs, inv_rs, img);
  MSFNO_TRY(launch_check("sk_prep"));
  SkipHParams p{};
  p.x = x; p.xs = xs; p.out = out; p.img = img; p.inv_rs = inv_rs; p.bias = bias; p.P = P;
  p.tiles_per_field = (int)cdiv(P, 64);
  const int64_t tiles = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(tiles < (1LL << 31), MSFNO_EINVAL, "skip_h: grid too large");
  // the persistent pipelined kernel (MSFNO_SKIP_P=0: one tile per workgroup, read on
  // every call so one process can run both); its x pieces and output stores move 4
  // pixels per lane (P % 4 == 0)
  const char* pe = getenv("MSFNO_SKIP_P");
  const bool persist = !(pe && pe[0] == '0');
  if (persist && P % 4 == 0) {
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    SkipHPParams q{};
    q.x = x; q.xs = xs; q.out = out; q.img = img; q.inv_rs = inv_rs; q.bias = bias; q.P = P;
    q.tiles_per_field = (int)cdiv(P, SP_PX);
    const int64_t t = (int64_t)B * q.tiles_per_field;
    MSFNO_REQUIRE(t < (1LL << 31), MSFNO_EINVAL, "skip_hp: grid too large");
    q.tiles = (int)t;
    // Workgroups per CU.  A workgroup fills its CU (142 KB of LDS, the whole register
    // file).  Alone (inline, or in a graph): 2 per CU, the second half of the grid starting
    // as the first retires.  On the block's side stream the grid size is the share of CUs
    // taken from the main stream's SHT kernels while the skip runs: 0.25 (64 of 256 CUs;
    // the skip then spans 2.35 ms under the SHT) measured 166.9 / 165.4 / 166.1 fields/s
    // against 163.6 / 164.3 / 162.8 for 2 per CU, 158.7 / 156.1 / 158.9 for 0.1875 and
    // 164.4 / 162.6 / 163.9 for 0.3125, three interleaved rounds (profiles/r06_f).
    // MSFNO_SKIP_GRID overrides both.
    const char* ge = getenv("MSFNO_SKIP_GRID");
    const double per_cu = ge ? atof(ge) : (side ? 0.25 : 2.0);
    const int64_t want = std::max<int64_t>(1, (int64_t)(per_cu * cus + 0.5));
    const int grid = (int)std::min<int64_t>(t, want);
    hipLaunchKernelGGL(skip_hp_kernel, dim3((unsigned)grid), dim3(64 * SP_W), 0, s, q);
    return launch_check("skip_hp");
  }
  // MSFNO_SKIP_NS=3: three ring slots, three workgroups per CU (A/B)
  static const int ns = [] {
    const char* e = getenv("MSFNO_SKIP_NS");
    return e && e[0] == '3' ? 3 : 4;
  }();
  if (ns == 3)
    hipLaunchKernelGGL((skip_h_kernel<3, 3>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((skip_h_kernel<MH_NS, 2>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  return launch_check("skip_h");
}

// the x3h engine is the default (measured as accurate as fp32 against fp64, more so
// than x6: tests/test_gpu_x3h.py); MSFNO_ENGINE=x6 selects the six-MFMA bf16 engine
bool mlp_fused_h_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_ENGINE");
    return !(e && std::string(e) == "x6");
  }();
  return on;
}

size_t mlp_fused_h_image_bytes() {
  return (size_t)MH_IMG_ELEMS * 2 + (size_t)(2 * MH_H + MH_C) * 4;
}

int launch_mlp_fused_h_images(const float* W1, const float* b1, const float* W2,
                              unsigned short* img, hipStream_t s) {
  float* sc = reinterpret_cast<float*>(img + MH_IMG_ELEMS);
  float* eta = sc + MH_H + MH_C;
  hipLaunchKernelGGL(mh_eta_kernel, dim3(MH_H / 256), dim3(256), 0, s, W1, b1, eta);
  MSFNO_TRY(launch_check("mh_eta"));
  hipLaunchKernelGGL(mh_scale_kernel, dim3((MH_H + MH_C + 255) / 256), dim3(256), 0, s, W1, W2, eta,
                     sc, sc + MH_H);
  MSFNO_TRY(launch_check("mh_scale"));
  hipLaunchKernelGGL(mh_w1_image_kernel, dim3(256), dim3(256), 0, s, W1, sc, img);
  MSFNO_TRY(launch_check("mh_w1_image"));
  hipLaunchKernelGGL(mh_w2_image_kernel, dim3(256), dim3(256), 0, s, W2, eta, sc + MH_H,
                     img + (int64_t)MH_HB * 2 * MH_SLICE);
  MSFNO_TRY(launch_check("mh_w2_image"));
  hipLaunchKernelGGL(mh_invert_kernel, dim3((MH_H + MH_C + 255) / 256), dim3(256), 0, s, sc);
  return launch_check("mh_invert");
}

int launch_mlp_fused_h(const float* x1, const float* scale, const float* shift,
                       const float* abound, const float* resid, float* out,
                       const unsigned short* img, const float* b1, const float* b2, int B,
                       int64_t P, hipStream_t s) {
  MSFNO_REQUIRE(x1 && scale && shift && abound && out && img && b1 && B > 0 && P >= 1,
                MSFNO_EINVAL, "mlp_fused_h: bad arguments");
  MlpHParams p{};
  p.x1 = x1; p.scale = scale; p.shift = shift; p.resid = resid; p.out = out;
  p.abound = abound;
  p.w1img = img;
  p.w2img = img + (int64_t)MH_HB * 2 * MH_SLICE;
  const float* sc = reinterpret_cast<const float*>(img + MH_IMG_ELEMS);
  p.inv_s1 = sc;
  p.inv_s2 = sc + MH_H;
  p.eta = sc + MH_H + MH_C;
  p.b1 = b1; p.b2 = b2; p.P = P;
  p.tiles_per_field = (int)cdiv(P, 16 * MH_WAVES);
  const int64_t tiles = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(tiles < (1LL << 31), MSFNO_EINVAL, "mlp_fused_h: grid too large");
  // MSFNO_MH_TRACE=<file> (diagnostic): each launch's per-workgroup CU ids and phase
  // timestamps are appended to <file> (synchronous; tools/mh_trace.py reads it)
  const char* te = getenv("MSFNO_MH_TRACE");
  if (te && te[0]) {
    uint64_t* tb = nullptr;
    MSFNO_CHECK_HIP(hipMalloc(&tb, (size_t)tiles * 5 * 8));
    MSFNO_CHECK_HIP(hipMemsetAsync(tb, 0, (size_t)tiles * 5 * 8, s));
    p.trace = tb;
    hipLaunchKernelGGL((mlp_fused_h_kernel<2, true, false>), dim3((unsigned)tiles), dim3(64 * MH_WAVES), 0, s, p);
    MSFNO_TRY(launch_check("mlp_fused_h"));
    std::vector<uint64_t> h((size_t)tiles * 5);
    MSFNO_CHECK_HIP(hipMemcpyAsync(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost, s));
    MSFNO_CHECK_HIP(hipStreamSynchronize(s));
    MSFNO_CHECK_HIP(hipFree(tb));
    if (FILE* f = fopen(te, "ab")) {
      const uint64_t n = (uint64_t)tiles;
      fwrite(&n, 8, 1, f);
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
    return MSFNO_OK;
  }
  // A fragments read two MFMA triples ahead (one or three: equal within 1 %, profiles/r06_i).
  // MSFNO_MH_BUF=1: raw-buffer addressing of x1 / residual / output (a field's plane below
  // 2 GB).  Not the default: as fast (1.96 ms) but 3.98 instead of 3.36 GB of HBM traffic
  // per launch (profiles/r06_v vs r06_j pmc_traffic.json)
  static const bool buf_env = [] {
    const char* e = getenv("MSFNO_MH_BUF");
    return e && e[0] == '1';
  }();
  static const bool ilv_env = [] {
    const char* e = getenv("MSFNO_MH_ILV");
    return !(e && e[0] == '0');
  }();
  const bool buf = buf_env && (int64_t)MH_C * P * 4 < (1LL << 31);
  if (buf && ilv_env)
    hipLaunchKernelGGL((mlp_fused_h_kernel<2, false, true, true>), dim3((unsigned)tiles), dim3(64 * MH_WAVES), 0, s, p);
  else if (buf)
    hipLaunchKernelGGL((mlp_fused_h_kernel<2, false, true>), dim3((unsigned)tiles), dim3(64 * MH_WAVES), 0, s, p);
  else if (ilv_env)
    hipLaunchKernelGGL((mlp_fused_h_kernel<2, false, false, true>), dim3((unsigned)tiles), dim3(64 * MH_WAVES), 0, s, p);
  else
    hipLaunchKernelGGL((mlp_fused_h_kernel<2, false, false>), dim3((unsigned)tiles), dim3(64 * MH_WAVES), 0, s, p);
  return launch_check("mlp_fused_h");
}

}  // namespace msfno
