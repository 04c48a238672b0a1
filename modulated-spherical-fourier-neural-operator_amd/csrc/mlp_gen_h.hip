// The network encoder / decoder MLP (sfnonet.py:513-523, 617-629; MLP.forward,
// layers.py:145-178) fused on the x3h engine:
//   out = W2 · GELU(W1 · [x ; x2] + b1) (+ b2) (+ addend)
// one launch, the hidden activation on-chip: the tiling of mlp_fused_h_kernel (16 pixels
// per wave, 64 per workgroup, two workgroups per CU, 16x16x32 fp16 MFMAs, three per fp32
// product; mlp_fused_h.hip has the engine and its error bound) with compile-time widths:
// KS k-steps of 32 input channels (Cin + Cin2 <= 32 KS), H hidden rows (runtime, a
// multiple of 64) and OT output tiles of 16 channels (Cout <= 16 OT).
//
// Range: every input of the block MLP has a per-channel bound from its norm statistics;
// the encoder's and decoder's inputs have none, so the scales are per PIXEL, formed from
// the pixel's own channels in registers (the four lanes that hold a pixel):
//   M = max_c |x[c]|,  xi = 2^(14 - e) for M = f 2^e  ->  |xi x| < 2^14;
//   |z_j| <= ||W1_j||_1 M + |b1_j| <= L_j (M + 1), L_j = max(||W1_j||_1, |b1_j|):
//   h_j is multiplied by eta_j = 2^-ceil(log2 L_j) (folded into W2's columns) and by
//   etap = 2^(14 - e') for M + 1 = f' 2^e', so |h'| < 2^14;
// the weights are row-scaled into [2^14, 2^15) as in mlp_fused_h.hip.  Each pixel's
// column of the product is then exact to the x3h bound relative to its own largest
// input, which is what an fp32 GEMM's own rounding gives.
//
// Weight image: a stream of 2-KB tiles (one 16 x 32 MFMA A operand, two fp16 planes,
// [pl][r 16][32] with the mh_swz k-group swizzle), consumed in units:
//   unit 0:        fc1 tiles of hidden block 0                   (2 KS tiles)
//   unit j (1..HB-1): fc1 tiles of block j, then fc2 tiles of block j - 1 (2 KS + OT)
//   unit HB:       fc2 tiles of block HB - 1                     (OT)
// each unit padded to whole 16-KB slices (8 tiles; the pad tiles are streamed, never
// multiplied) so every slice boundary falls at a compile-time tile position.  The slices
// stream through a four-slot LDS ring by LDS-DMA exactly as in mlp_fused_h.hip.
// fc1 tile (ks, t) of block j: W1 rows 32 j + 16 t + r, columns 32 ks + k;
// fc2 tile ot of block j: W2' rows 16 ot + r, hidden columns 32 j + mh_perm(k) (the C
// layout of the fc1 accumulators becomes fc2's B fragment in place).
#include "dma.h"
#include "gemm_common.h"
#include "kernels.h"

#include <algorithm>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>

namespace msfno {

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int MG_TILE = 1024;   // fp16 per 2-KB tile (two 512-element planes)
constexpr int MG_SLICE = 8;     // tiles per 16-KB slice
constexpr int MG_NS = 4;        // ring slots
constexpr int MG_WAVES = 4;
constexpr int MG_H_MAX = 256;

__host__ __device__ constexpr int mg_round8(int n) { return (n + 7) & ~7; }

// unit u's first tile (units of the padded stream)
__host__ __device__ constexpr int mg_unit_tile(int u, int KS, int OT) {
  return u == 0 ? 0 : mg_round8(2 * KS) + (u - 1) * mg_round8(2 * KS + OT);
}
__host__ __device__ constexpr int mg_tiles(int HB, int KS, int OT) {
  return mg_unit_tile(HB, KS, OT) + mg_round8(OT);
}

__host__ __device__ __forceinline__ int mg_swz(int r) { return ((r >> 2) & 1) << 1; }
__host__ __device__ __forceinline__ int mg_perm(int kappa) {
  const int g = kappa >> 3, e = kappa & 7;
  return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4);
}

__device__ __forceinline__ void mg_split(float a, float b, uint32_t& t0, uint32_t& t1) {
  const f2v v = {a, b};
  const half2v h0 = __builtin_convertvector(v, half2v);
  const f2v r = v - __builtin_convertvector(h0, f2v);
  const half2v h1 = __builtin_convertvector(r, half2v);
  t0 = __builtin_bit_cast(uint32_t, h0);
  t1 = __builtin_bit_cast(uint32_t, h1);
}

__device__ __forceinline__ half8 mg_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(half8, make_uint4(a, b, c, d));
}

// 2^(t - e) for v = f 2^e (f in [0.5, 1)); 1 for v = 0 / non-finite
__device__ __forceinline__ float mg_pow2_below(float v, int t) {
  if (!(v > 0.f) || !isfinite(v)) return 1.f;
  int e;
  frexpf(v, &e);
  return ldexpf(1.f, min(max(t - e, -120), 120));
}

template <int... I, class F>
__device__ __forceinline__ void mg_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void mg_for(F&& f) {
  mg_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// ---- weight image ------------------------------------------------------------------
// eta_j = 2^-ceil(log2 L_j), L_j = max(||W1_j||_1, |b1_j|); W1 (H x Ct).  One 256-thread
// workgroup per row (the row sum in fp64, a fixed reduction order)
__global__ __launch_bounds__(256) void mg_eta_kernel(const float* __restrict__ W1,
                                                     const float* __restrict__ b1, int Ct,
                                                     float* __restrict__ eta) {
  __shared__ double red[256];
  const int r = blockIdx.x, t = threadIdx.x;
  const float* row = W1 + (int64_t)r * Ct;
  double l1 = 0.0;
  for (int k = t; k < Ct; k += 256) l1 += fabs((double)row[k]);
  red[t] = l1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t != 0) return;
  const double L = fmax(red[0], fabs((double)b1[r])) * (1.0 + 1e-6);
  float e = 1.f;
  if (L > 0.0 && L < 1e30) {
    int x;
    frexp(L, &x);
    e = (float)ldexp(1.0, min(max(-x, -120), 120));
  }
  eta[r] = e;
}

// row scales 2^(15 - e), max |row| = f 2^e (W2 rows taken as W2 diag(1 / eta)); inverses
// into is1 [H] / is2 [16 OT] (0 past Cout).  One 256-thread workgroup per row
__global__ __launch_bounds__(256) void mg_scale_kernel(
    const float* __restrict__ W1, const float* __restrict__ W2, const float* __restrict__ eta,
    int H, int Ct, int Cout, float* __restrict__ s1, float* __restrict__ s2,
    float* __restrict__ is1, float* __restrict__ is2) {
  __shared__ float red[256];
  const int r = blockIdx.x, t = threadIdx.x;
  const bool first = r < H;
  if (!first && r - H >= Cout) {
    if (t == 0) { s2[r - H] = 0.f; is2[r - H] = 0.f; }
    return;
  }
  const float* row = first ? W1 + (int64_t)r * Ct : W2 + (int64_t)(r - H) * H;
  const int n = first ? Ct : H;
  float m = 0.f;
  for (int k = t; k < n; k += 256) m = fmaxf(m, fabsf(first ? row[k] : row[k] / eta[k]));
  red[t] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] = fmaxf(red[t], red[t + o]);
    __syncthreads();
  }
  if (t != 0) return;
  m = red[0];
  float sc = 1.f;
  if (m > 0.f && isfinite(m)) {
    int e;
    frexpf(m, &e);
    sc = ldexpf(1.f, 15 - e);
  }
  if (first) { s1[r] = sc; is1[r] = 1.f / sc; }
  else { s2[r - H] = sc; is2[r - H] = 1.f / sc; }
}

// one thread per fp16 pair of a real (non-pad) tile
// layout 0: the unit stream above; layout 1 (mlp_gen_hp_kernel): all fc1 tiles first,
// block-major (tile 2 KS j + i), then the fc2 tiles output-tile-major (tile 2 KS HB +
// HB ot + j), no pad tiles
__global__ void mg_image_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                const float* __restrict__ eta, const float* __restrict__ s1,
                                const float* __restrict__ s2, int H, int Ct, int Cout, int KS,
                                int OT, int layout, unsigned short* __restrict__ img) {
  const int HB = H / 32;
  const int64_t n1 = (int64_t)HB * 2 * KS * 256, n2 = (int64_t)HB * OT * 256;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n1 + n2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const bool fc1 = e < n1;
    const int64_t f = fc1 ? e : e - n1;
    const int kkp = (int)(f & 15), r = (int)((f >> 4) & 15);
    const int64_t tile_id = f >> 8;
    const int kk = 2 * kkp;
    const int kap = 8 * ((kk >> 3) ^ mg_swz(r)) + (kk & 7);  // k of the stored position kk
    float v0, v1;
    int64_t tile;
    if (fc1) {
      const int j = (int)(tile_id / (2 * KS)), i = (int)(tile_id % (2 * KS));
      const int ks = i >> 1, t = i & 1;
      const int row = 32 * j + 16 * t + r, k = 32 * ks + kap;
      const float sc = s1[row];
      const float* w = W1 + (int64_t)row * Ct;
      v0 = k < Ct ? w[k] * sc : 0.f;
      v1 = k + 1 < Ct ? w[k + 1] * sc : 0.f;
      tile = layout ? 2 * KS * j + i : mg_unit_tile(j, KS, OT) + i;
    } else {
      const int j = (int)(tile_id / OT), ot = (int)(tile_id % OT);
      const int orow = 16 * ot + r;
      const int k0 = 32 * j + mg_perm(kap), k1 = 32 * j + mg_perm(kap + 1);
      if (orow < Cout) {
        const float sc = s2[orow];
        const float* w = W2 + (int64_t)orow * H;
        v0 = w[k0] / eta[k0] * sc;
        v1 = w[k1] / eta[k1] * sc;
      } else {
        v0 = v1 = 0.f;
      }
      tile = layout ? (int64_t)2 * KS * HB + (int64_t)HB * ot + j
                    : mg_unit_tile(j + 1, KS, OT) + (j + 1 < HB ? 2 * KS : 0) + ot;
    }
    uint32_t t0, t1;
    mg_split(v0, v1, t0, t1);
    uint32_t* o = reinterpret_cast<uint32_t*>(img + tile * MG_TILE + r * 32 + kk);
    o[0] = t0;
    o[256] = t1;  // plane 1: +512 fp16
  }
}

struct MlpGParams {
  const float* x;       // [B][Cin][P]
  const float* x2;      // [B][Cin2][P] or null
  const float* xa;      // [B][Cin] per-channel affine of x (x -> xa x + xt) or null
  const float* xt;      // [B][Cin]
  const float* addend;  // [.][Cout][P] (batch stride add_bstride) or null
  float* out;           // [B][Cout][P]
  const unsigned short* img;
  const float* is1;     // [H] 1 / W1 row scale
  const float* is2;     // [16 OT] 1 / W2' row scale
  const float* eta;     // [H]
  const float* b1;      // [H]
  const float* b2;      // [Cout] or null
  int64_t P, add_bstride;
  int Cin, Cin2, Cout, H, nslice, tiles_per_field;
  int tiles;            // mlp_gen_hp_kernel: tiles of 128 pixels over all fields
};

// four wave-instructions (one m0 save / restore) of a 16-KB slice: lane l copies 16 B
// from sbase + voff[i] to LDS byte lds + i * LDS_STEP + 16 l
template <int LDS_STEP>
__device__ __forceinline__ void mg_glds16x4(uint64_t sbase, const uint32_t (&voff)[4], uint32_t lds) {
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

// BUF: x, x2, addend and output addressed as raw buffers (32-bit lane offsets; channels
// past Cin / Cin2 and rows past Cout fall outside the plane's range, which the buffer
// range check (lane offset only: the SGPR offset is not checked) reads as 0 / drops); the
// host takes it when every plane is below 2 GB and x2 starts on a k-step (Cin % 32 == 0)
template <int KS, int OT, bool EARLY, bool BUF>
__global__ __launch_bounds__(256, 2) void mlp_gen_h_kernel(MlpGParams p) {
  constexpr int W = MG_WAVES, NS = MG_NS;
  constexpr int SLICE_E = MG_SLICE * MG_TILE;    // fp16 per slice
  constexpr int RING_BYTES = NS * SLICE_E * 2;
  constexpr int NT1 = 2 * KS, NT2 = OT;
  constexpr int NU = mg_round8(NT1 + NT2);       // tiles per middle unit
  constexpr int N0 = mg_round8(NT1);
  constexpr int CP = 16 * OT;
  __shared__ __attribute__((aligned(16))) char lds_raw[RING_BYTES + (3 * MG_H_MAX + 2 * CP + 64 * KS) * 4];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const b1s = reinterpret_cast<float*>(lds_raw + RING_BYTES);
  float* const is1s = b1s + MG_H_MAX;
  float* const etas = is1s + MG_H_MAX;
  float* const b2s = etas + MG_H_MAX;
  float* const is2s = b2s + CP;
  float* const xas = is2s + CP;  // deferred input affine [32 KS]
  float* const xts = xas + 32 * KS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int z = lin / p.tiles_per_field;
  const int64_t P = p.P;
  const int64_t px = (int64_t)(lin - z * p.tiles_per_field) * (16 * W) + 16 * wave + r16;
  const int64_t pxc = px < P ? px : P - 1;
  const int H = p.H, HB = H >> 5, nslice = p.nslice;

  // ---- slices 0..NS-1 in flight ------------------------------------------------------
  const uint32_t ring_lds = lds_addr(ring);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  uint32_t piece_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) piece_off[i] = (uint32_t)(i * W * 1024 + lane * 16);
  auto issue = [&](int q) {
    const uint64_t src = reinterpret_cast<uint64_t>(p.img + (int64_t)q * SLICE_E) + (uint64_t)wave_u * 1024;
    mg_glds16x4<W * 1024>(src, piece_off, ring_lds + (uint32_t)((q % NS) * SLICE_E * 2 + wave_u * 1024));
  };
#pragma unroll
  for (int q = 0; q < NS; ++q)
    if (q < nslice) issue(q);

  // ---- x of the wave's 16 pixels (k-step ks: channels 32 ks + 8 g + e) -----------------
  const float* xb = p.x + (int64_t)z * p.Cin * P + pxc;
  const float* x2b = p.x2 ? p.x2 + (int64_t)z * p.Cin2 * P + pxc : nullptr;
  float xv[KS][8];
  const uint32_t P4 = (uint32_t)(P * 4);
  if constexpr (BUF) {
    const auto xr = buf_rsrc(p.x + (int64_t)z * p.Cin * P, (int64_t)p.Cin * P * 4);
    const auto x2r = buf_rsrc(p.x2 ? p.x2 + (int64_t)z * p.Cin2 * P : p.x, (int64_t)p.Cin2 * P * 4);
    const uint32_t vo = (uint32_t)(((int64_t)(8 * g) * P + pxc) * 4);
    const int ks1 = p.Cin >> 5;  // k-steps of x (Cin % 32 == 0 when x2 is given)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xv[ks][e] = (p.x2 && ks >= ks1) ? buf_ld_nt(x2r, vo + (uint32_t)(32 * (ks - ks1) + e) * P4, 0)
                                        : buf_ld_nt(xr, vo + (uint32_t)(32 * ks + e) * P4, 0);
  } else {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 32 * ks + 8 * g + e;
        float v = 0.f;
        if (c < p.Cin) v = __builtin_nontemporal_load(xb + (int64_t)c * P);
        else if (c - p.Cin < p.Cin2) v = __builtin_nontemporal_load(x2b + (int64_t)(c - p.Cin) * P);
        xv[ks][e] = v;
      }
  }

  for (int i = tid; i < H; i += 64 * W) {
    b1s[i] = p.b1[i];
    is1s[i] = p.is1[i];
    etas[i] = p.eta[i];
  }
  for (int i = tid; i < CP; i += 64 * W) {
    b2s[i] = (p.b2 && i < p.Cout) ? p.b2[i] : 0.f;
    is2s[i] = p.is2[i];
  }
  if (p.xa) {  // the producer's deferred per-channel affine (channels < Cin, 0 beyond)
    for (int i = tid; i < 32 * KS; i += 64 * W) {
      const bool in = i < p.Cin;
      xas[i] = in ? p.xa[(int64_t)z * p.Cin + i] : 1.f;
      xts[i] = in ? p.xt[(int64_t)z * p.Cin + i] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = 32 * ks + 8 * g;
      const float4 a0 = *reinterpret_cast<const float4*>(xas + c0);
      const float4 a1 = *reinterpret_cast<const float4*>(xas + c0 + 4);
      const float4 t0 = *reinterpret_cast<const float4*>(xts + c0);
      const float4 t1 = *reinterpret_cast<const float4*>(xts + c0 + 4);
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float tv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[ks][e] = fmaf(av[e], xv[ks][e], tv[e]);
    }
  }
  // the pixel's bound M over all its channels (the four lanes r16, r16 + 16, ...)
  float m = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(xv[ks][e]));
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  const float xi = mg_pow2_below(m, 14);          // |x xi| < 2^14
  const float etap = mg_pow2_below(m + 1.f, 14);  // |h eta_j etap| < 2^14
  const float ixi = 1.f / xi, ietap = 1.f / etap;
  half8 xf[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    uint32_t t[2][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      mg_split(xv[ks][2 * e] * xi, xv[ks][2 * e + 1] * xi, t[0][e], t[1][e]);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) xf[ks][pl] = mg_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
  }
  floatx4 oacc[OT];
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) oacc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
  // the addend of every output row: with EARLY (the default) its loads are issued here and
  // waited with x's, so the two latencies overlap; otherwise under the last unit's MFMAs
  float rv[OT][4];
  auto load_addend = [&]() {
    if (p.addend && BUF) {
      const auto ar = buf_rsrc(p.addend + (int64_t)z * p.add_bstride, (int64_t)p.Cout * P * 4);
      const uint32_t vo = (uint32_t)(((int64_t)(4 * g) * P + pxc) * 4);
#pragma unroll
      for (int ot = 0; ot < OT; ++ot)
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[ot][i] = buf_ld_nt(ar, vo + (uint32_t)(16 * ot + i) * P4, 0);
    } else if (p.addend) {
      const float* ad = p.addend + (int64_t)z * p.add_bstride + pxc;
#pragma unroll
      for (int ot = 0; ot < OT; ++ot)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * ot + 4 * g + i;
          rv[ot][i] = r < p.Cout ? __builtin_nontemporal_load(ad + (int64_t)r * P) : 0.f;
        }
    } else {
#pragma unroll
      for (int ot = 0; ot < OT; ++ot)
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[ot][i] = 0.f;
    }
  };
  if constexpr (EARLY) load_addend();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  floatx4 hacc[2][2];  // [parity][tile t]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int t = 0; t < 2; ++t) hacc[a][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  uint32_t hfu[2][4];  // fc2 B fragment of the converted block [plane][pair]
  half8 hb[2];
  const int a_lane = r16 * 32 + 8 * (g ^ mg_swz(r16));

  // slice q landed for every wave (up to NS - 2 later slices stay in flight); the slot of
  // slice q - 1 is free and takes slice q + NS - 1
  auto step_begin = [&](int q) {
    const int after = min(NS - 2, nslice - 1 - q);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (q >= 1 && q + NS - 1 < nslice) issue(q + NS - 1);
    return ring + (q % NS) * SLICE_E;
  };
  auto mfma3 = [](const half8 (&a)[2], const half8 (&b)[2], floatx4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
  };
  // pair e2 (0..3) of hidden block j in hacc[PAR]: unscale, + b1, GELU(erf), scale, split
  auto conv_pair = [&](int j, int e2, auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    const int t = e2 >> 1, i = 2 * (e2 & 1);
    const int row = 32 * j + 16 * t + 4 * g + i;
    const float2 b = *reinterpret_cast<const float2*>(b1s + row);
    const float2 is = *reinterpret_cast<const float2*>(is1s + row);
    const float2 hs = *reinterpret_cast<const float2*>(etas + row);
    f32x2 v = {fmaf(hacc[PAR][t][i], is.x * ixi, b.x), fmaf(hacc[PAR][t][i + 1], is.y * ixi, b.y)};
    v = gelu_erf2(v) * f32x2{hs.x * etap, hs.y * etap};
    mg_split(v.x, v.y, hfu[0][e2], hfu[1][e2]);
  };
  auto make_hb = [&]() {
    hb[0] = mg_frag(hfu[0][0], hfu[0][1], hfu[0][2], hfu[0][3]);
    hb[1] = mg_frag(hfu[1][0], hfu[1][1], hfu[1][2], hfu[1][3]);
  };

  // one unit: FC1 -> fc1 tiles of block j into hacc[PAR] (converting block j - 1 from
  // hacc[PAR ^ 1] on the way when FC2), FC2 -> fc2 tiles of block j - 1
  auto unit = [&](int j, int s0, auto par_c, auto fc1_c, auto fc2_c) {
    constexpr int PAR = decltype(par_c)::value;
    constexpr bool FC1 = decltype(fc1_c)::value, FC2 = decltype(fc2_c)::value;
    constexpr int n1 = FC1 ? NT1 : 0;
    constexpr int NTOT = n1 + (FC2 ? NT2 : 0);
    using PPrev = std::integral_constant<int, PAR ^ 1>;
    const unsigned short* slot = ring;
    mg_for<NTOT>([&](auto pc) {
      constexpr int pos = decltype(pc)::value;
      if constexpr (pos % MG_SLICE == 0) slot = step_begin(s0 + pos / MG_SLICE);
      const unsigned short* tp = slot + (pos % MG_SLICE) * MG_TILE + a_lane;
      const half8 a[2] = {*reinterpret_cast<const half8*>(tp),
                          *reinterpret_cast<const half8*>(tp + 512)};
      if constexpr (pos < n1) {
        mfma3(a, xf[pos >> 1], hacc[PAR][pos & 1]);
        if constexpr (FC2) {  // four conversions of block j - 1 spread over the fc1 tiles
          constexpr int c0 = (1 * NT1) / 5, c1 = (2 * NT1) / 5, c2 = (3 * NT1) / 5, c3 = (4 * NT1) / 5;
          if constexpr (pos == c0) conv_pair(j - 1, 0, PPrev{});
          if constexpr (pos == (c1 > c0 ? c1 : c0)) conv_pair(j - 1, 1, PPrev{});
          if constexpr (pos == (c2 > c1 ? c2 : c1)) conv_pair(j - 1, 2, PPrev{});
          if constexpr (pos == (c3 > c2 ? c3 : c2)) conv_pair(j - 1, 3, PPrev{});
        }
        if constexpr (FC2 && pos == n1 - 1) {
          make_hb();
#pragma unroll
          for (int t = 0; t < 2; ++t) hacc[PAR ^ 1][t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        mfma3(a, hb, oacc[pos - n1]);
      }
    });
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  using T = std::true_type;
  unit(0, 0, I0{}, T{}, F{});
  for (int j = 1; j < HB; j += 2) {
    unit(j, (N0 + (j - 1) * NU) / MG_SLICE, I1{}, T{}, T{});
    if (j + 1 < HB) unit(j + 1, (N0 + j * NU) / MG_SLICE, I0{}, T{}, T{});
  }
  // HB is even: block HB - 1 sits in hacc[1]
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) conv_pair(HB - 1, e2, I1{});
  make_hb();
  // (not EARLY: in flight under the last unit's MFMAs; three workgroups per CU with half
  // of it issued after that unit measured slower: 1.55 vs 1.33 ms for the encoder)
  if constexpr (!EARLY) load_addend();
  unit(HB, (N0 + (HB - 1) * NU) / MG_SLICE, I0{}, F{}, T{});

  // ---- epilogue: unscale + b2 + addend, store (rows 16 ot + 4 g + i) -------------------
  if (px >= P) return;
  float* o = p.out + (int64_t)z * p.Cout * P + px;
  const auto orr = buf_rsrc(p.out + (int64_t)z * p.Cout * P, (int64_t)p.Cout * P * 4);
  const uint32_t vo = (uint32_t)(((int64_t)(4 * g) * P + px) * 4);
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
    const int r0 = 16 * ot + 4 * g;
    const float4 is = *reinterpret_cast<const float4*>(is2s + r0);
    const float4 b = *reinterpret_cast<const float4*>(b2s + r0);
    const float isv[4] = {is.x * ietap, is.y * ietap, is.z * ietap, is.w * ietap};
    const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = fmaf(oacc[ot][i], isv[i], bv[i]) + rv[ot][i];
      if constexpr (BUF) buf_st_nt(v, orr, vo + (uint32_t)(16 * ot + i) * P4, 0);  // rows past Cout: out of range
      else if (r0 + i < p.Cout) o[(int64_t)(r0 + i) * P] = v;
    }
  }
}


// ---- persistent, pipelined form (the encoder: Ct <= 96, H = 256, no second input) ------
// mlp_gen_h_kernel runs one 64-pixel tile per workgroup: the x and addend loads, the
// slice steps and the 4-byte output stores are three phases that every CU enters at
// nearly the same time (PMC: MFMA busy 19 %, 56 % of wave cycles waiting on memory).
// Here one workgroup per CU walks a contiguous range of 128-pixel tiles (PG = 2, the
// default: four waves, one per SIMD with the whole register file, 32 pixels per wave as
// two 16-pixel groups, so each A fragment read from LDS feeds two MFMA triples; PG = 1:
// eight waves of 16 pixels, see GpShape); and the loop order is changed so that no HBM
// phase is left outside the slice steps:
//   - fc1 for all 8 hidden blocks first (6 slices), the GELU'd hidden activation of the
//     whole tile kept in registers as fc2 B fragments (fp16x2 pairs, 128 VGPRs);
//   - then fc2 one 16-row output tile per slice (the slice holds W2' rows 16 ot..+15 for
//     all 256 hidden channels), so an output tile is final after its own step: its
//     epilogue runs in the next step (scaled, + b2, transposed through a per-wave LDS
//     patch, + addend, 16-B stores of 128-B lines), under that step's MFMAs;
//   - the DMA group of a step carries, besides its 16-KB weight slice, PG-KB pieces per
//     wave: in the first fc1 steps 16 channels of the NEXT tile's x (raw fp32, into a
//     per-wave LDS buffer that is split into fp16 terms at the tile end, when the pixel's
//     range scale over all its channels is known), in the fc2 steps the 16 addend rows of
//     this tile's output tile (into the ring slot, read back by the lane that stores
//     them).  Each wave's pieces hold only its own pixels.
// Arithmetic per output element is that of mlp_gen_h_kernel (same MFMA order, same
// epilogue), so the two kernels agree bit for bit.
//
// vmcnt accounting (each wave, in issue order): group n = WD weight DMAs + PG per piece
// of step n (GpShape::grp), issued in step n - (NS - 1) after that step's epilogue stores
// (PG per lane, GpShape::sto).  The wait for group n counts the stores and groups of the NS - 2 steps
// in between (GpShape::younger, compile-time per step).  Groups 0..NS-2 are drained in
// the prologue; the last tile issues dummy groups (its own slices and pieces again) and
// the kernel drains every DMA before it exits.
constexpr int GP_PX = 128;                     // pixels per tile
constexpr int GP_HB = 8;                       // hidden blocks of 32 (H = 256)
constexpr int GP_WB = MG_SLICE * MG_TILE * 2;  // 16 KB of weight tiles per slice
constexpr int GP_SLOT = GP_WB + 8 * 1024;      // + the waves' addend pieces (8 KB)

// PG 16-pixel groups per wave, W = 8 / PG waves: PG = 2 -> one wave per SIMD with the
// whole register file, each A fragment read feeding two MFMA triples; PG = 1 -> two waves
// per SIMD (256 registers each), one wave's VALU, LDS and barrier time under the other's
// MFMAs.  A wave's piece (x or addend) is 16 rows x 16 PG pixels: PG KB, PG DMAs.
template <int KS, int OT, bool ADD, int NS_, int PG_>
struct GpShape {
  static constexpr int NS = NS_, PG = PG_, W = 8 / PG_;
  static constexpr int HB = GP_HB, NT1 = 2 * KS, NF = NT1 * HB;
  static constexpr int NQ1 = NF / MG_SLICE;  // fc1 steps
  static constexpr int NQ = NQ1 + OT;        // steps per tile
  static constexpr int CP = 16 * OT;
  static constexpr int WD = 16 / W;          // weight DMAs per wave and slice (1 KB each)
  static constexpr int ERS = 16 * PG + 4;    // epilogue patch row stride (floats)
  static constexpr int EPI = 16 * ERS * 4;   // per wave: 16 rows x 16 PG pixels
  // the next tile's x: 2 KS pieces (16 channels) per wave, carried by the groups of steps
  // XS .. XS + 2 KS - 1 (issued in this tile's first steps, after the previous tile's x
  // left the buffer) into a per-wave buffer read at the tile's end
  static constexpr int XS = NS - 1, NXP = 2 * KS, XW = NXP * PG * 1024;
  static constexpr int LDS = NS * GP_SLOT + W * XW + W * EPI + (3 * 32 * HB + 2 * CP) * 4;
  static_assert(NF % MG_SLICE == 0 && XS + NXP < NQ, "x pieces land before the tile's end");
  static_assert(OT % 2 == 0, "output tiles alternate between two accumulators");
  static_assert(LDS <= 160 * 1024, "mlp_gen_hp LDS");
  static_assert(NS >= 3 && (PG == 1 || PG == 2), "ring depth, pixel groups");
  __host__ __device__ static constexpr int md(int a) { return ((a % NQ) + NQ) % NQ; }
  __host__ __device__ static constexpr bool xp(int q) { return q >= XS && q < XS + NXP; }
  __host__ __device__ static constexpr bool ap(int q) { return ADD && q >= NQ1; }
  __host__ __device__ static constexpr int grp(int q) { return WD + (xp(q) ? PG : 0) + (ap(q) ? PG : 0); }
  __host__ __device__ static constexpr int sto(int q) { return (q == 0 || q > NQ1) ? PG : 0; }
  // vector-memory instructions a wave issues after group q
  __host__ __device__ static constexpr int younger(int q) {
    int k = 0;
    for (int d = 1; d <= NS - 2; ++d) k += sto(md(q - d)) + grp(md(q - d + NS - 1));
    return k;
  }
};

template <int N>
__device__ __forceinline__ void gp_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int KS, int OT, bool ADD, int NS_, int PG_>
__global__ __launch_bounds__(64 * (8 / PG_), 1) void mlp_gen_hp_kernel(MlpGParams p) {
  using S = GpShape<KS, OT, ADD, NS_, PG_>;
  constexpr int NS = S::NS, HB = S::HB, NT1 = S::NT1, NQ1 = S::NQ1, NQ = S::NQ, CP = S::CP;
  constexpr int PG = S::PG, W = S::W, ERS = S::ERS;
  __shared__ __attribute__((aligned(16))) char lds[S::LDS];
  char* const xbuf = lds + NS * GP_SLOT;
  float* const epi_all = reinterpret_cast<float*>(lds + NS * GP_SLOT + W * S::XW);
  float* const b1s = reinterpret_cast<float*>(lds + NS * GP_SLOT + W * S::XW + W * S::EPI);
  float* const is1s = b1s + 32 * HB;
  float* const etas = is1s + 32 * HB;
  float* const b2s = etas + 32 * HB;
  float* const is2s = b2s + CP;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t P = p.P;
  const int tpf = p.tiles_per_field;
  const int t0 = (int)((int64_t)blockIdx.x * p.tiles / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * p.tiles / gridDim.x);
  const int ntile = t1 - t0;  // >= 1: the host launches at most `tiles` workgroups
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t ring_lds = lds_addr(lds);
  const uint32_t xbuf_lds = ring_lds + NS * GP_SLOT;

  for (int i = tid; i < 32 * HB; i += 64 * W) {
    b1s[i] = p.b1[i];
    is1s[i] = p.is1[i];
    etas[i] = p.eta[i];
  }
  for (int i = tid; i < CP; i += 64 * W) {
    b2s[i] = (p.b2 && i < p.Cout) ? p.b2[i] : 0.f;
    is2s[i] = p.is2[i];
  }

  // tile tl of this workgroup (clamped to its last tile: the tail's dummy groups)
  struct Tile {
    int z;
    int64_t px0;
  };
  auto tile_of = [&](int tl) {
    const int t = t0 + (tl < ntile ? tl : ntile - 1);
    Tile r;
    r.z = t / tpf;
    r.px0 = (int64_t)(t - r.z * tpf) * GP_PX;
    return r;
  };

  // ---- DMA groups ----------------------------------------------------------------------
  // A piece DMA h2 (0..PG-1) of this wave: lane l -> LDS byte 16 l of the wave's 1-KB
  // half h2.  Addend pieces: row 8 h2 + (l >> 3) (PG 2) / l >> 2 (PG 1), pixel quad l & 7 /
  // l & 3 (read back by the same lane).  x pieces: the row / quad order chosen so that the
  // four lane groups reading a piece row hit distinct LDS banks: PG 2 as the addend with
  // quad (l & 7) ^ (R & 4); PG 1: position l >> 2 holds row R = 4 (pos & 3) + (pos >> 2).
  auto xrow_of = [&](int ln, int h2) {  // piece row R of lane ln's x DMA h2
    if constexpr (PG == 2) return 8 * h2 + (ln >> 3);
    else { const int pos = ln >> 2; return 4 * (pos & 3) + (pos >> 2); }
  };
  auto xquad_of = [&](int ln, int R) {  // pixel quad of lane ln's x DMA
    if constexpr (PG == 2) return (ln & 7) ^ (R & 4);
    else return ln & 3;
  };
  auto issue = [&](uint32_t slot_off, const Tile& tw, const Tile& tx, auto qc) {
    constexpr int Q = decltype(qc)::value;
    // opaque copies: keep the per-step address arithmetic at the step (hoisted to the
    // tile start, 22 steps of addresses overflow the SGPRs)
    uint64_t img = reinterpret_cast<uint64_t>(p.img), xg = reinterpret_cast<uint64_t>(p.x),
             ag = reinterpret_cast<uint64_t>(p.addend);
    asm volatile("" : "+s"(img), "+s"(xg), "+s"(ag));
    // (and an opaque lane index: the per-lane offsets of 22 steps are not precomputed)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t slot = ring_lds + slot_off;
    const uint64_t wsrc = img + (uint64_t)Q * MG_SLICE * MG_TILE * 2 + (uint64_t)wave_u * 1024;
#pragma unroll
    for (int i = 0; i < S::WD; ++i)
      glds16s(wsrc + (uint64_t)(i * W * 1024), (uint32_t)(ln * 16),
              slot + (uint32_t)(i * W * 1024 + wave_u * 1024));
    if constexpr (S::xp(Q)) {  // 16 channels of tile tx's x
      constexpr int k = Q - S::XS, ks = k >> 1, h = k & 1;
      const uint64_t base = xg + (uint64_t)((int64_t)tx.z * p.Cin * P * 4);
      const uint32_t xdst = xbuf_lds + (uint32_t)(wave_u * S::XW + k * PG * 1024);
#pragma unroll
      for (int h2 = 0; h2 < PG; ++h2) {
        const int R = xrow_of(ln, h2);
        const int c = min(32 * ks + 8 * (R >> 2) + 4 * h + (R & 3), p.Cin - 1);
        const int64_t px = min(tx.px0 + 16 * PG * wave + 4 * xquad_of(ln, R), P - 4);
        glds16s(base, (uint32_t)(((int64_t)c * P + px) * 4), xdst + (uint32_t)(h2 * 1024));
      }
    }
    if constexpr (S::ap(Q)) {  // addend rows 16 ot .. + 15 of tile tw
      constexpr int ot = Q - NQ1;
      const uint64_t base = ag + (uint64_t)((int64_t)tw.z * p.add_bstride * 4);
      const uint32_t pdst = slot + (uint32_t)(GP_WB + wave_u * PG * 1024);
#pragma unroll
      for (int h2 = 0; h2 < PG; ++h2) {
        const int row = PG == 2 ? 8 * h2 + (ln >> 3) : ln >> 2;
        const int quad = PG == 2 ? ln & 7 : ln & 3;
        const int r = min(16 * ot + row, p.Cout - 1);
        const int64_t px = min(tw.px0 + 16 * PG * wave + 4 * quad, P - 4);
        glds16s(base, (uint32_t)(((int64_t)r * P + px) * 4), pdst + (uint32_t)(h2 * 1024));
      }
    }
  };

  // ---- register state --------------------------------------------------------------------
  half8 xf[PG][KS][2];          // this tile's x (B fragments of fc1) [pg][ks][plane]
  uint32_t hf[HB][PG][2][4];    // hidden activation: fc2 B fragments [j][pg][plane][pair]
  floatx4 hacc[2][PG][2];       // fc1 accumulators [block parity][pg][t]
  floatx4 oacc[2][PG];          // fc2 accumulators [output-tile parity][pg]
  float ixi[PG], etap[PG], ietap[PG], iet_prev[PG];

  // x (per pixel: the range scales, then the fp16x2 split); xv[pg][ks][e] raw, 0 past Cin
  auto split_x = [&](const float (&xv)[PG][KS][8]) {
#pragma unroll
    for (int pg = 0; pg < PG; ++pg) {
      float m = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(xv[pg][ks][e]));
      m = fmaxf(m, __shfl_xor(m, 16));
      m = fmaxf(m, __shfl_xor(m, 32));
      const float xi = mg_pow2_below(m, 14);
      etap[pg] = mg_pow2_below(m + 1.f, 14);
      ixi[pg] = 1.f / xi;
      ietap[pg] = 1.f / etap[pg];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        uint32_t t[2][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          mg_split(xv[pg][ks][2 * e] * xi, xv[pg][ks][2 * e + 1] * xi, t[0][e], t[1][e]);
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) xf[pg][ks][pl] = mg_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
      }
    }
  };

  // ---- prologue: groups 0..NS-2 in flight, the first tile's x by plain loads --------------
  {
    const Tile c0 = tile_of(0), c1 = tile_of(1);
    mg_for<NS - 1>([&](auto qc) { issue((uint32_t)(decltype(qc)::value * GP_SLOT), c0, c1, qc); });
    const float* xb = p.x + (int64_t)c0.z * p.Cin * P;
    float xr[PG][KS][8];
#pragma unroll
    for (int pg = 0; pg < PG; ++pg) {
      const int64_t px = min(c0.px0 + 16 * PG * wave + 16 * pg + r16, P - 1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 32 * ks + 8 * g + e;
          xr[pg][ks][e] = c < p.Cin ? __builtin_nontemporal_load(xb + (int64_t)c * P + px) : 0.f;
        }
    }
    split_x(xr);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int pg = 0; pg < PG; ++pg) {
#pragma unroll
      for (int t = 0; t < 2; ++t) hacc[a][pg][t] = floatx4{0.f, 0.f, 0.f, 0.f};
      oacc[a][pg] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

  const int a_lane = r16 * 32 + 8 * (g ^ mg_swz(r16));
  float* const ep = epi_all + wave * 16 * ERS;
  auto mfma3 = [](const half8 (&a)[2], const half8 (&b)[2], floatx4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
  };
  // pair e2 of hidden block j, pixel group pg (hacc[j & 1]): unscale, + b1, GELU, scale, split
  auto conv = [&](auto jc, auto pgc, auto e2c) {
    constexpr int j = decltype(jc)::value, pg = decltype(pgc)::value, e2 = decltype(e2c)::value;
    constexpr int t = e2 >> 1, i = 2 * (e2 & 1);
    const int row = 32 * j + 16 * t + 4 * g + i;
    const float2 b = *reinterpret_cast<const float2*>(b1s + row);
    const float2 is = *reinterpret_cast<const float2*>(is1s + row);
    const float2 hs = *reinterpret_cast<const float2*>(etas + row);
    const floatx4& h = hacc[j & 1][pg][t];
    f32x2 v = {fmaf(h[i], is.x * ixi[pg], b.x), fmaf(h[i + 1], is.y * ixi[pg], b.y)};
    v = gelu_erf2(v) * f32x2{hs.x * etap[pg], hs.y * etap[pg]};
    mg_split(v.x, v.y, hf[j][pg][0][e2], hf[j][pg][1][e2]);
  };
  // the conversions of a block: 4 pairs per pixel group, spread over the next block's tiles
  constexpr int NCONV = 4 * PG;
  // step n's entry (run in step n - 1 under its last two tiles' MFMAs): group n landed
  // for every wave, all reads of step n - 1's slot issued by now complete (so the group
  // issued in step n may overwrite it), then the first two A fragments
  // A fragments of tiles u (mod NA), AH tiles ahead (PG 1: one ahead, two waves per SIMD
  // hide the rest; the register budget is 256)
  constexpr int AH = PG == 1 ? 1 : 2, NA = 2 * AH;
  half8 a[NA][2];
  auto prep = [&](auto qc, uint32_t slot_off) {
    constexpr int Q = decltype(qc)::value;
    gp_wait_vm<S::younger(Q)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned short* ws = reinterpret_cast<const unsigned short*>(lds + slot_off);
#pragma unroll
    for (int k = 0; k < AH; ++k)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        a[k][pl] = *reinterpret_cast<const half8*>(ws + k * MG_TILE + pl * 512 + a_lane);
  };

  // epilogue in two halves: (1) unscale + b2 into the wave's patch, (2) rows back as 16-B
  // vectors, + the addend piece of aslot, buffer stores
  auto epi_patch = [&](int ot, const floatx4 (&acc)[PG], const float (&iet)[PG]) {
    const int r0 = 16 * ot + 4 * g;
    const float4 is = *reinterpret_cast<const float4*>(is2s + r0);
    const float4 bb = *reinterpret_cast<const float4*>(b2s + r0);
#pragma unroll
    for (int pg = 0; pg < PG; ++pg) {
      float* e0 = ep + (4 * g) * ERS + 16 * pg + r16;
      e0[0] = fmaf(acc[pg][0], is.x * iet[pg], bb.x);
      e0[ERS] = fmaf(acc[pg][1], is.y * iet[pg], bb.y);
      e0[2 * ERS] = fmaf(acc[pg][2], is.z * iet[pg], bb.z);
      e0[3 * ERS] = fmaf(acc[pg][3], is.w * iet[pg], bb.w);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto epi_store = [&](int ot, const Tile& tw, const char* aslot) {
    // buffer stores: every wave issues all PG (the vmcnt counts stay exact); a lane past
    // the field's last pixel or row points outside the field's range and is dropped
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        p.out + (int64_t)tw.z * p.Cout * P, (short)0, (int)((int64_t)p.Cout * P * 4), 0x00020000);
#pragma unroll
    for (int k = 0; k < PG; ++k) {
      const int row = PG == 2 ? 8 * k + (lane >> 3) : lane >> 2;
      const int quad = PG == 2 ? lane & 7 : lane & 3;
      const int64_t pxl = tw.px0 + 16 * PG * wave + 4 * quad;
      floatx4 v = *reinterpret_cast<const floatx4*>(ep + row * ERS + 4 * quad);
      if constexpr (ADD)
        v += *reinterpret_cast<const floatx4*>(aslot + GP_WB + wave * PG * 1024 + k * 1024 + lane * 16);
      // (a row past Cout lies past the field's range by itself)
      const uint32_t off = pxl < P ? (uint32_t)(((int64_t)(16 * ot + row) * P + pxl) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), orsrc, off, 0, 2 /* nt */);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  prep(std::integral_constant<int, 0>{}, 0u);
  Tile prev = tile_of(0);
  // byte offsets of the slots of the current and the previous step (a running pair,
  // opaque to the compiler so that 22 steps of slot addresses are not precomputed)
  uint32_t so = 0, so_prev = (NS - 1) * GP_SLOT;
  for (int tl = 0; tl < ntile; ++tl) {
    const Tile cur = tile_of(tl), nx1 = tile_of(tl + 1), nx2 = tile_of(tl + 2);
    mg_for<NQ>([&](auto qc) {
      constexpr int Q = decltype(qc)::value;
      constexpr int QN = Q + NS - 1;  // the step whose group this step issues
      asm volatile("" : "+s"(so), "+s"(so_prev));
      const char* pslot = lds + so_prev;  // step n - 1
      const uint32_t so_next = so + GP_SLOT == NS * GP_SLOT ? 0u : so + GP_SLOT;
      const unsigned short* ws = reinterpret_cast<const unsigned short*>(lds + so);
      // the previous output tile (this tile's, or the last of the previous tile)
      constexpr bool EPI = Q > NQ1 || Q == 0;
      const bool epi = Q > NQ1 || (Q == 0 && tl > 0);
      if constexpr (Q == NQ1) {  // the last hidden block (its MFMAs ran in the last fc1 step)
        mg_for<NCONV>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          conv(std::integral_constant<int, HB - 1>{}, std::integral_constant<int, (c >> 2)>{},
               std::integral_constant<int, (c & 3)>{});
        });
#pragma unroll
        for (int pg = 0; pg < PG; ++pg)
#pragma unroll
          for (int t = 0; t < 2; ++t) hacc[(HB - 1) & 1][pg][t] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      mg_for<MG_SLICE>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u + AH < MG_SLICE) {
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            a[(u + AH) % NA][pl] = *reinterpret_cast<const half8*>(ws + (u + AH) * MG_TILE + pl * 512 + a_lane);
        }
        const half8(&av)[2] = a[u % NA];
        if constexpr (Q < NQ1) {  // fc1 tile f: block j, k-step ks, row half t
          constexpr int f = MG_SLICE * Q + u, j = f / NT1, i = f % NT1;
#pragma unroll
          for (int pg = 0; pg < PG; ++pg) mfma3(av, xf[pg][i >> 1], hacc[j & 1][pg][i & 1]);
          if constexpr (j >= 1) {  // block j - 1 converted under block j's tiles
            mg_for<NCONV>([&](auto cc) {
              constexpr int c = decltype(cc)::value;
              if constexpr ((c * NT1) / NCONV == i)
                conv(std::integral_constant<int, j - 1>{}, std::integral_constant<int, (c >> 2)>{},
                     std::integral_constant<int, (c & 3)>{});
            });
            if constexpr (i == ((NCONV - 1) * NT1) / NCONV) {
#pragma unroll
              for (int pg = 0; pg < PG; ++pg)
#pragma unroll
                for (int t = 0; t < 2; ++t) hacc[(j - 1) & 1][pg][t] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
          }
        } else {  // fc2 of output tile ot, hidden block u
          constexpr int ot = Q - NQ1;
          if constexpr (u == 0) {
#pragma unroll
            for (int pg = 0; pg < PG; ++pg) oacc[ot & 1][pg] = floatx4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int pg = 0; pg < PG; ++pg) {
            const half8 hb[2] = {mg_frag(hf[u][pg][0][0], hf[u][pg][0][1], hf[u][pg][0][2], hf[u][pg][0][3]),
                                 mg_frag(hf[u][pg][1][0], hf[u][pg][1][1], hf[u][pg][1][2], hf[u][pg][1][3])};
            mfma3(av, hb, oacc[ot & 1][pg]);
          }
        }
        if constexpr (EPI && u == 1) {
          if (epi) {
            if constexpr (Q == 0) epi_patch(OT - 1, oacc[(OT - 1) & 1], iet_prev);
            else epi_patch(Q - NQ1 - 1, oacc[(Q - NQ1 - 1) & 1], ietap);
          }
        }
        if constexpr (u == 3) {
          // the epilogue's stores, then this step's group (into the slot of step n - 1,
          // whose addend piece the stores have just read)
          if constexpr (EPI) {
            if (epi) {
              if constexpr (Q == 0) epi_store(OT - 1, prev, pslot);
              else epi_store(Q - NQ1 - 1, cur, pslot);
            }
          }
          if constexpr (QN < NQ) issue(so_prev, cur, nx1, std::integral_constant<int, QN>{});
          else issue(so_prev, nx1, nx2, std::integral_constant<int, QN - NQ>{});
        }
        if constexpr (u == 6) {
          if constexpr (Q + 1 < NQ) {
            prep(std::integral_constant<int, Q + 1>{}, so_next);
          } else {
            // the tile's end: the next tile's x (range scales, split; this tile's 1 / etap
            // kept for its last output tile, whose epilogue runs in the next tile's first
            // step), then the next tile's first step
#pragma unroll
            for (int pg = 0; pg < PG; ++pg) iet_prev[pg] = ietap[pg];
            if (tl + 1 < ntile) {
              // the next tile's x from the wave's buffer (channels 32 ks + 8 g + e of
              // piece 2 ks + e / 4, row 4 g + e % 4); channels past Cin read 0 (opaque:
              // loop-invariant lane masks would be hoisted into SGPRs)
              int cin = p.Cin;
              asm volatile("" : "+s"(cin));
              const char* xw = xbuf + wave * S::XW;
              auto xval = [&](int pg, int ks, int e8) {
                const int px = 16 * pg + r16, quad = px >> 2;
                const int k = 2 * ks + (e8 >> 2), R = 4 * g + (e8 & 3);
                int off;
                if constexpr (PG == 2)
                  off = k * 2048 + (R >> 3) * 1024 + ((R & 7) * 8 + (quad ^ (R & 4))) * 16 + (px & 3) * 4;
                else
                  off = k * 1024 + (4 * (e8 & 3) + g) * 64 + px * 4;
                const float v = *reinterpret_cast<const float*>(xw + off);
                return 32 * ks + 8 * g + e8 < cin ? v : 0.f;
              };
              // two passes over the buffer (range, then split) instead of 24 PG raw
              // values in registers beside the new fragments
#pragma unroll
              for (int pg = 0; pg < PG; ++pg) {
                float m = 0.f;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                  for (int e8 = 0; e8 < 8; ++e8) m = fmaxf(m, fabsf(xval(pg, ks, e8)));
                m = fmaxf(m, __shfl_xor(m, 16));
                m = fmaxf(m, __shfl_xor(m, 32));
                const float xi = mg_pow2_below(m, 14);
                etap[pg] = mg_pow2_below(m + 1.f, 14);
                ixi[pg] = 1.f / xi;
                ietap[pg] = 1.f / etap[pg];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                  uint32_t t[2][4];
#pragma unroll
                  for (int e = 0; e < 4; ++e)
                    mg_split(xval(pg, ks, 2 * e) * xi, xval(pg, ks, 2 * e + 1) * xi, t[0][e], t[1][e]);
#pragma unroll
                  for (int pl = 0; pl < 2; ++pl) xf[pg][ks][pl] = mg_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
                }
              }
              prep(std::integral_constant<int, 0>{}, so_next);
            }
          }
        }
      });
      so_prev = so;
      so = so_next;
    });
    prev = cur;
  }
  // the last output tile of the last tile (its addend piece is in the last step's slot)
  epi_patch(OT - 1, oacc[(OT - 1) & 1], iet_prev);
  epi_store(OT - 1, prev, lds + so_prev);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's dummy DMAs land before exit
}

// the instantiated widths: (KS, OT) = (3, 16): the encoder 73 -> 256 -> 256;
// (11, 5): the decoder 329 -> 256 -> 73
bool mg_shape(int Ct, int Cout, int* ks, int* ot) {
  const int k = (Ct + 31) / 32, o = (Cout + 15) / 16;
  if ((k == 3 && o == 16) || (k == 11 && o == 5)) {
    *ks = k;
    *ot = o;
    return true;
  }
  return false;
}

}  // namespace

// MSFNO_MLP_GEN_H=0 keeps the two-GEMM x6 path for the standalone MLP
static bool mlp_gen_h_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_MLP_GEN_H");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool mlp_gen_h_supported(int Ct, int H, int Cout) {
  int ks, ot;
  return mlp_gen_h_env() && mlp_fused_h_env() && gemm_use_x6() && H > 0 && H % 64 == 0 && H <= MG_H_MAX &&
         mg_shape(Ct, Cout, &ks, &ot);
}

size_t mlp_gen_h_workspace(int Ct, int H, int Cout) {
  int ks, ot;
  if (!mg_shape(Ct, Cout, &ks, &ot)) return 0;
  const int64_t tiles = mg_tiles(H / 32, ks, ot);
  return (size_t)round_up(tiles * MG_TILE * 2, 256) + (size_t)(3 * H + 4 * 16 * ot) * 4 + 256;
}

int launch_mlp_gen_h(const float* x, const float* xa, const float* xt, const float* x2, int Cin,
                     int Cin2, const float* W1,
                     const float* b1, const float* W2, const float* b2, int H, int Cout,
                     const float* addend, int64_t add_bstride, float* out, int B, int64_t P,
                     void* ws, size_t ws_bytes, hipStream_t s, void* cache, int cache_valid) {
  const int Ct = Cin + Cin2;
  int KS, OT;
  MSFNO_REQUIRE((xa == nullptr) == (xt == nullptr) && x && W1 && b1 && W2 && out && B > 0 && P >= 1 && Cin > 0 && Cin2 >= 0 &&
                    (Cin2 == 0) == (x2 == nullptr) && mlp_gen_h_supported(Ct, H, Cout) &&
                    mg_shape(Ct, Cout, &KS, &OT) &&
                    (cache || (ws && ws_bytes >= mlp_gen_h_workspace(Ct, H, Cout))),
                MSFNO_EINVAL, "mlp_gen_h: bad arguments");
  const int HB = H / 32, Cp = 16 * OT;
  const int64_t tiles = mg_tiles(HB, KS, OT);
  // the persistent pipelined kernel (the encoder shape; MSFNO_MG_P=0 keeps one tile per
  // workgroup).  Its pieces and stores move 4 pixels per lane (P % 4 == 0) with 32-bit
  // byte offsets into a field
  static const bool persist_env = [] {
    const char* e = getenv("MSFNO_MG_P");
    return !(e && e[0] == '0');
  }();
  const bool persist = persist_env && KS == 3 && OT == 16 && HB == GP_HB && !xa && !x2 &&
                       P % 4 == 0 && P >= 4 && (int64_t)Cin * P * 4 < (1LL << 32) &&
                       (int64_t)Cout * P * 4 < (1LL << 31);
  const int layout = persist ? 1 : 0;
  // the weight image and its scale vectors: in the caller's prepared-weight cache when
  // given (rebuilt only when cache_valid is 0), else in the workspace on every call
  char* base = static_cast<char*>(cache ? cache : ws);
  unsigned short* img = reinterpret_cast<unsigned short*>(base);
  float* eta = reinterpret_cast<float*>(base + round_up(tiles * MG_TILE * 2, 256));
  float* s1 = eta + H;
  float* is1 = s1 + H;
  float* s2 = is1 + H;
  float* is2 = s2 + Cp;
  // the image layout each cache was built with: a cached image of the other layout (a
  // call of the same weights that the persistent kernel cannot take) is rebuilt
  if (cache) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> built;
    std::lock_guard<std::mutex> lk(mu);
    auto it = built.find(cache);
    if (it == built.end() || it->second != layout) cache_valid = 0;
    built[cache] = layout;
  }
  if (!(cache && cache_valid)) {
    // the pad tiles are streamed (never multiplied): keep them finite
    if (hipMemsetAsync(img, 0, tiles * MG_TILE * 2, s) != hipSuccess) {
      set_error("mlp_gen_h: image clear failed");
      return MSFNO_EHIP;
    }
    hipLaunchKernelGGL(mg_eta_kernel, dim3(H), dim3(256), 0, s, W1, b1, Ct, eta);
    MSFNO_TRY(launch_check("mg_eta"));
    hipLaunchKernelGGL(mg_scale_kernel, dim3(H + Cp), dim3(256), 0, s, W1, W2, eta, H, Ct, Cout,
                       s1, s2, is1, is2);
    MSFNO_TRY(launch_check("mg_scale"));
    hipLaunchKernelGGL(mg_image_kernel, dim3(256), dim3(256), 0, s, W1, W2, eta, s1, s2, H, Ct,
                       Cout, KS, OT, layout, img);
    MSFNO_TRY(launch_check("mg_image"));
  }
  MlpGParams p{};
  p.x = x; p.xa = xa; p.xt = xt; p.x2 = x2; p.addend = addend; p.out = out; p.img = img;
  p.is1 = is1; p.is2 = is2; p.eta = eta; p.b1 = b1; p.b2 = b2;
  p.P = P; p.add_bstride = add_bstride;
  p.Cin = Cin; p.Cin2 = Cin2; p.Cout = Cout; p.H = H;
  p.nslice = (int)(tiles / MG_SLICE);
  if (persist) {
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    p.tiles_per_field = (int)cdiv(P, GP_PX);
    const int64_t t = (int64_t)B * p.tiles_per_field;
    MSFNO_REQUIRE(t < (1LL << 31), MSFNO_EINVAL, "mlp_gen_hp: grid too large");
    p.tiles = (int)t;
    const int grid = (int)std::min<int64_t>(t, cus);  // one workgroup fills a CU
    // ring depth 4 (5 and 6 measured equal with the x pieces in the ring slots,
    // profiles/r06_l; with the x buffer only 4 fits)
    const dim3 gd((unsigned)grid);
    // (the two pixel groups' MFMA triples interleaved: equal, 132.0 / 132.0 vs 132.0 /
    // 131.5 steps/s, profiles/r06_p/ab_mfma_pairs.txt).  MSFNO_MG_PG = 1 / 2: pixel groups
    // per wave (8 / 4 waves): equal, net 130.1 / 129.9 / 130.0 vs 130.0 / 130.5 / 130.5
    // steps/s (profiles/r06_q/summary_q.txt).  Phase costs (summary_r.txt, diagnostic builds):
    // without the GELU 0.16 ms less per net step, without the addend, x or store streams
    // 0.01-0.05 ms less each; the fc1 steps' VALU forced between their MFMAs
    // (sched_group_barrier, 2 / 4 / 6 per MFMA) changed nothing (summary_s.txt)
    static const int pg = [] {
      const char* e = getenv("MSFNO_MG_PG");
      return e && e[0] == '1' ? 1 : 2;
    }();
    const dim3 bd2(64 * (8 / pg));
    if (pg == 1) {
      if (addend) hipLaunchKernelGGL((mlp_gen_hp_kernel<3, 16, true, 4, 1>), gd, bd2, 0, s, p);
      else hipLaunchKernelGGL((mlp_gen_hp_kernel<3, 16, false, 4, 1>), gd, bd2, 0, s, p);
    } else {
      if (addend) hipLaunchKernelGGL((mlp_gen_hp_kernel<3, 16, true, 4, 2>), gd, bd2, 0, s, p);
      else hipLaunchKernelGGL((mlp_gen_hp_kernel<3, 16, false, 4, 2>), gd, bd2, 0, s, p);
    }
    return launch_check("mlp_gen_hp");
  }
  p.tiles_per_field = (int)cdiv(P, 16 * MG_WAVES);
  const int64_t grid = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(grid < (1LL << 31), MSFNO_EINVAL, "mlp_gen_h: grid too large");
  // the encoder's addend (pos_embed) loads issued with x's: mlp_gen 2.48 / 2.51 / 2.46 ->
  // 2.35 / 2.33 / 2.34 ms per 12-block step, net 124.5 / 124.0 / 123.9 -> 125.6 / 125.7 /
  // 125.7 steps/s (three interleaved pairs, profiles/r06_h); MSFNO_MG_EARLY=0 restores
  // the late form
  const char* ee = getenv("MSFNO_MG_EARLY");
  const bool early = !(ee && ee[0] == '0');
  // raw-buffer addressing (MSFNO_MG_BUF=0: 64-bit addresses, A/B)
  static const bool buf_env = [] {
    const char* e = getenv("MSFNO_MG_BUF");
    return !(e && e[0] == '0');
  }();
  const int64_t lim = 1LL << 31;
  const bool buf = buf_env && (x2 == nullptr || Cin % 32 == 0) && (int64_t)Cin * P * 4 < lim &&
                   (int64_t)Cin2 * P * 4 < lim && (int64_t)Cout * P * 4 < lim;
  const dim3 gd((unsigned)grid), bd(64 * MG_WAVES);
  if (KS == 3 && early && buf) hipLaunchKernelGGL((mlp_gen_h_kernel<3, 16, true, true>), gd, bd, 0, s, p);
  else if (KS == 3 && early) hipLaunchKernelGGL((mlp_gen_h_kernel<3, 16, true, false>), gd, bd, 0, s, p);
  else if (KS == 3) hipLaunchKernelGGL((mlp_gen_h_kernel<3, 16, false, false>), gd, bd, 0, s, p);
  else if (buf) hipLaunchKernelGGL((mlp_gen_h_kernel<11, 5, false, true>), gd, bd, 0, s, p);
  else hipLaunchKernelGGL((mlp_gen_h_kernel<11, 5, false, false>), gd, bd, 0, s, p);
  return launch_check("mlp_gen_h");
}

}  // namespace msfno
