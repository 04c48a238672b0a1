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

#include <string>
#include <type_traits>
#include <utility>

namespace msfno {

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

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
__global__ void mg_image_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                const float* __restrict__ eta, const float* __restrict__ s1,
                                const float* __restrict__ s2, int H, int Ct, int Cout, int KS,
                                int OT, unsigned short* __restrict__ img) {
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
      tile = mg_unit_tile(j, KS, OT) + i;
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
      tile = mg_unit_tile(j + 1, KS, OT) + (j + 1 < HB ? 2 * KS : 0) + ot;
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

template <int KS, int OT, bool EARLY>
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
    if (p.addend) {
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
#pragma unroll
  for (int ot = 0; ot < OT; ++ot) {
    const int r0 = 16 * ot + 4 * g;
    const float4 is = *reinterpret_cast<const float4*>(is2s + r0);
    const float4 b = *reinterpret_cast<const float4*>(b2s + r0);
    const float isv[4] = {is.x * ietap, is.y * ietap, is.z * ietap, is.w * ietap};
    const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (r0 + i < p.Cout) o[(int64_t)(r0 + i) * P] = fmaf(oacc[ot][i], isv[i], bv[i]) + rv[ot][i];
  }
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
  // the weight image and its scale vectors: in the caller's prepared-weight cache when
  // given (rebuilt only when cache_valid is 0), else in the workspace on every call
  char* base = static_cast<char*>(cache ? cache : ws);
  unsigned short* img = reinterpret_cast<unsigned short*>(base);
  float* eta = reinterpret_cast<float*>(base + round_up(tiles * MG_TILE * 2, 256));
  float* s1 = eta + H;
  float* is1 = s1 + H;
  float* s2 = is1 + H;
  float* is2 = s2 + Cp;
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
                       Cout, KS, OT, img);
    MSFNO_TRY(launch_check("mg_image"));
  }
  MlpGParams p{};
  p.x = x; p.xa = xa; p.xt = xt; p.x2 = x2; p.addend = addend; p.out = out; p.img = img;
  p.is1 = is1; p.is2 = is2; p.eta = eta; p.b1 = b1; p.b2 = b2;
  p.P = P; p.add_bstride = add_bstride;
  p.Cin = Cin; p.Cin2 = Cin2; p.Cout = Cout; p.H = H;
  p.nslice = (int)(tiles / MG_SLICE);
  p.tiles_per_field = (int)cdiv(P, 16 * MG_WAVES);
  const int64_t grid = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(grid < (1LL << 31), MSFNO_EINVAL, "mlp_gen_h: grid too large");
  // the encoder's addend (pos_embed) loads issued with x's: mlp_gen 2.48 / 2.51 / 2.46 ->
  // 2.35 / 2.33 / 2.34 ms per 12-block step, net 124.5 / 124.0 / 123.9 -> 125.6 / 125.7 /
  // 125.7 steps/s (three interleaved pairs, profiles/r06_h); MSFNO_MG_EARLY=0 restores
  // the late form
  const char* ee = getenv("MSFNO_MG_EARLY");
  const bool early = !(ee && ee[0] == '0');
  if (KS == 3 && early)
    hipLaunchKernelGGL((mlp_gen_h_kernel<3, 16, true>), dim3((unsigned)grid), dim3(64 * MG_WAVES), 0, s, p);
  else if (KS == 3)
    hipLaunchKernelGGL((mlp_gen_h_kernel<3, 16, false>), dim3((unsigned)grid), dim3(64 * MG_WAVES), 0, s, p);
  else
    hipLaunchKernelGGL((mlp_gen_h_kernel<11, 5, false>), dim3((unsigned)grid), dim3(64 * MG_WAVES), 0, s, p);
  return launch_check("mlp_gen_h");
}

}  // namespace msfno
