// Fused block MLP, two workgroups per CU (gfx950): the same contraction as
// mlp_fused.hip — out = W2·GELU(W1·(a ⊙ x1 + t) + b1) + b2 + resid, C = 256,
// H = 512, x6 engine (six bf16 products of the exact three-term splits, fp32
// accumulation), hidden activation on-chip — re-tiled so that two waves share
// every SIMD:
//
//  * 16x16x32 bf16 MFMAs; a wave owns 16 pixels, a workgroup (4 waves, one per
//    SIMD) 64 pixels, and the register budget is 256 per wave, so TWO workgroups
//    run on each CU.  One workgroup's GELU/split VALU work, ring barriers, tile
//    prologue (x1 loads) and epilogue (residual + stores) run while the other's
//    MFMAs keep the matrix pipe busy — the one-wave-per-SIMD kernel exposed all of
//    them (DESIGN.md §4 phase clock: 98 k of 187 k cycles per tile were MFMAs).
//  * x1 goes straight from global memory into the fc1 B fragments (lane (px, g)
//    holds channels 32 ks + 8 g + 0..7 of its pixel; 64-B runs per 16 lanes), no
//    LDS staging.  The residual is read the same way in the accumulator layout.
//  * fc1 produces a 32-row hidden block as two 16x16 tiles; bias + GELU + split turn
//    them IN PLACE into fc2's B fragment for that block: lane (px, g) holds rows
//    4g..4g+3 (tile 0) and 16+4g..16+4g+3 (tile 1) = k positions 8g..8g+7 of a
//    32-deep k-step under the permutation m2_perm, which fc2's weight image carries.
//  * Weights stream through a 3-slot ring of 24-KB slices (LDS-DMA, counted vmcnt
//    + raw s_barrier), the slice order of mlp_fused.hip:
//      W1(0,0) W1(0,1) | W1(j,0) W1(j,1) W2(j-1,0) W2(j-1,1) j = 1..15 | W2(15,0) W2(15,1)
//    W1(j,kh): hidden rows 32j..+31, channels 128kh..+127: [pl][ks 4][t 2][r 16][32]
//    W2(j,oh): out rows 128oh..+127, hidden block j:       [pl][ot 8][r 16][32 (perm)]
//    Each slice is 8 units of (3 A fragments, 6 MFMAs) per wave.
//  * A-fragment rows of 64 B: the 16-B k-group g sits at g ^ m2_swz(r) (ds_read_b128
//    conflict-free for the 16x16x32 operand pattern).
#include "dma.h"
#include "gemm_common.h"
#include "kernels.h"

#include <type_traits>

namespace msfno {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int M2_C = 256, M2_H = 512;
constexpr int M2_WAVES = 4, M2_PX = 16 * M2_WAVES;  // pixels per workgroup tile
constexpr int M2_HB = M2_H / 32;                    // hidden blocks
constexpr int M2_SLICE = 12288;                     // bf16 per 24-KB slice
constexpr int M2_PLANE = 4096;                      // bf16 per plane within a slice
constexpr int M2_NS = 3;                            // ring slots
constexpr int M2_NSLICE = 4 * M2_HB;                // slices per tile
constexpr int M2_RING_BYTES = M2_NS * M2_SLICE * 2;
constexpr int M2_LDS = M2_RING_BYTES + M2_H * 4;    // ring + b1

struct Mlp2Params {
  const float* x1;      // [B][C][P]
  const float* scale;   // [B][C]  x1 affine (norm1 + FiLM): a
  const float* shift;   // [B][C]  t
  const float* resid;   // [B][C][P] or null
  float* out;           // [B][C][P]
  const unsigned short* w1img;  // [HB][2 kh] slices
  const unsigned short* w2img;  // [HB][2 oh] slices
  const float* b1;      // [H]
  const float* b2;      // [C] or null
  int64_t P;
  int tiles_per_field;
};

// physical 16-B k-group of logical group g in A-image row r (see header)
__host__ __device__ __forceinline__ int m2_swz(int r) { return ((r >> 2) & 1) << 1; }

// hidden row (within a block) of fc2 k position kappa = 8 g + e
__host__ __device__ __forceinline__ int m2_perm(int kappa) {
  const int g = kappa >> 3, e = kappa & 7;
  return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4);
}

__device__ __forceinline__ bf16x8 m2_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8, make_uint4(a, b, c, d));
}

// W1 (H x C fp32) -> [j][kh][pl][ks][t][r][32]
__global__ void m2_w1_image_kernel(const float* __restrict__ W1, unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)M2_HB * 2 * 4 * 2 * 16 * 16;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 15);        // pair within the 32-wide row
    const int r = (int)((e >> 4) & 15);
    const int t = (int)((e >> 8) & 1);
    const int ks = (int)((e >> 9) & 3);
    const int kh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;               // physical position
    const int g = (kk >> 3) ^ m2_swz(r);  // logical k-group stored there
    const int k = 128 * kh + 32 * ks + 8 * g + (kk & 7);
    const float* src = W1 + (int64_t)(32 * j + 16 * t + r) * M2_C + k;
    uint32_t t0, t1, t2;
    split2(src[0], src[1], t0, t1, t2);
    uint32_t* o = reinterpret_cast<uint32_t*>(
        img + (int64_t)(j * 2 + kh) * M2_SLICE + ((ks * 2 + t) * 16 + r) * 32 + kk);
    o[0] = t0;
    o[M2_PLANE / 2] = t1;
    o[M2_PLANE] = t2;
  }
}

// W2 (C x H fp32) -> [j][oh][pl][ot][r][32] with the hidden index permuted by m2_perm
__global__ void m2_w2_image_kernel(const float* __restrict__ W2, unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)M2_HB * 2 * 8 * 16 * 16;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 15);
    const int r = (int)((e >> 4) & 15);
    const int ot = (int)((e >> 8) & 7);
    const int oh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;
    const int kap = 8 * ((kk >> 3) ^ m2_swz(r)) + (kk & 7);
    const float* row = W2 + (int64_t)(128 * oh + 16 * ot + r) * M2_H + 32 * j;
    uint32_t t0, t1, t2;
    split2(row[m2_perm(kap)], row[m2_perm(kap + 1)], t0, t1, t2);
    uint32_t* o = reinterpret_cast<uint32_t*>(
        img + (int64_t)(j * 2 + oh) * M2_SLICE + (ot * 16 + r) * 32 + kk);
    o[0] = t0;
    o[M2_PLANE / 2] = t1;
    o[M2_PLANE] = t2;
  }
}

// global source of slice q of a tile (element offset)
__device__ __forceinline__ const unsigned short* m2_slice_src(const Mlp2Params& p, int q) {
  if (q < 2) return p.w1img + (int64_t)q * M2_SLICE;
  if (q >= M2_NSLICE - 2)
    return p.w2img + (int64_t)(2 * (M2_HB - 1) + (q - (M2_NSLICE - 2))) * M2_SLICE;
  const int j = 1 + ((q - 2) >> 2), r = (q - 2) & 3;
  return r < 2 ? p.w1img + (int64_t)(2 * j + r) * M2_SLICE
               : p.w2img + (int64_t)(2 * (j - 1) + (r - 2)) * M2_SLICE;
}

template <int AHEAD>
__global__ __launch_bounds__(256, 2) void mlp_fused2_kernel(Mlp2Params p) {
  __shared__ __attribute__((aligned(16))) char lds_raw[M2_LDS];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const b1s = reinterpret_cast<float*>(lds_raw + M2_RING_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int z = lin / p.tiles_per_field;
  const int64_t P = p.P;
  const int64_t px = (int64_t)(lin - z * p.tiles_per_field) * M2_PX + 16 * wave + r16;
  const bool valid = px < P;
  const int64_t pxc = valid ? px : P - 1;

  // ---- slices 0..2 in flight (this wave's 1-KB pieces wave + 4 i) ------------------
  const uint32_t ring_lds = lds_addr(ring);
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  uint32_t piece_off[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) piece_off[i] = (uint32_t)(i * M2_WAVES * 1024 + lane * 16);
  auto issue = [&](int q) {
    const uint64_t src = reinterpret_cast<uint64_t>(m2_slice_src(p, q)) + (uint64_t)wave_u * 1024;
    const uint32_t base = ring_lds + (uint32_t)((q % M2_NS) * M2_SLICE * 2 + wave_u * 1024);
    glds16x6<M2_WAVES * 1024>(src, piece_off, base);
  };
  issue(0);
  issue(1);
  issue(2);

  // ---- x1 -> normalised bf16x3 B fragments (k-step ks: channels 32 ks + 8 g + 0..7) --
  const float* xcol = p.x1 + (int64_t)z * M2_C * P + pxc;
  const float* sc = p.scale + (int64_t)z * M2_C;
  const float* sh = p.shift + (int64_t)z * M2_C;
  bf16x8 xf[8][3];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int c0 = 32 * ks + 8 * g;
    float xv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = __builtin_nontemporal_load(xcol + (int64_t)(c0 + e) * P);
    const float4 sa = *reinterpret_cast<const float4*>(sc + c0);
    const float4 sb = *reinterpret_cast<const float4*>(sc + c0 + 4);
    const float4 ta = *reinterpret_cast<const float4*>(sh + c0);
    const float4 tb = *reinterpret_cast<const float4*>(sh + c0 + 4);
    const float sv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float tv[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    uint32_t t[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      split2(fmaf(sv[2 * e], xv[2 * e], tv[2 * e]), fmaf(sv[2 * e + 1], xv[2 * e + 1], tv[2 * e + 1]),
             t[0][e], t[1][e], t[2][e]);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) xf[ks][pl] = m2_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
  }
  // output accumulators: tile ot = out rows 16 ot + 4 g + 0..3 of this lane's pixel; b2 first
  floatx4 oacc[16];
#pragma unroll
  for (int ot = 0; ot < 16; ++ot) {
    if (p.b2) {
      const float4 b = *reinterpret_cast<const float4*>(p.b2 + 16 * ot + 4 * g);
      oacc[ot] = floatx4{b.x, b.y, b.z, b.w};
    } else {
      oacc[ot] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  for (int i = tid; i < M2_H; i += 256) b1s[i] = p.b1[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slices 0-2 and every load landed
  __syncthreads();

  floatx4 hacc[2][2];  // [parity][tile]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int t = 0; t < 2; ++t) hacc[a][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  uint32_t hfu[3][4];  // fc2 B fragment of the converted block [plane][pair]

  const int a_lane = r16 * 32 + 8 * (g ^ m2_swz(r16));

  // step q: slice q landed for every wave; the slot of slice q - 1 is free (every
  // wave passed this barrier after reading it) and takes slice q + 2
  auto step_begin = [&](int q) {
    if (q + 1 < M2_NSLICE)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // slice q + 1 may stay in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    return ring + (q % M2_NS) * M2_SLICE;
  };
  auto refill = [&](int q) {
    if (q >= 1 && q + 2 < M2_NSLICE) issue(q + 2);
  };

  auto mfma6 = [](const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
    return c;
  };

  // pair e2 (0..3) of hidden block j held in hacc[PAR]: + b1, GELU(erf), split -> hfu
  auto conv_pair = [&](int j, int e2, auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    const int t = e2 >> 1, i = 2 * (e2 & 1);
    const float2 b = *reinterpret_cast<const float2*>(b1s + 32 * j + 16 * t + 4 * g + i);
    f32x2 v = {hacc[PAR][t][i] + b.x, hacc[PAR][t][i + 1] + b.y};
    v = gelu_erf2(v);
    split2(v.x, v.y, hfu[0][e2], hfu[1][e2], hfu[2][e2]);
  };

  // one slice = 8 units of (3 A fragments, 6 MFMAs); A fragments read AHEAD units ahead
  // fc1 slice W1(j, KH): unit u = (ks = u >> 1, t = u & 1) into hacc[PAR][t]; CONV:
  // pairs 2 KH, 2 KH + 1 of block jc (hacc[PAR ^ 1]) converted under it
  auto fc1_step = [&](const unsigned short* slot, int q, auto kh_c, auto par_c, auto conv_c,
                      int jc) {
    constexpr int KH = decltype(kh_c)::value, PAR = decltype(par_c)::value;
    constexpr bool CONV = decltype(conv_c)::value;
    using PPrev = std::integral_constant<int, PAR ^ 1>;
    auto aoff = [&](int u, int pl) { return ((pl * 4 + (u >> 1)) * 2 + (u & 1)) * 512 + a_lane; };
    bf16x8 a[AHEAD + 1][3];
#pragma unroll
    for (int k = 0; k < AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[k][pl] = *reinterpret_cast<const bf16x8*>(slot + aoff(k, pl));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + AHEAD < 8) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[(u + AHEAD) % (AHEAD + 1)][pl] = *reinterpret_cast<const bf16x8*>(slot + aoff(u + AHEAD, pl));
      }
      hacc[PAR][u & 1] = mfma6(a[u % (AHEAD + 1)], xf[KH * 4 + (u >> 1)], hacc[PAR][u & 1]);
      if (u == 0) refill(q);
      if constexpr (CONV) {
        if (u == 2 || u == 6) conv_pair(jc, 2 * KH + (u >> 2), PPrev{});
      }
    }
    if constexpr (CONV && KH == 1) {
#pragma unroll
      for (int t = 0; t < 2; ++t) hacc[PAR ^ 1][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // fc2 slice W2(j, OH) with the converted block in hfu: unit u = out tile 8 OH + u
  auto fc2_step = [&](const unsigned short* slot, int q, auto oh_c) {
    constexpr int OH = decltype(oh_c)::value;
    auto aoff = [&](int u, int pl) { return (pl * 8 + u) * 512 + a_lane; };
    const bf16x8 hb[3] = {m2_frag(hfu[0][0], hfu[0][1], hfu[0][2], hfu[0][3]),
                          m2_frag(hfu[1][0], hfu[1][1], hfu[1][2], hfu[1][3]),
                          m2_frag(hfu[2][0], hfu[2][1], hfu[2][2], hfu[2][3])};
    bf16x8 a[AHEAD + 1][3];
#pragma unroll
    for (int k = 0; k < AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[k][pl] = *reinterpret_cast<const bf16x8*>(slot + aoff(k, pl));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u + AHEAD < 8) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[(u + AHEAD) % (AHEAD + 1)][pl] = *reinterpret_cast<const bf16x8*>(slot + aoff(u + AHEAD, pl));
      }
      oacc[OH * 8 + u] = mfma6(a[u % (AHEAD + 1)], hb, oacc[OH * 8 + u]);
      if (u == 0) refill(q);
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
  for (int j = 1; j < M2_HB; j += 2) {
    do_round(j, I1{});
    if (j + 1 < M2_HB) do_round(j + 1, I0{});
  }
  // block 15 (in hacc[1]) converted, then its fc2 slices
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) conv_pair(M2_HB - 1, e2, I1{});
  fc2_step(step_begin(M2_NSLICE - 2), M2_NSLICE - 2, I0{});
  fc2_step(step_begin(M2_NSLICE - 1), M2_NSLICE - 1, I1{});

  // ---- epilogue: + residual, store (rows 16 ot + 4 g + i of this lane's pixel) --------
  if (valid) {
    float* o = p.out + (int64_t)z * M2_C * P + px;
    if (p.resid) {
      const float* rs = p.resid + (int64_t)z * M2_C * P + px;
#pragma unroll
      for (int ot = 0; ot < 16; ++ot)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          oacc[ot][i] += __builtin_nontemporal_load(rs + (int64_t)(16 * ot + 4 * g + i) * P);
    }
#pragma unroll
    for (int ot = 0; ot < 16; ++ot)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[(int64_t)(16 * ot + 4 * g + i) * P] = oacc[ot][i];
  }
}

}  // namespace

bool mlp_fused2_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_MF2");
    return e && e[0] == '1';
  }();
  return on;
}

int launch_mlp_fused2_images(const float* W1, const float* W2, unsigned short* img, hipStream_t s) {
  unsigned short* w2img = img + (int64_t)M2_HB * 2 * M2_SLICE;
  hipLaunchKernelGGL(m2_w1_image_kernel, dim3(256), dim3(256), 0, s, W1, img);
  MSFNO_TRY(launch_check("m2_w1_image"));
  hipLaunchKernelGGL(m2_w2_image_kernel, dim3(256), dim3(256), 0, s, W2, w2img);
  return launch_check("m2_w2_image");
}

int launch_mlp_fused2(const float* x1, const float* scale, const float* shift, const float* resid,
                      float* out, const unsigned short* img, const float* b1, const float* b2,
                      int B, int64_t P, hipStream_t s) {
  MSFNO_REQUIRE(x1 && scale && shift && out && img && b1 && B > 0 && P >= 1, MSFNO_EINVAL,
                "mlp_fused2: bad arguments");
  Mlp2Params p{};
  p.x1 = x1; p.scale = scale; p.shift = shift; p.resid = resid; p.out = out;
  p.w1img = img;
  p.w2img = img + (int64_t)M2_HB * 2 * M2_SLICE;
  p.b1 = b1; p.b2 = b2; p.P = P;
  p.tiles_per_field = (int)cdiv(P, M2_PX);
  const int64_t tiles = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(tiles < (1LL << 31), MSFNO_EINVAL, "mlp_fused2: grid too large");
  static const int ahead = [] {
    const char* e = getenv("MSFNO_MF2_AHEAD");
    return e ? atoi(e) : 2;
  }();
  if (ahead == 1)
    hipLaunchKernelGGL((mlp_fused2_kernel<1>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((mlp_fused2_kernel<2>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  return launch_check("mlp_fused2");
}

}  // namespace msfno
