// Fused block MLP for gfx950 (layers.py:145-178 with norm1 + FiLM, sfnonet.py:
// 377-393): out = W2·GELU(W1·(a ⊙ x1 + t) + b1) + b2 + resid, C = 256, H = 512,
// fp32-accurate on the bf16 matrix cores (the x6 engine of gemm_x6.hip: six
// products of the exact three-term bf16 splits, fp32 accumulation).
//
// The hidden activation never leaves the CU.  A workgroup (4 waves, one per
// SIMD) owns 128 pixels; a wave owns 32 of them for the whole MLP:
//  * x1 (its 256 channels x 32 pixels, normalised and split into bf16x3) stays
//    in registers as the B operand of fc1 for every hidden block;
//  * fc1 produces one 32-row hidden block at a time in a 32x32 accumulator;
//  * bias + GELU + the bf16x3 split turn that accumulator IN PLACE into fc2's B
//    operand: lane (n, half) holds rows (r>>2)*8 + 4 half + (r&3) of the block,
//    and the slots r = 0..7 / 8..15 are exactly a 16-deep k-step of rows
//    {0..15} / {16..31} in a lane-dependent order.  fc2's weight image carries
//    that order (the contraction over k is invariant under a permutation of k
//    applied to both operands), so no LDS round trip and no shuffle is needed;
//  * the 256 x 32 output accumulator (residual + b2 at the start) is stored
//    once at the end.
// Weights stream through LDS: a ring of four 24-KB slots filled by LDS-DMA
// (global_load_lds_dwordx4, inline asm, counted vmcnt + raw s_barrier;
// cdna_hip_programming.md §5.7), two slices in flight while one is multiplied.
// Slice sequence of a tile (hidden block j, 16 blocks):
//   W1(0,0) W1(0,1) | W1(j,0) W1(j,1) W2(j-1,0) W2(j-1,1) for j = 1..15 | W2(15,0) W2(15,1)
// W1(j,kh): rows 32j..32j+31 of W1, k = 128 kh .. +127    (8 k-steps, 48 MFMAs)
// W2(j,oh): rows 128 oh .. +127 of W2, k = block j         (4 x 2 k-steps, 48 MFMAs)
// The GELU/split of block j-1 runs under the MFMAs of W1(j, *) (a second fc1
// accumulator), so fc2 of a block starts while fc1 of the next one runs.
//
// Per field at config 2 this moves x1 (1.06 GB), the residual (1.06 GB) and the
// output (1.06 GB) through HBM, against 10.4 GB for fc1 + fc2 with h
// materialised as planes.
#include "dma.h"
#include "gemm_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <vector>

namespace msfno {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int MF_C = 256, MF_H = 512;
constexpr int MF_WAVES = 4, MF_PX = 32 * MF_WAVES;  // pixels per workgroup tile
constexpr int MF_HB = MF_H / 32;                    // hidden blocks
constexpr int MF_SLICE_ELEMS = 12288;               // bf16 per 24-KB slice
constexpr int MF_NS = 4;                            // ring slots
constexpr int MF_NSLICE = 4 * MF_HB;                // slices per tile
constexpr int MF_PIECES = MF_SLICE_ELEMS * 2 / 1024 / MF_WAVES;  // 1-KB DMA pieces per wave (6)
constexpr int MF_VEC_OFF = 160 * 1024 - (MF_H + 3 * MF_C) * 4;  // b1, a, t, b2
constexpr int MF_LDS = 160 * 1024;
constexpr int MF_RES_CHUNK = 32 * MF_PX * 4;  // residual rows of one output block
static_assert(MF_NS * MF_SLICE_ELEMS * 2 + 2 * MF_RES_CHUNK <= MF_VEC_OFF, "residual staging");
static_assert(MF_SLICE_ELEMS * 2 + MF_C * MF_PX * 4 <= MF_VEC_OFF, "x1 staging below the vectors");
static_assert(MF_NS * MF_SLICE_ELEMS * 2 <= MF_VEC_OFF, "ring below the vectors");

struct MlpFusedParams {
  const float* x1;      // [B][C][P]
  const float* scale;   // [B][C]  x1 affine (norm1 + FiLM): a
  const float* shift;   // [B][C]  t
  const float* resid;   // [B][C][P] or null
  float* out;           // [B][C][P]
  const unsigned short* w1img;  // [HB][2 kh][3 pl][8 ks][32 m][16]
  const unsigned short* w2img;  // [HB][2 oh][3 pl][2 s][128 m][16]
  const float* b1;      // [H]
  const float* b2;      // [C] or null
  int64_t P;
  int tiles_per_field;
  unsigned long long* stamps;  // diagnostic build only (STAMP): [workgroup][8] s_memtime
};

// physical 16-B half of logical k-half h in an A-image row m (conflict-free
// ds_read_b128: the two halves swap on row bit 3, as in gemm_x6p's A stage)
__device__ __forceinline__ int mf_swz(int m) { return (m >> 3) & 1; }

__device__ __forceinline__ bf16x8 mf_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint4 u = make_uint4(a, b, c, d);
  return __builtin_bit_cast(bf16x8, u);
}

// ---- weight images ----------------------------------------------------------------
// W1 (H x C fp32, row-major) -> [j][kh][pl][ks][m][16]; k = 128 kh + 16 ks + 8 h + e,
// physical half = h ^ swz(m)
__global__ void mf_w1_image_kernel(const float* __restrict__ W1, unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)MF_HB * 2 * 8 * 32 * 8;  // pairs per plane-set
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 7);  // pair within the 16-wide row
    const int m = (int)((e >> 3) & 31);
    const int ks = (int)((e >> 8) & 7);
    const int kh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;
    const int lh = (kk >> 3) ^ mf_swz(m);
    const int k = 128 * kh + 16 * ks + 8 * lh + (kk & 7);
    const float* src = W1 + (int64_t)(32 * j + m) * MF_C + k;
    uint32_t t0, t1, t2;
    split2(src[0], src[1], t0, t1, t2);
    const int64_t slice = (int64_t)(j * 2 + kh) * MF_SLICE_ELEMS;
    const int64_t off = ((int64_t)ks * 32 + m) * 16 + kk;
    constexpr int PL = 8 * 32 * 16;
    uint32_t* o = reinterpret_cast<uint32_t*>(img + slice + off);
    o[0] = t0;
    o[PL / 2] = t1;
    o[PL] = t2;
  }
}

// hidden row of k position kappa (0..15) of fc2's k-step s (0, 1) within a block:
// the fc1 accumulator slot r = 8 s + (kappa & 7) of a lane with half = kappa >> 3
__device__ __forceinline__ int mf_perm(int s, int kappa) {
  const int r = 8 * s + (kappa & 7);
  return (r >> 2) * 8 + (kappa >> 3) * 4 + (r & 3);
}

// W2 (C x H fp32, row-major) -> [j][oh][pl][s][m][16] with k permuted by mf_perm
__global__ void mf_w2_image_kernel(const float* __restrict__ W2, unsigned short* __restrict__ img) {
  constexpr int64_t PAIRS = (int64_t)MF_HB * 2 * 2 * 128 * 8;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < PAIRS;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int kkp = (int)(e & 7);
    const int m = (int)((e >> 3) & 127);
    const int s = (int)((e >> 10) & 1);
    const int oh = (int)((e >> 11) & 1);
    const int j = (int)(e >> 12);
    const int kk = 2 * kkp;
    const int kap = 8 * ((kk >> 3) ^ mf_swz(m)) + (kk & 7);
    const float* row = W2 + (int64_t)(128 * oh + m) * MF_H + 32 * j;
    uint32_t t0, t1, t2;
    split2(row[mf_perm(s, kap)], row[mf_perm(s, kap + 1)], t0, t1, t2);
    const int64_t slice = (int64_t)(j * 2 + oh) * MF_SLICE_ELEMS;
    const int64_t off = ((int64_t)s * 128 + m) * 16 + kk;
    constexpr int PL = 2 * 128 * 16;
    uint32_t* o = reinterpret_cast<uint32_t*>(img + slice + off);
    o[0] = t0;
    o[PL / 2] = t1;
    o[PL] = t2;
  }
}

// global source (element offset) of slice q of a tile
__device__ __forceinline__ const unsigned short* mf_slice_src(const MlpFusedParams& p, int q) {
  if (q < 2) return p.w1img + (int64_t)q * MF_SLICE_ELEMS;            // W1(0, q)
  if (q >= MF_NSLICE - 2)                                               // W2(15, q - 62)
    return p.w2img + (int64_t)(2 * (MF_HB - 1) + (q - (MF_NSLICE - 2))) * MF_SLICE_ELEMS;
  const int j = 1 + ((q - 2) >> 2), r = (q - 2) & 3;
  return r < 2 ? p.w1img + (int64_t)(2 * j + r) * MF_SLICE_ELEMS
               : p.w2img + (int64_t)(2 * (j - 1) + (r - 2)) * MF_SLICE_ELEMS;
}

// MF_AHEAD: k-steps of A fragments read ahead of the MFMAs (LDS latency cover)
// XS: the read-ahead crosses slice boundaries (XS = 1: two k-steps ahead, always;
// the next slice's barrier runs inside the current step, see xstep below)
template <int SCHED, int STAMP, int DBG = 0, int MF_AHEAD = 2, int XS = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void mlp_fused_kernel(MlpFusedParams p) {
  // DBG (diagnostic timing builds only, wrong results): 1 no ring waits / barriers /
  // refills in the steps, 2 no MFMAs, 4 no GELU / split of the hidden blocks, 8 the
  // A fragments of every k-step re-use the first k-step's (no ds_reads in the loop)
  // diagnostic phase clock (MSFNO_MF_STAMPS=1; never in the product launch): wave 0 of
  // each workgroup records s_memtime at phase boundaries and the cycles it spent in
  // the ring waits + barriers
  unsigned long long st_wait = 0;
  auto stamp = [&](int k, unsigned long long v) {
    if constexpr (STAMP) {
      if (threadIdx.x == 0) p.stamps[(int64_t)blockIdx.x * 8 + k] = v;
    }
  };
  if constexpr (STAMP) stamp(0, __builtin_amdgcn_s_memtime());
  const unsigned long long rt0 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;
  // LDS: ring slots [0, 96K); x1 staging [24K, 152K) at the tile start (only slot 0
  // is live then); two 16-KB residual chunks [96K, 128K) during the steps; vectors at
  // the top
  __shared__ __attribute__((aligned(16))) char lds_raw[MF_LDS];
  unsigned short* const ring = reinterpret_cast<unsigned short*>(lds_raw);
  float* const stage_x = reinterpret_cast<float*>(lds_raw + MF_SLICE_ELEMS * 2);
  float* const stage_res = reinterpret_cast<float*>(lds_raw + MF_NS * MF_SLICE_ELEMS * 2);
  float* const b1s = reinterpret_cast<float*>(lds_raw + MF_VEC_OFF);
  float* const scs = b1s + MF_H;  // x1 affine a, t and b2 of this tile's field
  float* const shs = scs + MF_C;
  float* const b2s = shs + MF_C;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int z = lin / p.tiles_per_field;
  const int64_t P = p.P;
  const int64_t px0 = (int64_t)(lin - z * p.tiles_per_field) * MF_PX;
  const int64_t px = px0 + 32 * wave + l32;
  const bool valid = px < P;

  const uint32_t ring_lds = lds_addr(ring);
  // slice q -> ring slot q % 4: this wave's 1-KB pieces wave + 4 i, one asm block with
  // SGPR bases (wave-uniform) and the lane offset in a VGPR
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  static_assert(MF_PIECES == 6, "glds16x6");
  uint32_t piece_off[6];  // piece wave + 4 i: byte offset i * 4 KB + the lane's 16 B
#pragma unroll
  for (int i = 0; i < 6; ++i) piece_off[i] = (uint32_t)(i * MF_WAVES * 1024 + lane * 16);
  auto issue = [&](int q) {
    const uint64_t src = reinterpret_cast<uint64_t>(mf_slice_src(p, q)) + (uint64_t)wave_u * 1024;
    const uint32_t base = ring_lds + (uint32_t)((q % MF_NS) * MF_SLICE_ELEMS * 2 + wave_u * 1024);
    glds16x6<MF_WAVES * 1024>(src, piece_off, base);
  };
  // a [256 channel][128 pixel] fp32 tile of a (B, C, P) tensor -> LDS by LDS-DMA:
  // 1-KB piece i = channel rows 2i, 2i + 1; pixels past P are clamped (P % 4 == 0)
  auto stage_tile = [&](const float* t, float* dst) {
    const float* src = t + (int64_t)z * MF_C * P + (int64_t)(lane >> 5) * P +
                       min(px0 + 4 * l32, P - 4);
    const uint32_t base = lds_addr(dst);
#pragma unroll
    for (int k = 0; k < MF_C / 2 / MF_WAVES; ++k) {
      const int piece = wave + MF_WAVES * k;
      glds16(src + (int64_t)(2 * piece) * P, base + (uint32_t)(piece * 1024));
    }
  };
  // ---- tile start: x1 staged, slice 0 in flight, per-field vectors --------------
  stage_tile(p.x1, stage_x);
  issue(0);
  for (int r = tid; r < MF_H; r += 256) b1s[r] = p.b1[r];
  for (int r = tid; r < MF_C; r += 256) {
    scs[r] = p.scale[(int64_t)z * MF_C + r];
    shs[r] = p.shift[(int64_t)z * MF_C + r];
    b2s[r] = p.b2 ? p.b2[r] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (STAMP) stamp(1, __builtin_amdgcn_s_memtime());

  // ---- x1 -> normalised bf16x3 B fragments: k-step ks holds channels 16 ks + 8 half + 0..7
  bf16x8 xf[16][3];
  const float* xs = stage_x + 32 * wave + l32;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const float4 sa = *reinterpret_cast<const float4*>(scs + 16 * ks + 8 * half);
    const float4 sb = *reinterpret_cast<const float4*>(scs + 16 * ks + 8 * half + 4);
    const float4 ta = *reinterpret_cast<const float4*>(shs + 16 * ks + 8 * half);
    const float4 tb = *reinterpret_cast<const float4*>(shs + 16 * ks + 8 * half + 4);
    const float sv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float tv[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    float xv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = xs[(16 * ks + 8 * half + e) * MF_PX];
    uint32_t t[3][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      split2(fmaf(sv[2 * e], xv[2 * e], tv[2 * e]),
             fmaf(sv[2 * e + 1], xv[2 * e + 1], tv[2 * e + 1]), t[0][e], t[1][e], t[2][e]);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) xf[ks][pl] = mf_frag(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
  }
  floatx16 oacc[8];  // output accumulators (C layout rows of out block ob): b2 first
#pragma unroll
  for (int ob = 0; ob < 8; ++ob)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(b2s + 32 * ob + 8 * q + 4 * half);
      oacc[ob][4 * q] = b.x;
      oacc[ob][4 * q + 1] = b.y;
      oacc[ob][4 * q + 2] = b.z;
      oacc[ob][4 * q + 3] = b.w;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the staging area is free: slices 1, 2 may land in it
  issue(1);
  issue(2);
  if constexpr (STAMP) stamp(2, __builtin_amdgcn_s_memtime());
  floatx16 hacc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[i][r] = 0.f;

  const int a_lane = l32 * 16 + 8 * (half ^ mf_swz(l32));  // A fragment offset in a row group

  // wait for slice q and make it visible; the step then refills the slot of slice
  // q - 1 with slice q + 3 after its first k-step (refill(q)), so the MFMA pipe starts
  // right after the barrier and the DMA issue runs under the MFMAs
  // extra: residual-chunk DMA instructions this wave issued after slice q (below)
  auto step_begin = [&](int q, int extra = 0) {
    if constexpr ((DBG & 1) != 0) return ring + (q % MF_NS) * MF_SLICE_ELEMS;
    unsigned long long w0 = 0;
    if constexpr (STAMP) w0 = __builtin_amdgcn_s_memtime();
    const int after = min(2, MF_NSLICE - 1 - q);  // slices issued after q
    if (after >= 2 && extra)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (after >= 2)
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (after == 1)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (STAMP) st_wait += __builtin_amdgcn_s_memtime() - w0;
    return ring + (q % MF_NS) * MF_SLICE_ELEMS;
  };

  auto mfma6 = [](const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 c) {
    if constexpr ((DBG & 2) != 0) {
      c[0] += (float)a[0][0] + (float)b[0][0];  // keep the operands live, no MFMA
      return c;
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
    return c;
  };

  // Scheduling: every k-step is one region (sched_barrier) laid out as
  //   [ds_read x3 of the NEXT k-step] then 6 x [MFMA, up to 6 VALU]
  // so the A-fragment reads run one k-step ahead and the GELU/split VALU work of
  // the block being converted fills the MFMA issue gaps (an MFMA holds the SIMD's
  // vector issue for 8 of its 32 cycles; MI355X_MICROARCH.md) instead of running
  // ahead of them as one serial stretch.
  auto kstep_schedule = [](bool reads) {
    if constexpr (SCHED == 0) return;
    if (reads) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // DS read
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
      __builtin_amdgcn_sched_group_barrier(0x402, 6, 0);    // VALU incl. transcendental
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // one pair (slots r = 2 e2, 2 e2 + 1) of hidden block j in hacc[PAR] -> hfu:
  // + b1, GELU(erf), bf16x3 split
  uint32_t hfu[2][3][4];  // fc2 B fragments as bf16 pairs [k-step s][plane][pair]
  auto conv_pair = [&](int j, int e2, auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    uint32_t (&h)[2][3][4] = hfu;
    if constexpr ((DBG & 4) != 0) {
      h[e2 >> 2][0][e2 & 3] = __float_as_uint(hacc[PAR][2 * e2]);
      return;
    }
    const int r = 2 * e2;
    const float2 b = *reinterpret_cast<const float2*>(b1s + 32 * j + (r >> 2) * 8 + 4 * half + (r & 3));
    f32x2 v = {hacc[PAR][r] + b.x, hacc[PAR][r + 1] + b.y};
    v = gelu_erf2(v);
    split2(v.x, v.y, h[e2 >> 2][0][e2 & 3], h[e2 >> 2][1][e2 & 3], h[e2 >> 2][2][e2 & 3]);
  };

  // fc1 slice W1(j, KH) into hacc[PAR]; CONV: pairs 4 KH .. 4 KH + 3 of block jc
  // (in hacc[PAR ^ 1]) are converted under its MFMAs, one per odd k-step
  auto refill = [&](int q) {
    if constexpr ((DBG & 1) != 0) return;
    if (q + 3 < MF_NSLICE) issue(q + 3);
  };
  auto fc1_step = [&](const unsigned short* slot, int q, auto kh_c, auto par_c, auto conv_c,
                      int jc) {
    constexpr int KH = decltype(kh_c)::value, PAR = decltype(par_c)::value;
    constexpr bool CONV = decltype(conv_c)::value;
    using PPrev = std::integral_constant<int, PAR ^ 1>;
    bf16x8 a[MF_AHEAD + 1][3];
#pragma unroll
    for (int k = 0; k < MF_AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[k][pl] = *reinterpret_cast<const bf16x8*>(slot + (pl * 8 + k) * 512 + a_lane);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + MF_AHEAD < 8 && (DBG & 8) == 0) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[(ks + MF_AHEAD) % (MF_AHEAD + 1)][pl] =
              *reinterpret_cast<const bf16x8*>(slot + (pl * 8 + ks + MF_AHEAD) * 512 + a_lane);
      }
      hacc[PAR] = mfma6(a[(DBG & 8) ? 0 : ks % (MF_AHEAD + 1)], xf[KH * 8 + ks], hacc[PAR]);
      if (ks == 0) refill(q);
      if constexpr (CONV) {
        if (ks & 1) conv_pair(jc, 4 * KH + (ks >> 1), PPrev{});
      }
      kstep_schedule(ks + MF_AHEAD < 8);
    }
    if constexpr (CONV && KH == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) hacc[PAR ^ 1][r] = 0.f;
    }
  };
  // fc2 slice W2(j, OH) with the current hfu
  auto fc2_step = [&](const unsigned short* slot, int q, auto oh_c) {
    constexpr int OH = decltype(oh_c)::value;
    auto aoff = [&](int it, int pl) {  // it = 2 ob + s
      return ((pl * 2 + (it & 1)) * 128 + (it >> 1) * 32) * 16 + a_lane;
    };
    bf16x8 a[MF_AHEAD + 1][3];
#pragma unroll
    for (int k = 0; k < MF_AHEAD; ++k)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[k][pl] = *reinterpret_cast<const bf16x8*>(slot + aoff(k, pl));
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      if (it + MF_AHEAD < 8 && (DBG & 8) == 0) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[(it + MF_AHEAD) % (MF_AHEAD + 1)][pl] =
              *reinterpret_cast<const bf16x8*>(slot + aoff(it + MF_AHEAD, pl));
      }
      const int s = it & 1;
      const uint32_t (&h)[2][3][4] = hfu;
      const bf16x8 hb[3] = {mf_frag(h[s][0][0], h[s][0][1], h[s][0][2], h[s][0][3]),
                            mf_frag(h[s][1][0], h[s][1][1], h[s][1][2], h[s][1][3]),
                            mf_frag(h[s][2][0], h[s][2][1], h[s][2][2], h[s][2][3])};
      oacc[OH * 4 + (it >> 1)] =
          mfma6(a[(DBG & 8) ? 0 : it % (MF_AHEAD + 1)], hb, oacc[OH * 4 + (it >> 1)]);
      if (it == 0) refill(q);
      kstep_schedule(it + MF_AHEAD < 8);
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  using T = std::true_type;
  // round j (1..15): W1(j, 0..1) into hacc[j & 1] with block j - 1 converted under
  // their MFMAs, then W2(j - 1, 0..1)
  // The residual streams in near the end of the tile, 16-KB chunk c = channels
  // 32 c .. +31 (out block c) into staging region c % 3 above the ring: chunks 0-2
  // at step 50 (round 13), consumed at step 58 (round 15); 3-5 issued there, consumed
  // at step 62; 6-7 issued at step 62, consumed after the last step.  Consumption
  // is in the peeled rounds, where the accumulator index is a compile-time constant;
  // each consuming step has waited for a slice issued after the chunk, then barriered.
  const bool has_res = p.resid != nullptr;
  auto issue_res = [&](int c) {
    const float* src = p.resid + (int64_t)z * MF_C * P + (int64_t)(32 * c + (lane >> 5)) * P +
                       min(px0 + 4 * l32, P - 4);
    const uint32_t base = lds_addr(stage_res) + (uint32_t)((c % 3) * MF_RES_CHUNK);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int piece = wave + MF_WAVES * k;  // channel rows 2 piece, 2 piece + 1 of the chunk
      glds16(src + (int64_t)(2 * piece) * P, base + (uint32_t)(piece * 1024));
    }
  };
  auto add_res = [&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    const float* rs = stage_res + (c % 3) * (MF_RES_CHUNK / 4) + 32 * wave + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      oacc[c][r] += rs[((r >> 2) * 8 + 4 * half + (r & 3)) * MF_PX];
  };
  auto do_round = [&](int j, auto par_c) {
    const int q = 2 + 4 * (j - 1);
    const bool res_issue = has_res && j == MF_HB - 3;
    fc1_step(step_begin(q), q, I0{}, par_c, T{}, j - 1);
    if (res_issue) {  // after the step's refill (the vmcnt accounting relies on the order)
      issue_res(0);
      issue_res(1);
      issue_res(2);
    }
    const int ex = res_issue ? 12 : 0;
    fc1_step(step_begin(q + 1, ex), q + 1, I1{}, par_c, T{}, j - 1);
    fc2_step(step_begin(q + 2, ex), q + 2, I0{});
    fc2_step(step_begin(q + 3, ex), q + 3, I1{});
  };

  if constexpr (XS) {
    // ---- cross-step schedule --------------------------------------------------------
    // Fragment f of the current slice lives in af[f & 3].  Inside step q, after the
    // MFMAs of k-step 6, slice_wait(q + 1) makes slice q + 1 visible (every wave's DMA
    // of it landed, and every wave has finished reading slice q: its slot takes slice
    // q + 4 right away), and the first two fragments of slice q + 1 are read under
    // k-steps 6 and 7: the MFMA pipe does not restart from an LDS read at each slice.
    using K1 = std::integral_constant<int, 0>;  // W1 slice
    using K2 = std::integral_constant<int, 1>;  // W2 slice
    using KN = std::integral_constant<int, 2>;  // no next slice
    constexpr int QA = 2 + 4 * (MF_HB - 4), QB = 2 + 4 * (MF_HB - 2);  // residual issue steps
    bf16x8 af[4][3];
    auto load_frag = [&](int q, auto kind_c, int f) {
      constexpr int KIND = decltype(kind_c)::value;
      const unsigned short* slot = ring + (q % MF_NS) * MF_SLICE_ELEMS;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const int off = KIND == 0 ? (pl * 8 + f) * 512 + a_lane
                                  : ((pl * 2 + (f & 1)) * 128 + (f >> 1) * 32) * 16 + a_lane;
        af[f & 3][pl] = *reinterpret_cast<const bf16x8*>(slot + off);
      }
    };
    // slice q visible to every wave; DMA instructions this wave issued after slice q:
    // slices q + 1, q + 2 (6 each) and, around the residual issues, 12 more
    auto slice_wait = [&](int q) {
      if constexpr ((DBG & 1) != 0) return;
      unsigned long long w0 = 0;
      if constexpr (STAMP) w0 = __builtin_amdgcn_s_memtime();
      const int after = min(2, MF_NSLICE - 1 - q);
      const bool ex = has_res && ((q >= QA + 2 && q <= QA + 4) || (q >= QB + 2 && q <= QB + 3));
      if (after >= 2 && ex)
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else if (after >= 2)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (after == 1)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if constexpr (STAMP) st_wait += __builtin_amdgcn_s_memtime() - w0;
    };
    // step q: a W1 slice (KIND 0: hidden block into hacc[PAR], converting block jc of
    // hacc[PAR ^ 1] under it when CONV) or a W2 slice (KIND 1: out rows 128 SUB ..)
    auto xstep = [&](int q, auto kind_c, auto next_c, auto sub_c, auto par_c, auto conv_c,
                     int jc) {
      constexpr int KIND = decltype(kind_c)::value, NEXT = decltype(next_c)::value;
      constexpr int SUB = decltype(sub_c)::value, PAR = decltype(par_c)::value;
      constexpr bool CONV = decltype(conv_c)::value;
      using PPrev = std::integral_constant<int, PAR ^ 1>;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        if (ks + 2 < 8 && (DBG & 8) == 0) load_frag(q, kind_c, ks + 2);
        const int fi = (DBG & 8) ? 0 : (ks & 3);
        if constexpr (KIND == 0) {
          hacc[PAR] = mfma6(af[fi], xf[SUB * 8 + ks], hacc[PAR]);
          if constexpr (CONV) {
            if (ks & 1) conv_pair(jc, 4 * SUB + (ks >> 1), PPrev{});
          }
        } else {
          const int sh = ks & 1;
          const uint32_t (&h)[2][3][4] = hfu;
          const bf16x8 hb[3] = {mf_frag(h[sh][0][0], h[sh][0][1], h[sh][0][2], h[sh][0][3]),
                                mf_frag(h[sh][1][0], h[sh][1][1], h[sh][1][2], h[sh][1][3]),
                                mf_frag(h[sh][2][0], h[sh][2][1], h[sh][2][2], h[sh][2][3])};
          oacc[SUB * 4 + (ks >> 1)] = mfma6(af[fi], hb, oacc[SUB * 4 + (ks >> 1)]);
        }
        kstep_schedule(ks + 2 < 8 && (DBG & 8) == 0);
        if constexpr (NEXT != 2) {
          if (ks == 6) {
            slice_wait(q + 1);
            refill(q + 1);
          }
          if (ks >= 6 && (DBG & 8) == 0)
            load_frag(q + 1, std::integral_constant<int, NEXT>{}, ks - 6);
        }
      }
      if constexpr (KIND == 0 && CONV && SUB == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r) hacc[PAR ^ 1][r] = 0.f;
      }
    };
    auto xround = [&](int j, auto par_c) {
      const int q = 2 + 4 * (j - 1);
      xstep(q, K1{}, K1{}, I0{}, par_c, T{}, j - 1);
      if (has_res && j == MF_HB - 3) {  // q == QA; slices up to q + 4 issued
        issue_res(0);
        issue_res(1);
        issue_res(2);
      }
      xstep(q + 1, K1{}, K2{}, I1{}, par_c, T{}, j - 1);
      xstep(q + 2, K2{}, K2{}, I0{}, I0{}, F{}, 0);
      xstep(q + 3, K2{}, K1{}, I1{}, I0{}, F{}, 0);
    };
    // slice 0 landed (prologue); its slot's successor slice 3 (the x1 staging is free)
    issue(3);
    load_frag(0, K1{}, 0);
    load_frag(0, K1{}, 1);
    xstep(0, K1{}, K1{}, I0{}, I0{}, F{}, 0);
    xstep(1, K1{}, K1{}, I1{}, I0{}, F{}, 0);
    for (int j = 1; j < MF_HB - 1; j += 2) {
      xround(j, I1{});
      xround(j + 1, I0{});
    }
    // round 15 (peeled): residual chunks 0-2 in (slice_wait(58) retired them), 3-5 out
    if (has_res) {
      add_res(I0{});
      add_res(I1{});
      add_res(std::integral_constant<int, 2>{});
    }
    xstep(QB, K1{}, K1{}, I0{}, I1{}, T{}, MF_HB - 2);
    if (has_res) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // regions 0-2 read by every wave
      issue_res(3);
      issue_res(4);
      issue_res(5);
    }
    xstep(QB + 1, K1{}, K2{}, I1{}, I1{}, T{}, MF_HB - 2);
    xstep(QB + 2, K2{}, K2{}, I0{}, I0{}, F{}, 0);
    xstep(QB + 3, K2{}, K2{}, I1{}, I0{}, F{}, 0);  // slice_wait(62): vmcnt(6) retired chunks 3-5
    if (has_res) {
      add_res(std::integral_constant<int, 3>{});
      add_res(std::integral_constant<int, 4>{});
      add_res(std::integral_constant<int, 5>{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue_res(6);
      issue_res(7);
    }
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) conv_pair(MF_HB - 1, e2, I1{});
    xstep(MF_NSLICE - 2, K2{}, K2{}, I0{}, I0{}, F{}, 0);  // slice_wait(63): vmcnt(0), chunks 6, 7
    xstep(MF_NSLICE - 1, K2{}, KN{}, I1{}, I0{}, F{}, 0);
    if (has_res) {
      add_res(std::integral_constant<int, 6>{});
      add_res(std::integral_constant<int, 7>{});
    }
  } else {
  fc1_step(step_begin(0), 0, I0{}, I0{}, F{}, 0);
  fc1_step(step_begin(1), 1, I1{}, I0{}, F{}, 0);
  for (int j = 1; j < MF_HB - 1; j += 2) {
    do_round(j, I1{});
    do_round(j + 1, I0{});
  }
  {
    // round 15 (peeled): residual chunks 0-2 in, 3-5 out
    constexpr int j = MF_HB - 1;
    const int q = 2 + 4 * (j - 1);
    const unsigned short* s0 = step_begin(q);
    const int ex = has_res ? 12 : 0;
    if (has_res) {
      add_res(I0{});
      add_res(I1{});
      add_res(std::integral_constant<int, 2>{});
    }
    fc1_step(s0, q, I0{}, I1{}, T{}, j - 1);
    if (has_res) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // regions 0-2 read by every wave before the refill
      issue_res(3);
      issue_res(4);
      issue_res(5);
    }
    fc1_step(step_begin(q + 1, ex), q + 1, I1{}, I1{}, T{}, j - 1);
    fc2_step(step_begin(q + 2, ex), q + 2, I0{});
    fc2_step(step_begin(q + 3, ex), q + 3, I1{});
  }
  {
    // block 15 (hacc[1]) converted without MFMAs to hide it, then its fc2 slices
    const unsigned short* s0 = step_begin(MF_NSLICE - 2);  // its wait covers chunks 3-5
    if (has_res) {
      add_res(std::integral_constant<int, 3>{});
      add_res(std::integral_constant<int, 4>{});
      add_res(std::integral_constant<int, 5>{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue_res(6);
      issue_res(7);
    }
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) conv_pair(MF_HB - 1, e2, I1{});
    fc2_step(s0, MF_NSLICE - 2, I0{});
    fc2_step(step_begin(MF_NSLICE - 1), MF_NSLICE - 1, I1{});  // vmcnt(0): chunks 6, 7 landed
    if (has_res) {
      add_res(std::integral_constant<int, 6>{});
      add_res(std::integral_constant<int, 7>{});
    }
  }
  }  // XS

  if constexpr (STAMP) stamp(3, __builtin_amdgcn_s_memtime());
  // ---- store (all DMA retired: the last step waited vmcnt(0)) ------------------------
  if (valid) {
    float* o = p.out + (int64_t)z * MF_C * P + px;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[(int64_t)(32 * ob + (r >> 2) * 8 + 4 * half + (r & 3)) * P] = oacc[ob][r];
  }
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(4, __builtin_amdgcn_s_memtime());
    stamp(5, st_wait);
    stamp(6, (unsigned long long)__smid());
    stamp(7, __builtin_amdgcn_s_memrealtime() - rt0);
  }
}

// diagnostic launch (MSFNO_MF_STAMPS=1): synchronises, prints the median cycles of
// each phase over the workgroups to stderr
int mlp_fused_stamped(MlpFusedParams p, int64_t tiles, int sched, hipStream_t s) {
  std::vector<unsigned long long> h((size_t)tiles * 8);
  unsigned long long* d = nullptr;
  MSFNO_CHECK_HIP(hipMalloc(&d, h.size() * 8));
  p.stamps = d;
  static const int dbg = [] {
    const char* e = getenv("MSFNO_MF_DBG");
    return e ? atoi(e) : 0;
  }();
  if (dbg == 1)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1, 1>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else if (dbg == 2)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1, 2>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else if (dbg == 4)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1, 4>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else if (dbg == 8)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1, 8>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else if (dbg == 13)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1, 13>), dim3((unsigned)tiles), dim3(256), 0, s, p);

  else if (sched)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 1>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((mlp_fused_kernel<0, 1>), dim3((unsigned)tiles), dim3(256), 0, s, p);
  MSFNO_CHECK_HIP(hipStreamSynchronize(s));
  MSFNO_CHECK_HIP(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  MSFNO_CHECK_HIP(hipFree(d));
  auto med = [&](auto f) {
    std::vector<double> v;
    for (int64_t t = 0; t < tiles; ++t) v.push_back(f(&h[(size_t)t * 8]));
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::fprintf(stderr,
               "mlp_fused stamps (median cycles over %lld workgroups): prologue-load %.0f, "
               "split %.0f, steps %.0f (of which ring waits %.0f), store %.0f, total %.0f "
               "(%.2f us at 100 MHz realtime)\n",
               (long long)tiles, med([](auto* x) { return (double)(x[1] - x[0]); }),
               med([](auto* x) { return (double)(x[2] - x[1]); }),
               med([](auto* x) { return (double)(x[3] - x[2]); }),
               med([](auto* x) { return (double)x[5]; }),
               med([](auto* x) { return (double)(x[4] - x[3]); }),
               med([](auto* x) { return (double)(x[4] - x[0]); }),
               med([](auto* x) { return (double)x[7] / 100.0; }));
  return MSFNO_OK;
}

bool mlp_fused_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_MLP_FUSED");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

bool mlp_fused_supported(int C, int H) { return mlp_fused_env() && C == MF_C && H == MF_H; }

size_t mlp_fused_image_bytes() {
  return std::max((size_t)2 * MF_HB * 2 * MF_SLICE_ELEMS * 2, mlp_fused_h_image_bytes());
}

int launch_mlp_fused_images(const float* W1, const float* b1, const float* W2,
                            unsigned short* img, hipStream_t s) {
  MSFNO_REQUIRE(W1 && W2 && img && (reinterpret_cast<uintptr_t>(img) & 15) == 0, MSFNO_EINVAL,
                "mlp_fused: bad weight image arguments");
  if (mlp_fused_h_env()) return launch_mlp_fused_h_images(W1, b1, W2, img, s);
  unsigned short* w2img = img + (int64_t)MF_HB * 2 * MF_SLICE_ELEMS;
  hipLaunchKernelGGL(mf_w1_image_kernel, dim3(256), dim3(256), 0, s, W1, img);
  MSFNO_TRY(launch_check("mf_w1_image"));
  hipLaunchKernelGGL(mf_w2_image_kernel, dim3(256), dim3(256), 0, s, W2, w2img);
  return launch_check("mf_w2_image");
}

int launch_mlp_fused(const float* x1, const float* scale, const float* shift, const float* abound,
                     const float* resid, float* out, const unsigned short* img, const float* b1,
                     const float* b2, int B, int64_t P, hipStream_t s) {
  MSFNO_REQUIRE(x1 && scale && shift && out && img && b1 && B > 0 && P >= 4 && P % 4 == 0,
                MSFNO_EINVAL, "mlp_fused: bad arguments");
  MSFNO_REQUIRE(((reinterpret_cast<uintptr_t>(x1) | reinterpret_cast<uintptr_t>(resid)) & 15) == 0,
                MSFNO_EINVAL, "mlp_fused: x1 / resid must be 16-B aligned");
  if (mlp_fused_h_env())
    return launch_mlp_fused_h(x1, scale, shift, abound, resid, out, img, b1, b2, B, P, s);
  MlpFusedParams p{};
  p.x1 = x1; p.scale = scale; p.shift = shift; p.resid = resid; p.out = out;
  p.w1img = img;
  p.w2img = img + (int64_t)MF_HB * 2 * MF_SLICE_ELEMS;
  p.b1 = b1; p.b2 = b2; p.P = P;
  p.tiles_per_field = (int)cdiv(P, MF_PX);
  const int64_t tiles = (int64_t)B * p.tiles_per_field;
  MSFNO_REQUIRE(tiles < (1LL << 31), MSFNO_EINVAL, "mlp_fused: grid too large");
  // MSFNO_MF_SCHED=0: no explicit MFMA / VALU interleave (the compiler's schedule), for A/B
  static const int sched = [] {
    const char* e = getenv("MSFNO_MF_SCHED");
    return e ? atoi(e) : 1;
  }();
  static const bool stamps = [] {
    const char* e = getenv("MSFNO_MF_STAMPS");
    return e && e[0] == '1';
  }();
  // MSFNO_MF_AHEAD=1|3: A-fragment read-ahead depth (default 2), for A/B
  static const int ahead = [] {
    const char* e = getenv("MSFNO_MF_AHEAD");
    return e ? atoi(e) : 2;
  }();
  // MSFNO_MF_XS=1: cross-step A-fragment prefetch (the next slice's barrier inside the
  // current step), for A/B
  static const int xs = [] {
    const char* e = getenv("MSFNO_MF_XS");
    return e ? atoi(e) : 0;
  }();
  if (stamps) return mlp_fused_stamped(p, tiles, sched, s);
  const dim3 grid((unsigned)tiles), blk(256);
  if (xs)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 0, 0, 2, 1>), grid, blk, 0, s, p);
  else if (!sched)
    hipLaunchKernelGGL((mlp_fused_kernel<0, 0, 0, 2>), grid, blk, 0, s, p);

  else if (ahead == 1)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 0, 0, 1>), grid, blk, 0, s, p);
  else if (ahead == 3)
    hipLaunchKernelGGL((mlp_fused_kernel<1, 0, 0, 3>), grid, blk, 0, s, p);
  else
    hipLaunchKernelGGL((mlp_fused_kernel<1, 0, 0, 2>), grid, blk, 0, s, p);
  return launch_check("mlp_fused");
}

}  // namespace msfno
