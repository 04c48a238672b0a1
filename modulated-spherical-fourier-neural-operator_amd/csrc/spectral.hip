// Layout, statistics and streaming kernels around the Legendre/spectral GEMMs:
//   * Xn <-> Xt transposes (natural per-row spectrum <-> m-major GEMM operand),
//     with InstanceNorm-0 folded into the forward one,
//   * InstanceNorm statistics combination (Chan/Welford in fp64) + FiLM fold,
//   * weight preparation (complex block expansion, norm/FiLM folding into fc1),
//   * the linear filter's per-mode complex contraction (HBM weight stream),
//   * S-layout conversions (reference dense (l,m) / torch.tril_indices order).
#include <cstring>
#include <string>

#include "bf16x3.h"
#include "dma.h"
#include "kernels.h"

namespace msfno {

constexpr float kTwoPi = 6.28318530717958647692f;

// ---------------------------------------------------------------------------
// transposes
// ---------------------------------------------------------------------------
constexpr int TK = 64, TMM = 32;
// symmetric transposes, tiles (latitudes x m) measured at 721 x 1440 among 64x32,
// 32x64, 64x64 and 32x32: forward 64 x 32 (0.31 ms), inverse 32 x 64 (0.27 vs 0.30 ms)
constexpr int TK_FWD = 64, TM_FWD = 32, TK_INV = 32, TM_INV = 64;

__global__ __launch_bounds__(256) void transpose_fwd_kernel(const float2* __restrict__ Xn,
                                                            float* __restrict__ Xt, int B, int C,
                                                            int nlat, int mmax, int ldk,
                                                            const float* __restrict__ nscale,
                                                            const float* __restrict__ nshift,
                                                            const int* __restrict__ slab,
                                                            int kpad) {
  __shared__ float2 tile[TMM][TK + 1];
  const int k0 = blockIdx.x * TK, m0 = blockIdx.y * TMM;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const float2* src = Xn + (int64_t)bc * nlat * mmax;
  for (int i = threadIdx.x; i < TK * TMM; i += 256) {
    const int kk = i / TMM, mm = i - kk * TMM;
    const int k = k0 + kk, m = m0 + mm;
    float2 v = make_float2(0.f, 0.f);
    if (k < nlat && m < mmax) v = src[(int64_t)k * mmax + m];
    tile[mm][kk] = v;
  }
  __syncthreads();
  const float sc = nscale ? nscale[bc] : 1.f;
  const float sh = nshift ? nshift[bc] * kTwoPi : 0.f;
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  for (int i = threadIdx.x; i < TK * TMM; i += 256) {
    const int mm = i / TK, kk = i - mm * TK;
    const int k = k0 + kk, m = m0 + mm;
    const int sl = (m < mmax) ? (slab ? slab[m] : m) : -1;
    if (k < nlat && sl >= 0) {
      float2 v = tile[mm][kk];
      v.x = v.x * sc + (m == 0 ? sh : 0.f);
      v.y = v.y * sc;
      float* dst = Xt + (int64_t)sl * R * ldk;
      dst[rre * ldk + k] = v.x;
      dst[rim * ldk + k] = v.y;
    } else if (k < kpad && sl >= 0) {  // band exchange pads (read by the GEMM)
      float* dst = Xt + (int64_t)sl * R * ldk;
      dst[rre * ldk + k] = 0.f;
      dst[rim * ldk + k] = 0.f;
    }
  }
}

__global__ void dc_fixup_kernel(float* __restrict__ Xt, int B, int C, int nlat, int ldk,
                                const float* __restrict__ nscale,
                                const float* __restrict__ nshift) {
  const int64_t R = 2LL * B * C;
  const int64_t n = R * nlat;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / nlat;
    const int k = (int)(e - r * nlat);
    const int b = (int)(r / (2 * C));
    const int ri = (int)((r / C) & 1);
    const int c = (int)(r % C);
    const int bc = b * C + c;
    float* p = Xt + r * ldk + k;
    *p = ri ? nscale[bc] * *p : fmaf(nscale[bc], *p, kTwoPi * nshift[bc]);
  }
}

int launch_dc_fixup(float* Xt, int B, int C, int nlat, int ldk, const float* nscale,
                    const float* nshift, hipStream_t s) {
  const int64_t n = 2LL * B * C * nlat;
  hipLaunchKernelGGL(dc_fixup_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 4096)),
                     dim3(256), 0, s, Xt, B, C, nlat, ldk, nscale, nshift);
  return launch_check("dc_fixup");
}

int launch_transpose_fwd(const float2* Xn, float* Xt, int B, int C, int nlat, int mmax, int ldk,
                         const float* nscale, const float* nshift, hipStream_t s,
                         const int* slab, int kpad) {
  dim3 grid((unsigned)cdiv(std::max(nlat, kpad), TK), (unsigned)cdiv(mmax, TMM), (unsigned)(B * C));
  hipLaunchKernelGGL(transpose_fwd_kernel, grid, dim3(256), 0, s, Xn, Xt, B, C, nlat, mmax, ldk,
                     nscale, nshift, slab, kpad);
  return launch_check("transpose_fwd");
}

__global__ __launch_bounds__(256) void transpose_inv_kernel(const float* __restrict__ Yt,
                                                            float2* __restrict__ Yn, int B, int C,
                                                            int nlat, int mmax, int mact,
                                                            int ldk,
                                                            const int* __restrict__ slab) {
  __shared__ float2 tile[TMM][TK + 1];
  const int k0 = blockIdx.x * TK, m0 = blockIdx.y * TMM;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  for (int i = threadIdx.x; i < TK * TMM; i += 256) {
    const int mm = i / TK, kk = i - mm * TK;
    const int k = k0 + kk, m = m0 + mm;
    float2 v = make_float2(0.f, 0.f);
    const int sl = (m < mact) ? (slab ? slab[m] : m) : -1;
    if (k < nlat && sl >= 0) {
      const float* src = Yt + (int64_t)sl * R * ldk;
      v = make_float2(src[rre * ldk + k], src[rim * ldk + k]);
    }
    tile[mm][kk] = v;
  }
  __syncthreads();
  float2* dst = Yn + (int64_t)bc * nlat * mmax;
  for (int i = threadIdx.x; i < TK * TMM; i += 256) {
    const int kk = i / TMM, mm = i - kk * TMM;
    const int k = k0 + kk, m = m0 + mm;
    if (k < nlat && m < mmax) dst[(int64_t)k * mmax + m] = tile[mm][kk];
  }
}

int launch_transpose_inv(const float* Yt, float2* Yn, int B, int C, int nlat, int mmax, int mact,
                         int ldk, hipStream_t s, const int* slab) {
  dim3 grid((unsigned)cdiv(nlat, TK), (unsigned)cdiv(mmax, TMM), (unsigned)(B * C));
  hipLaunchKernelGGL(transpose_inv_kernel, grid, dim3(256), 0, s, Yt, Yn, B, C, nlat, mmax, mact,
                     ldk, slab);
  return launch_check("transpose_inv");
}

// Equatorially symmetric plans (msfno_sht_plan_s::sym): the forward transpose
// also folds the hemispheres, Xs_k = X_k + X_{n-1-k} (k < Ke; the centre row of
// an odd grid once) into slab columns [0, Ke) and Xa_k = X_k - X_{n-1-k} (k < Ko)
// into [ldke, ldke + Ko); the inverse one unfolds Y_k = E_k + O_k,
// Y_{n-1-k} = E_k - O_k from the even/odd Legendre outputs.
template <int TKx, int TMx>
__global__ __launch_bounds__(256) void transpose_fwd_sym_kernel(
    const float2* __restrict__ Xn, float* __restrict__ Xt, int B, int C, LatGeom g, int mmax,
    const float* __restrict__ nscale, const float* __restrict__ nshift,
    const int* __restrict__ slab, int kpad) {
  __shared__ float2 tn[TMx][TKx + 1], ts[TMx][TKx + 1];
  const int k0 = blockIdx.x * TKx, m0 = blockIdx.y * TMx;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const float2* src = Xn + (int64_t)bc * g.nlat * mmax;
  for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
    const int kk = i / TMx, mm = i - kk * TMx;
    const int k = k0 + kk, m = m0 + mm;
    float2 vn = make_float2(0.f, 0.f), vs = vn;
    if (k < g.Ke && m < mmax) {
      vn = src[(int64_t)k * mmax + m];
      if (k < g.nh) vs = src[(int64_t)(g.nlat - 1 - k) * mmax + m];
    }
    tn[mm][kk] = vn;
    ts[mm][kk] = vs;
  }
  __syncthreads();
  const float sc = nscale ? nscale[bc] : 1.f;
  const float sh = nshift ? nshift[bc] * kTwoPi : 0.f;
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
    const int mm = i / TKx, kk = i - mm * TKx;
    const int k = k0 + kk, m = m0 + mm;
    if (m >= mmax) continue;
    const int sl = slab ? slab[m] : m;
    if (sl < 0) continue;
    float* dst = Xt + (int64_t)sl * R * g.ldk;
    if (k >= g.Ke) {  // band exchange pads (read by the GEMM): Xs [Ke, kpad), Xa [nh, kpad)
      if (k < kpad) {
        dst[rre * g.ldk + k] = 0.f;
        dst[rim * g.ldk + k] = 0.f;
        dst[rre * g.ldk + g.ldke + k] = 0.f;
        dst[rim * g.ldk + g.ldke + k] = 0.f;
      }
      continue;
    }
    const float2 n = tn[mm][kk], q = ts[mm][kk];
    const float shm = (m == 0) ? sh : 0.f;
    const bool pair = k < g.nh;
    // affine per row, then fold: s(N + S) + 2t  /  s(N - S)
    dst[rre * g.ldk + k] = pair ? fmaf(sc, n.x + q.x, 2.f * shm) : fmaf(sc, n.x, shm);
    dst[rim * g.ldk + k] = pair ? sc * (n.y + q.y) : sc * n.y;
    if (pair) {
      dst[rre * g.ldk + g.ldke + k] = sc * (n.x - q.x);
      dst[rim * g.ldk + g.ldke + k] = sc * (n.y - q.y);
    } else if (k < kpad) {
      dst[rre * g.ldk + g.ldke + k] = 0.f;
      dst[rim * g.ldk + g.ldke + k] = 0.f;
    }
  }
}

// Two-phase variants: ONE LDS tile, written twice (Xs then Xa forward, north then
// south rows inverse) from values the threads hold in registers, so a 32 x 128 tile
// fits in 33 KB: rows of 128 m (1 KB) on the spectrum side and whole 128-B lines of
// 32 latitudes on the slab side (the one-phase 16 x 128 / 64 x 32 tiles fetch half
// lines: PMC read bytes 2.0x / 1.5x the algorithmic ones)
template <int TKx, int TMx>
__global__ __launch_bounds__(256) void transpose_fwd_sym2_kernel(
    const float2* __restrict__ Xn, float* __restrict__ Xt, int B, int C, LatGeom g, int mmax,
    const float* __restrict__ nscale, const float* __restrict__ nshift,
    const int* __restrict__ slab, int kpad) {
  constexpr int PER = TKx * TMx / 256;
  static_assert(PER * 256 == TKx * TMx, "tile");
  __shared__ float2 tile[TMx][TKx + 1];
  const int k0 = blockIdx.x * TKx, m0 = blockIdx.y * TMx;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const float2* src = Xn + (int64_t)bc * g.nlat * mmax;
  const float sc = nscale ? nscale[bc] : 1.f;
  const float sh = nshift ? nshift[bc] * kTwoPi : 0.f;
  float2 xs[PER], xa[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int i = threadIdx.x + 256 * q;
    const int kk = i / TMx, mm = i - kk * TMx;
    const int k = k0 + kk, m = m0 + mm;
    float2 n = make_float2(0.f, 0.f), t = n;
    if (k < g.Ke && m < mmax) {
      n = src[(int64_t)k * mmax + m];
      if (k < g.nh) t = src[(int64_t)(g.nlat - 1 - k) * mmax + m];
    }
    const bool pair = k < g.nh;
    const float shm = (m == 0) ? sh : 0.f;
    // affine per row, then fold: s(N + S) + 2t  /  s(N - S)
    xs[q] = k >= g.Ke ? make_float2(0.f, 0.f)  // band pads
            : pair ? make_float2(fmaf(sc, n.x + t.x, 2.f * shm), sc * (n.y + t.y))
                   : make_float2(fmaf(sc, n.x, shm), sc * n.y);
    xa[q] = pair ? make_float2(sc * (n.x - t.x), sc * (n.y - t.y)) : make_float2(0.f, 0.f);
  }
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  const int kend = max(g.Ke, kpad);
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    if (ph) __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int kk = i / TMx, mm = i - kk * TMx;
      tile[mm][kk] = ph ? xa[q] : xs[q];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
      const int mm = i / TKx, kk = i - mm * TKx;
      const int k = k0 + kk, m = m0 + mm;
      if (k >= kend || m >= mmax) continue;
      const int sl = slab ? slab[m] : m;
      if (sl < 0) continue;
      // real values for k < Ke (Xs) / k < nh (Xa); zeros on the pads up to kpad
      if (k >= (ph ? (kpad > 0 ? kend : g.nh) : kend)) continue;
      const float2 v = tile[mm][kk];
      float* dst = Xt + (int64_t)sl * R * g.ldk + (ph ? g.ldke : 0) + k;
      dst[rre * g.ldk] = v.x;
      dst[rim * g.ldk] = v.y;
    }
  }
}

// Vector-store variant: the fold + affine in registers on the load side (8-B loads of
// the north and mirror rows), the four slab rows of one m (Xs re / im, Xa re / im)
// as LDS rows of TKx floats, stored as 16-B vectors (a 64-lane instruction writes
// four 256-B row segments; the scalar-store kernels above write one).  Whole float4
// units up to round4(end of the valid k range) are written, zeros past it (pads).
template <int TKx, int TMx>
__global__ __launch_bounds__(256) void transpose_fwd_sym4_kernel(
    const float2* __restrict__ Xn, float* __restrict__ Xt, int B, int C, LatGeom g, int mmax,
    const float* __restrict__ nscale, const float* __restrict__ nshift,
    const int* __restrict__ slab, int kpad) {
  constexpr int LD = TKx + 4;  // 16-B aligned LDS rows
  constexpr int KV = TKx / 4;  // float4 units per row
  __shared__ __attribute__((aligned(16))) float tile[4 * TMx * LD];  // [h][c][m][k]
  const int k0 = blockIdx.x * TKx, m0 = blockIdx.y * TMx;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const float2* src = Xn + (int64_t)bc * g.nlat * mmax;
  const float sc = nscale ? nscale[bc] : 1.f;
  const float sh = nshift ? nshift[bc] * kTwoPi : 0.f;
  for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
    const int kk = i / TMx, mm = i - kk * TMx;
    const int k = k0 + kk, m = m0 + mm;
    float2 n = make_float2(0.f, 0.f), t = n;
    if (k < g.Ke && m < mmax) {
      n = src[(int64_t)k * mmax + m];
      if (k < g.nh) t = src[(int64_t)(g.nlat - 1 - k) * mmax + m];
    }
    const bool pair = k < g.nh;
    const float shm = (m == 0) ? sh : 0.f;
    // affine per row, then fold: s(N + S) + 2t  /  s(N - S); zeros past Ke / nh
    const float sre = pair ? fmaf(sc, n.x + t.x, 2.f * shm) : (k < g.Ke ? fmaf(sc, n.x, shm) : 0.f);
    const float sim = pair ? sc * (n.y + t.y) : sc * n.y;
    tile[(0 * TMx + mm) * LD + kk] = sre;
    tile[(1 * TMx + mm) * LD + kk] = sim;
    tile[(2 * TMx + mm) * LD + kk] = pair ? sc * (n.x - t.x) : 0.f;
    tile[(3 * TMx + mm) * LD + kk] = pair ? sc * (n.y - t.y) : 0.f;
  }
  __syncthreads();
  const int64_t R = 2LL * B * C;
  const int kend = max(g.Ke, kpad);
  const int kend_a = kpad > 0 ? kend : g.nh;
  for (int i = threadIdx.x; i < 4 * TMx * KV; i += 256) {
    const int row = i / KV, kv = i - row * KV;
    const int hc = row / TMx, mm = row - hc * TMx;
    const int h = hc >> 1, ri = hc & 1;
    const int k = k0 + 4 * kv, m = m0 + mm;
    if (m >= mmax || k >= (h ? kend_a : kend)) continue;
    const int sl = slab ? slab[m] : m;
    if (sl < 0) continue;
    const float4 v = *reinterpret_cast<const float4*>(tile + row * LD + 4 * kv);
    float* dst = Xt + (int64_t)sl * R * g.ldk + ((int64_t)(b * 2 + ri) * C + c) * g.ldk +
                 (h ? g.ldke : 0) + k;
    *reinterpret_cast<float4*>(dst) = v;
  }
}

// x3h-plane variant of the vector-store kernel, for the register-B forward Legendre
// (legendre_x3f): the slab as two fp16 terms per value (v = v0 + v1, v0 = fp16(v),
// v1 = fp16(v - v0): the same 4 bytes per value as fp32), interleaved per 8 k
// ([slab][R][ldk / 8][plane][8]: a thread's 8 values are 32 contiguous bytes) under ONE
// power-of-two scale per channel, sigma_bc = lsig[bc] from chan_affine: a bound of the
// whole folded slab row (|x^| <= |s| sqrt(M2) + |s mean + t| for the norm0 output,
// the rfft scaled by 2 pi / nlon gives |X^_m| <= 2 pi max |x^|, the fold doubles it)
// mapped into [2^14, 2^15).
// 1 / sigma goes to isr[r] for both slab rows r of the channel.  Pads are written as
// zeros up to ldke (Xs) and ldk - ldke (Xa), so every 16-B piece the GEMM stages
// below its K holds finite values.
__device__ __forceinline__ void split_h2(float a, float b, uint32_t& t0, uint32_t& t1) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t v = {a, b};
  const h2_t h0 = __builtin_convertvector(v, h2_t);
  const f2_t r = v - __builtin_convertvector(h0, f2_t);
  const h2_t h1 = __builtin_convertvector(r, h2_t);
  t0 = __builtin_bit_cast(uint32_t, h0);
  t1 = __builtin_bit_cast(uint32_t, h1);
}

// Block order of the symmetric transposes (XR): the spectra rows (mmax float2 = 2888 B at
// 721x1440) and the slab rows start off the 128-B line grid, so two neighbouring tiles
// share the lines at their common edge; the hardware deals blocks round-robin over the
// 8 XCDs, which puts neighbours in different L2s, and each fetches the shared line from
// HBM (PMC: reads 1.5x the algorithmic bytes, profiles/r06_v).  XR = 1 / 2: a 1-D grid
// whose ids tr_remap makes contiguous per XCD, decoded m-tile fastest (1) or
// latitude-tile fastest (2: the hardware's own order, but with neighbours in one XCD).
// XR = 0: the plain 3-D grid.
__device__ __forceinline__ int tr_remap(int orig, int nwg) {  // = gemm_common.h xcd_remap
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <int XR>
__device__ __forceinline__ int3 tr_block(int nx, int ny) {
  if constexpr (XR == 0) {
    return make_int3((int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
  } else if constexpr (XR == 1) {
    const int lin = tr_remap((int)blockIdx.x, (int)gridDim.x);
    const int y = lin % ny, r = lin / ny;
    return make_int3(r % nx, y, r / nx);
  } else {
    const int lin = tr_remap((int)blockIdx.x, (int)gridDim.x);
    const int x = lin % nx, r = lin / nx;
    return make_int3(x, r % ny, r / ny);
  }
}

static dim3 tr_grid(int xr, int nx, int ny, int nz) {
  return xr ? dim3((unsigned)(nx * ny * nz)) : dim3((unsigned)nx, (unsigned)ny, (unsigned)nz);
}

// MSFNO_TR_XCD = "<forward><inverse>" block orders (A/B; "00": the plain 3-D grids)
static int tr_xcd(int which) {
  static const std::string v = [] {
    const char* e = getenv("MSFNO_TR_XCD");
    return std::string(e && strlen(e) == 2 ? e : "22");
  }();
  const int d = v[which] - '0';
  return d >= 0 && d <= 2 ? d : 2;
}

template <int TKx, int TMx>
static void fwd_sym4h_launch(const float2* Xn, unsigned short* Xp, int B, int C, const LatGeom& g,
                             int mmax, const float* nscale, const float* nshift,
                             const float* lsig, float* isr, const int* perm, int kext,
                             hipStream_t s);

template <int TKx, int TMx, int XR, bool PRE>
__global__ __launch_bounds__(256) void transpose_fwd_sym4h_kernel(
    const float2* __restrict__ Xn, unsigned short* __restrict__ Xp, int B, int C,
    LatGeom g, int mmax, const float* __restrict__ nscale, const float* __restrict__ nshift,
    const float* __restrict__ lsig, float* __restrict__ isr, const int* __restrict__ slab,
    int nx, int ny) {
  constexpr int LD = TKx + 4;
  __shared__ __attribute__((aligned(16))) float tile[4 * TMx * LD];  // [h][c][m][k]
  const int3 blk = tr_block<XR>(nx, ny);
  const int k0 = blk.x * TKx, m0 = blk.y * TMx;
  const int bc = blk.z;
  const int b = bc / C, c = bc - b * C;
  const float2* src = Xn + (int64_t)bc * g.nlat * mmax;
  const float sc = nscale[bc];
  const float sh = nshift[bc] * kTwoPi;
  const float sig = lsig[bc];
  const int64_t R = 2LL * B * C;
  if (blk.x == 0 && blk.y == 0 && threadIdx.x < 2)
    isr[(int64_t)(b * 2 + threadIdx.x) * C + c] = 1.f / sig;
  // the tile's values: every load of a thread issued before the first is used (PRE; the
  // rolled loop kept two 8-B loads per wave in flight), then folded into the LDS tile
  auto put = [&](int kk, int mm, float2 n, float2 t) {
    const int k = k0 + kk, m = m0 + mm;
    const bool pair = k < g.nh;
    const float shm = (m == 0) ? sh : 0.f;
    const float sre = pair ? fmaf(sc, n.x + t.x, 2.f * shm) : (k < g.Ke ? fmaf(sc, n.x, shm) : 0.f);
    const float sim = pair ? sc * (n.y + t.y) : sc * n.y;
    tile[(0 * TMx + mm) * LD + kk] = sre * sig;
    tile[(1 * TMx + mm) * LD + kk] = sim * sig;
    tile[(2 * TMx + mm) * LD + kk] = pair ? sc * (n.x - t.x) * sig : 0.f;
    tile[(3 * TMx + mm) * LD + kk] = pair ? sc * (n.y - t.y) * sig : 0.f;
  };
  auto fetch = [&](int kk, int mm, float2& n, float2& t) {
    const int k = k0 + kk, m = m0 + mm;
    n = make_float2(0.f, 0.f);
    t = n;
    if (k < g.Ke && m < mmax) {
      n = src[(int64_t)k * mmax + m];
      if (k < g.nh) t = src[(int64_t)(g.nlat - 1 - k) * mmax + m];
    }
  };
  if constexpr (PRE) {
    constexpr int PER = TKx * TMx / 256;
    static_assert(PER * 256 == TKx * TMx, "tile");
    float2 nv[PER], tv[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      fetch(i / TMx, i % TMx, nv[q], tv[q]);
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      put(i / TMx, i % TMx, nv[q], tv[q]);
    }
  } else {
    for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
      float2 n, t;
      fetch(i / TMx, i % TMx, n, t);
      put(i / TMx, i % TMx, n, t);
    }
  }
  __syncthreads();
  // 8 k per thread: one 16-B store per plane (ldke, ldk are multiples of 8)
  constexpr int KV8 = TKx / 8;
  const int kend_s = g.ldke, kend_a = g.ldk - g.ldke;  // pads as zeros
  for (int i = threadIdx.x; i < 4 * TMx * KV8; i += 256) {
    const int row = i / KV8, kv = i - row * KV8;
    const int hc = row / TMx, mm = row - hc * TMx;
    const int h = hc >> 1, ri = hc & 1;
    const int k = k0 + 8 * kv, m = m0 + mm;
    if (m >= mmax || k >= (h ? kend_a : kend_s)) continue;
    const int sl = slab ? slab[m] : m;  // (band pack: the slab of m in the send order)
    if (sl < 0) continue;
    const float4 v = *reinterpret_cast<const float4*>(tile + row * LD + 8 * kv);
    const float4 w = *reinterpret_cast<const float4*>(tile + row * LD + 8 * kv + 4);
    uint4 hi, lo;
    split_h2(v.x, v.y, hi.x, lo.x);
    split_h2(v.z, v.w, hi.y, lo.y);
    split_h2(w.x, w.y, hi.z, lo.z);
    split_h2(w.z, w.w, hi.w, lo.w);
    // interleaved planes: 8 k of the high plane, then the same 8 k of the low plane
    unsigned short* dst = Xp + 2 * ((int64_t)sl * R * g.ldk +
                                    ((int64_t)(b * 2 + ri) * C + c) * g.ldk + (h ? g.ldke : 0) + k);
    *reinterpret_cast<uint4*>(dst) = hi;
    *reinterpret_cast<uint4*>(dst + 8) = lo;
  }
}

int launch_transpose_fwd_sym_h(const float2* Xn, unsigned short* Xp, int B, int C,
                               const LatGeom& g, int mmax, const float* nscale,
                               const float* nshift, const float* lsig, float* isr,
                               hipStream_t s) {
  if (!nscale || !nshift || !lsig || !isr || !g.sym || (g.ldke & 7) || (g.ldk & 7) ||
      std::max(g.ldke, g.ldk - g.ldke) > cdiv(g.Ke, 64) * 64)
    return MSFNO_EINVAL;
  fwd_sym4h_launch<64, 32>(Xn, Xp, B, C, g, mmax, nscale, nshift, lsig, isr, nullptr, g.Ke, s);
  return launch_check("transpose_fwd_sym_h");
}

// the latitude-band pack on x3h pairs (band.cpp stage 1, symmetric plans): this rank's
// spectra -> the phase-0 send buffer as launch_band_pack lays it out (slab perm[m], rows
// of 2W: [Xs | Xa], pads zero), each value as the two fp16 terms of
// transpose_fwd_sym4h_kernel under the channel's sigma; 1 / sigma to isr (every row)
int launch_band_pack_h(const float2* Xn, unsigned short* send, int B, int C, const LatGeom& g,
                       int mmax, const float* nscale, const float* nshift, const float* lsig,
                       float* isr, const int* perm, int W, hipStream_t s) {
  MSFNO_REQUIRE(g.sym && nscale && nshift && lsig && isr && perm && W % 8 == 0 &&
                    g.ldke == W && g.ldk == 2 * W,
                MSFNO_EINVAL, "band_pack_h: symmetric band geometry with W % 8 == 0");
  fwd_sym4h_launch<64, 32>(Xn, send, B, C, g, mmax, nscale, nshift, lsig, isr, perm,
                           std::max(g.Ke, W), s);
  return launch_check("band_pack_h");
}

template <int TKx, int TMx>
static void fwd_sym4h_launch(const float2* Xn, unsigned short* Xp, int B, int C, const LatGeom& g,
                             int mmax, const float* nscale, const float* nshift,
                             const float* lsig, float* isr, const int* perm, int kext,
                             hipStream_t s) {
  const int nx = cdiv(kext, TKx), ny = cdiv(mmax, TMx), xr = tr_xcd(0);
  const dim3 grid = tr_grid(xr, nx, ny, B * C);
  static const bool pre = [] {
    const char* e = getenv("MSFNO_TR_FWD_PRE");
    return !(e && e[0] == '0');
  }();
#define MSFNO_SYM4H(XR, PRE)                                                                     \
  hipLaunchKernelGGL((transpose_fwd_sym4h_kernel<TKx, TMx, XR, PRE>), grid, dim3(256), 0, s, Xn, \
                     Xp, B, C, g, mmax, nscale, nshift, lsig, isr, perm, nx, ny)
  if (xr == 2 && pre) MSFNO_SYM4H(2, true);
  else if (xr == 2) MSFNO_SYM4H(2, false);
  else if (xr == 1) MSFNO_SYM4H(1, false);
  else MSFNO_SYM4H(0, false);
#undef MSFNO_SYM4H
}

// BF: the loads are branch-free (clamped addresses, the values selected afterwards), so a
// thread's 64 loads are all in flight at once; with the range tests as branches the
// compiler drained them per branch (33 vmcnt(0) waits, at most 4 loads in flight)
template <int TKx, int TMx, int XR, bool BF>
__global__ __launch_bounds__(256) void transpose_inv_sym2_kernel(const float* __restrict__ Yt,
                                                                 float2* __restrict__ Yn, int B,
                                                                 int C, LatGeom g, int mmax,
                                                                 int mact,
                                                                 const int* __restrict__ slab,
                                                                 int nx, int ny) {
  constexpr int PER = TKx * TMx / 256;
  static_assert(PER * 256 == TKx * TMx, "tile");
  __shared__ float2 tile[TMx][TKx + 1];
  const int3 blk = tr_block<XR>(nx, ny);
  const int k0 = blk.x * TKx, m0 = blk.y * TMx;
  const int bc = blk.z;
  const int b = bc / C, c = bc - b * C;
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  float2 yn[PER], ys[PER];
  if constexpr (BF) {
    // the slab of every m first (one wait), then all 4 PER loads at clamped addresses;
    // the empty asm uses each value unconditionally, so the compiler cannot sink a
    // load into the branch of its range test
    int slq[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int m = m0 + (threadIdx.x + 256 * q) / TKx;
      slq[q] = (m < mact) ? (slab ? slab[min(m, mact - 1)] : m) : -1;
    }
    float er[PER], ei[PER], orr[PER], oi[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int k = k0 + (i % TKx);
      const bool ok = k < g.Ke && slq[q] >= 0, pr = ok && k < g.nh;
      const float* srcp = Yt + (int64_t)(ok ? slq[q] : 0) * R * g.ldk;
      const int ke = ok ? k : 0, ko = g.ldke + (pr ? k : 0);
      er[q] = srcp[rre * g.ldk + ke];
      ei[q] = srcp[rim * g.ldk + ke];
      orr[q] = srcp[rre * g.ldk + ko];
      oi[q] = srcp[rim * g.ldk + ko];
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      asm volatile("" : "+v"(er[q]), "+v"(ei[q]), "+v"(orr[q]), "+v"(oi[q]));
      const int i = threadIdx.x + 256 * q;
      const int k = k0 + (i % TKx);
      const bool ok = k < g.Ke && slq[q] >= 0, pr = ok && k < g.nh;
      const float2 e = ok ? make_float2(er[q], ei[q]) : make_float2(0.f, 0.f);
      const float2 o = pr ? make_float2(orr[q], oi[q]) : make_float2(0.f, 0.f);
      yn[q] = make_float2(e.x + o.x, e.y + o.y);
      ys[q] = pr ? make_float2(e.x - o.x, e.y - o.y) : make_float2(0.f, 0.f);
    }
  } else {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int mm = i / TKx, kk = i - mm * TKx;
      const int k = k0 + kk, m = m0 + mm;
      float2 n = make_float2(0.f, 0.f), t = n;
      const int sl = (m < mact) ? (slab ? slab[m] : m) : -1;
      if (k < g.Ke && sl >= 0) {
        const float* srcp = Yt + (int64_t)sl * R * g.ldk;
        const float2 e = make_float2(srcp[rre * g.ldk + k], srcp[rim * g.ldk + k]);
        if (k < g.nh) {
          const float2 o = make_float2(srcp[rre * g.ldk + g.ldke + k], srcp[rim * g.ldk + g.ldke + k]);
          n = make_float2(e.x + o.x, e.y + o.y);
          t = make_float2(e.x - o.x, e.y - o.y);
        } else {
          n = e;
        }
      }
      yn[q] = n;
      ys[q] = t;
    }
  }
  float2* dst = Yn + (int64_t)bc * g.nlat * mmax;
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    if (ph) __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int mm = i / TKx, kk = i - mm * TKx;
      tile[mm][kk] = ph ? ys[q] : yn[q];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
      const int kk = i / TMx, mm = i - kk * TMx;
      const int k = k0 + kk, m = m0 + mm;
      if (m >= mmax || k >= (ph ? g.nh : g.Ke)) continue;
      dst[(int64_t)(ph ? g.nlat - 1 - k : k) * mmax + m] = tile[mm][kk];
    }
  }
}

// tile shape (latitudes x m) of the symmetric transposes: MSFNO_TR_FWD / MSFNO_TR_INV =
// "64x32" | "32x64" | "32x128" | "16x128" | "2p" | "v4" (A/B; defaults v4 forward: the
// 64x32 tile with 16-B stores, 0.265 vs 0.280 ms for 64x32 in two interleaved in-block
// runs (round 3); 2p inverse: 0.247-0.248 vs 0.255-0.258 ms for 16x128 in four interleaved in-block runs
// at 721x1440, C = 256 (16x128: 0.257 vs 0.268 ms for 32x64); the 32x128 one-phase
// tiles (67 KB of LDS) lose occupancy: 0.58 / 0.34 ms)
static int tr_tile(const char* var, int dflt) {
  const char* e = getenv(var);
  if (!e) return dflt;
  const std::string v(e);
  return v == "64x32" ? 0 : v == "32x64" ? 1 : v == "32x128" ? 2 : v == "16x128" ? 3
         : v == "2p" ? 4 : v == "v4" ? 5 : dflt;
}

template <int TKx, int TMx>
static void fwd_sym_launch(const float2* Xn, float* Xt, int B, int C, const LatGeom& g, int mmax,
                           const float* nscale, const float* nshift, const int* perm, int kpad,
                           hipStream_t s) {
  dim3 grid((unsigned)cdiv(std::max(g.Ke, kpad), TKx), (unsigned)cdiv(mmax, TMx),
            (unsigned)(B * C));
  hipLaunchKernelGGL((transpose_fwd_sym_kernel<TKx, TMx>), grid, dim3(256), 0, s, Xn, Xt, B, C,
                     g, mmax, nscale, nshift, perm, kpad);
}

static void fwd_sym_dispatch(const float2* Xn, float* Xt, int B, int C, const LatGeom& g,
                             int mmax, const float* nscale, const float* nshift, const int* perm,
                             int kpad, hipStream_t s) {
  static const int t = tr_tile("MSFNO_TR_FWD", 5);
  switch (t) {
    case 1: fwd_sym_launch<32, 64>(Xn, Xt, B, C, g, mmax, nscale, nshift, perm, kpad, s); break;
    case 2: fwd_sym_launch<32, 128>(Xn, Xt, B, C, g, mmax, nscale, nshift, perm, kpad, s); break;
    case 3: fwd_sym_launch<16, 128>(Xn, Xt, B, C, g, mmax, nscale, nshift, perm, kpad, s); break;
    case 4: {
      dim3 grid((unsigned)cdiv(std::max(g.Ke, kpad), 32), (unsigned)cdiv(mmax, 128),
                (unsigned)(B * C));
      hipLaunchKernelGGL((transpose_fwd_sym2_kernel<32, 128>), grid, dim3(256), 0, s, Xn, Xt, B,
                         C, g, mmax, nscale, nshift, perm, kpad);
      break;
    }
    case 5: {
      dim3 grid((unsigned)cdiv(std::max(g.Ke, kpad), 64), (unsigned)cdiv(mmax, 32),
                (unsigned)(B * C));
      hipLaunchKernelGGL((transpose_fwd_sym4_kernel<64, 32>), grid, dim3(256), 0, s, Xn, Xt, B,
                         C, g, mmax, nscale, nshift, perm, kpad);
      break;
    }
    default: fwd_sym_launch<TK_FWD, TM_FWD>(Xn, Xt, B, C, g, mmax, nscale, nshift, perm, kpad, s);
  }
}

int launch_transpose_fwd_sym(const float2* Xn, float* Xt, int B, int C, const LatGeom& g, int mmax,
                             const float* nscale, const float* nshift, hipStream_t s) {
  fwd_sym_dispatch(Xn, Xt, B, C, g, mmax, nscale, nshift, nullptr, 0, s);
  return launch_check("transpose_fwd_sym");
}

// Latitude-band pack (band.cpp stage 1): this rank's spectra Xn (local rows, geometry
// g: rows [0, Ke) its band, [Ke, nlat) the mirrors of its first nh rows) -> the
// phase-0 send buffer, slab perm[m] (ordered by owner), slab rows of ldk = 2W:
// folded [Xs | Xa] on a symmetric plan, the local rows on a general one; pads zero.
int launch_band_pack(const float2* Xn, float* send, int B, int C, const LatGeom& g, int mmax,
                     const float* nscale, const float* nshift, const int* perm, int W,
                     hipStream_t s) {
  if (!g.sym)
    return launch_transpose_fwd(Xn, send, B, C, g.nlat, mmax, g.ldk, nscale, nshift, s, perm,
                                2 * W);
  fwd_sym_dispatch(Xn, send, B, C, g, mmax, nscale, nshift, perm, W, s);
  return launch_check("band_pack");
}


template <int TKx, int TMx>
__global__ __launch_bounds__(256) void transpose_inv_sym_kernel(const float* __restrict__ Yt,
                                                                float2* __restrict__ Yn, int B,
                                                                int C, LatGeom g, int mmax,
                                                                int mact,
                                                                const int* __restrict__ slab) {
  __shared__ float2 tn[TMx][TKx + 1], ts[TMx][TKx + 1];
  const int k0 = blockIdx.x * TKx, m0 = blockIdx.y * TMx;
  const int bc = blockIdx.z;
  const int b = bc / C, c = bc - b * C;
  const int64_t R = 2LL * B * C;
  const int64_t rre = (int64_t)(b * 2 + 0) * C + c;
  const int64_t rim = (int64_t)(b * 2 + 1) * C + c;
  for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
    const int mm = i / TKx, kk = i - mm * TKx;
    const int k = k0 + kk, m = m0 + mm;
    float2 n = make_float2(0.f, 0.f), q = n;
    const int sl = (m < mact) ? (slab ? slab[m] : m) : -1;
    if (k < g.Ke && sl >= 0) {
      const float* src = Yt + (int64_t)sl * R * g.ldk;
      const float2 e = make_float2(src[rre * g.ldk + k], src[rim * g.ldk + k]);
      if (k < g.nh) {
        const float2 o = make_float2(src[rre * g.ldk + g.ldke + k], src[rim * g.ldk + g.ldke + k]);
        n = make_float2(e.x + o.x, e.y + o.y);
        q = make_float2(e.x - o.x, e.y - o.y);
      } else {
        n = e;
      }
    }
    tn[mm][kk] = n;
    ts[mm][kk] = q;
  }
  __syncthreads();
  float2* dst = Yn + (int64_t)bc * g.nlat * mmax;
  for (int i = threadIdx.x; i < TKx * TMx; i += 256) {
    const int kk = i / TMx, mm = i - kk * TMx;
    const int k = k0 + kk, m = m0 + mm;
    if (k >= g.Ke || m >= mmax) continue;
    dst[(int64_t)k * mmax + m] = tn[mm][kk];
    if (k < g.nh) dst[(int64_t)(g.nlat - 1 - k) * mmax + m] = ts[mm][kk];
  }
}

template <int TKx, int TMx>
static void inv_sym_launch(const float* Yt, float2* Yn, int B, int C, const LatGeom& g, int mmax,
                           int mact, const int* perm, hipStream_t s) {
  dim3 grid((unsigned)cdiv(g.Ke, TKx), (unsigned)cdiv(mmax, TMx), (unsigned)(B * C));
  hipLaunchKernelGGL((transpose_inv_sym_kernel<TKx, TMx>), grid, dim3(256), 0, s, Yt, Yn, B, C,
                     g, mmax, mact, perm);
}

static void inv_sym_dispatch(const float* Yt, float2* Yn, int B, int C, const LatGeom& g,
                             int mmax, int mact, const int* perm, hipStream_t s) {
  static const int t = tr_tile("MSFNO_TR_INV", 4);
  switch (t) {
    case 0: inv_sym_launch<64, 32>(Yt, Yn, B, C, g, mmax, mact, perm, s); break;
    case 1: inv_sym_launch<TK_INV, TM_INV>(Yt, Yn, B, C, g, mmax, mact, perm, s); break;
    case 2: inv_sym_launch<32, 128>(Yt, Yn, B, C, g, mmax, mact, perm, s); break;
    case 4: {
      const int nx = cdiv(g.Ke, 32), ny = cdiv(mmax, 128);
      const int xr = tr_xcd(1);
      const dim3 grid = tr_grid(xr, nx, ny, B * C);
      static const bool bf = [] {
        const char* e = getenv("MSFNO_TR_INV_BF");
        return !(e && e[0] == '0');
      }();
      if (xr == 2 && bf)
        hipLaunchKernelGGL((transpose_inv_sym2_kernel<32, 128, 2, true>), grid, dim3(256), 0, s,
                           Yt, Yn, B, C, g, mmax, mact, perm, nx, ny);
      else if (xr == 1)
        hipLaunchKernelGGL((transpose_inv_sym2_kernel<32, 128, 1, false>), grid, dim3(256), 0, s,
                           Yt, Yn, B, C, g, mmax, mact, perm, nx, ny);
      else if (xr == 2)
        hipLaunchKernelGGL((transpose_inv_sym2_kernel<32, 128, 2, false>), grid, dim3(256), 0, s,
                           Yt, Yn, B, C, g, mmax, mact, perm, nx, ny);
      else
        hipLaunchKernelGGL((transpose_inv_sym2_kernel<32, 128, 0, false>), grid, dim3(256), 0, s, Yt,
                           Yn, B, C, g, mmax, mact, perm, nx, ny);
      break;
    }
    default: inv_sym_launch<16, 128>(Yt, Yn, B, C, g, mmax, mact, perm, s);
  }
}

int launch_transpose_inv_sym(const float* Yt, float2* Yn, int B, int C, const LatGeom& g, int mmax,
                             int mact, hipStream_t s) {
  inv_sym_dispatch(Yt, Yn, B, C, g, mmax, mact, nullptr, s);
  return launch_check("transpose_inv_sym");
}

// Latitude-band unpack (band.cpp stage 3): the phase-1 receive buffer (slab perm[m],
// rows of ldk = 2W holding [E | O] or the local rows) -> this rank's spectra Yn
int launch_band_unpack(const float* recv, float2* Yn, int B, int C, const LatGeom& g, int mmax,
                       int mact, const int* perm, hipStream_t s) {
  if (!g.sym) return launch_transpose_inv(recv, Yn, B, C, g.nlat, mmax, mact, g.ldk, s, perm);
  inv_sym_dispatch(recv, Yn, B, C, g, mmax, mact, perm, s);
  return launch_check("band_unpack");
}

// ---------------------------------------------------------------------------
// statistics: combine (mean, M2) partials per channel, fp64 (Chan et al.)
// ---------------------------------------------------------------------------
struct Welford {
  double n, mean, m2;
};
__device__ __forceinline__ Welford wcombine(Welford a, Welford b) {
  if (b.n == 0) return a;
  if (a.n == 0) return b;
  const double n = a.n + b.n;
  const double d = b.mean - a.mean;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * (b.n / n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
  return r;
}

// the x3h skip GEMM's B-row scale of a channel with mean mu and sum of squared
// deviations m2: every element satisfies |x| <= |mu| + sqrt(m2), mapped below 2^14
__device__ __forceinline__ float x3_bound_scale(double mu, double m2) {
  const double bound = (fabs(mu) + sqrt(m2)) * (1.0 + 1e-3);
  if (!(bound > 0.0 && bound < 1e300)) return 1.f;
  int e;
  frexp(bound, &e);
  return (float)ldexp(1.0, min(max(14 - e, -100), 100));
}

// a bound of |sc x + sh| over a channel with mean mu and sum of squared deviations m2
// (|x - mu| <= sqrt(m2)), with 0.1 % headroom for the fp32 evaluation
__device__ __forceinline__ float affine_bound(double sc, double sh, double mu, double m2) {
  const double b = (fabs(sc) * sqrt(m2) + fabs(sc * mu + sh)) * (1.0 + 1e-3);
  return (float)fmin(b, 3.0e38);
}

// transpose_fwd_sym4h_kernel's sigma: |x^| <= |sc| sqrt(M2) + |sc mu + sh|, |X^_m| <= 2 pi
// max |x^|, folded x 2; mapped into [2^14, 2^15)
__device__ __forceinline__ float slab_sigma(double sc, double sh, double mu, double m2) {
  const double bound = 2.0 * 6.283185307179586 * (fabs(sc) * sqrt(m2) + fabs(sc * mu + sh)) *
                       (1.0 + 1e-3);
  float sig = 1.f;
  if (bound > 0.0 && bound < 1e300) {
    int e;
    frexp(bound, &e);
    sig = (float)ldexp(1.0, min(max(15 - e, -100), 100));
  }
  return sig;
}

__global__ __launch_bounds__(256) void chan_affine_kernel(
    const float2* __restrict__ part, int64_t np, int64_t cnt, int64_t cnt_last, int C,
    const float* __restrict__ w, const float* __restrict__ bsh, float eps,
    const float* __restrict__ gamma, const float* __restrict__ beta, float film_scale,
    float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ xscale,
    float* __restrict__ lsig, float* __restrict__ abound) {
  __shared__ double sn[256], smean[256], sm2[256];
  const int bc = blockIdx.x;
  const int c = bc % C;
  const float2* p = part + (int64_t)bc * np;
  Welford acc{0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < np; i += 256) {
    const float2 v = p[i];
    Welford x{(double)(i == np - 1 ? cnt_last : cnt), (double)v.x, (double)v.y};
    acc = wcombine(acc, x);
  }
  sn[threadIdx.x] = acc.n;
  smean[threadIdx.x] = acc.mean;
  sm2[threadIdx.x] = acc.m2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      Welford a{sn[threadIdx.x], smean[threadIdx.x], sm2[threadIdx.x]};
      Welford b{sn[threadIdx.x + o], smean[threadIdx.x + o], sm2[threadIdx.x + o]};
      a = wcombine(a, b);
      sn[threadIdx.x] = a.n;
      smean[threadIdx.x] = a.mean;
      sm2[threadIdx.x] = a.m2;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double var = sm2[0] / sn[0];  // biased, as InstanceNorm
    const double rstd = 1.0 / sqrt(var + (double)eps);
    const double mu = smean[0];
    double sc = (w ? (double)w[c] : 1.0) * rstd;
    double sh = (bsh ? (double)bsh[c] : 0.0) - sc * mu;
    if (gamma) {  // FiLM: (1 + γ·s)·x̂ + β·s   (sfnonet.py:694-697)
      const double g = 1.0 + (double)gamma[bc] * (double)film_scale;
      sc *= g;
      sh = sh * g + (double)beta[bc] * (double)film_scale;
    }
    scale[bc] = (float)sc;
    shift[bc] = (float)sh;
    if (xscale) xscale[bc] = x3_bound_scale(mu, sm2[0]);
    if (abound) abound[bc] = affine_bound(sc, sh, mu, sm2[0]);
    if (lsig) lsig[bc] = slab_sigma(sc, sh, mu, sm2[0]);
  }
}

int launch_chan_affine(const float2* partials, int64_t np, int64_t cnt, int64_t cnt_last, int B,
                       int C, const float* w, const float* b, float eps, const float* gamma,
                       const float* beta, float film_scale, float* scale, float* shift,
                       hipStream_t s, float* xscale, float* lsig, float* abound) {
  hipLaunchKernelGGL(chan_affine_kernel, dim3(B * C), dim3(256), 0, s, partials, np, cnt,
                     cnt_last, C, w, b, eps, gamma, beta, film_scale, scale, shift, xscale, lsig,
                     abound);
  return launch_check("chan_affine");
}

// ---------------------------------------------------------------------------
// latitude-band sharding: per-rank statistics partials and the
// band <-> full-latitude re-layout around the all-to-all exchanges
// ---------------------------------------------------------------------------
// rowstats (BC, np) (mean, M2) over cnt elements each -> out (BC, 3) fp64 {n, mean, M2}
__global__ __launch_bounds__(256) void stats_partial_kernel(const float2* __restrict__ part,
                                                            int64_t np, int64_t cnt,
                                                            double* __restrict__ out,
                                                            float* __restrict__ xscale) {
  __shared__ double sn[256], smean[256], sm2[256];
  const int bc = blockIdx.x;
  const float2* p = part + (int64_t)bc * np;
  Welford acc{0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < np; i += 256) {
    const float2 v = p[i];
    acc = wcombine(acc, Welford{(double)cnt, (double)v.x, (double)v.y});
  }
  sn[threadIdx.x] = acc.n;
  smean[threadIdx.x] = acc.mean;
  sm2[threadIdx.x] = acc.m2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      Welford a{sn[threadIdx.x], smean[threadIdx.x], sm2[threadIdx.x]};
      a = wcombine(a, Welford{sn[threadIdx.x + o], smean[threadIdx.x + o], sm2[threadIdx.x + o]});
      sn[threadIdx.x] = a.n;
      smean[threadIdx.x] = a.mean;
      sm2[threadIdx.x] = a.m2;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[3 * (int64_t)bc + 0] = sn[0];
    out[3 * (int64_t)bc + 1] = smean[0];
    out[3 * (int64_t)bc + 2] = sm2[0];
    if (xscale) xscale[bc] = x3_bound_scale(smean[0], sm2[0]);
  }
}

int launch_stats_partial(const float2* rowstats, int64_t np, int64_t cnt, int64_t BC, double* out,
                         hipStream_t s, float* xscale) {
  hipLaunchKernelGGL(stats_partial_kernel, dim3((unsigned)BC), dim3(256), 0, s, rowstats, np, cnt,
                     out, xscale);
  return launch_check("stats_partial");
}

// parts (nparts, BC, 3) -> InstanceNorm (+FiLM) affine, same math as chan_affine_kernel
__global__ void chan_affine_parts_kernel(const double* __restrict__ parts, int nparts, int BC,
                                         int C, const float* __restrict__ w,
                                         const float* __restrict__ bsh, float eps,
                                         const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float film_scale,
                                         float* __restrict__ scale, float* __restrict__ shift,
                                         float* __restrict__ xscale, float* __restrict__ abound,
                                         float* __restrict__ lsig) {
  const int bc = blockIdx.x * blockDim.x + threadIdx.x;
  if (bc >= BC) return;
  const int c = bc % C;
  Welford acc{0.0, 0.0, 0.0};
  for (int p = 0; p < nparts; ++p) {
    const double* q = parts + 3 * ((int64_t)p * BC + bc);
    acc = wcombine(acc, Welford{q[0], q[1], q[2]});
  }
  const double var = acc.m2 / acc.n;
  const double rstd = 1.0 / sqrt(var + (double)eps);
  double sc = (w ? (double)w[c] : 1.0) * rstd;
  double sh = (bsh ? (double)bsh[c] : 0.0) - sc * acc.mean;
  if (gamma) {
    const double g = 1.0 + (double)gamma[bc] * (double)film_scale;
    sc *= g;
    sh = sh * g + (double)beta[bc] * (double)film_scale;
  }
  scale[bc] = (float)sc;
  shift[bc] = (float)sh;
  if (xscale) xscale[bc] = x3_bound_scale(acc.mean, acc.m2);
  if (abound) abound[bc] = affine_bound(sc, sh, acc.mean, acc.m2);
  if (lsig) lsig[bc] = slab_sigma(sc, sh, acc.mean, acc.m2);
}

int launch_chan_affine_parts(const double* parts, int nparts, int B, int C, const float* w,
                             const float* b, float eps, const float* gamma, const float* beta,
                             float film_scale, float* scale, float* shift, hipStream_t s,
                             float* xscale, float* abound, float* lsig) {
  const int BC = B * C;
  hipLaunchKernelGGL(chan_affine_parts_kernel, dim3((unsigned)cdiv(BC, 256)), dim3(256), 0, s,
                     parts, nparts, BC, C, w, b, eps, gamma, beta, film_scale, scale, shift,
                     xscale, abound, lsig);
  return launch_check("chan_affine_parts");
}

// W'[b][o][i] = W[o][i]·scale[b][i];  b'[b][o] = bias[o] + Σ_i W[o][i]·shift[b][i]
__global__ __launch_bounds__(256) void fold_affine_kernel(const float* __restrict__ W,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          float* __restrict__ Wf,
                                                          float* __restrict__ bf, int O, int I) {
  __shared__ float red[256];
  const int o = blockIdx.x, b = blockIdx.y;
  const float* wr = W + (int64_t)o * I;
  float* wo = Wf + ((int64_t)b * O + o) * I;
  const float* sc = scale + (int64_t)b * I;
  const float* sh = shift + (int64_t)b * I;
  float acc = 0.f;
  for (int i = threadIdx.x; i < I; i += 256) {
    const float wv = wr[i];
    wo[i] = wv * sc[i];
    acc += wv * sh[i];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) bf[(int64_t)b * O + o] = (bias ? bias[o] : 0.f) + red[0];
}

int launch_fold_affine(const float* W, const float* bias, const float* scale, const float* shift,
                       float* Wf, float* bf, int B, int O, int I, hipStream_t s) {
  hipLaunchKernelGGL(fold_affine_kernel, dim3(O, B), dim3(256), 0, s, W, bias, scale, shift, Wf,
                     bf, O, I);
  return launch_check("fold_affine");
}

__device__ __forceinline__ float gelu_erf(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}

// one block-row of 1024 elements per workgroup; stats partial per (bc, tile)
__global__ __launch_bounds__(256) void affine_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ addend, float* __restrict__ out, int64_t P, int act,
    float2* __restrict__ stats, int stats_ld) {
  __shared__ float rs[256], rq[256];
  const int64_t bc = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * 1024;
  const float sc = scale ? scale[bc] : 1.f;
  const float sh = shift ? shift[bc] : 0.f;
  const float* xr = x + bc * P;
  const float* ar = addend ? addend + bc * P : nullptr;
  float* orow = out + bc * P;
  float s = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < 1024; i += 256) {
    const int64_t p = p0 + i;
    if (p < P) {
      float v = xr[p] * sc + sh;
      if (ar) v += ar[p];
      if (act == 1) v = gelu_erf(v);
      orow[p] = v;
      s += v;
      q += v * v;
    }
  }
  if (!stats) return;
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      rq[threadIdx.x] += rq[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float n = (float)min((int64_t)1024, P - p0);
    const float mean = rs[0] / n;
    stats[bc * stats_ld + blockIdx.x] = make_float2(mean, fmaxf(rq[0] - rs[0] * mean, 0.f));
  }
}

int launch_affine_rows(const float* x, const float* scale, const float* shift,
                       const float* addend, float* out, int64_t BC, int64_t P, int act,
                       float2* stats, int stats_ld, hipStream_t s) {
  dim3 grid((unsigned)cdiv(P, 1024), (unsigned)BC);
  hipLaunchKernelGGL(affine_rows_kernel, grid, dim3(256), 0, s, x, scale, shift, addend, out, P,
                     act, stats, stats_ld);
  return launch_check("affine_rows");
}

// ---------------------------------------------------------------------------
// weight preparation
// ---------------------------------------------------------------------------
__global__ void expand_complex_weight_kernel(const float* __restrict__ w, float* __restrict__ We,
                                             int Ci, int Co) {
  const int64_t n = 4LL * Ci * Co;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / (2 * Ci), col = e - row * (2 * Ci);
    const int ro = (int)(row / Co), o = (int)(row - (int64_t)ro * Co);
    const int ri = (int)(col / Ci), i = (int)(col - (int64_t)ri * Ci);
    const float wr = w[((int64_t)i * Co + o) * 2 + 0];
    const float wi = w[((int64_t)i * Co + o) * 2 + 1];
    float v;
    if (ro == 0) v = (ri == 0) ? wr : -wi;   // Re y = Σ xr·wr − xi·wi
    else v = (ri == 0) ? wi : wr;            // Im y = Σ xr·wi + xi·wr
    We[e] = v;
  }
}

int launch_expand_complex_weight(const float* w, float* Wexp, int Ci, int Co, hipStream_t s) {
  const int64_t n = 4LL * Ci * Co;
  hipLaunchKernelGGL(expand_complex_weight_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 4096)),
                     dim3(256), 0, s, w, Wexp, Ci, Co);
  return launch_check("expand_complex_weight");
}

// forward table:  Wf[m][k][j] = weights[m][m+j][k]   (ld Lp_m, zero pad j >= L_m)
// inverse table:  Pi[m][j][k] = pct[m][m+j][k]       (ld ldk,  zero pad k >= nlat)
// (mmax, lmax, nlat) reference table -> per-m plan GEMM blocks (common.h:
// set_table_offsets); columns / rows in the parity-split S order, pads zero.
__global__ void relayout_table_kernel(const float* __restrict__ tab, float* __restrict__ out,
                                      const int64_t* __restrict__ tab_off,
                                      const int* __restrict__ Lp, const int* __restrict__ Lpe,
                                      int lmax, LatGeom g, int inverse,
                                      const int* __restrict__ kmap, int Kb) {
  const int m = blockIdx.y;
  const int L = lmax - m;
  const int lp = Lp[m], lpe = Lpe[m], lpo = lp - lpe;
  if (L <= 0 || lp == 0) return;  // lp == 0: m outside a sharded plan's m-set
  float* o = out + tab_off[m];
  const float* t = tab + (int64_t)m * lmax * g.nlat;
  // value of row j (= l - m) at latitude k, 0 outside the triangle
  auto at = [&](int j, int k) -> float {
    return (j < L) ? t[(int64_t)(m + j) * g.nlat + k] : 0.f;
  };
  auto jcol = [&](int c) { return c < lpe ? 2 * c : 2 * (c - lpe) + 1; };
  if (kmap) {
    // band plan (common.h): the K (forward) / N (inverse) index is an exchange
    // column k' whose latitude is kmap[k'] (-1: pad)
    const int64_t n = (int64_t)Kb * lp;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
      int kb, j;
      if (g.sym) {
        const int64_t ne = (int64_t)Kb * lpe;
        const bool ev = e < ne;
        const int64_t f = ev ? e : e - ne;
        const int w = ev ? lpe : lpo;
        int c;
        if (inverse) { c = (int)(f / Kb); kb = (int)(f - (int64_t)c * Kb); }
        else { kb = (int)(f / w); c = (int)(f - (int64_t)kb * w); }
        j = ev ? 2 * c : 2 * c + 1;
      } else {
        int c;
        if (inverse) { c = (int)(e / Kb); kb = (int)(e - (int64_t)c * Kb); }
        else { kb = (int)(e / lp); c = (int)(e - (int64_t)kb * lp); }
        j = jcol(c);
      }
      const int k = kmap[kb];
      o[e] = k >= 0 ? at(j, k) : 0.f;
    }
    return;
  }
  const int ldko = (g.Ko + 3) & ~3;
  int64_t n;
  if (!g.sym) n = inverse ? (int64_t)lp * g.ldk : (int64_t)g.nlat * lp;
  else n = inverse ? (int64_t)lpe * g.ldke + (int64_t)lpo * ldko
                   : (int64_t)g.Ke * lpe + (int64_t)g.Ko * lpo;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (!g.sym) {
      if (inverse) {  // (lp x ldk)
        const int c = (int)(e / g.ldk), k = (int)(e - (int64_t)c * g.ldk);
        if (k < g.nlat) v = at(jcol(c), k);
      } else {        // (nlat x lp)
        const int k = (int)(e / lp), c = (int)(e - (int64_t)k * lp);
        v = at(jcol(c), k);
      }
    } else if (inverse) {
      const int64_t ne = (int64_t)lpe * g.ldke;
      if (e < ne) {   // Pe (lpe x ldke)
        const int c = (int)(e / g.ldke), k = (int)(e - (int64_t)c * g.ldke);
        if (k < g.Ke) v = at(2 * c, k);
      } else {        // Po (lpo x ldko)
        const int64_t f = e - ne;
        const int c = (int)(f / ldko), k = (int)(f - (int64_t)c * ldko);
        if (k < g.Ko) v = at(2 * c + 1, k);
      }
    } else {
      const int64_t ne = (int64_t)g.Ke * lpe;
      if (e < ne) {   // We (Ke x lpe)
        const int k = (int)(e / lpe), c = (int)(e - (int64_t)k * lpe);
        v = at(2 * c, k);
      } else {        // Wo (Ko x lpo)
        const int64_t f = e - ne;
        const int k = (int)(f / lpo), c = (int)(f - (int64_t)k * lpo);
        v = at(2 * c + 1, k);
      }
    }
    o[e] = v;
  }
}

int launch_relayout_table(const msfno_sht_plan_s& p, const float* table, hipStream_t s) {
  dim3 grid(256, (unsigned)p.mmax);
  hipLaunchKernelGGL(relayout_table_kernel, grid, dim3(256), 0, s, table, p.table, p.d_tab_off,
                     p.d_Lp, p.d_Lpe, p.lmax, p.geom(), p.inverse,
                     p.band_world ? p.d_kmap : nullptr, p.band_world ? p.band_K() : 0);
  return launch_check("relayout_table");
}

// flag |= 1 when some row (m, l) of the table breaks
// t[nlat-1-k] = (-1)^(l-m) t[k] beyond 1e-5 of the row's max magnitude
__global__ __launch_bounds__(256) void check_symmetry_kernel(const float* __restrict__ tab,
                                                             int lmax, int nlat,
                                                             int* __restrict__ flag) {
  __shared__ float red[256];
  const int m = blockIdx.y, l = blockIdx.x;
  const float* t = tab + ((int64_t)m * lmax + l) * nlat;
  float mx = 0.f;
  for (int k = threadIdx.x; k < nlat; k += 256) mx = fmaxf(mx, fabsf(t[k]));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  const float tol = 1e-5f * red[0];
  const float sgn = ((l - m) & 1) ? -1.f : 1.f;
  bool bad = false;
  for (int k = threadIdx.x; k < nlat / 2; k += 256)
    bad |= !(fabsf(t[nlat - 1 - k] - sgn * t[k]) <= tol);  // NaN-safe
  if (bad) atomicOr(flag, 1);
}

int launch_check_symmetry(const float* table, int mmax, int lmax, int nlat, int* d_flag,
                          hipStream_t s) {
  hipLaunchKernelGGL(check_symmetry_kernel, dim3((unsigned)lmax, (unsigned)mmax), dim3(256), 0, s,
                     table, lmax, nlat, d_flag);
  return launch_check("check_symmetry");
}

// ---------------------------------------------------------------------------
// S layout conversions
// ---------------------------------------------------------------------------
__device__ __forceinline__ int find_m(const int* off, int mact, int64_t t) {
  int lo = 0, hi = mact - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// column t of an S row -> (m, j = l - m); j < 0 for padding
__device__ __forceinline__ void spec_col_inv(const int* off, const int* Lpe, const int* Lp,
                                             int mact, int64_t t, int lmax, int& m, int& j) {
  m = find_m(off, mact, t);
  const int u = (int)(t - off[m]);
  const int lpe = Lpe[m];
  j = u < lpe ? 2 * u : 2 * (u - lpe) + 1;
  if (u >= Lp[m] || m + j >= lmax) j = -1;
}

// out (bc, lmax, mmax) complex dense (zeros where l < m)
__global__ void spec_to_ref_kernel(const float* __restrict__ S, float2* __restrict__ out, int B,
                                   int C, int lmax, int mmax, int mact, int64_t ldT,
                                   const int* __restrict__ off, const int* __restrict__ Lpe) {
  const int64_t n = (int64_t)B * C * lmax * mmax;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(e % mmax);
    const int l = (int)((e / mmax) % lmax);
    const int64_t bc = e / ((int64_t)mmax * lmax);
    const int b = (int)(bc / C), c = (int)(bc % C);
    float2 v = make_float2(0.f, 0.f);
    if (l >= m && m < mact) {
      const int64_t t = spec_col(off, Lpe, m, l);
      v.x = S[((int64_t)(b * 2 + 0) * C + c) * ldT + t];
      v.y = S[((int64_t)(b * 2 + 1) * C + c) * ldT + t];
    }
    out[e] = v;
  }
}

int launch_spec_to_ref(const msfno_sht_plan_s& p, const float* S, float2* out, int B, int C,
                       const int* d_off, hipStream_t s) {
  const int64_t n = (int64_t)B * C * p.lmax * p.mmax;
  hipLaunchKernelGGL(spec_to_ref_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 65535)),
                     dim3(256), 0, s, S, out, B, C, p.lmax, p.mmax, p.spec.mact, p.spec.ldT,
                     d_off, p.d_Lpe);
  return launch_check("spec_to_ref");
}

__global__ void ref_to_spec_kernel(const float2* __restrict__ in, float* __restrict__ S, int B,
                                   int C, int lmax, int mmax, int mact, int64_t Tp, int64_t ldT,
                                   const int* __restrict__ off, const int* __restrict__ Lpe,
                                   const int* __restrict__ Lp) {
  const int64_t n = (int64_t)B * C * Tp;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e % Tp;
    const int64_t bc = e / Tp;
    const int b = (int)(bc / C), c = (int)(bc % C);
    int m, j;
    spec_col_inv(off, Lpe, Lp, mact, t, lmax, m, j);
    float2 v = make_float2(0.f, 0.f);
    if (j >= 0) v = in[(bc * lmax + m + j) * mmax + m];
    S[((int64_t)(b * 2 + 0) * C + c) * ldT + t] = v.x;
    S[((int64_t)(b * 2 + 1) * C + c) * ldT + t] = v.y;
  }
}

int launch_ref_to_spec(const msfno_sht_plan_s& p, const float2* in, float* S, int B, int C,
                       const int* d_off, hipStream_t s) {
  const int64_t n = (int64_t)B * C * p.spec.Tp;
  hipLaunchKernelGGL(ref_to_spec_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 65535)),
                     dim3(256), 0, s, in, S, B, C, p.lmax, p.mmax, p.spec.mact, p.spec.Tp,
                     p.spec.ldT, d_off, p.d_Lpe, p.d_Lp);
  return launch_check("ref_to_spec");
}

// tril order (torch.tril_indices(lmax, mmax)): row l holds m = 0..min(l, mmax-1)
__device__ __forceinline__ int64_t tril_row_off(int l, int mmax) {
  if (l <= mmax) return (int64_t)l * (l + 1) / 2;
  return (int64_t)mmax * (mmax + 1) / 2 + (int64_t)(l - mmax) * mmax;
}

// S -> xt (B, C, T, 2);  one thread per (bc, t) of the S row (coalesced reads)
__global__ void spec_to_tril_kernel(const float* __restrict__ S, float* __restrict__ xt, int B,
                                    int C, int lmax, int mmax, int mact, int64_t Tp, int64_t T,
                                    int64_t ldT, const int* __restrict__ off,
                                    const int* __restrict__ Lpe, const int* __restrict__ Lp,
                                    const int* __restrict__ tmap) {
  const int64_t n = (int64_t)B * C * Tp;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e % Tp;
    const int64_t bc = e / Tp;
    const int b = (int)(bc / C), c = (int)(bc % C);
    int m, j;
    spec_col_inv(off, Lpe, Lp, mact, t, lmax, m, j);
    if (j < 0) continue;
    int64_t nn = tril_row_off(m + j, mmax) + m;
    if (tmap) nn = tmap[nn];  // m-set plan: position among this rank's modes
    const float re = S[((int64_t)(b * 2 + 0) * C + c) * ldT + t];
    const float im = S[((int64_t)(b * 2 + 1) * C + c) * ldT + t];
    reinterpret_cast<float2*>(xt)[bc * T + nn] = make_float2(re, im);
  }
}

__global__ void tril_to_spec_kernel(const float* __restrict__ yt, float* __restrict__ S, int B,
                                    int C, int lmax, int mmax, int mact, int64_t Tp, int64_t T,
                                    int64_t ldT, const int* __restrict__ off,
                                    const int* __restrict__ Lpe, const int* __restrict__ Lp,
                                    const int* __restrict__ tmap) {
  const int64_t n = (int64_t)B * C * Tp;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e % Tp;
    const int64_t bc = e / Tp;
    const int b = (int)(bc / C), c = (int)(bc % C);
    int m, j;
    spec_col_inv(off, Lpe, Lp, mact, t, lmax, m, j);
    float2 v = make_float2(0.f, 0.f);
    if (j >= 0) {
      int64_t nn = tril_row_off(m + j, mmax) + m;
      if (tmap) nn = tmap[nn];
      v = reinterpret_cast<const float2*>(yt)[bc * T + nn];
    }
    S[((int64_t)(b * 2 + 0) * C + c) * ldT + t] = v.x;
    S[((int64_t)(b * 2 + 1) * C + c) * ldT + t] = v.y;
  }
}

// the S columns no mode maps to, zeroed in every row of the output S
__global__ void zero_spec_pads_kernel(float* __restrict__ Y, const int* __restrict__ tpad,
                                      int npad, int rows, int64_t ldT) {
  const int64_t n = (int64_t)rows * npad;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x)
    Y[(e / npad) * ldT + tpad[e % npad]] = 0.f;
}

// Tiled form of the two re-layouts for full plans: the (l, m) triangle in tiles of
// 64 l x 16 m through LDS, so both sides move whole runs (S: per m the even and odd
// j = l - m of the tile, 32 contiguous floats each in the Re and in the Im row; tril:
// per l the tile's 16 m, 128 contiguous bytes).  The scattered 8-B writes of the
// per-element kernels above cost 0.38 / 0.17 ms at config 2 for 0.27 GB.
constexpr int TT_L = 64, TT_M = 16;

template <bool TO_TRIL>
__global__ __launch_bounds__(256) void spec_tril_tiled_kernel(
    const float* __restrict__ S, float* __restrict__ Sout, const float2* __restrict__ tin,
    float2* __restrict__ tout, int C, int lmax, int mmax, int64_t T, int64_t ldT,
    const int* __restrict__ off, const int* __restrict__ Lpe) {
  __shared__ float2 tile[TT_L][TT_M + 1];
  const int l0 = blockIdx.x * TT_L, m0 = blockIdx.y * TT_M;
  const int64_t bc = blockIdx.z;
  const int b = (int)(bc / C), c = (int)(bc - (int64_t)b * C);
  if (m0 > l0 + TT_L - 1 || m0 >= mmax || l0 >= lmax) return;
  const int tid = threadIdx.x;
  const int64_t rre = ((int64_t)(b * 2 + 0) * C + c) * ldT;
  const int64_t rim = ((int64_t)(b * 2 + 1) * C + c) * ldT;
  // S side: thread (ml = tid >> 4, q = tid & 15): m = m0 + ml; for each parity the
  // j = l - m of the tile's l range are a run of 32 (u = j >> 1 consecutive)
  auto s_side = [&](auto store_c) {
    constexpr bool STORE = decltype(store_c)::value;
    const int ml = tid >> 4, q = tid & 15;
    const int m = m0 + ml;
    if (m >= mmax || m >= lmax) return;
    const int lpe = Lpe[m];
    const int64_t base = off[m];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      // first j >= l0 - m of this parity (j >= 0)
      int j0 = max(l0 - m, 0);
      if ((j0 & 1) != par) ++j0;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j = j0 + 2 * (q + 16 * k);
        const int l = m + j;
        if (l >= l0 + TT_L || l >= lmax) continue;
        const int64_t t = base + (par ? lpe : 0) + (j >> 1);
        if constexpr (STORE) {
          const float2 v = tile[l - l0][ml];
          Sout[rre + t] = v.x;
          Sout[rim + t] = v.y;
        } else {
          tile[l - l0][ml] = make_float2(S[rre + t], S[rim + t]);
        }
      }
    }
  };
  // tril side: thread (ll = tid >> 2, mq = tid & 3): l = l0 + ll, m = m0 + 4 mq .. + 3
  auto t_side = [&](auto store_c) {
    constexpr bool STORE = decltype(store_c)::value;
    const int ll = tid >> 2, mq = tid & 3;
    const int l = l0 + ll;
    if (l >= lmax) return;
    const int64_t row = (l <= mmax) ? (int64_t)l * (l + 1) / 2
                                    : (int64_t)mmax * (mmax + 1) / 2 + (int64_t)(l - mmax) * mmax;
    const int mend = min(l + 1, mmax);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + 4 * mq + e;
      if (m >= mend) continue;
      if constexpr (STORE)
        tout[bc * T + row + m] = tile[ll][4 * mq + e];
      else
        tile[ll][4 * mq + e] = tin[bc * T + row + m];
    }
  };
  using F = std::false_type;
  using Tt = std::true_type;
  if constexpr (TO_TRIL) {
    s_side(F{});
    __syncthreads();
    t_side(Tt{});
  } else {
    t_side(F{});
    __syncthreads();
    s_side(Tt{});
  }
}

static bool tril_tiled(const msfno_sht_plan_s& p) { return p.d_tcol != nullptr; }

static dim3 tril_grid(const SpecLayout& L, int B, int C) {
  return dim3((unsigned)cdiv(L.lmax, TT_L), (unsigned)cdiv(std::min(L.mmax, L.lmax), TT_M),
              (unsigned)(B * C));
}

int launch_spec_to_tril(const msfno_sht_plan_s& p, const float* S, float* xt, int B, int C,
                        hipStream_t s) {
  const SpecLayout& L = p.spec;
  if (tril_tiled(p)) {  // full plans (the m-set plans of the band path map through tmap)
    hipLaunchKernelGGL((spec_tril_tiled_kernel<true>), tril_grid(L, B, C), dim3(256), 0, s, S,
                       nullptr, nullptr, reinterpret_cast<float2*>(xt), C, L.lmax, L.mmax, L.T,
                       L.ldT, p.d_off, p.d_Lpe);
    return launch_check("spec_to_tril_tiled");
  }
  const int64_t n = (int64_t)B * C * L.Tp;
  hipLaunchKernelGGL(spec_to_tril_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 65535)),
                     dim3(256), 0, s, S, xt, B, C, L.lmax, L.mmax, L.mact, L.Tp, L.T, L.ldT,
                     p.d_off, p.d_Lpe, p.d_Lp, p.d_tril_local);
  return launch_check("spec_to_tril");
}

int launch_tril_to_spec(const msfno_sht_plan_s& p, const float* yt, float* S, int B, int C,
                        hipStream_t s) {
  const SpecLayout& L = p.spec;
  if (tril_tiled(p)) {
    hipLaunchKernelGGL((spec_tril_tiled_kernel<false>), tril_grid(L, B, C), dim3(256), 0, s,
                       nullptr, S, reinterpret_cast<const float2*>(yt), nullptr, C, L.lmax,
                       L.mmax, L.T, L.ldT, p.d_off, p.d_Lpe);
    MSFNO_TRY(launch_check("tril_to_spec_tiled"));
    if (p.npad > 0) {  // the pad columns of every row, zero (as tril_to_spec_kernel wrote)
      const int64_t n = 2LL * B * C * p.npad;
      hipLaunchKernelGGL(zero_spec_pads_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 4096)),
                         dim3(256), 0, s, S, p.d_tpad, p.npad, 2 * B * C, L.ldT);
      MSFNO_TRY(launch_check("zero_spec_pads"));
    }
    return MSFNO_OK;
  }
  const int64_t n = (int64_t)B * C * L.Tp;
  hipLaunchKernelGGL(tril_to_spec_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 65535)),
                     dim3(256), 0, s, yt, S, B, C, L.lmax, L.mmax, L.mact, L.Tp, L.T, L.ldT,
                     p.d_off, p.d_Lpe, p.d_Lp, p.d_tril_local);
  return launch_check("tril_to_spec");
}

// ---------------------------------------------------------------------------
// linear filter: y[b,k,n] = Σ_i a[b,i,n]·w[k,i,n]   (complex, per mode n)
// HBM-bound on w (C·C·T complex).  Each thread owns MPT consecutive modes and
// KC output channels for NB batch entries; every weight element is read once
// (16-B loads, 1 KiB per wave instruction), activations re-read Co/KC times
// from L2.
// ---------------------------------------------------------------------------
template <int NB, int KC, int MPT>
__global__ __launch_bounds__(256) void compl_contract_kernel(const float* __restrict__ a,
                                                             const float* __restrict__ w,
                                                             float* __restrict__ y, int B, int Ci,
                                                             int Co, int64_t T, int nkc) {
  const int nmt = (int)gridDim.x / nkc;  // mode tiles
  // consecutive block ids -> same mode tile (shared activations stay in L2)
  const int kc = blockIdx.x % nkc;
  const int mt = blockIdx.x / nkc;
  (void)nmt;
  const int64_t n0 = ((int64_t)mt * 256 + threadIdx.x) * MPT;
  const int b0 = blockIdx.y * NB;
  const int k0 = kc * KC;
  if (n0 >= T) return;
  const bool full = (n0 + MPT <= T);
  float2 acc[NB][KC][MPT];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int q = 0; q < MPT; ++q) acc[b][k][q] = make_float2(0.f, 0.f);
  const float2* a2 = reinterpret_cast<const float2*>(a);
  const float2* w2 = reinterpret_cast<const float2*>(w);
  for (int i = 0; i < Ci; ++i) {
    float2 xv[NB][MPT];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int bb = b0 + b;
      const float2* src = a2 + ((int64_t)(bb < B ? bb : 0) * Ci + i) * T + n0;
      if (MPT == 2 && full) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        xv[b][0] = make_float2(v.x, v.y);
        xv[b][MPT - 1] = make_float2(v.z, v.w);
      } else {
#pragma unroll
        for (int q = 0; q < MPT; ++q) xv[b][q] = (n0 + q < T) ? src[q] : make_float2(0.f, 0.f);
      }
    }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int kk = k0 + k < Co ? k0 + k : 0;
      const float2* ws = w2 + ((int64_t)kk * Ci + i) * T + n0;
      float2 wv[MPT];
      if (MPT == 2 && full) {
        const float4 v = *reinterpret_cast<const float4*>(ws);
        wv[0] = make_float2(v.x, v.y);
        wv[MPT - 1] = make_float2(v.z, v.w);
      } else {
#pragma unroll
        for (int q = 0; q < MPT; ++q) wv[q] = (n0 + q < T) ? ws[q] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < MPT; ++q) {
          acc[b][k][q].x += xv[b][q].x * wv[q].x - xv[b][q].y * wv[q].y;
          acc[b][k][q].y += xv[b][q].x * wv[q].y + xv[b][q].y * wv[q].x;
        }
    }
  }
  float2* y2 = reinterpret_cast<float2*>(y);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int bb = b0 + b;
    if (bb >= B) continue;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      if (k0 + k >= Co) continue;
      float2* dst = y2 + ((int64_t)bb * Co + k0 + k) * T + n0;
      if (MPT == 2 && full) {
        *reinterpret_cast<float4*>(dst) =
            make_float4(acc[b][k][0].x, acc[b][k][0].y, acc[b][k][MPT - 1].x, acc[b][k][MPT - 1].y);
      } else {
#pragma unroll
        for (int q = 0; q < MPT; ++q)
          if (n0 + q < T) dst[q] = acc[b][k][q];
      }
    }
  }
}

template <int NB, int KC, int MPT>
static int launch_contract_t(const float* a, const float* w, float* y, int B, int Ci, int Co,
                             int64_t T, hipStream_t s) {
  const int nkc = (int)cdiv(Co, KC);
  const int64_t nmt = cdiv(T, 256 * MPT);
  MSFNO_REQUIRE(nmt * nkc < (1LL << 31), MSFNO_EINVAL, "contract grid too large");
  dim3 grid((unsigned)(nmt * nkc), (unsigned)cdiv(B, NB));
  hipLaunchKernelGGL((compl_contract_kernel<NB, KC, MPT>), grid, dim3(256), 0, s, a, w, y, B, Ci,
                     Co, T, nkc);
  return launch_check("compl_contract");
}

// Batch 1 (the weight is read exactly once): the weight stream goes HBM -> LDS by
// LDS-DMA (dma.h), NS - 1 channel steps ahead (MSFNO_CONTRACT_NS, default 2; 2 % faster
// than the register-load kernel below, which batches > 1 use).  A workgroup owns 256 modes (one per
// thread) and 16 output channels; a stage holds, for one input channel i, the 16
// weight rows w[k0 + s, i, n0 .. n0 + 255] and the activation row a[i, n0 ..] (17
// segments of 2 KB, 34 DMA pieces of 1 KB).
constexpr int CDMA_KC = 16, CDMA_NT = 256, CDMA_SEG = CDMA_KC + 1, CDMA_PIECES = 2 * CDMA_SEG;

template <int NS>
__global__ __launch_bounds__(256) void compl_contract_dma_kernel(const float* __restrict__ a,
                                                                 const float* __restrict__ w,
                                                                 float* __restrict__ y, int Ci,
                                                                 int Co, int64_t T, int nkc) {
  constexpr int STAGE = CDMA_SEG * CDMA_NT * 8;  // bytes
  __shared__ __attribute__((aligned(16))) char lds[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kc = blockIdx.x % nkc, mt = blockIdx.x / nkc;
  const int k0 = kc * CDMA_KC;
  const int64_t n0 = (int64_t)mt * CDMA_NT;
  const int64_t rowb = T * 8;  // bytes per (k, i) weight row / per activation row
  // this wave's pieces p = wave + 4 q (p < 34): segment p / 2 (16 = activation), half p % 2
  constexpr int QMAX = (CDMA_PIECES + 3) / 4;
  const int nq = (CDMA_PIECES - wave + 3) / 4;
  const char* src[QMAX];
  int64_t istep[QMAX];
  uint32_t dst[QMAX];
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int pc = min(wave + 4 * q, CDMA_PIECES - 1);
    const int seg = pc >> 1, half = pc & 1;
    const int64_t off = min(n0 * 8 + half * 1024 + lane * 16, rowb - 16);
    const int k = min(k0 + seg, Co - 1);
    src[q] = seg < CDMA_KC ? reinterpret_cast<const char*>(w) + (int64_t)k * Ci * rowb + off
                           : reinterpret_cast<const char*>(a) + off;
    istep[q] = rowb;  // next input channel: next row of the same (k) block / of a
    dst[q] = (uint32_t)(seg * CDMA_NT * 8 + half * 1024);
  }
  const uint32_t lds0 = lds_addr(lds);
  auto issue = [&](int i, int slot) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q)
      if (q < nq) glds16(src[q] + i * istep[q], lds0 + (uint32_t)(slot * STAGE) + dst[q]);
  };
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < Ci) issue(j, j);
  float2 acc[CDMA_KC];
#pragma unroll
  for (int k = 0; k < CDMA_KC; ++k) acc[k] = make_float2(0.f, 0.f);
  for (int i = 0; i < Ci; ++i) {
    // stage i landed (stages i + 1 .. i + NS - 2 may stay in flight)
    const int ahead = min(NS - 2, Ci - 1 - i);
    wait_vmcnt(ahead * nq);
    // raw barrier (a __syncthreads fence could drain the DMA still in flight): every
    // wave's pieces landed, and every wave's reads of slot (i - 1) % NS have returned
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (i + NS - 1 < Ci) issue(i + NS - 1, (i + NS - 1) % NS);
    const float2* st = reinterpret_cast<const float2*>(lds + (i % NS) * STAGE);
    const float2 av = st[CDMA_KC * CDMA_NT + tid];
#pragma unroll
    for (int k = 0; k < CDMA_KC; ++k) {
      const float2 wv = st[k * CDMA_NT + tid];
      acc[k].x = fmaf(av.x, wv.x, fmaf(-av.y, wv.y, acc[k].x));
      acc[k].y = fmaf(av.x, wv.y, fmaf(av.y, wv.x, acc[k].y));
    }
  }
  const int64_t n = n0 + tid;
  if (n < T) {
    float2* y2 = reinterpret_cast<float2*>(y);
#pragma unroll
    for (int k = 0; k < CDMA_KC; ++k)
      if (k0 + k < Co) y2[(int64_t)(k0 + k) * T + n] = acc[k];
  }
}

// MSFNO_CONTRACT_DMA=0 keeps the register-load kernel at batch 1 (A/B)
static bool contract_dma() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_CONTRACT_DMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

int launch_compl_contract(const float* a, const float* w, float* y, int B, int Ci, int Co,
                          int64_t T, hipStream_t s) {
  if (B == 1 && contract_dma() && T % 2 == 0 && T >= 8 && Ci > 0 &&
      ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(w)) & 15) == 0) {
    const int nkc = (int)cdiv(Co, CDMA_KC);
    const int64_t nmt = cdiv(T, CDMA_NT);
    MSFNO_REQUIRE(nmt * nkc < (1LL << 31), MSFNO_EINVAL, "contract grid too large");
    static const int ns = [] {
      const char* e = getenv("MSFNO_CONTRACT_NS");
      return e ? atoi(e) : 2;  // two 68-KB workgroups per CU: 5.88 ms vs 6.16 (3) / 6.19 (4)
    }();
    if (ns == 2)
      hipLaunchKernelGGL(compl_contract_dma_kernel<2>, dim3((unsigned)(nmt * nkc)), dim3(256), 0,
                         s, a, w, y, Ci, Co, T, nkc);
    else if (ns == 4)
      hipLaunchKernelGGL(compl_contract_dma_kernel<4>, dim3((unsigned)(nmt * nkc)), dim3(256), 0,
                         s, a, w, y, Ci, Co, T, nkc);
    else
      hipLaunchKernelGGL(compl_contract_dma_kernel<3>, dim3((unsigned)(nmt * nkc)), dim3(256), 0,
                         s, a, w, y, Ci, Co, T, nkc);
    return launch_check("compl_contract_dma");
  }
  const bool even = (T % 2 == 0) && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(w) |
                                      reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  if (B >= 8) {
    return even ? launch_contract_t<8, 4, 2>(a, w, y, B, Ci, Co, T, s)
                : launch_contract_t<8, 4, 1>(a, w, y, B, Ci, Co, T, s);
  }
  if (B >= 4) {
    return even ? launch_contract_t<4, 8, 2>(a, w, y, B, Ci, Co, T, s)
                : launch_contract_t<4, 8, 1>(a, w, y, B, Ci, Co, T, s);
  }
  if (B == 2 || B == 3) {
    return even ? launch_contract_t<2, 8, 2>(a, w, y, B, Ci, Co, T, s)
                : launch_contract_t<2, 8, 1>(a, w, y, B, Ci, Co, T, s);
  }
  return even ? launch_contract_t<1, 16, 2>(a, w, y, B, Ci, Co, T, s)
              : launch_contract_t<1, 16, 1>(a, w, y, B, Ci, Co, T, s);
}

// compl_mul2d_fwd_c in reference layout (standalone op, not on the fused path):
// y[b,o,p] = Σ_i a[b,i,p]·w[i,o]; one thread per (b, p), 8 outputs per pass.
__global__ __launch_bounds__(256) void compl_mul2d_kernel(const float2* __restrict__ a,
                                                          const float2* __restrict__ w,
                                                          float2* __restrict__ y, int B, int Ci,
                                                          int Co, int64_t XY, int relu) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= XY) return;
  const float2* ab = a + (int64_t)b * Ci * XY + p;
  for (int o0 = 0; o0 < Co; o0 += 8) {
    float2 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = make_float2(0.f, 0.f);
    for (int i = 0; i < Ci; ++i) {
      const float2 x = ab[(int64_t)i * XY];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (o0 + q < Co) {
          const float2 wv = w[(int64_t)i * Co + o0 + q];
          acc[q].x += x.x * wv.x - x.y * wv.y;
          acc[q].y += x.x * wv.y + x.y * wv.x;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (o0 + q < Co) {
        float2 v = acc[q];
        if (relu) v.x = fmaxf(v.x, 0.f);
        y[((int64_t)b * Co + o0 + q) * XY + p] = v;
      }
    }
  }
}

int launch_compl_mul2d(const float* a, const float* w, float* y, int B, int Ci, int Co,
                       int64_t XY, int relu_real, hipStream_t s) {
  dim3 grid((unsigned)cdiv(XY, 256), (unsigned)B);
  hipLaunchKernelGGL(compl_mul2d_kernel, grid, dim3(256), 0, s,
                     reinterpret_cast<const float2*>(a), reinterpret_cast<const float2*>(w),
                     reinterpret_cast<float2*>(y), B, Ci, Co, XY, relu_real);
  return launch_check("compl_mul2d");
}

}  // namespace msfno
