// Longitudinal real FFTs of the SHT (torch_harmonics RealSHT/InverseRealSHT:
// 2π·rfft(x, norm="forward") and irfft(n=nlon, norm="forward")).
//
// One wavefront per latitude row, 4 rows per 256-thread workgroup.  A real row
// of even length N is packed as H = N/2 complex points, transformed with a
// mixed-radix (4,2,3,5,7,11,13) Stockham FFT in LDS (ping-pong buffers, natural
// order, twiddles from an fp64-built table), then unpacked into the bins
// 0..mmax-1 that the Legendre stage consumes (only 361 of 721 for 1440).  Odd N
// falls back to a full complex transform.  The forward kernel also emits the
// per-row (mean, M2) used for InstanceNorm statistics, so norm0 costs no extra
// pass over HBM; the inverse kernel can apply GELU and emit output-row stats.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "bf16x3.h"
#include "dma.h"
#include "kernels.h"

namespace msfno {

struct FFTArgs {
  int N, H, packed, nrad, inplace, codelet;
  int radices[kMaxRadices];
  const float2* twH;
  const float2* twN;
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
  return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

// e^{∓2πi t/R} for the internal twiddles of the nested radix-16 / radix-9 butterflies
template <int R, bool INV>
__device__ __forceinline__ float2 root(int t) {
  float c = 1.f, sn = 0.f;
  if constexpr (R == 16) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f;
    constexpr float R2 = 0.70710678118654752440f;
    switch (t) {
      case 1: c = C1; sn = S1; break;
      case 2: c = R2; sn = R2; break;
      case 3: c = S1; sn = C1; break;
      case 4: c = 0.f; sn = 1.f; break;
      case 6: c = -R2; sn = R2; break;
      case 9: c = -C1; sn = -S1; break;
      default: break;
    }
  } else {  // R == 9
    switch (t) {
      case 1: c = 0.76604444311897803520f; sn = 0.64278760968653932632f; break;
      case 2: c = 0.17364817766693034885f; sn = 0.98480775301220805936f; break;
      case 4: c = -0.93969262078590838405f; sn = 0.34202014332566873304f; break;
      default: break;
    }
  }
  return make_float2(c, INV ? sn : -sn);
}

template <int R, bool INV>
__device__ __forceinline__ void butterfly(float2 (&v)[R], const float2* twH, int H);

template <int R, bool INV>
__device__ __forceinline__ void butterfly(float2 (&v)[R], const float2* twH, int H) {
  if constexpr (R == 2) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const float2 a2 = cadd(v[1], v[3]), a3 = csub(v[1], v[3]);
    v[0] = cadd(a0, a2);
    v[2] = csub(a0, a2);
    const float2 t = mul_mi<INV>(a3);
    v[1] = cadd(a1, t);
    v[3] = csub(a1, t);
  } else if constexpr (R == 3) {
    const float h = 0.86602540378443864676f;
    const float2 s = cadd(v[1], v[2]);
    const float2 d = csub(v[1], v[2]);
    const float2 t1 = make_float2(v[0].x - 0.5f * s.x, v[0].y - 0.5f * s.y);
    const float2 t2 = mul_mi<INV>(make_float2(h * d.x, h * d.y));  // ∓i·(√3/2)(v1-v2)
    v[0] = cadd(v[0], s);
    v[1] = cadd(t1, t2);
    v[2] = csub(t1, t2);
  } else if constexpr (R == 5) {
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const float2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
    const float2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
    const float2 a1 = make_float2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
    const float2 a2 = make_float2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
    const float2 b1 = mul_mi<INV>(make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y));
    const float2 b2 = mul_mi<INV>(make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y));
    v[0] = cadd(v[0], cadd(t1, t2));
    v[1] = cadd(a1, b1);
    v[4] = csub(a1, b1);
    v[2] = cadd(a2, b2);
    v[3] = csub(a2, b2);
  } else if constexpr (R == 16 || R == 9) {
    // R = P·P: inner P-point DFTs over a (stride P), internal twiddles W_R^{b·k1},
    // outer P-point DFTs over b.  Output index k1 + P·k2.
    constexpr int P = R == 16 ? 4 : 3;
    float2 y[P][P];  // y[b][k1]
#pragma unroll
    for (int b = 0; b < P; ++b) {
      float2 t[P];
#pragma unroll
      for (int a = 0; a < P; ++a) t[a] = v[P * a + b];
      butterfly<P, INV>(t, twH, H);
#pragma unroll
      for (int k1 = 0; k1 < P; ++k1) y[b][k1] = (b * k1 == 0) ? t[k1] : cmul(t[k1], root<R, INV>(b * k1));
    }
#pragma unroll
    for (int k1 = 0; k1 < P; ++k1) {
      float2 t[P];
#pragma unroll
      for (int b = 0; b < P; ++b) t[b] = y[b][k1];
      butterfly<P, INV>(t, twH, H);
#pragma unroll
      for (int k2 = 0; k2 < P; ++k2) v[k1 + P * k2] = t[k2];
    }
  } else {
    // generic small prime: y_q = Σ_r v_r·w_q^r by Horner's rule (one root per output)
    float2 y[R];
    const int st = H / R;
    y[0] = v[0];
#pragma unroll
    for (int r = 1; r < R; ++r) y[0] = cadd(y[0], v[r]);
#pragma unroll
    for (int q = 1; q < R; ++q) {
      float2 w = twH[q * st];
      if (INV) w.y = -w.y;
      float2 acc = v[R - 1];
#pragma unroll
      for (int r = R - 2; r >= 0; --r) acc = cadd(cmul(acc, w), v[r]);
      y[q] = acc;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = y[q];
  }
}

// v[r] *= w^r with w = tw[idx]: the powers are built from one table read (two
// for R = P·P: w and w^P), at most three complex products per factor.
template <int R, bool INV>
__device__ __forceinline__ void apply_twiddles(float2 (&v)[R], const float2* tw, int idx) {
  float2 w1 = tw[idx];
  if (INV) w1.y = -w1.y;
  if constexpr (R == 16 || R == 9) {
    constexpr int P = R == 16 ? 4 : 3;
    float2 wp = tw[P * idx];
    if (INV) wp.y = -wp.y;
    float2 pb[P], pa[P];  // w^b, (w^P)^a
    pb[0] = make_float2(1.f, 0.f);
    pa[0] = make_float2(1.f, 0.f);
    pb[1] = w1;
    pa[1] = wp;
#pragma unroll
    for (int e = 2; e < P; ++e) {
      pb[e] = cmul(pb[e - 1], w1);
      pa[e] = cmul(pa[e - 1], wp);
    }
#pragma unroll
    for (int a = 0; a < P; ++a)
#pragma unroll
      for (int b = 0; b < P; ++b) {
        if (a == 0 && b == 0) continue;
        const float2 wr = a == 0 ? pb[b] : (b == 0 ? pa[a] : cmul(pa[a], pb[b]));
        v[P * a + b] = cmul(v[P * a + b], wr);
      }
  } else {
    float2 wr = w1;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      if (r > 1) wr = (r == 2) ? cmul(w1, w1) : cmul(wr, w1);
      v[r] = cmul(v[r], wr);
    }
  }
}

// One Stockham pass, in place in the wave's LDS row buffer: every lane first
// reads all inputs of its butterflies into registers, then (after the reads
// have returned — they feed the arithmetic) writes the outputs.  LDS accesses
// of one wavefront are performed in order, so no barrier is needed: each row
// belongs to exactly one wave.
// ST (first pass of the forward transform only): the (mean, M2) of the row's 2 H real
// values from the inputs the lane has just read, before the butterflies overwrite them:
// each lane's own two-pass mean / M2 over its registers, combined over the wave with
// Chan's formula M2 = sum_l (M2_l + n_l (mean_l - mean)^2); no LDS pass of its own.
// LD (first pass only): the pass's inputs come from ld(k) instead of buf[k] (the
// inverse transform's Hermitian pre-twiddle computed straight from the spectrum row, so
// the row is not written to buf and read back)
struct NoLoader {};
// SO (last pass only): the pass's outputs go to so(it, r, k, value) instead of buf[k] (the
// inverse transform's output row stored from registers)
// SWI / SWO: the pass reads / writes buf through fft_swz (pass 2 -> pass 3 of the
// 4 x 4 x ... codelets, FixedFFT::SWZ)
__device__ __forceinline__ int fft_swz(int a) { return a ^ (((a >> 5) & 3) << 2); }
template <int R, int IT, bool INV, bool ST = false, class LD = NoLoader, class SO = NoLoader,
          bool SWI = false, bool SWO = false>
__device__ __forceinline__ void stockham_pass_inplace(float2* buf, int H, int Ns,
                                                      const float2* tw, int lane,
                                                      float2* stats = nullptr,
                                                      const LD& ld = LD{}, const SO& so = SO{}) {
  const int nb = H / R;
  const int step = H / (Ns * R);
  float2 v[IT][R];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (!std::is_same<LD, NoLoader>::value)
          v[it][r] = ld(j + r * nb);
        else if constexpr (SWI)
          v[it][r] = buf[fft_swz(j + r * nb)];
        else
          v[it][r] = buf[j + r * nb];
      }
    }
  }
  if constexpr (ST) {
    float s = 0.f;
    int cnt = 0;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      if (lane + 64 * it < nb) {
#pragma unroll
        for (int r = 0; r < R; ++r) s += v[it][r].x + v[it][r].y;
        cnt += 2 * R;
      }
    }
    const float ml = cnt ? s / (float)cnt : 0.f;
    float q = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      if (lane + 64 * it < nb) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          q += (v[it][r].x - ml) * (v[it][r].x - ml) + (v[it][r].y - ml) * (v[it][r].y - ml);
      }
    }
    float tot = s;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) tot += __shfl_xor(tot, o);
    const float mean = tot / (float)(2 * H);
    const float d = ml - mean;
    float m2 = q + (float)cnt * d * d;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m2 += __shfl_xor(m2, o);
    *stats = make_float2(mean, m2);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
      const int k = j % Ns;
      if (Ns > 1) apply_twiddles<R, INV>(v[it], tw, k * step);
      butterfly<R, INV>(v[it], tw, H);
    }
  }
  if constexpr (!std::is_same<SO, NoLoader>::value) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int j = lane + 64 * it;
      if (j < nb) {
        const int base = (j / Ns) * Ns * R + j % Ns;
#pragma unroll
        for (int r = 0; r < R; ++r) so(it, r, base + r * Ns, v[it][r]);
      }
    }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
      const int k = j % Ns;
      const int base = (j / Ns) * Ns * R + k;
      if ((R % 2) == 0 && Ns == 1) {
        // first pass: a lane's R outputs are contiguous; 16-B stores halve the
        // bank conflicts of R strided 8-B stores
#pragma unroll
        for (int r = 0; r < R; r += 2)
          *reinterpret_cast<float4*>(buf + base + r) =
              make_float4(v[it][r].x, v[it][r].y, v[it][r + 1].x, v[it][r + 1].y);
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) buf[SWO ? fft_swz(base + r * Ns) : base + r * Ns] = v[it][r];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ constexpr int pass_iters(int H, int R) { return (H / R + 63) / 64; }

// Out-of-place pass (ping-pong), one butterfly at a time: the generic fallback
// for sizes without a compiled codelet.
template <int R, bool INV>
__device__ __forceinline__ void stockham_pass_pp(const float2* in, float2* out, int H, int Ns,
                                                 const float2* tw, int lane) {
  const int nb = H / R;
  const int step = H / (Ns * R);
  for (int j = lane; j < nb; j += 64) {
    const int k = j % Ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = in[j + r * nb];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float2 w = tw[r * k * step];
        if (INV) w.y = -w.y;
        v[r] = cmul(v[r], w);
      }
    }
    butterfly<R, INV>(v, tw, H);
    const int base = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) out[base + r * Ns] = v[r];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// Compile-time codelet: the radix sequence is a template parameter, so every
// pass has constant size, stride and butterfly count (in-place, no ping-pong).
template <int... Rs>
struct FixedFFT {
  static constexpr int H = (Rs * ...);
  static constexpr int kBufs = 1;
  static constexpr int NPASS = sizeof...(Rs);
  static constexpr int RADS[NPASS] = {Rs...};
  static constexpr int RL = RADS[NPASS - 1];            // last radix
  static constexpr int ITL = pass_iters(H, RL);         // its butterflies per lane
  // pass 2 of a 4 x 4 x ... codelet writes at base + 4 r (base = 16 (j >> 2) + (j & 3)):
  // for one r, the 8 lane quads of a half-wave fall on 2 bank groups (4-way conflicts);
  // through fft_swz (bits 2-3 of the index XORed with bits 5-6, a permutation of every
  // 16-aligned block, so H % 16 == 0) the 8 quads fall on 8 distinct groups.  Pass 3
  // reads through the same map; every other pass is untouched.
  static constexpr bool SWZ = NPASS >= 3 && RADS[0] == 4 && RADS[1] == 4 && H % 16 == 0;
  template <bool INV>
  __device__ __forceinline__ static void run(float2* buf, float2*, const struct FFTArgs& f, const float2* tw,
                             int lane) {
    step<INV, 0, false>(buf, tw, lane, 1, nullptr, NoLoader{}, [] {}, NoLoader{});
  }
  // the forward transform with the row's (mean, M2) taken in its first pass
  __device__ __forceinline__ static float2 run_stats(float2* buf, const float2* tw, int lane) {
    float2 st = make_float2(0.f, 0.f);
    step<false, 0, true>(buf, tw, lane, 1, &st, NoLoader{}, [] {}, NoLoader{});
    return st;
  }
  // the transform with its first pass reading ld(k) instead of buf; after() runs once the
  // first pass is done (its reads of whatever ld reads have returned)
  template <bool INV, class LD, class AF>
  __device__ __forceinline__ static void run_loaded(float2* buf, const float2* tw, int lane,
                                                    const LD& ld, const AF& after) {
    step<INV, 0, false>(buf, tw, lane, 1, nullptr, ld, after, NoLoader{});
  }
  // ... and its last pass handing every output to so(it, r, k, value) instead of buf
  template <bool INV, class LD, class AF, class SO, bool SWINV = false>
  __device__ __forceinline__ static void run_io(float2* buf, const float2* tw, int lane,
                                                const LD& ld, const AF& after, const SO& so) {
    static_assert(NPASS >= 2, "run_io: a first and a last pass");
    step<INV, 0, false, LD, AF, SO, SWINV>(buf, tw, lane, 1, nullptr, ld, after, so);
  }
  template <bool INV, int I, bool STATS, class LD, class AF, class SO, bool SWINV = false>
  __device__ __forceinline__ static void step(float2* buf, const float2* tw, int lane, int Ns,
                                              float2* st, const LD& ld, const AF& after,
                                              const SO& so) {
    constexpr int R = RADS[I], IT = pass_iters(H, R);
    // (the forward transform; the inverse only where its kernel asks for it, SWINV: at 4
    // waves per SIMD the swizzle's address arithmetic pushed the inverse kernel past 128
    // VGPRs into scratch, irfft 0.58 -> 0.66 ms)
    constexpr bool SW = SWZ && (!INV || SWINV);
    constexpr bool SWI = SW && I == 2, SWO = SW && I == 1;
    if constexpr (I == 0 && I == NPASS - 1)
      stockham_pass_inplace<R, IT, INV, STATS, LD, SO>(buf, H, Ns, tw, lane, st, ld, so);
    else if constexpr (I == 0)
      stockham_pass_inplace<R, IT, INV, STATS, LD>(buf, H, Ns, tw, lane, st, ld);
    else if constexpr (I == NPASS - 1)
      stockham_pass_inplace<R, IT, INV, false, NoLoader, SO, SWI>(buf, H, Ns, tw, lane, nullptr,
                                                                  NoLoader{}, so);
    else
      stockham_pass_inplace<R, IT, INV, false, NoLoader, NoLoader, SWI, SWO>(buf, H, Ns, tw, lane);
    if constexpr (I == 0) after();
    if constexpr (I + 1 < NPASS)
      step<INV, I + 1, STATS, LD, AF, SO, SWINV>(buf, tw, lane, Ns * R, st, ld, after, so);
  }
};

struct GenericFFT {
  static constexpr int H = 0;  // runtime
  static constexpr int kBufs = 2;
  template <bool INV>
  __device__ __forceinline__ static void run(float2* buf, float2* buf2, const struct FFTArgs& f, const float2* tw,
                             int lane) {
    int Ns = 1;
    float2* a = buf;
    float2* b = buf2;
    for (int p = 0; p < f.nrad; ++p) {
      const int R = f.radices[p];
      switch (R) {
        case 4: stockham_pass_pp<4, INV>(a, b, f.H, Ns, tw, lane); break;
        case 2: stockham_pass_pp<2, INV>(a, b, f.H, Ns, tw, lane); break;
        case 3: stockham_pass_pp<3, INV>(a, b, f.H, Ns, tw, lane); break;
        case 5: stockham_pass_pp<5, INV>(a, b, f.H, Ns, tw, lane); break;
        case 7: stockham_pass_pp<7, INV>(a, b, f.H, Ns, tw, lane); break;
        case 11: stockham_pass_pp<11, INV>(a, b, f.H, Ns, tw, lane); break;
        default: stockham_pass_pp<13, INV>(a, b, f.H, Ns, tw, lane); break;
      }
      Ns *= R;
      float2* t = a; a = b; b = t;
    }
    if (a != buf) {
      for (int n = lane; n < f.H; n += 64) buf[n] = a[n];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

constexpr int kWaves = 4;  // rows in flight per workgroup (one per wave)
constexpr int kStageMax = 512;  // prefetched inverse-FFT input row (complex bins)

// LDS: [twiddles (H)] [per-wave row buffer (H) x kWaves]
__device__ __forceinline__ void load_twiddles(float2* tw, const FFTArgs& f) {
  for (int t = threadIdx.x; t < f.H; t += blockDim.x) tw[t] = f.twH[t];
  __syncthreads();
}

template <class CL>
__global__ __launch_bounds__(256) void fft_r2c_rows_kernel(const float* __restrict__ x,
                                                           float2* __restrict__ out,
                                                           float2* __restrict__ rowstats,
                                                           int64_t rows, int mmax, float scale,
                                                           FFTArgs f) {
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int H = CL::H > 0 ? CL::H : f.H;
  const int N = f.N;
  float2* tw = smem;
  const int per = CL::kBufs * H;
  float2* buf = smem + H + (size_t)w * per;
  float2* buf2 = buf + H;
  load_twiddles(tw, f);
  constexpr int NV = CL::H > 0 ? (CL::H / 2 + 63) / 64 : 1;  // float4 per lane per row
  float4 pf[NV];
  const int64_t stride = (int64_t)gridDim.x * kWaves;
  auto fetch = [&](int64_t r) {
    if constexpr (CL::H > 0) {
      if (r < rows) {
        const float4* x4 = reinterpret_cast<const float4*>(x + r * (2 * CL::H));
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int n = lane + 64 * j;
          if (n < CL::H / 2) pf[j] = x4[n];
        }
      }
    }
  };
  fetch((int64_t)blockIdx.x * kWaves + w);
  for (int64_t row = (int64_t)blockIdx.x * kWaves + w; row < rows; row += stride) {
    const float* xr = x + row * N;
    float s = 0.f;
    if constexpr (CL::H > 0) {  // codelet: rows arrive through the register prefetch
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int n = lane + 64 * j;
        if (n < CL::H / 2) {
          const float4 v = pf[j];
          buf[2 * n] = make_float2(v.x, v.y);
          buf[2 * n + 1] = make_float2(v.z, v.w);
          s += (v.x + v.y) + (v.z + v.w);
        }
      }
      fetch(row + stride);
    } else if (f.packed) {
      if ((N & 3) == 0) {
        const float4* x4 = reinterpret_cast<const float4*>(xr);
        for (int n = lane; n < N / 4; n += 64) {
          const float4 v = x4[n];
          buf[2 * n] = make_float2(v.x, v.y);
          buf[2 * n + 1] = make_float2(v.z, v.w);
          s += (v.x + v.y) + (v.z + v.w);
        }
      } else {
        const float2* x2 = reinterpret_cast<const float2*>(xr);
        for (int n = lane; n < H; n += 64) {
          const float2 v = x2[n];
          buf[n] = v;
          s += v.x + v.y;
        }
      }
    } else {
      for (int n = lane; n < N; n += 64) {
        const float v = xr[n];
        buf[n] = make_float2(v, 0.f);
        s += v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (rowstats) {
      const float mean = wave_sum(s) / (float)N;
      float q = 0.f;
      for (int n = lane; n < H; n += 64) {
        const float2 v = buf[n];
        const float d0 = v.x - mean;
        q += d0 * d0;
        if (f.packed) {
          const float d1 = v.y - mean;
          q += d1 * d1;
        }
      }
      q = wave_sum(q);
      if (lane == 0) rowstats[row] = make_float2(mean, q);
    }
    CL::template run<false>(buf, buf2, f, tw, lane);
    float2* o = out + row * mmax;
    if (f.packed) {
      for (int k = lane; k < mmax; k += 64) {
        const float2 zk = buf[k % H];
        const float2 zc = cconj(buf[(H - k) % H]);
        const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
        const float2 D = csub(zk, zc);
        const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);  // D / (2i)
        const float2 X = cadd(E, cmul(f.twN[k], O));
        o[k] = make_float2(scale * X.x, scale * X.y);
      }
    } else {
      for (int k = lane; k < mmax; k += 64) {
        const float2 X = buf[k];
        o[k] = make_float2(scale * X.x, scale * X.y);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

__device__ __forceinline__ float gelu_erf_f(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}

template <class CL>
__global__ __launch_bounds__(256) void fft_c2r_rows_kernel(const float2* __restrict__ in,
                                                           float* x, const float* addsrc,
                                                           float2* __restrict__ rowstats,
                                                           int64_t rows, int mmax, int act,
                                                           FFTArgs f) {
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int H = CL::H > 0 ? CL::H : f.H;
  const int N = f.N;
  float2* tw = smem;
  // per wave: FFT buffer(s) + (codelets) a staging row for the prefetched input
  const int per = CL::kBufs * H + (CL::H > 0 ? kStageMax : 0);
  float2* buf = smem + H + (size_t)w * per;
  float2* buf2 = buf + H;
  float2* stage = buf + CL::kBufs * H;
  load_twiddles(tw, f);
  constexpr int NVI = kStageMax / 64;
  float2 pf[NVI];
  const int64_t stride = (int64_t)gridDim.x * kWaves;
  const bool use_pf = CL::H > 0 && mmax <= kStageMax;
  auto fetch = [&](int64_t r) {
    if (use_pf && r < rows) {
      const float2* yr = in + r * mmax;
#pragma unroll
      for (int j = 0; j < NVI; ++j) {
        const int k = lane + 64 * j;
        if (k < mmax) pf[j] = yr[k];
      }
    }
  };
  fetch((int64_t)blockIdx.x * kWaves + w);
  for (int64_t row = (int64_t)blockIdx.x * kWaves + w; row < rows; row += stride) {
    const float2* yr = in + row * mmax;
    if (use_pf) {
#pragma unroll
      for (int j = 0; j < NVI; ++j) {
        const int k = lane + 64 * j;
        if (k < mmax) stage[k] = pf[j];
      }
      fetch(row + stride);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      yr = stage;
    }
    if (f.packed) {
      for (int k = lane; k < H; k += 64) {
        float2 xk = k < mmax ? yr[k] : make_float2(0.f, 0.f);
        if (k == 0) xk.y = 0.f;
        const int k2 = H - k;
        float2 xh = k2 < mmax ? yr[k2] : make_float2(0.f, 0.f);
        if (k2 == H || k2 == 0) xh.y = 0.f;  // DC / Nyquist imaginary parts are ignored
        const float2 xc = cconj(xh);
        const float2 A = cadd(xk, xc);
        const float2 D = csub(xk, xc);
        const float2 T = cmul(cconj(f.twN[k]), D);
        buf[k] = make_float2(A.x - T.y, A.y + T.x);
      }
    } else {
      for (int k = lane; k < N; k += 64) {
        float2 v = make_float2(0.f, 0.f);
        if (k < mmax) {
          v = yr[k];
          if (k == 0) v.y = 0.f;
        } else if (N - k < mmax) {
          v = cconj(yr[N - k]);
        }
        buf[k] = v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    CL::template run<true>(buf, buf2, f, tw, lane);
    float* xo = x + row * N;
    const float* ao = addsrc ? addsrc + row * N : nullptr;
    float s = 0.f;
    if (f.packed) {
      if ((N & 3) == 0) {
        float4* x4 = reinterpret_cast<float4*>(xo);
        for (int n = lane; n < N / 4; n += 64) {
          float2 a = buf[2 * n], b = buf[2 * n + 1];
          if (ao) {  // skip branch: x1 = act(x1_skip + filter)
            const float4 r = reinterpret_cast<const float4*>(ao)[n];
            a.x += r.x; a.y += r.y; b.x += r.z; b.y += r.w;
          }
          if (act == 1 || ao) {
            if (act == 1) {
              a.x = gelu_erf_f(a.x); a.y = gelu_erf_f(a.y);
              b.x = gelu_erf_f(b.x); b.y = gelu_erf_f(b.y);
            }
            buf[2 * n] = a;
            buf[2 * n + 1] = b;
          }
          x4[n] = make_float4(a.x, a.y, b.x, b.y);
          s += (a.x + a.y) + (b.x + b.y);
        }
      } else {
        float2* x2 = reinterpret_cast<float2*>(xo);
        for (int n = lane; n < H; n += 64) {
          float2 v = buf[n];
          if (ao) { v.x += ao[2 * n]; v.y += ao[2 * n + 1]; }
          if (act == 1) { v.x = gelu_erf_f(v.x); v.y = gelu_erf_f(v.y); }
          buf[n] = v;
          x2[n] = v;
          s += v.x + v.y;
        }
      }
    } else {
      for (int n = lane; n < N; n += 64) {
        float v = buf[n].x;
        if (ao) v += ao[n];
        if (act == 1) v = gelu_erf_f(v);
        buf[n].x = v;
        xo[n] = v;
        s += v;
      }
    }
    if (rowstats) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const float mean = wave_sum(s) / (float)N;
      float q = 0.f;
      if (f.packed) {
        for (int n = lane; n < H; n += 64) {
          const float2 v = buf[n];
          q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean);
        }
      } else {
        for (int n = lane; n < N; n += 64) {
          const float v = buf[n].x;
          q += (v - mean) * (v - mean);
        }
      }
      q = wave_sum(q);
      if (lane == 0) rowstats[row] = make_float2(mean, q);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA row kernels (compiled codelets, N % 8 == 0; the block's path).  Each
// wave keeps its next row in flight as an asynchronous global->LDS copy
// (dma.h) while it transforms the current one, so the HBM latency is covered
// without parking rows in VGPRs: the register-prefetch kernels above hold ~3
// workgroups per CU and their waves wait on memory most of the time (the
// inverse one also reads its skip-branch row synchronously).  The FFT runs in
// place in the LDS row the DMA filled; both twiddle tables live in LDS (a
// global twiddle read would make hipcc drain the copies in flight).
// ---------------------------------------------------------------------------
template <class CL, int WV, bool PL, int NS = 3>
__global__ __launch_bounds__(64 * WV) void fft_r2c_dma_kernel(const float* __restrict__ x,
                                                              float2* __restrict__ out,
                                                              float2* __restrict__ rowstats,
                                                              int64_t rows, int mmax, float scale,
                                                              FFTArgs f, C2RPlanes pp) {
  constexpr int H = CL::H, N = 2 * H, RB = N * 4;
  constexpr int NCH = (RB + 1023) / 1024;  // DMA wave-instructions per row
  // slots are exactly one row (16-B multiple): the last 1-KB piece is issued by the
  // lanes that cover the row only (a masked LDS-DMA still counts once in vmcnt).
  // Same time as 1-KB-rounded slots at 721 x 1440 (0.718 vs 0.719 ms, same box); 13
  // waves, which the smaller slots would allow, were slower
  constexpr int SLOT = (RB + 15) / 16 * 16;
  // NS row slots per wave: NS - 1 rows in flight while one is transformed
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float2* tw = smem;
  float2* twN = smem + H;
  char* slots = reinterpret_cast<char*>(smem + 2 * H + 2) + (size_t)w * NS * SLOT;
  for (int t = threadIdx.x; t < H; t += blockDim.x) tw[t] = f.twH[t];
  for (int t = threadIdx.x; t <= H; t += blockDim.x) twN[t] = f.twN[t];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * WV;
  const int64_t row0 = (int64_t)blockIdx.x * WV + w;
  auto issue = [&](int64_t r, int sl) {
    const char* src = reinterpret_cast<const char*>(x + r * N);
    const uint32_t dst = lds_addr(slots + sl * SLOT);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (c + 1 < NCH || c * 1024 + lane * 16 < RB)
        glds16(src + min(c * 1024 + lane * 16, RB - 16), dst + c * 1024);
  };
  if (row0 < rows) issue(row0, 0);
  if (NS > 1 && row0 + stride < rows) issue(row0 + stride, 1);
  constexpr bool PL8 = PL && N % 8 == 0;  // 16-B plane stores (8 values per lane)
  constexpr int NSP = PL8 ? 3 * ((N / 8 + 63) / 64) : (PL ? 3 * ((N / 4 + 63) / 64) : 0);
  const int nst = (mmax + 63) / 64 + (rowstats ? 1 : 0) + NSP;  // vector stores per row
  int sl = 0;
  int i = 0;
  for (int64_t row = row0; row < rows; row += stride, ++i) {
    // this row's copy has landed: count what this wave issued after it (the next
    // row's copy, if any, and the stores of the previous one or two rows)
    const bool next = row + stride < rows;
    if constexpr (NS == 1) {  // the only slot: this row was issued after the last stores
      wait_vmcnt(0);
    } else if constexpr (NS == 3) {
      wait_vmcnt((i >= 2 ? nst : 0) + (next ? NCH : 0) + (i >= 1 ? nst : 0));
      if (row + 2 * stride < rows) issue(row + 2 * stride, sl == 0 ? 2 : sl - 1);
    } else {  // the next row was issued after the previous row's stores
      wait_vmcnt((i >= 1 ? nst : 0) + (next ? NCH : 0));
    }
    float2* buf = reinterpret_cast<float2*>(slots + sl * SLOT);
    if constexpr (PL) {  // the raw row as bf16x3 planes, (b, c, lat) of row = (b*C + c)*nlat + lat
      const int64_t bc = row / pp.nlat, lat = row - bc * pp.nlat;
      const int64_t b = bc / pp.C, c = bc - b * pp.C;
      const int64_t P = (int64_t)pp.nlat * N, ps = (int64_t)pp.C * P;
      unsigned short* xq = pp.xp + b * 3 * ps + c * P + lat * N;
      const float4* b4 = reinterpret_cast<const float4*>(buf);
#pragma unroll
      for (int j = 0; j < (PL8 ? NSP / 3 : 0); ++j) {
        const int m = lane + 64 * j;  // 8 values: each plane as one 16-B vector
        if (m < N / 8) {
          const float4 v0 = b4[2 * m], v1 = b4[2 * m + 1];
          uint32_t t[3][4];
          split2(v0.x, v0.y, t[0][0], t[1][0], t[2][0]);
          split2(v0.z, v0.w, t[0][1], t[1][1], t[2][1]);
          split2(v1.x, v1.y, t[0][2], t[1][2], t[2][2]);
          split2(v1.z, v1.w, t[0][3], t[1][3], t[2][3]);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            *reinterpret_cast<uint4*>(xq + pl * ps + 8 * m) =
                make_uint4(t[pl][0], t[pl][1], t[pl][2], t[pl][3]);
        }
      }
#pragma unroll
      for (int j = 0; j < (PL8 ? 0 : NSP / 3); ++j) {
        const int n = lane + 64 * j;
        if (n < N / 4) {
          const float4 v = b4[n];
          uint32_t a0, a1, a2, c0, c1, c2;
          split2(v.x, v.y, a0, a1, a2);
          split2(v.z, v.w, c0, c1, c2);
          *reinterpret_cast<uint2*>(xq + 4 * n) = make_uint2(a0, c0);
          *reinterpret_cast<uint2*>(xq + ps + 4 * n) = make_uint2(a1, c1);
          *reinterpret_cast<uint2*>(xq + 2 * ps + 4 * n) = make_uint2(a2, c2);
        }
      }
    }
    if (rowstats) {  // (mean, M2) from the first FFT pass's registers (stockham_pass_inplace)
      const float2 st = CL::run_stats(buf, tw, lane);
      if (lane == 0) rowstats[row] = st;
    } else {
      CL::template run<false>(buf, nullptr, f, tw, lane);
    }
    float2* o = out + row * mmax;
    auto bin = [&](int k) {
      const float2 zk = buf[k % H];
      const float2 zc = cconj(buf[(H - k) % H]);
      const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
      const float2 D = csub(zk, zc);
      const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);  // D / (2i)
      const float2 X = cadd(E, cmul(twN[k], O));
      return make_float2(scale * X.x, scale * X.y);
    };
    for (int k = lane; k < mmax; k += 64) o[k] = bin(k);

    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if constexpr (NS == 1) {
      // every read of the slot has returned: refill it with the next row
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (next) issue(row + stride, 0);
    } else if constexpr (NS == 3) {
      sl = sl == 2 ? 0 : sl + 1;
    } else {
      // every read of this slot has returned: refill it with the row after next
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (row + 2 * stride < rows) issue(row + 2 * stride, sl);
      sl ^= 1;
    }
  }
}

// inverse: Yn row (mmax bins, DMA from the 16-B aligned address below the row
// start) and, with ADD, the skip-branch row x1 (x = act(x1 + irfft)); output
// rows stored from registers, row stats for InstanceNorm-1.  AH (1 or 2) rows in
// flight per wave (AH Yn and AH skip slots).  Measured at 721x1440: one row ahead
// with two 4-wave workgroups per CU beats two rows ahead with one 6-wave one
// (0.81 vs 0.98 ms): the row FFT itself is VALU/LDS-latency bound, so waves per
// CU matter more than bytes in flight.
// AR: the skip row is read into registers after the FFT instead of an LDS slot
// (8.8 instead of 14.8 KB of LDS per wave: more waves per CU)
// SWI_: the FFT codelet's pass-2 swizzle in this inverse kernel too (FixedFFT::SWZ; for
// wave counts that leave the registers it needs)
template <class CL, bool ADD, int WV, int AH, bool PL, bool AR = false, bool SWI_ = false>
__global__ __launch_bounds__(64 * WV) void fft_c2r_dma_kernel(const float2* __restrict__ in,
                                                              float* x, const float* addsrc,
                                                              float2* __restrict__ rowstats,
                                                              int64_t rows, int mmax, int act,
                                                              int ncy, FFTArgs f, C2RPlanes pp) {
  constexpr int H = CL::H, N = 2 * H, RB = N * 4;
  constexpr int NCA = (RB + 1023) / 1024;  // DMA instructions per skip row
  // store instructions per row (8-B plane stores: 16-B ones measured 2.5 % slower here,
  // unlike the forward kernel)
  constexpr int NST = (PL ? 3 : 1) * ((N / 4 + 63) / 64);
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float2* tw = smem;
  float2* twN = smem + H;
  const int YS = ncy * 1024;
  static_assert(!AR || (ADD && AH == 1), "register skip rows: one row ahead");
  constexpr bool ADMA = ADD && !AR;  // skip row staged by LDS-DMA
  const int per = RB + AH * YS + (ADMA ? AH * NCA * 1024 : 0);
  char* wb = reinterpret_cast<char*>(smem + 2 * H + 2) + (size_t)w * per;
  float2* buf = reinterpret_cast<float2*>(wb);
  char* yst = wb + RB;                  // AH slots of YS
  char* ast = wb + RB + AH * YS;        // AH slots of NCA KB
  for (int t = threadIdx.x; t < H; t += blockDim.x) tw[t] = f.twH[t];
  for (int t = threadIdx.x; t <= H; t += blockDim.x) twN[t] = f.twN[t];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * WV;
  const int YB = mmax * 8;
  const int64_t yend = (((int64_t)rows * YB) & ~(int64_t)15) - 16;  // last chunk inside Yn
  auto issue_y = [&](int64_t r, int sl) {
    const int64_t a0 = ((int64_t)r * YB) & ~(int64_t)15;
    const char* src = reinterpret_cast<const char*>(in);
    const uint32_t dst = lds_addr(yst + sl * YS);
    for (int c = 0; c < ncy; ++c)
      glds16(src + min(a0 + c * 1024 + lane * 16, yend), dst + c * 1024);
  };
  auto issue_a = [&](int64_t r, int sl) {
    const char* src = reinterpret_cast<const char*>(addsrc + r * N);
    const uint32_t dst = lds_addr(ast + sl * NCA * 1024);
#pragma unroll
    for (int c = 0; c < NCA; ++c)
      glds16(src + min(c * 1024 + lane * 16, RB - 16), dst + c * 1024);
  };
  const int64_t row0 = (int64_t)blockIdx.x * WV + w;
  if (row0 < rows) {
    issue_y(row0, 0);
    if constexpr (ADMA) issue_a(row0, 0);
  }
  if (AH == 2 && row0 + stride < rows) {
    issue_y(row0 + stride, 1);
    if constexpr (ADMA) issue_a(row0 + stride, 1);
  }
  // store instructions per row: the plane path's NST, or one 8-B store per output of the
  // last pass's butterflies (every butterfly iteration has an active lane)
  constexpr int NSTR = PL ? NST : CL::ITL * CL::RL;
  const int nst = NSTR + (rowstats ? 1 : 0);
  const int na = ADMA ? NCA : 0;
  int i = 0;
  for (int64_t row = row0; row < rows; row += stride, ++i) {
    const int sl = AH == 2 ? (i & 1) : 0;
    const bool e1 = row + stride < rows, e2 = row + 2 * stride < rows;
    // Yn(row) landed: count what this wave issued after it (dma.h)
    if (AH == 2)
      wait_vmcnt((i >= 2 ? nst : 0) + na + (i >= 1 ? nst : 0) + (e1 ? ncy + na : 0));
    else
      wait_vmcnt(na + (i >= 1 ? nst : 0));
    const float2* yr = reinterpret_cast<const float2*>(yst + sl * YS) + (((int64_t)row * YB) & 15) / 8;
    // the Hermitian pre-twiddle of bin k, read by the first FFT pass straight from the Yn slot
    auto pre = [&](int k) -> float2 {
      float2 xk = k < mmax ? yr[k] : make_float2(0.f, 0.f);
      if (k == 0) xk.y = 0.f;
      const int k2 = H - k;
      float2 xh = k2 < mmax ? yr[k2] : make_float2(0.f, 0.f);
      if (k2 == H || k2 == 0) xh.y = 0.f;  // DC / Nyquist imaginary parts are ignored
      const float2 xc = cconj(xh);
      const float2 A = cadd(xk, xc);
      const float2 D = csub(xk, xc);
      const float2 T = cmul(cconj(twN[k]), D);
      return make_float2(A.x - T.y, A.y + T.x);
    };
    if constexpr (!PL) {
      // the last pass hands its outputs over in registers: + skip, activation, 8-B stores
      // of the row (lanes contiguous), the row statistics from the same registers; the
      // skip values (AR) are loaded after the first pass, under the middle passes
      constexpr int RL = CL::RL, ITL = CL::ITL, NsL = H / RL;
      float2 skv[AR ? ITL : 1][AR ? RL : 1];
      float2 vo[ITL][RL];
      float s = 0.f;
      const float2* a2 = reinterpret_cast<const float2*>(ast + sl * NCA * 1024);
      float2* x2 = reinterpret_cast<float2*>(x + row * N);
      auto after = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (AH == 2 ? e2 : e1) issue_y(row + AH * stride, sl);  // this Yn slot was consumed
        if constexpr (ADMA) {  // skip row landed (counts as in the plane path below)
          if (AH == 2)
            wait_vmcnt((e1 ? ncy + na : 0) + (i >= 1 ? nst : 0) + (e2 ? ncy : 0));
          else
            wait_vmcnt(e1 ? ncy : 0);
        }
        if constexpr (AR) {
          const float2* g2 = reinterpret_cast<const float2*>(addsrc + row * N);
#pragma unroll
          for (int it = 0; it < ITL; ++it)
#pragma unroll
            for (int r = 0; r < RL; ++r) {
              const int j = lane + 64 * it;
              skv[it][r] = j < NsL ? g2[j + r * NsL] : make_float2(0.f, 0.f);
            }
        }
      };
      auto so = [&](int it, int r, int k, float2 a) {
        if constexpr (ADD) {
          const float2 sv = AR ? skv[AR ? it : 0][AR ? r : 0] : a2[k];
          a.x += sv.x;
          a.y += sv.y;
        }
        if (act == 1) {
          a.x = gelu_erf_f(a.x);
          a.y = gelu_erf_f(a.y);
        }
        x2[k] = a;
        vo[it][r] = a;
        s += a.x + a.y;
      };
      CL::template run_io<true, decltype(pre), decltype(after), decltype(so), SWI_>(buf, tw, lane,
                                                                                pre, after, so);
      if (rowstats) {
        const float mean = wave_sum(s) / (float)N;
        float q = 0.f;
#pragma unroll
        for (int it = 0; it < ITL; ++it)
          if (lane + 64 * it < NsL) {
#pragma unroll
            for (int r = 0; r < RL; ++r)
              q += (vo[it][r].x - mean) * (vo[it][r].x - mean) +
                   (vo[it][r].y - mean) * (vo[it][r].y - mean);
          }
        q = wave_sum(q);
        if (lane == 0) rowstats[row] = make_float2(mean, q);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if constexpr (ADMA) {
        if (AH == 2 ? e2 : e1) issue_a(row + AH * stride, sl);  // this skip slot was consumed
      }
      continue;
    }
    CL::template run_loaded<true>(buf, tw, lane, pre, [&]() {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      if (AH == 2 ? e2 : e1) issue_y(row + AH * stride, sl);  // this Yn slot was consumed
    });
    constexpr int NA4 = (N / 4 + 63) / 64;  // skip-row float4 per lane
    float4 areg[AR ? NA4 : 1];
    if constexpr (AR) {  // all of this lane's skip values in flight at once
      const float4* g4 = reinterpret_cast<const float4*>(addsrc + row * N);
#pragma unroll
      for (int j = 0; j < NA4; ++j) {
        const int n = lane + 64 * j;
        areg[j] = n < N / 4 ? g4[n] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if constexpr (ADMA) {  // skip row landed
      if (AH == 2)
        wait_vmcnt((e1 ? ncy + na : 0) + (i >= 1 ? nst : 0) + (e2 ? ncy : 0));
      else
        wait_vmcnt(e1 ? ncy : 0);
    }
    const float4* a4 = reinterpret_cast<const float4*>(ast + sl * NCA * 1024);
    float4* x4 = reinterpret_cast<float4*>(x + row * N);
    unsigned short* xq = nullptr;
    int64_t ps = 0;
    if constexpr (PL) {  // plane row: (b, c, lat) of row = (b*C + c)*nlat + lat
      const int64_t bc = row / pp.nlat, lat = row - bc * pp.nlat;
      const int64_t b = bc / pp.C, c = bc - b * pp.C;
      const int64_t P = (int64_t)pp.nlat * N;
      ps = (int64_t)pp.C * P;
      xq = pp.xp + b * 3 * ps + c * P + lat * N;
    }
    // the output values stay in registers for the row statistics' second pass (no LDS
    // write-back and re-read)
    constexpr int NV4 = (N / 4 + 63) / 64;
    float4 vout[NV4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int n = lane + 64 * j;
      if (j < NV4) vout[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < N / 4) {
        float2 a = buf[2 * n], b = buf[2 * n + 1];
        if constexpr (ADD) {
          const float4 r = AR ? areg[j < NA4 ? j : 0] : a4[n];
          a.x += r.x; a.y += r.y; b.x += r.z; b.y += r.w;
        }
        if (act == 1) {
          a.x = gelu_erf_f(a.x); a.y = gelu_erf_f(a.y);
          b.x = gelu_erf_f(b.x); b.y = gelu_erf_f(b.y);
        }
        if (j < NV4) vout[j] = make_float4(a.x, a.y, b.x, b.y);
        if constexpr (PL) {
          uint32_t a0, a1, a2, b0, b1, b2;
          split2(a.x, a.y, a0, a1, a2);
          split2(b.x, b.y, b0, b1, b2);
          uint2* q = reinterpret_cast<uint2*>(xq + 4 * n);
          q[0] = make_uint2(a0, b0);
          *reinterpret_cast<uint2*>(xq + ps + 4 * n) = make_uint2(a1, b1);
          *reinterpret_cast<uint2*>(xq + 2 * ps + 4 * n) = make_uint2(a2, b2);
        } else {
          x4[n] = make_float4(a.x, a.y, b.x, b.y);
        }
        s += (a.x + a.y) + (b.x + b.y);
      }
    }
    if (rowstats) {
      const float mean = wave_sum(s) / (float)N;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < NV4; ++j) {
        if (lane + 64 * j < N / 4) {
          const float4 v = vout[j];
          q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean) +
               ((v.z - mean) * (v.z - mean) + (v.w - mean) * (v.w - mean));
        }
      }
      q = wave_sum(q);
      if (lane == 0) rowstats[row] = make_float2(mean, q);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if constexpr (ADMA) {
      if (AH == 2 ? e2 : e1) issue_a(row + AH * stride, sl);  // this skip slot was consumed
    }
  }
}

// ---------------------------------------------------------------------------
// Fused FFT + transpose kernels (the block's path).  A workgroup owns TK
// consecutive latitudes of one (b,c) plane; each wave transforms TK/4 rows with
// the next row's global loads in flight (register prefetch) while it computes.
//   forward: x rows -> LDS tile [m][TK] -> Xt[m][(b,ri,c)][k0..k0+TK)   (m-major
//            GEMM operand of the Legendre stage; spectrum NOT normalised: the
//            InstanceNorm-0 affine is applied later, see dc_fixup / GEMM rowscale)
//   inverse: Yt[m][(b,ri,c)][k0..) -> LDS tile [m][TK] -> irfft rows -> output
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap_1d(int orig, int nwg) {
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// LDS tile: separate real / imaginary planes [mmax][TK + pad] so that four
// consecutive latitudes move as one float4 between LDS and HBM.
template <int TK>
struct TileGeom {
  static constexpr int TS = TK + 4;  // plane row stride (floats), keeps float4 alignment
};

template <class CL, int TK>
__global__ __launch_bounds__(256) void fft_r2c_tile_kernel(const float* __restrict__ x,
                                                           float* __restrict__ Xt,
                                                           float2* __restrict__ rowstats, int C,
                                                           int nlat, int mmax, int ldk, int64_t R,
                                                           int ntiles, float scale, FFTArgs f) {
  extern __shared__ float2 smem[];
  constexpr int H = CL::H;
  constexpr int N = 2 * H;
  constexpr int NV = (N / 4 + 63) / 64;
  constexpr int TS = TileGeom<TK>::TS;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float2* tw = smem;
  float* pre = reinterpret_cast<float*>(smem + H);
  float* pim = pre + (size_t)mmax * TS;
  float2* buf = reinterpret_cast<float2*>(pim + (size_t)mmax * TS) + (size_t)w * H;
  load_twiddles(tw, f);
  const int lin = xcd_remap_1d(blockIdx.x, gridDim.x);
  const int tile = lin % ntiles;
  const int bc = lin / ntiles;
  const int k0 = tile * TK;
  const float4* plane = reinterpret_cast<const float4*>(x + (int64_t)bc * nlat * N);
  float4 pf[NV];
  auto prefetch = [&](int kk) {
    const int k = k0 + kk;
    if (kk < TK && k < nlat) {
      const float4* r4 = plane + (int64_t)k * (N / 4);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int n = lane + 64 * j;
        if (n < N / 4) pf[j] = r4[n];
      }
    }
  };
  prefetch(w);
  for (int kk = w; kk < TK && k0 + kk < nlat; kk += 4) {
    const int k = k0 + kk;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int n = lane + 64 * j;
      if (n < N / 4) {
        const float4 v = pf[j];
        buf[2 * n] = make_float2(v.x, v.y);
        buf[2 * n + 1] = make_float2(v.z, v.w);
        s += (v.x + v.y) + (v.z + v.w);
      }
    }
    prefetch(kk + 4);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (rowstats) {
      const float mean = wave_sum(s) / (float)N;
      float q = 0.f;
      for (int n = lane; n < H; n += 64) {
        const float2 v = buf[n];
        q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean);
      }
      q = wave_sum(q);
      if (lane == 0) rowstats[(int64_t)bc * nlat + k] = make_float2(mean, q);
    }
    CL::template run<false>(buf, nullptr, f, tw, lane);
    for (int m = lane; m < mmax; m += 64) {
      const float2 zk = buf[m % H];
      const float2 zc = cconj(buf[(H - m) % H]);
      const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
      const float2 D = csub(zk, zc);
      const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);
      const float2 X = cadd(E, cmul(f.twN[m], O));
      pre[m * TS + kk] = scale * X.x;
      pim[m * TS + kk] = scale * X.y;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  __syncthreads();
  const int b = bc / C, c = bc - b * C;
  const int64_t rre = (int64_t)(b * 2) * C + c, rim = rre + C;
  constexpr int Q = TK / 4;
  const int total = mmax * 2 * Q;
  for (int e = threadIdx.x; e < total; e += 256) {
    const int m = e / (2 * Q);
    const int rem = e - m * 2 * Q;
    const int ri = rem / Q, q = rem - ri * Q;
    const int k = k0 + 4 * q;
    if (k < nlat) {  // k < nlat <= ldk, ldk % 4 == 0: the float4 stays inside the row
      const float4 v = *reinterpret_cast<const float4*>((ri ? pim : pre) + m * TS + 4 * q);
      *reinterpret_cast<float4*>(Xt + ((int64_t)m * R + (ri ? rim : rre)) * ldk + k) = v;
    }
  }
}

template <class CL, int TK>
__global__ __launch_bounds__(256) void fft_c2r_tile_kernel(const float* __restrict__ Yt,
                                                           float* __restrict__ out,
                                                           float2* __restrict__ rowstats, int C,
                                                           int nlat, int mmax, int mact, int ldk,
                                                           int64_t R, int ntiles, int act,
                                                           FFTArgs f) {
  extern __shared__ float2 smem[];
  constexpr int H = CL::H;
  constexpr int N = 2 * H;
  constexpr int TS = TileGeom<TK>::TS;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float2* tw = smem;
  float* pre = reinterpret_cast<float*>(smem + H);
  float* pim = pre + (size_t)mmax * TS;
  float2* buf = reinterpret_cast<float2*>(pim + (size_t)mmax * TS) + (size_t)w * H;
  const int lin = xcd_remap_1d(blockIdx.x, gridDim.x);
  const int tile = lin % ntiles;
  const int bc = lin / ntiles;
  const int k0 = tile * TK;
  const int b = bc / C, c = bc - b * C;
  const int64_t rre = (int64_t)(b * 2) * C + c, rim = rre + C;
  for (int t = threadIdx.x; t < H; t += 256) tw[t] = f.twH[t];
  constexpr int Q = TK / 4;
  const int total = mmax * 2 * Q;
  // all loads of the tile issued before any LDS write (kLoadBatch in flight per lane)
  constexpr int kLoadBatch = 8;
  for (int e0 = 0; e0 < total; e0 += 256 * kLoadBatch) {
    float4 v[kLoadBatch];
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) {
      const int e = e0 + u * 256 + threadIdx.x;
      const int m = e / (2 * Q);
      const int rem = e - m * 2 * Q;
      const int ri = rem / Q, q = rem - ri * Q;
      const int k = k0 + 4 * q;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < total && k < nlat && m < mact)
        v[u] = *reinterpret_cast<const float4*>(Yt + ((int64_t)m * R + (ri ? rim : rre)) * ldk + k);
    }
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) {
      const int e = e0 + u * 256 + threadIdx.x;
      if (e < total) {
        const int m = e / (2 * Q);
        const int rem = e - m * 2 * Q;
        const int ri = rem / Q, q = rem - ri * Q;
        *reinterpret_cast<float4*>((ri ? pim : pre) + m * TS + 4 * q) = v[u];
      }
    }
  }
  __syncthreads();
  for (int kk = w; kk < TK && k0 + kk < nlat; kk += 4) {
    const int k = k0 + kk;
    for (int q = lane; q < H; q += 64) {
      float2 xk = q < mmax ? make_float2(pre[q * TS + kk], pim[q * TS + kk]) : make_float2(0.f, 0.f);
      if (q == 0) xk.y = 0.f;
      const int q2 = H - q;
      float2 xh = q2 < mmax ? make_float2(pre[q2 * TS + kk], pim[q2 * TS + kk]) : make_float2(0.f, 0.f);
      if (q2 == H || q2 == 0) xh.y = 0.f;
      const float2 xc = cconj(xh);
      const float2 A = cadd(xk, xc);
      const float2 D = csub(xk, xc);
      const float2 T = cmul(cconj(f.twN[q]), D);
      buf[q] = make_float2(A.x - T.y, A.y + T.x);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    CL::template run<true>(buf, nullptr, f, tw, lane);
    float4* o4 = reinterpret_cast<float4*>(out + ((int64_t)bc * nlat + k) * N);
    float s = 0.f;
    for (int n = lane; n < N / 4; n += 64) {
      float2 a = buf[2 * n], bb = buf[2 * n + 1];
      if (act == 1) {
        a.x = gelu_erf_f(a.x); a.y = gelu_erf_f(a.y);
        bb.x = gelu_erf_f(bb.x); bb.y = gelu_erf_f(bb.y);
        buf[2 * n] = a;
        buf[2 * n + 1] = bb;
      }
      o4[n] = make_float4(a.x, a.y, bb.x, bb.y);
      s += (a.x + a.y) + (bb.x + bb.y);
    }
    if (rowstats) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const float mean = wave_sum(s) / (float)N;
      float q = 0.f;
      for (int n = lane; n < H; n += 64) {
        const float2 v = buf[n];
        q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean);
      }
      q = wave_sum(q);
      if (lane == 0) rowstats[(int64_t)bc * nlat + k] = make_float2(mean, q);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

static FFTArgs make_args(const FFTPlan& p) {
  FFTArgs a{};
  a.N = p.N; a.H = p.H; a.packed = p.packed; a.nrad = p.nrad; a.inplace = p.inplace;
  a.codelet = p.codelet;
  for (int i = 0; i < kMaxRadices; ++i) a.radices[i] = p.radices[i];
  a.twH = p.twH; a.twN = p.twN;
  return a;
}

static int64_t fft_grid(int64_t rows) {
  // enough workgroups to fill the chip several times over; waves loop over rows
  return std::min<int64_t>(cdiv(rows, kWaves), 256 * 20);
}

// compiled codelets (radix order as produced by fft_plan_build)
using FFT1440 = FixedFFT<4, 4, 3, 3, 5>;  // nlon 1440 (721x1440 grid)
using FFT240 = FixedFFT<4, 2, 3, 5>;      // nlon 240  (120x240 Gauss grid)
using FFT64 = FixedFFT<4, 4, 2>;          // nlon 64
using FFT48 = FixedFFT<4, 2, 3>;          // nlon 48
using FFT180 = FixedFFT<2, 3, 3, 5>;      // nlon 180
using FFT32 = FixedFFT<4, 4>;             // nlon 32
#define MSFNO_FFT_CODELETS(X) \
  X(1, FFT1440)               \
  X(2, FFT240)                \
  X(3, FFT64)                 \
  X(4, FFT48)                 \
  X(5, FFT180)                \
  X(6, FFT32)

// LDS-DMA row kernels for compiled codelets (MSFNO_FFT_DMA=0: register-prefetch
// kernels, kept for A/B)
static bool use_fft_dma() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_FFT_DMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int set_lds_limit(const void* fn, size_t lds);

// persistent grid of the DMA row kernels: one workgroup per CU
static int64_t dma_grid() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

template <class CL>
static int launch_r2c(const FFTArgs& a, const float* x, float2* out, float2* rowstats,
                      int64_t rows, int mmax, float scale, hipStream_t s,
                      const C2RPlanes* planes) {
  if constexpr (CL::H > 0) {
    if (use_fft_dma() && (2 * CL::H) % 8 == 0 && mmax <= CL::H + 1) {
      // waves x row slots per workgroup, one workgroup per CU: 12 x 2 (one row in
      // flight, 12 waves) measured 4 % faster than 8 x 3 (two rows in flight, 8
      // waves) at 721 x 1440 and 5 x 2 (two workgroups) slower; the row FFT is
      // latency bound, waves per CU beat rows in flight.  MSFNO_R2C_CFG=8x3|5x2 (A/B)
      static const int cfg = [] {
        const char* e = getenv("MSFNO_R2C_CFG");
        if (e && std::string(e) == "8x3") return 0;
        if (e && std::string(e) == "5x2") return 2;
        if (e && std::string(e) == "16x1") return 3;
        return 1;
      }();
      const size_t slot = (size_t)(2 * CL::H * 4 + 15) / 16 * 16;  // = the kernel's SLOT
      auto go = [&](auto kern, int WV, int NS) -> int {
        const size_t lds = (size_t)(2 * CL::H + 2) * sizeof(float2) + WV * NS * slot;
        MSFNO_REQUIRE(lds <= 160 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
        const int64_t grid =
            std::min<int64_t>(cdiv(rows, WV), dma_grid() * (WV == 5 ? 2 : 1));  // WGs per CU
        MSFNO_TRY(set_lds_limit(reinterpret_cast<const void*>(kern), lds));
        C2RPlanes pp{};
        if (planes) pp = *planes;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * WV), lds, s, x, out, rowstats,
                           rows, mmax, scale, a, pp);
        return launch_check("fft_r2c_dma");
      };
      if (cfg == 1)
        return planes ? go(fft_r2c_dma_kernel<CL, 12, true, 2>, 12, 2)
                      : go(fft_r2c_dma_kernel<CL, 12, false, 2>, 12, 2);
      if (cfg == 2)
        return planes ? go(fft_r2c_dma_kernel<CL, 5, true, 2>, 5, 2)
                      : go(fft_r2c_dma_kernel<CL, 5, false, 2>, 5, 2);
      if (cfg == 3)
        return planes ? go(fft_r2c_dma_kernel<CL, 16, true, 1>, 16, 1)
                      : go(fft_r2c_dma_kernel<CL, 16, false, 1>, 16, 1);
      return planes ? go(fft_r2c_dma_kernel<CL, 8, true>, 8, 3)
                    : go(fft_r2c_dma_kernel<CL, 8, false>, 8, 3);
    }
  }
  MSFNO_REQUIRE(!planes, MSFNO_EUNSUPPORTED, "r2c plane output needs the LDS-DMA row FFT");
  const size_t lds = (size_t)(kWaves * CL::kBufs + 1) * a.H * sizeof(float2);
  MSFNO_REQUIRE(lds <= 64 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  hipLaunchKernelGGL((fft_r2c_rows_kernel<CL>), dim3((unsigned)fft_grid(rows)), dim3(256), lds, s,
                     x, out, rowstats, rows, mmax, scale, a);
  return launch_check("fft_r2c_rows");
}

static bool c2r_swz() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_C2R_SWZ");
    return e && e[0] == '1';
  }();
  return on;
}

template <class CL>
static int launch_c2r(const FFTArgs& a, const float2* in, float* x, const float* addsrc,
                      float2* rowstats, int64_t rows, int mmax, int act, hipStream_t s,
                      const C2RPlanes* planes) {
  if constexpr (CL::H > 0) {
    const int ncy = (mmax * 8 + 16 + 1023) / 1024;
    C2RPlanes pp{};
    if (planes) pp = *planes;
    if (use_fft_dma() && (2 * CL::H) % 8 == 0 && mmax <= CL::H + 1 && ncy <= 5) {
      const int rb = 2 * CL::H * 4, nca = (rb + 1023) / 1024;
      // one row ahead, 4-wave workgroups, as many per CU as the LDS holds
      // skip rows through registers (no LDS slot): 16 waves per CU instead of 10,
      // irfft 0.86 -> 0.74 ms at 721 x 1440.  MSFNO_C2R_AREG=0 stages them by LDS-DMA
      static const bool areg = [] {
        const char* e = getenv("MSFNO_C2R_AREG");
        return !(e && e[0] == '0');
      }();
      // LDS per wave: row + Yn slot (+ the skip-row slot of the LDS-DMA variants)
      const size_t per_reg = (size_t)rb + ncy * 1024;
      const size_t per = per_reg + (addsrc ? nca * 1024 : 0);
      const size_t tw = (size_t)(2 * CL::H + 2) * sizeof(float2);
      const int wg_cu = (int)std::max<size_t>(1, (160 * 1024) / (tw + 4 * per));
      MSFNO_REQUIRE(tw + 4 * per <= 160 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
      auto go = [&](auto kern, int WV, size_t pw) -> int {
        const size_t lds = tw + WV * pw;
        MSFNO_TRY(set_lds_limit(reinterpret_cast<const void*>(kern), lds));
        const int wgs = WV == 4 ? wg_cu : (int)std::max<size_t>(1, (160 * 1024) / lds);
        const int64_t grid = std::min<int64_t>(cdiv(rows, WV), dma_grid() * wgs);
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * WV), lds, s, in, x, addsrc,
                           rowstats, rows, mmax, act, ncy, a, pp);
        return MSFNO_OK;
      };
      // block path (skip add + planes): one 10-wave workgroup per CU when the LDS holds
      // it (one twiddle copy per CU instead of two): 3 % faster than two 4-wave ones at
      // 721 x 1440.  MSFNO_C2R_WV=4 keeps the 4-wave workgroups (A/B)
      static const bool wide = [] {
        const char* e = getenv("MSFNO_C2R_WV");
        return !(e && atoi(e) == 4);
      }();
      if (planes && addsrc && areg && tw + 16 * per_reg <= 160 * 1024)
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 16, 1, true, true>, 16, per_reg));
      else if (planes && addsrc && wide && tw + 10 * per <= 160 * 1024)
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 10, 1, true>, 10, per));
      else if (planes && addsrc)
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 4, 1, true>, 4, per));
      else if (planes)
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, false, 4, 1, true>, 4, per));
      else if (addsrc && areg && c2r_swz() && tw + 12 * per_reg <= 160 * 1024)
        // MSFNO_C2R_SWZ=1 (A/B): 12 waves with the codelet's pass-2 swizzle
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 12, 1, false, true, true>, 12, per_reg));
      else if (addsrc && areg && tw + 16 * per_reg <= 160 * 1024)
        // fp32 x1 for the fused MLP: the same 16-wave register-skip kernel
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 16, 1, false, true>, 16, per_reg));
      else if (addsrc)
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, true, 4, 1, false>, 4, per));
      else
        MSFNO_TRY(go(fft_c2r_dma_kernel<CL, false, 4, 1, false>, 4, per));
      return launch_check("fft_c2r_dma");
    }
  }
  MSFNO_REQUIRE(!planes, MSFNO_EUNSUPPORTED, "plane output needs the LDS-DMA inverse FFT");
  const size_t lds =
      ((size_t)(kWaves * CL::kBufs + 1) * a.H + (CL::H > 0 ? kWaves * kStageMax : 0)) *
      sizeof(float2);
  MSFNO_REQUIRE(lds <= 64 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  hipLaunchKernelGGL((fft_c2r_rows_kernel<CL>), dim3((unsigned)fft_grid(rows)), dim3(256), lds, s,
                     in, x, addsrc, rowstats, rows, mmax, act, a);
  return launch_check("fft_c2r_rows");
}

int launch_fft_r2c_rows(const FFTPlan& f, const float* x, float2* out, float2* rowstats,
                        int64_t rows, int mmax, float scale, hipStream_t s,
                        const C2RPlanes* planes) {
  if (rows <= 0) return MSFNO_OK;
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_r2c<CL>(a, x, out, rowstats, rows, mmax, scale, s, planes);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: return launch_r2c<GenericFFT>(a, x, out, rowstats, rows, mmax, scale, s, planes);
  }
}

int launch_fft_c2r_rows(const FFTPlan& f, const float2* in, float* x, const float* addsrc,
                        float2* rowstats, int64_t rows, int mmax, int act, hipStream_t s,
                        const C2RPlanes* planes) {
  if (rows <= 0) return MSFNO_OK;
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_c2r<CL>(a, in, x, addsrc, rowstats, rows, mmax, act, s, planes);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: return launch_c2r<GenericFFT>(a, in, x, addsrc, rowstats, rows, mmax, act, s, planes);
  }
}

bool fft_r2c_planes_supported(const FFTPlan& f, int mmax) {
  return use_fft_dma() && f.codelet != 0 && f.packed && f.N % 8 == 0 && mmax <= f.H + 1;
}

bool fft_c2r_planes_supported(const FFTPlan& f, int mmax) {
  const int ncy = (mmax * 8 + 16 + 1023) / 1024;
  return use_fft_dma() && f.codelet != 0 && f.packed && f.N % 8 == 0 && mmax <= f.H + 1 &&
         ncy <= 5;
}

template <class CL, int TK>
static size_t tile_lds(int mmax) {
  return (size_t)CL::H * 5 * sizeof(float2) + (size_t)2 * mmax * TileGeom<TK>::TS * sizeof(float);
}

static int set_lds_limit(const void* fn, size_t lds) {
  if (lds > 64 * 1024)
    MSFNO_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return MSFNO_OK;
}

static int tile_k() {
  static int tk = -1;
  if (tk < 0) {
    const char* e = getenv("MSFNO_FFT_TK");
    tk = (e && atoi(e) == 8) ? 8 : 16;
  }
  return tk;
}

template <class CL, int TK>
static int launch_r2c_tile_t(const FFTArgs& a, const float* x, float* Xt, float2* rowstats, int B,
                             int C, int nlat, int mmax, int ldk, float scale, hipStream_t s) {
  const size_t lds = tile_lds<CL, TK>(mmax);
  MSFNO_REQUIRE(lds <= 160 * 1024, MSFNO_EUNSUPPORTED, "FFT tile exceeds LDS");
  MSFNO_TRY(set_lds_limit(reinterpret_cast<const void*>(&fft_r2c_tile_kernel<CL, TK>), lds));
  const int ntiles = (int)cdiv(nlat, TK);
  hipLaunchKernelGGL((fft_r2c_tile_kernel<CL, TK>), dim3((unsigned)(ntiles * B * C)), dim3(256),
                     lds, s, x, Xt, rowstats, C, nlat, mmax, ldk, 2LL * B * C, ntiles, scale, a);
  return launch_check("fft_r2c_tile");
}

template <class CL, int TK>
static int launch_c2r_tile_t(const FFTArgs& a, const float* Yt, float* out, float2* rowstats,
                             int B, int C, int nlat, int mmax, int mact, int ldk, int act,
                             hipStream_t s) {
  const size_t lds = tile_lds<CL, TK>(mmax);
  MSFNO_REQUIRE(lds <= 160 * 1024, MSFNO_EUNSUPPORTED, "FFT tile exceeds LDS");
  MSFNO_TRY(set_lds_limit(reinterpret_cast<const void*>(&fft_c2r_tile_kernel<CL, TK>), lds));
  const int ntiles = (int)cdiv(nlat, TK);
  hipLaunchKernelGGL((fft_c2r_tile_kernel<CL, TK>), dim3((unsigned)(ntiles * B * C)), dim3(256),
                     lds, s, Yt, out, rowstats, C, nlat, mmax, mact, ldk, 2LL * B * C, ntiles, act,
                     a);
  return launch_check("fft_c2r_tile");
}

template <class CL>
static int launch_r2c_tile(const FFTArgs& a, const float* x, float* Xt, float2* rowstats, int B,
                           int C, int nlat, int mmax, int ldk, float scale, hipStream_t s) {
  return tile_k() == 8
             ? launch_r2c_tile_t<CL, 8>(a, x, Xt, rowstats, B, C, nlat, mmax, ldk, scale, s)
             : launch_r2c_tile_t<CL, 16>(a, x, Xt, rowstats, B, C, nlat, mmax, ldk, scale, s);
}

template <class CL>
static int launch_c2r_tile(const FFTArgs& a, const float* Yt, float* out, float2* rowstats,
                           int B, int C, int nlat, int mmax, int mact, int ldk, int act,
                           hipStream_t s) {
  return tile_k() == 8
             ? launch_c2r_tile_t<CL, 8>(a, Yt, out, rowstats, B, C, nlat, mmax, mact, ldk, act, s)
             : launch_c2r_tile_t<CL, 16>(a, Yt, out, rowstats, B, C, nlat, mmax, mact, ldk, act, s);
}

bool fft_tile_supported(const FFTPlan& f) { return f.codelet != 0 && (f.N % 4) == 0; }

int launch_fft_r2c_tile(const FFTPlan& f, const float* x, float* Xt, float2* rowstats, int B,
                        int C, int nlat, int mmax, int ldk, float scale, hipStream_t s) {
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_r2c_tile<CL>(a, x, Xt, rowstats, B, C, nlat, mmax, ldk, scale, s);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: set_error("no FFT codelet for this nlon"); return MSFNO_EUNSUPPORTED;
  }
}

int launch_fft_c2r_tile(const FFTPlan& f, const float* Yt, float* out, float2* rowstats, int B,
                        int C, int nlat, int mmax, int mact, int ldk, int act, hipStream_t s) {
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_c2r_tile<CL>(a, Yt, out, rowstats, B, C, nlat, mmax, mact, ldk, act, s);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: set_error("no FFT codelet for this nlon"); return MSFNO_EUNSUPPORTED;
  }
}

template <int... Rs>
static bool matches(const FFTPlan& p, FixedFFT<Rs...>*) {
  return p.packed && FixedFFT<Rs...>::H == p.H;  // the codelet brings its own radix plan
}

// ---------------------------------------------------------------------------
int fft_plan_build(FFTPlan& p, int N) {
  MSFNO_REQUIRE(N >= 2, MSFNO_EINVAL, "nlon must be >= 2");
  p.N = N;
  p.packed = (N % 2 == 0) ? 1 : 0;
  p.H = p.packed ? N / 2 : N;
  int h = p.H;
  p.nrad = 0;
  const int prefs[] = {4, 2, 3, 5, 7, 11, 13};
  for (int r : prefs) {
    while (h % r == 0 && h > 1) {
      MSFNO_REQUIRE(p.nrad < kMaxRadices, MSFNO_EUNSUPPORTED, "too many FFT passes");
      p.radices[p.nrad++] = r;
      h /= r;
    }
  }
  MSFNO_REQUIRE(h == 1, MSFNO_EUNSUPPORTED,
                "nlon has a prime factor > 13 (unsupported by the longitude FFT)");
  p.codelet = 0;
#define X(id, CL) \
  if (!p.codelet && matches(p, (CL*)nullptr)) p.codelet = id;
  MSFNO_FFT_CODELETS(X)
#undef X
  p.inplace = p.codelet != 0;
  std::vector<float2> twH(p.H), twN(p.N / 2 + 1);
  for (int t = 0; t < p.H; ++t) {
    const double a = -2.0 * M_PI * (double)t / (double)p.H;
    twH[t] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  for (int k = 0; k <= p.N / 2; ++k) {
    const double a = -2.0 * M_PI * (double)k / (double)p.N;
    twN[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  MSFNO_CHECK_HIP(hipMalloc(&p.twH, twH.size() * sizeof(float2)));
  MSFNO_CHECK_HIP(hipMalloc(&p.twN, twN.size() * sizeof(float2)));
  MSFNO_CHECK_HIP(hipMemcpy(p.twH, twH.data(), twH.size() * sizeof(float2), hipMemcpyHostToDevice));
  MSFNO_CHECK_HIP(hipMemcpy(p.twN, twN.data(), twN.size() * sizeof(float2), hipMemcpyHostToDevice));
  return MSFNO_OK;
}

void fft_plan_free(FFTPlan& p) {
  if (p.twH) (void)hipFree(p.twH);
  if (p.twN) (void)hipFree(p.twN);
  p.twH = p.twN = nullptr;
}

}  // namespace msfno
