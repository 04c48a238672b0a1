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

// One Stockham pass, in place in the wave's LDS row buffer: every lane first
// reads all inputs of its butterflies into registers, then (after the reads
// have returned — they feed the arithmetic) writes the outputs.  LDS accesses
// of one wavefront are performed in order, so no barrier is needed: each row
// belongs to exactly one wave.
template <int R, int IT, bool INV>
__device__ __forceinline__ void stockham_pass_inplace(float2* buf, int H, int Ns,
                                                      const float2* tw, int lane) {
  const int nb = H / R;
  const int step = H / (Ns * R);
  float2 v[IT][R];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[it][r] = buf[j + r * nb];
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
      const int k = j % Ns;
      if (Ns > 1) {
#pragma unroll
        for (int r = 1; r < R; ++r) {
          float2 w = tw[r * k * step];
          if (INV) w.y = -w.y;
          v[it][r] = cmul(v[it][r], w);
        }
      }
      butterfly<R, INV>(v[it], tw, H);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (j < nb) {
      const int k = j % Ns;
      const int base = (j / Ns) * Ns * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[base + r * Ns] = v[it][r];
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
  template <bool INV>
  __device__ static void run(float2* buf, float2*, const struct FFTArgs&, const float2* tw,
                             int lane) {
    int Ns = 1;
    ((stockham_pass_inplace<Rs, pass_iters(H, Rs), INV>(buf, H, Ns, tw, lane), Ns *= Rs), ...);
  }
};

struct GenericFFT {
  static constexpr int H = 0;  // runtime
  static constexpr int kBufs = 2;
  template <bool INV>
  __device__ static void run(float2* buf, float2* buf2, const struct FFTArgs& f, const float2* tw,
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
  for (int64_t row = (int64_t)blockIdx.x * kWaves + w; row < rows;
       row += (int64_t)gridDim.x * kWaves) {
    const float* xr = x + row * N;
    float s = 0.f;
    if (f.packed) {
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
                                                           float* __restrict__ x,
                                                           float2* __restrict__ rowstats,
                                                           int64_t rows, int mmax, int act,
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
  for (int64_t row = (int64_t)blockIdx.x * kWaves + w; row < rows;
       row += (int64_t)gridDim.x * kWaves) {
    const float2* yr = in + row * mmax;
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
    float s = 0.f;
    if (f.packed) {
      if ((N & 3) == 0) {
        float4* x4 = reinterpret_cast<float4*>(xo);
        for (int n = lane; n < N / 4; n += 64) {
          float2 a = buf[2 * n], b = buf[2 * n + 1];
          if (act == 1) {
            a.x = gelu_erf_f(a.x); a.y = gelu_erf_f(a.y);
            b.x = gelu_erf_f(b.x); b.y = gelu_erf_f(b.y);
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
          if (act == 1) { v.x = gelu_erf_f(v.x); v.y = gelu_erf_f(v.y); buf[n] = v; }
          x2[n] = v;
          s += v.x + v.y;
        }
      }
    } else {
      for (int n = lane; n < N; n += 64) {
        float v = buf[n].x;
        if (act == 1) { v = gelu_erf_f(v); buf[n].x = v; }
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

template <class CL>
static int launch_r2c(const FFTArgs& a, const float* x, float2* out, float2* rowstats,
                      int64_t rows, int mmax, float scale, hipStream_t s) {
  const size_t lds = (size_t)(kWaves * CL::kBufs + 1) * a.H * sizeof(float2);
  MSFNO_REQUIRE(lds <= 64 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  hipLaunchKernelGGL((fft_r2c_rows_kernel<CL>), dim3((unsigned)fft_grid(rows)), dim3(256), lds, s,
                     x, out, rowstats, rows, mmax, scale, a);
  return launch_check("fft_r2c_rows");
}

template <class CL>
static int launch_c2r(const FFTArgs& a, const float2* in, float* x, float2* rowstats,
                      int64_t rows, int mmax, int act, hipStream_t s) {
  const size_t lds = (size_t)(kWaves * CL::kBufs + 1) * a.H * sizeof(float2);
  MSFNO_REQUIRE(lds <= 64 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  hipLaunchKernelGGL((fft_c2r_rows_kernel<CL>), dim3((unsigned)fft_grid(rows)), dim3(256), lds, s,
                     in, x, rowstats, rows, mmax, act, a);
  return launch_check("fft_c2r_rows");
}

int launch_fft_r2c_rows(const FFTPlan& f, const float* x, float2* out, float2* rowstats,
                        int64_t rows, int mmax, float scale, hipStream_t s) {
  if (rows <= 0) return MSFNO_OK;
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_r2c<CL>(a, x, out, rowstats, rows, mmax, scale, s);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: return launch_r2c<GenericFFT>(a, x, out, rowstats, rows, mmax, scale, s);
  }
}

int launch_fft_c2r_rows(const FFTPlan& f, const float2* in, float* x, float2* rowstats,
                        int64_t rows, int mmax, int act, hipStream_t s) {
  if (rows <= 0) return MSFNO_OK;
  const FFTArgs a = make_args(f);
  switch (f.codelet) {
#define X(id, CL) \
  case id: return launch_c2r<CL>(a, in, x, rowstats, rows, mmax, act, s);
    MSFNO_FFT_CODELETS(X)
#undef X
    default: return launch_c2r<GenericFFT>(a, in, x, rowstats, rows, mmax, act, s);
  }
}

template <int... Rs>
static bool matches(const FFTPlan& p, FixedFFT<Rs...>*) {
  const int want[] = {Rs...};
  if (p.nrad != (int)sizeof...(Rs)) return false;
  for (int i = 0; i < p.nrad; ++i)
    if (p.radices[i] != want[i]) return false;
  return true;
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
