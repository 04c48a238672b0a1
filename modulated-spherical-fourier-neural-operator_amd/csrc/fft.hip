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
#include <cmath>

#include "kernels.h"

namespace msfno {

struct FFTArgs {
  int N, H, packed, nrad;
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
    // generic small prime: direct DFT with roots from the H-point table
    float2 y[R];
    const int st = H / R;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      float2 acc = v[0];
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float2 w = twH[((q * r) % R) * st];
        if (INV) w.y = -w.y;
        acc = cadd(acc, cmul(v[r], w));
      }
      y[q] = acc;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = y[q];
  }
}

template <int R, bool INV>
__device__ __forceinline__ void stockham_pass(const float2* __restrict__ in, float2* __restrict__ out,
                                              int H, int Ns, const float2* twH, int lane) {
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
        float2 w = twH[r * k * step];
        if (INV) w.y = -w.y;
        v[r] = cmul(v[r], w);
      }
    }
    butterfly<R, INV>(v, twH, H);
    const int base = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) out[base + r * Ns] = v[r];
  }
}

// Runs all passes; returns the buffer holding the natural-order result.
template <bool INV>
__device__ float2* run_fft(float2* a, float2* b, const FFTArgs& f, int lane) {
  int Ns = 1;
  for (int p = 0; p < f.nrad; ++p) {
    const int R = f.radices[p];
    switch (R) {
      case 4: stockham_pass<4, INV>(a, b, f.H, Ns, f.twH, lane); break;
      case 2: stockham_pass<2, INV>(a, b, f.H, Ns, f.twH, lane); break;
      case 3: stockham_pass<3, INV>(a, b, f.H, Ns, f.twH, lane); break;
      case 5: stockham_pass<5, INV>(a, b, f.H, Ns, f.twH, lane); break;
      case 7: stockham_pass<7, INV>(a, b, f.H, Ns, f.twH, lane); break;
      case 11: stockham_pass<11, INV>(a, b, f.H, Ns, f.twH, lane); break;
      default: stockham_pass<13, INV>(a, b, f.H, Ns, f.twH, lane); break;
    }
    Ns *= R;
    __syncthreads();
    float2* t = a; a = b; b = t;
  }
  return a;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

constexpr int kRowsPerWG = 4;

__global__ __launch_bounds__(256) void fft_r2c_rows_kernel(const float* __restrict__ x,
                                                           float2* __restrict__ out,
                                                           float2* __restrict__ rowstats,
                                                           int64_t rows, int mmax, float scale,
                                                           FFTArgs f) {
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerWG + w;
  const bool valid = row < rows;
  const int H = f.H, N = f.N;
  float2* bA = smem + (size_t)w * 2 * H;
  float2* bB = bA + H;

  float s = 0.f;
  if (valid) {
    const float* xr = x + row * N;
    if (f.packed) {
      const float2* x2 = reinterpret_cast<const float2*>(xr);
      for (int n = lane; n < H; n += 64) {
        const float2 v = x2[n];
        bA[n] = v;
        s += v.x + v.y;
      }
    } else {
      for (int n = lane; n < N; n += 64) {
        const float v = xr[n];
        bA[n] = make_float2(v, 0.f);
        s += v;
      }
    }
  }
  if (rowstats) {
    const float mean = wave_sum(s) / (float)N;
    float q = 0.f;
    if (valid) {
      for (int n = lane; n < H; n += 64) {
        const float2 v = bA[n];
        const float d0 = v.x - mean;
        q += d0 * d0;
        if (f.packed) {
          const float d1 = v.y - mean;
          q += d1 * d1;
        }
      }
    }
    q = wave_sum(q);
    if (valid && lane == 0) rowstats[row] = make_float2(mean, q);
  }
  __syncthreads();
  float2* Z = run_fft<false>(bA, bB, f, lane);
  if (!valid) return;
  float2* o = out + row * mmax;
  if (f.packed) {
    for (int k = lane; k < mmax; k += 64) {
      const float2 zk = Z[k % H];
      const float2 zc = cconj(Z[(H - k) % H]);
      const float2 E = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
      const float2 D = csub(zk, zc);
      const float2 O = make_float2(0.5f * D.y, -0.5f * D.x);  // D / (2i)
      const float2 X = cadd(E, cmul(f.twN[k], O));
      o[k] = make_float2(scale * X.x, scale * X.y);
    }
  } else {
    for (int k = lane; k < mmax; k += 64) {
      const float2 X = Z[k];
      o[k] = make_float2(scale * X.x, scale * X.y);
    }
  }
}

__device__ __forceinline__ float gelu_erf_f(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}

__global__ __launch_bounds__(256) void fft_c2r_rows_kernel(const float2* __restrict__ in,
                                                           float* __restrict__ x,
                                                           float2* __restrict__ rowstats,
                                                           int64_t rows, int mmax, int act,
                                                           FFTArgs f) {
  extern __shared__ float2 smem[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerWG + w;
  const bool valid = row < rows;
  const int H = f.H, N = f.N;
  float2* bA = smem + (size_t)w * 2 * H;
  float2* bB = bA + H;
  if (valid) {
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
        bA[k] = make_float2(A.x - T.y, A.y + T.x);
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
        bA[k] = v;
      }
    }
  }
  __syncthreads();
  float2* Z = run_fft<true>(bA, bB, f, lane);
  if (!valid) return;
  float* xo = x + row * N;
  float s = 0.f;
  if (f.packed) {
    float2* x2 = reinterpret_cast<float2*>(xo);
    for (int n = lane; n < H; n += 64) {
      float2 v = Z[n];
      if (act == 1) { v.x = gelu_erf_f(v.x); v.y = gelu_erf_f(v.y); }
      x2[n] = v;
      Z[n] = v;
      s += v.x + v.y;
    }
  } else {
    for (int n = lane; n < N; n += 64) {
      float v = Z[n].x;
      if (act == 1) v = gelu_erf_f(v);
      xo[n] = v;
      Z[n].x = v;
      s += v;
    }
  }
  if (rowstats) {
    const float mean = wave_sum(s) / (float)N;
    float q = 0.f;
    if (f.packed) {
      for (int n = lane; n < H; n += 64) {
        const float2 v = Z[n];
        q += (v.x - mean) * (v.x - mean) + (v.y - mean) * (v.y - mean);
      }
    } else {
      for (int n = lane; n < N; n += 64) {
        const float v = Z[n].x;
        q += (v - mean) * (v - mean);
      }
    }
    q = wave_sum(q);
    if (lane == 0) rowstats[row] = make_float2(mean, q);
  }
}

static FFTArgs make_args(const FFTPlan& p) {
  FFTArgs a{};
  a.N = p.N; a.H = p.H; a.packed = p.packed; a.nrad = p.nrad;
  for (int i = 0; i < kMaxRadices; ++i) a.radices[i] = p.radices[i];
  a.twH = p.twH; a.twN = p.twN;
  return a;
}

int launch_fft_r2c_rows(const FFTPlan& f, const float* x, float2* out, float2* rowstats,
                        int64_t rows, int mmax, float scale, hipStream_t s) {
  if (rows <= 0) return MSFNO_OK;
  const size_t lds = (size_t)kRowsPerWG * 2 * f.H * sizeof(float2);
  MSFNO_REQUIRE(lds <= 160 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  const int64_t grid = cdiv(rows, kRowsPerWG);
  hipLaunchKernelGGL(fft_r2c_rows_kernel, dim3((unsigned)grid), dim3(256), lds, s, x, out,
                     rowstats, rows, mmax, scale, make_args(f));
  return launch_check("fft_r2c_rows");
}

int launch_fft_c2r_rows(const FFTPlan& f, const float2* in, float* x, float2* rowstats,
                        int64_t rows, int mmax, int act, hipStream_t s) {
  if (rows <= 0) return MSFNO_OK;
  const size_t lds = (size_t)kRowsPerWG * 2 * f.H * sizeof(float2);
  MSFNO_REQUIRE(lds <= 160 * 1024, MSFNO_EUNSUPPORTED, "nlon too large for the LDS FFT");
  const int64_t grid = cdiv(rows, kRowsPerWG);
  hipLaunchKernelGGL(fft_c2r_rows_kernel, dim3((unsigned)grid), dim3(256), lds, s, in, x,
                     rowstats, rows, mmax, act, make_args(f));
  return launch_check("fft_c2r_rows");
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
