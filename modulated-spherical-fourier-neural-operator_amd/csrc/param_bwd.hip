// Kernels of the parameter gradients (--retrain-film, MSFNO/Models/sfno/model.py:922-923,
// 1016-1019 and main.py:958-960: the decoder and the last film_layers blocks train with
// the FiLM generator; block_bwd.cpp, api.cpp msfno_mlp_backward_params):
//   * wgrad_nt: C[m][n] = sum_b sum_k A_b[m][k] B'_b[n][k] -- a weight gradient whose
//     reduction runs over pixels (1x1 convs: dW = dY X^T) or over spectral modes (the
//     spectral MLP: dW = conj(X)^T G as two real products on interleaved complex rows).
//     B' is B, or B with a per-(batch, row) affine (the MLP input a x1 + t), GELU(B) (the
//     fc2 input), or the complex pair swap (re, im) -> (im, -re) (the imaginary part of
//     conj(x) g).  Split over K; fp32 partial sums per chunk, combined in fp64.
//   * lin_wgrad: the linear filter's per-mode gradient dw[k][i][t] = sum_b g[b][k][t]
//     conj(a[b][i][t]) (einsum "bin,kin->bkn", contractions.py:37-41).
//   * norm_param_grad: InstanceNorm affine gradients dw_c = sum_b f_bc sum_p g n,
//     db_c = sum_b f_bc sum_p g (n the normalised input, f = 1 + gamma s for a FiLM'd norm1)
//     and plain bias gradients (x null: db only), row sums in fp64.
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace msfno {

namespace {

constexpr int WG_T = 64;   // C tile (rows and columns)
constexpr int WG_K = 32;   // k per LDS stage
constexpr int WG_KC = 4096;  // k per workgroup (one fp32 partial)

template <int MODE>
__device__ __forceinline__ float wg_bval(const float* __restrict__ row, int64_t k, int64_t K,
                                         float sc, float sh) {
  if (k >= K) return 0.f;
  if constexpr (MODE == WGRAD_PLAIN) return row[k];
  if constexpr (MODE == WGRAD_AFFINE) return fmaf(sc, row[k], sh);
  if constexpr (MODE == WGRAD_GELU) return gelu_erf(row[k]);
  // WGRAD_CSWAP: (re, im) pairs -> (im, -re)
  return (k & 1) ? -row[k - 1] : row[k + 1];
}

// grid (N tiles, M tiles, batch * ksplit); 256 threads, 4 x 4 outputs each
template <int MODE>
__global__ __launch_bounds__(256) void wgrad_nt_kernel(
    const float* __restrict__ A, int64_t lda, int64_t sA, const float* __restrict__ B,
    int64_t ldb, int64_t sB, int M, int N, int64_t K, int ksplit, const float* __restrict__ bsc,
    const float* __restrict__ bsh, float* __restrict__ part) {
  __shared__ float As[WG_K][WG_T + 4], Bs[WG_K][WG_T + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int n0 = blockIdx.x * WG_T, m0 = blockIdx.y * WG_T;
  const int b = blockIdx.z / ksplit, ks = blockIdx.z % ksplit;
  const int64_t kb = (int64_t)ks * WG_KC, ke = min(K, kb + WG_KC);
  const float* Ab = A + (int64_t)b * sA;
  const float* Bb = B + (int64_t)b * sB;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  // staging: element e = tid + 256 i of the 64 x 32 tile: row e / 32, k e % 32
  for (int64_t k0 = kb; k0 < ke; k0 += WG_K) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, r = e >> 5, kk = e & 31;
      const int64_t k = k0 + kk;
      const int m = m0 + r, n = n0 + r;
      As[kk][r] = (m < M && k < ke) ? Ab[(int64_t)m * lda + k] : 0.f;
      float bv = 0.f;
      if (n < N && k < ke) {
        const float sc = MODE == WGRAD_AFFINE ? bsc[(int64_t)b * N + n] : 1.f;
        const float sh = MODE == WGRAD_AFFINE ? bsh[(int64_t)b * N + n] : 0.f;
        bv = wg_bval<MODE>(Bb + (int64_t)n * ldb, k, ke, sc, sh);
      }
      Bs[kk][r] = bv;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < WG_K; ++kk) {
      const float4 a = *reinterpret_cast<const float4*>(&As[kk][4 * ty]);
      const float4 v = *reinterpret_cast<const float4*>(&Bs[kk][4 * tx]);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* pp = part + (int64_t)blockIdx.z * M * N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 4 * ty + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 4 * tx + j;
      if (n < N) pp[(int64_t)m * N + n] = acc[i][j];
    }
  }
}

// C[m * ldc + n * cs] = sum over the partials (fp64)
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int nparts, int M, int N,
                                    float* __restrict__ C, int64_t ldc, int cs) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  double s = 0.0;
  for (int p = 0; p < nparts; ++p) s += (double)part[(int64_t)p * M * N + e];
  const int m = (int)(e / N), n = (int)(e % N);
  C[(int64_t)m * ldc + (int64_t)n * cs] = (float)s;
}

// dw[k][i][t] (complex) = sum_b g[b][k][t] conj(a[b][i][t])
__global__ void lin_wgrad_kernel(const float2* __restrict__ g, const float2* __restrict__ a,
                                 float2* __restrict__ dw, int B, int Co, int Ci, int64_t T) {
  const int64_t n = (int64_t)Co * Ci * T;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e % T;
    const int64_t ki = e / T;
    const int i = (int)(ki % Ci), k = (int)(ki / Ci);
    float re = 0.f, im = 0.f;
    for (int b = 0; b < B; ++b) {
      const float2 gv = g[((int64_t)b * Co + k) * T + t];
      const float2 av = a[((int64_t)b * Ci + i) * T + t];
      re = fmaf(gv.x, av.x, fmaf(gv.y, av.y, re));
      im = fmaf(gv.y, av.x, fmaf(-gv.x, av.y, im));
    }
    dw[e] = make_float2(re, im);
  }
}

// per row r = (b, c): s1 = sum_p g (x - mean) rstd (x null: 0), s0 = sum_p g, in fp64
__global__ __launch_bounds__(256) void norm_rows_kernel(const float* __restrict__ g,
                                                        const float* __restrict__ x,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int64_t P,
                                                        double* __restrict__ rows) {
  __shared__ double r0[256], r1[256];
  const int r = blockIdx.x;
  const float* gp = g + (int64_t)r * P;
  const float* xp = x ? x + (int64_t)r * P : nullptr;
  const float mu = x ? mean[r] : 0.f, rs = x ? rstd[r] : 0.f;
  double s0 = 0.0, s1 = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 256) {
    const double gv = (double)gp[p];
    s0 += gv;
    if (xp) s1 += gv * (double)((xp[p] - mu) * rs);
  }
  r0[threadIdx.x] = s0;
  r1[threadIdx.x] = s1;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r0[threadIdx.x] += r0[threadIdx.x + o];
      r1[threadIdx.x] += r1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    rows[2 * r] = r0[0];
    rows[2 * r + 1] = r1[0];
  }
}

// dw_c = sum_b f_bc s1_bc, db_c = sum_b f_bc s0_bc;  f = 1 + gamma s (gamma null: 1)
__global__ void norm_combine_kernel(const double* __restrict__ rows, const float* __restrict__ gamma,
                                    float film_scale, int B, int C, float* __restrict__ dw,
                                    float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double w = 0.0, bb = 0.0;
  for (int b = 0; b < B; ++b) {
    const int r = b * C + c;
    const double f = gamma ? 1.0 + (double)gamma[r] * (double)film_scale : 1.0;
    bb += f * rows[2 * r];
    w += f * rows[2 * r + 1];
  }
  if (dw) dw[c] = (float)w;
  if (db) db[c] = (float)bb;
}

}  // namespace

size_t wgrad_nt_workspace(int M, int N, int64_t K, int batch) {
  const int64_t ksplit = (K + WG_KC - 1) / WG_KC;
  return (size_t)batch * ksplit * M * N * sizeof(float);
}

int launch_wgrad_nt(const float* A, int64_t lda, int64_t sA, const float* B, int64_t ldb,
                    int64_t sB, int M, int N, int64_t K, int batch, int mode, const float* bsc,
                    const float* bsh, float* C, int64_t ldc, int cs, void* ws, size_t ws_bytes,
                    hipStream_t s) {
  MSFNO_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && batch > 0 && ws, MSFNO_EINVAL,
                "wgrad_nt: bad arguments");
  MSFNO_REQUIRE(mode != WGRAD_AFFINE || (bsc && bsh), MSFNO_EINVAL, "wgrad_nt: affine needs scales");
  MSFNO_REQUIRE(mode != WGRAD_CSWAP || K % 2 == 0, MSFNO_EINVAL, "wgrad_nt: complex rows");
  MSFNO_REQUIRE(ws_bytes >= wgrad_nt_workspace(M, N, K, batch), MSFNO_EWORKSPACE,
                "wgrad_nt: workspace too small");
  const int64_t ksplit = (K + WG_KC - 1) / WG_KC;
  MSFNO_REQUIRE(ksplit * batch < 65536, MSFNO_EINVAL, "wgrad_nt: K too large");
  float* part = static_cast<float*>(ws);
  const dim3 grid((unsigned)((N + WG_T - 1) / WG_T), (unsigned)((M + WG_T - 1) / WG_T),
                  (unsigned)(ksplit * batch));
#define WG_LAUNCH(MD)                                                                        \
  hipLaunchKernelGGL(wgrad_nt_kernel<MD>, grid, dim3(256), 0, s, A, lda, sA, B, ldb, sB, M, N, \
                     K, (int)ksplit, bsc, bsh, part)
  switch (mode) {
    case WGRAD_PLAIN: WG_LAUNCH(WGRAD_PLAIN); break;
    case WGRAD_AFFINE: WG_LAUNCH(WGRAD_AFFINE); break;
    case WGRAD_GELU: WG_LAUNCH(WGRAD_GELU); break;
    case WGRAD_CSWAP: WG_LAUNCH(WGRAD_CSWAP); break;
    default: MSFNO_REQUIRE(false, MSFNO_EINVAL, "wgrad_nt: bad mode");
  }
#undef WG_LAUNCH
  MSFNO_TRY(launch_check("wgrad_nt"));
  const int64_t mn = (int64_t)M * N;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, s, part,
                     (int)(ksplit * batch), M, N, C, ldc, cs);
  return launch_check("wgrad_reduce");
}

int launch_lin_wgrad(const float* g, const float* a, float* dw, int B, int Co, int Ci, int64_t T,
                     hipStream_t s) {
  MSFNO_REQUIRE(g && a && dw && B > 0 && Co > 0 && Ci > 0 && T > 0, MSFNO_EINVAL,
                "lin_wgrad: bad arguments");
  const int64_t n = (int64_t)Co * Ci * T;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(lin_wgrad_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<const float2*>(g), reinterpret_cast<const float2*>(a),
                     reinterpret_cast<float2*>(dw), B, Co, Ci, T);
  return launch_check("lin_wgrad");
}

size_t norm_param_grad_workspace(int B, int C) { return (size_t)B * C * 2 * sizeof(double); }

int launch_norm_param_grad(const float* g, const float* x, const float* mean, const float* rstd,
                           const float* gamma, float film_scale, int B, int C, int64_t P,
                           float* dw, float* db, void* ws, hipStream_t s) {
  MSFNO_REQUIRE(g && ws && B > 0 && C > 0 && P > 0 && (dw == nullptr || (x && mean && rstd)),
                MSFNO_EINVAL, "norm_param_grad: bad arguments");
  if (!dw && !db) return MSFNO_OK;
  double* rows = static_cast<double*>(ws);
  hipLaunchKernelGGL(norm_rows_kernel, dim3((unsigned)(B * C)), dim3(256), 0, s, g,
                     dw ? x : nullptr, mean, rstd, P, rows);
  MSFNO_TRY(launch_check("norm_rows"));
  hipLaunchKernelGGL(norm_combine_kernel, dim3((C + 255) / 256), dim3(256), 0, s, rows, gamma,
                     film_scale, B, C, dw, db);
  return launch_check("norm_combine");
}

}  // namespace msfno
