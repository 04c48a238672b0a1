// Kernels of the FiLM backward (gradients to gamma and beta
// only, the SFNO weights frozen; MSFNO/train.py fine-tunes the FiLM generator):
//   * transpose of a small weight matrix (the GEMMs of the backward need W^T),
//   * dh *= GELU'(pre) (exact erf GELU, activations of layers.py:145-178),
//   * per-(b, c) reductions  dgamma = s * sum_p du * xhat,  dbeta = s * sum_p du
//     with xhat = a * x1 + t the InstanceNorm-1 output (sfnonet.py:376-378,
//     FiLM sfnonet.py:689-697), accumulated in fp64.
#include "kernels.h"

namespace msfno {

// AT (cols x rows, ld rows) = A (rows x cols, ld lda)^T
__global__ void transpose_mat_kernel(const float* __restrict__ A, int rows, int cols, int lda,
                                     float* __restrict__ AT) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (r < rows && c < cols) ? A[(int64_t)r * lda + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (c < cols && r < rows) AT[(int64_t)c * rows + r] = tile[threadIdx.x][i];
  }
}

int launch_transpose_mat(const float* A, int rows, int cols, int lda, float* AT, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return MSFNO_OK;
  dim3 grid((unsigned)cdiv(cols, 32), (unsigned)cdiv(rows, 32));
  hipLaunchKernelGGL(transpose_mat_kernel, grid, dim3(32, 8), 0, s, A, rows, cols, lda, AT);
  return launch_check("transpose_mat");
}

// d/dz [0.5 z (1 + erf(z / sqrt 2))] = Phi(z) + z phi(z)
__global__ void gelu_grad_mul_kernel(float* __restrict__ dh, const float* __restrict__ pre,
                                     int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float z = pre[e];
    const float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752440f));
    const float pdf = 0.39894228040143267794f * expf(-0.5f * z * z);
    dh[e] *= cdf + z * pdf;
  }
}

int launch_gelu_grad_mul(float* dh, const float* pre, int64_t n, hipStream_t s) {
  if (n <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(gelu_grad_mul_kernel, dim3(blocks), dim3(256), 0, s, dh, pre, n);
  return launch_check("gelu_grad_mul");
}

// one workgroup per (b, c) row of P pixels
__global__ __launch_bounds__(256) void film_grad_reduce_kernel(
    const float* __restrict__ du, const float* __restrict__ x1, const float* __restrict__ an,
    const float* __restrict__ tn, float scale, int64_t P, float* __restrict__ dgamma,
    float* __restrict__ dbeta) {
  __shared__ double sg[256], sb[256];
  const int bc = blockIdx.x;
  const float a = an[bc], t = tn[bc];
  const float* g = du + (int64_t)bc * P;
  const float* v = x1 + (int64_t)bc * P;
  double accg = 0.0, accb = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 256) {
    const float gp = g[p];
    accg += (double)gp * (double)fmaf(a, v[p], t);
    accb += (double)gp;
  }
  sg[threadIdx.x] = accg;
  sb[threadIdx.x] = accb;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sg[threadIdx.x] += sg[threadIdx.x + o];
      sb[threadIdx.x] += sb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    dgamma[bc] = (float)(scale * sg[0]);
    dbeta[bc] = (float)(scale * sb[0]);
  }
}

int launch_film_grad_reduce(const float* du, const float* x1, const float* an, const float* tn,
                            float scale, int BC, int64_t P, float* dgamma, float* dbeta,
                            hipStream_t s) {
  if (BC <= 0) return MSFNO_OK;
  hipLaunchKernelGGL(film_grad_reduce_kernel, dim3(BC), dim3(256), 0, s, du, x1, an, tn, scale, P,
                     dgamma, dbeta);
  return launch_check("film_grad_reduce");
}


// ---------------------------------------------------------------------------
// Kernels of the full block backward (dL/dx through a filmed block, block_bwd.cpp)
// ---------------------------------------------------------------------------

// per row r = (b, c) of P values: mean, 1 / sqrt(var + eps) (biased variance, two passes
// in fp64: InstanceNorm2d, sfnonet.py:491-499) and the affine of the normalised row,
// scale = w_c rstd, shift = b_c - w_c mean rstd (w, b null: 1, 0)
__global__ __launch_bounds__(256) void row_moments_kernel(
    const float* __restrict__ x, int C, int64_t P, const float* __restrict__ w,
    const float* __restrict__ b, float eps, float* __restrict__ mean, float* __restrict__ rstd,
    float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ double red[256];
  const int r = blockIdx.x, c = r % C;
  const float* v = x + (int64_t)r * P;
  double acc = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 256) acc += (double)v[p];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double mu = red[0] / (double)P;
  __syncthreads();
  acc = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 256) {
    const double d = (double)v[p] - mu;
    acc += d * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double rs = 1.0 / sqrt(red[0] / (double)P + (double)eps);
    const double wc = w ? (double)w[c] : 1.0, bc = b ? (double)b[c] : 0.0;
    mean[r] = (float)mu;
    rstd[r] = (float)rs;
    if (scale) scale[r] = (float)(wc * rs);
    if (shift) shift[r] = (float)(bc - wc * mu * rs);
  }
}

int launch_row_moments(const float* x, int64_t rows, int C, int64_t P, const float* w,
                       const float* b, float eps, float* mean, float* rstd, float* scale,
                       float* shift, hipStream_t s) {
  MSFNO_REQUIRE(rows > 0 && rows < (1LL << 31) && C > 0 && P > 0, MSFNO_EINVAL,
                "row_moments: bad sizes");
  hipLaunchKernelGGL(row_moments_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, C, P, w, b, eps,
                     mean, rstd, scale, shift);
  return launch_check("row_moments");
}

// InstanceNorm backward per row r = (b, c):  y = w_c n + b_c, n = (x - mean) rstd;
// dn = w_c f_r g with the FiLM factor f_r = 1 + gamma_r s (gamma null: 1);
// dx = rstd (dn - mean(dn) - n mean(dn n)) (+ add1 + add2)
__global__ __launch_bounds__(256) void inorm_backward_kernel(
    const float* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ w, const float* __restrict__ gamma, float film_scale,
    const float* __restrict__ g, const float* __restrict__ add1, const float* __restrict__ add2,
    float* __restrict__ dx, int C, int64_t P) {
  __shared__ double r1[256], r2[256];
  const int r = blockIdx.x, c = r % C;
  const float f = (w ? w[c] : 1.f) * (gamma ? 1.f + gamma[r] * film_scale : 1.f);
  const float mu = mean[r], rs = rstd[r];
  const int64_t o = (int64_t)r * P;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 256) {
    const double dn = (double)(f * g[o + p]);
    s1 += dn;
    s2 += dn * (double)((x[o + p] - mu) * rs);
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      r1[threadIdx.x] += r1[threadIdx.x + k];
      r2[threadIdx.x] += r2[threadIdx.x + k];
    }
    __syncthreads();
  }
  const float m1 = (float)(r1[0] / (double)P), m2 = (float)(r2[0] / (double)P);
  for (int64_t p = threadIdx.x; p < P; p += 256) {
    const float n = (x[o + p] - mu) * rs;
    float v = rs * (f * g[o + p] - m1 - n * m2);
    if (add1) v += add1[o + p];
    if (add2) v += add2[o + p];
    dx[o + p] = v;
  }
}

int launch_inorm_backward(const float* x, const float* mean, const float* rstd, const float* w,
                          const float* gamma, float film_scale, const float* g, const float* add1,
                          const float* add2, float* dx, int64_t rows, int C, int64_t P,
                          hipStream_t s) {
  MSFNO_REQUIRE(rows > 0 && rows < (1LL << 31) && C > 0 && P > 0, MSFNO_EINVAL,
                "inorm_backward: bad sizes");
  hipLaunchKernelGGL(inorm_backward_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, mean, rstd, w,
                     gamma, film_scale, g, add1, add2, dx, C, P);
  return launch_check("inorm_backward");
}

// ComplexReLU("real") backward (activations.py:42-46): the real part of the gradient
// passes where the forward's real part was positive (h = the post-ReLU activation)
__global__ void relu_real_mask_kernel(float2* __restrict__ dh, const float2* __restrict__ h,
                                      int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x)
    if (!(h[e].x > 0.f)) dh[e].x = 0.f;
}

int launch_relu_real_mask(float* dh, const float* h, int64_t n, hipStream_t s) {
  if (n <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(relu_real_mask_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<float2*>(dh), reinterpret_cast<const float2*>(h), n);
  return launch_check("relu_real_mask");
}

// wt[k][i][t] = conj(w[i][k][t]) for complex w (I, K, T): the adjoint of a complex
// linear map y = w x (T = 1: the spectral-MLP weights (Ci, Co, 2) -> (Co, Ci, 2); T = the
// tril modes: the linear filter's (Co, Ci, T, 2) -> (Ci, Co, T, 2))
__global__ void conj_swap01_kernel(const float2* __restrict__ w, float2* __restrict__ wt, int I,
                                   int K, int64_t T) {
  const int64_t pairs = (int64_t)I * K;
  for (int64_t q = blockIdx.x; q < pairs; q += gridDim.x) {
    const int i = (int)(q / K), k = (int)(q - (int64_t)i * K);
    const float2* src = w + q * T;
    float2* dst = wt + ((int64_t)k * I + i) * T;
    for (int64_t t = threadIdx.x; t < T; t += blockDim.x) {
      const float2 v = src[t];
      dst[t] = make_float2(v.x, -v.y);
    }
  }
}

int launch_conj_swap01(const float* w, int I, int K, int64_t T, float* wt, hipStream_t s) {
  if (I <= 0 || K <= 0 || T <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>((int64_t)I * K, 65536);
  hipLaunchKernelGGL(conj_swap01_kernel, dim3(blocks), dim3(T >= 256 ? 256 : 64), 0, s,
                     reinterpret_cast<const float2*>(w), reinterpret_cast<float2*>(wt), I, K, T);
  return launch_check("conj_swap01");
}

// index of (l, m) in torch.tril_indices(lmax, mmax) order (layers.py:368): row l holds
// m = 0 .. min(l, mmax - 1)
__device__ __forceinline__ int64_t tril_index(int l, int m, int mmax) {
  const int64_t lc = min(l, mmax);
  return lc * (lc + 1) / 2 + (int64_t)(l - lc) * mmax + m;
}

// dense (rows, lmax, mmax) complex <-> tril (rows, T) complex; scatter writes zeros off the
// triangle
template <bool GATHER>
__global__ void tril_map_kernel(const float2* __restrict__ src, float2* __restrict__ dst,
                                int lmax, int mmax, int64_t T) {
  const int64_t LM = (int64_t)lmax * mmax;
  const int64_t r = blockIdx.y;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < LM;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(e / mmax), m = (int)(e - (int64_t)l * mmax);
    const bool in = m <= l;
    if constexpr (GATHER) {
      if (in) dst[r * T + tril_index(l, m, mmax)] = src[r * LM + e];
    } else {
      dst[r * LM + e] = in ? src[r * T + tril_index(l, m, mmax)] : make_float2(0.f, 0.f);
    }
  }
}

int launch_tril_map(const float* src, float* dst, int64_t rows, int lmax, int mmax, int64_t T,
                    bool gather, hipStream_t s) {
  MSFNO_REQUIRE(rows > 0 && rows < 65536 && lmax > 0 && mmax > 0, MSFNO_EINVAL,
                "tril_map: bad sizes");
  const int64_t LM = (int64_t)lmax * mmax;
  dim3 grid((unsigned)std::min<int64_t>(cdiv(LM, 256), 1024), (unsigned)rows);
  const float2* a = reinterpret_cast<const float2*>(src);
  float2* b = reinterpret_cast<float2*>(dst);
  if (gather)
    hipLaunchKernelGGL(tril_map_kernel<true>, grid, dim3(256), 0, s, a, b, lmax, mmax, T);
  else
    hipLaunchKernelGGL(tril_map_kernel<false>, grid, dim3(256), 0, s, a, b, lmax, mmax, T);
  return launch_check("tril_map");
}

__global__ void fill_kernel(float* __restrict__ p, int64_t n, float v) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x)
    p[e] = v;
}

int launch_fill(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return MSFNO_OK;
  const int blocks = (int)std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(fill_kernel, dim3(blocks), dim3(256), 0, s, p, n, v);
  return launch_check("fill");
}

// u = (1 + gamma s)(an x1 + tn) + beta s = sc x1 + sh per (b, c) (FiLM, sfnonet.py:689-697)
__global__ void film_affine_kernel(const float* __restrict__ an, const float* __restrict__ tn,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float s, float* __restrict__ sc, float* __restrict__ sh,
                                   int64_t n) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float f = 1.f + gamma[e] * s;
    sc[e] = f * an[e];
    sh[e] = f * tn[e] + beta[e] * s;
  }
}

int launch_film_affine(const float* an, const float* tn, const float* gamma, const float* beta,
                       float film_scale, float* sc, float* sh, int64_t n, hipStream_t s) {
  if (n <= 0) return MSFNO_OK;
  hipLaunchKernelGGL(film_affine_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, an, tn,
                     gamma, beta, film_scale, sc, sh, n);
  return launch_check("film_affine");
}

}  // namespace msfno
