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

}  // namespace msfno
