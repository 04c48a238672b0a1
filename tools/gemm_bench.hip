// Microbenchmark of the fp32 MFMA GEMM variants on the block's shapes.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench.hip -lrocblas -o tools/bin/gemm_bench
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>
#include <rocblas/rocblas.h>

#include "../modulated-spherical-fourier-neural-operator_amd/csrc/gemm.hip"

using namespace msfno;

void msfno::set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); }

template <int BM, int BN, int BK>
float run(const char* name, int M, int N, int K, float* A, float* B, float* C, const GemmEpi& e,
          int reps, double flops) {
  GemmParams p = make_params(A, B, C, e);
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = N; p.ldc = N;
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + BN - 1) / BN;
  p.vecA = p.vecB = 1;
  dim3 grid(p.tiles_m * p.tiles_n, 1, 1);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) launch<BM, BN, BK>(p, grid, 0);
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) launch<BM, BN, BK>(p, grid, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  printf("%-10s BM=%d BN=%d BK=%d M=%d N=%d K=%d: %.3f ms  %.1f TF/s\n", name, BM, BN, BK, M, N, K,
         ms, flops / ms / 1e9);
  return ms;
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  const int P = 721 * 1440;
  size_t maxA = 1024 * 1024, maxB = (size_t)512 * P, maxC = (size_t)512 * P;
  float *A, *B, *C, *D, *bias;
  hipMalloc(&A, maxA * 4);
  hipMalloc(&B, maxB * 4);
  hipMalloc(&C, maxC * 4);
  hipMalloc(&D, maxC * 4);
  hipMalloc(&bias, 4096 * 4);
  std::vector<float> h(maxA);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), maxA * 4, hipMemcpyHostToDevice);
  hipMemset(B, 0, maxB * 4);
  {  // random-ish B
    std::vector<float> hb(1 << 24);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = (float)((i * 40503u) % 997) / 997.f - 0.5f;
    for (size_t off = 0; off < maxB; off += hb.size())
      hipMemcpy(B + off, hb.data(), std::min(hb.size(), maxB - off) * 4, hipMemcpyHostToDevice);
  }
  GemmEpi plain;
  GemmEpi gelu; gelu.bias = bias; gelu.act = 1;
  GemmEpi skipe; skipe.bias = bias; skipe.addend = D; skipe.ldd = P;
  GemmEpi skipb; skipb.bias = bias;
  GemmEpi relu; relu.relu_period = 1024; relu.relu_rows = 512;
  GemmEpi fc2e; fc2e.bias = bias; fc2e.addend = D; fc2e.ldd = P;
  GemmEpi fc2g = fc2e; fc2g.act = 2;
  GemmEpi geluB; geluB.act = 2; geluB.bias = bias;
  const int T = 65536;
  struct S { const char* n; int M, N, K; GemmEpi e; };
  std::vector<S> shapes = {
      {"fc2", 256, P, 512, plain}, {"fc2-geluB", 256, P, 512, geluB}, {"spec-relu", 1024, 65536, 1024, relu}, {"fc1", 512, P, 256, plain}, {"fc1-gelu", 512, P, 256, gelu},
      {"fc2-badd", 256, P, 512, fc2e}, {"skip", 256, P, 256, skipb}, {"spec", 1024, 65536, 1024, plain},
      {"fc2-full", 256, P, 512, fc2g}};
  for (auto& s : shapes) {
    if (only && std::string(s.n) != only) continue;
    const double fl = 2.0 * s.M * (double)s.N * s.K;
    run<128, 128, 16>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
    run<128, 64, 16>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
    run<256, 64, 16>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
    run<256, 128, 16>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
    run<128, 256, 16>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
    run<128, 128, 32>(s.n, s.M, s.N, s.K, A, B, C, s.e, 5, fl);
  }
  // rocBLAS sgemm on the same row-major problem: C^T = B^T A^T (column-major)
  if (only) return 0;
  rocblas_handle rh;
  rocblas_create_handle(&rh);
  const float one = 1.f, zero = 0.f;
  struct G { int M, N, K; };
  for (G g : {G{256, P, 512}, G{512, P, 256}, G{256, P, 256}, G{1024, 65536, 1024}}) {
    for (int i = 0; i < 2; ++i)
      rocblas_sgemm(rh, rocblas_operation_none, rocblas_operation_none, g.N, g.M, g.K, &one, B, g.N,
                    A, g.K, &zero, C, g.N);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    for (int i = 0; i < 5; ++i)
      rocblas_sgemm(rh, rocblas_operation_none, rocblas_operation_none, g.N, g.M, g.K, &one, B, g.N,
                    A, g.K, &zero, C, g.N);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("rocblas M=%d N=%d K=%d: %.3f ms %.1f TF/s\n", g.M, g.N, g.K, ms,
           2.0 * g.M * (double)g.N * g.K / ms / 1e9);
  }
  return 0;
}
