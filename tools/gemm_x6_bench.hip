// fp32 MFMA GEMM vs the bf16x6 split GEMM: speed on the block's 1x1-conv shapes
// and accuracy against an fp64 host reference.
// Build: see tools/build_tools.sh (links the in-tree libmsfno.so)
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "common.h"

using namespace msfno;

static float frand(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((s >> 40) & 0xffffff) / (float)0x1000000 * 2.f - 1.f;
}

int main(int argc, char** argv) {
  // usage: gemm_x6_bench [shape [x6 tile id]]  (tile only: run just that x6 config)
  const char* only = argc > 1 ? argv[1] : nullptr;
  const int only_tile = argc > 2 ? atoi(argv[2]) : -1;
  const int P = 721 * 1440;
  size_t maxB = (size_t)512 * P;
  float *A, *B, *C, *D, *bias;
  void* ws;
  hipMalloc(&A, 1024 * 1024 * 4);
  hipMalloc(&B, maxB * 4);
  hipMalloc(&C, maxB * 4);
  hipMalloc(&D, maxB * 4);
  hipMalloc(&bias, 4096 * 4);
  const size_t wsb = gemm_x6_workspace(1024, 4096, 1);
  hipMalloc(&ws, wsb);
  uint64_t seed = 1;
  {
    std::vector<float> h(1024 * 1024);
    for (auto& v : h) v = 0.05f * frand(seed);
    hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> hb(1 << 24);
    for (auto& v : hb) v = frand(seed);
    for (size_t off = 0; off < maxB; off += hb.size()) {
      hipMemcpy(B + off, hb.data(), std::min(hb.size(), maxB - off) * 4, hipMemcpyHostToDevice);
      hipMemcpy(D + off, hb.data(), std::min(hb.size(), maxB - off) * 4, hipMemcpyHostToDevice);
    }
    hipMemcpy(bias, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  }
  GemmEpi gelu; gelu.bias = bias; gelu.act = 1;
  GemmEpi badd; badd.bias = bias; badd.addend = D; badd.ldd = P;
  GemmEpi sb; sb.bias = bias;
  struct S { const char* n; int M, K; GemmEpi e; GemmTile t32; };
  std::vector<S> shapes = {{"fc1-gelu", 512, 256, gelu, TILE_128x256},
                           {"fc2-badd", 256, 512, badd, TILE_256x128},
                           {"skip", 256, 256, sb, TILE_128x256}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](auto&& fn) {
    for (int i = 0; i < 2; ++i) fn();
    hipEventRecord(e0, 0);
    for (int i = 0; i < 5; ++i) fn();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
  };
  for (auto& s : shapes) {
    if (only && std::string(s.n) != only) continue;
    const double fl = 2.0 * s.M * (double)P * s.K;
    float ms;
    if (only_tile < 0) {
      ms = timeit([&] {
        gemm_uniform(s.t32, A, B, C, s.M, P, s.K, s.K, P, P, 0, 0, 0, 1, s.e, 0);
      });
      printf("%-9s f32  tile=%d: %.3f ms %.1f TF/s\n", s.n, (int)s.t32, ms, fl / ms / 1e9);
    }
    for (GemmTile t : {TILE_128x128, TILE_256x128, TILE_128x256, TILE_256x256}) {
      if (only_tile >= 0 && (int)t != only_tile) continue;
      ms = timeit([&] {
        gemm_x6(t, A, B, C, s.M, P, s.K, s.K, P, P, 0, 0, 0, 1, s.e, ws, wsb, 0);
      });
      printf("%-9s x6   tile=%d: %.3f ms %.1f TF/s (fp32-equivalent)\n", s.n, (int)t, ms,
             fl / ms / 1e9);
    }
  }
  // custom x6 shape (fp32 B split in-kernel): gemm_x6_bench x6 M N K [epi bits: 1 bias,
  // 2 add, 4 gelu] [tile id]
  if (only && std::string(only) == "x6" && argc >= 5) {
    const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), ep = argc > 5 ? atoi(argv[5]) : 0;
    const GemmTile t = argc > 6 ? (GemmTile)atoi(argv[6]) : TILE_256x256;
    GemmEpi e;
    if (ep & 1) e.bias = bias;
    if (ep & 2) { e.addend = D; e.ldd = N; }
    if (ep & 4) e.act = 1;
    const double fl = 2.0 * M * (double)N * K;
    float ms = timeit([&] { gemm_x6(t, A, B, C, M, N, K, K, N, N, 0, 0, 0, 1, e, ws, wsb, 0); });
    printf("x6 M=%d N=%d K=%d epi=%d tile=%d: %.3f ms %.1f TF/s (fp32-equivalent)\n", M, N, K, ep,
           (int)t, ms, fl / ms / 1e9);
    return 0;
  }
  // custom x6p shape: gemm_x6_bench x6p M N K [epi: 0 none, 1 bias, 3 bias+add]
  if (only && std::string(only) == "x6p" && argc >= 6) {
    const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), ep = argc > 5 ? atoi(argv[5]) : 0;
    const int ldp = (N + 7) / 8 * 8;
    unsigned short* Bp;
    hipMalloc(&Bp, (size_t)3 * K * ldp * 2);
    launch_split_planes(B, Bp, K, N, N, 0, ldp, (int64_t)K * ldp, 0, 1, 0);
    GemmEpi e;
    if (ep & 1) e.bias = bias;
    if (ep & 2) { e.addend = D; e.ldd = N; }
    e.b_planes = Bp;
    e.b_plane_stride = (int64_t)K * ldp;
    const double fl = 2.0 * M * (double)N * K;
    float ms = timeit([&] { gemm_x6p(A, C, M, N, K, K, ldp, N, 0, 0, 0, 1, e, ws, wsb, 0); });
    printf("x6p M=%d N=%d K=%d epi=%d: %.3f ms %.1f TF/s (fp32-equivalent)\n", M, N, K, ep, ms,
           fl / ms / 1e9);
    return 0;
  }
  // x6p (both operands as bf16x3 planes, LDS-DMA ring): fc2 shape, B = h planes
  if (!only || std::string(only) == "fc2p" || std::string(only) == "fc1p") {
    const bool f1 = only && std::string(only) == "fc1p";
    const int M = f1 ? 512 : 256, K = f1 ? 256 : 512;
    const int ldp = (P + 7) / 8 * 8;
    unsigned short* Bp;
    hipMalloc(&Bp, (size_t)3 * K * ldp * 2);
    launch_split_planes(B, Bp, K, P, P, 0, ldp, (int64_t)K * ldp, 0, 1, 0);
    GemmEpi e = f1 ? gelu : badd;
    if (f1) e.act = 0;  // fp32-output x6p has no GELU epilogue (fc1 writes planes)
    e.b_planes = Bp;
    e.b_plane_stride = (int64_t)K * ldp;
    const double fl = 2.0 * M * (double)P * K;
    float ms = timeit([&] { gemm_x6p(A, C, M, P, K, K, ldp, P, 0, 0, 0, 1, e, ws, wsb, 0); });
    printf("%-9s x6p  256x256: %.3f ms %.1f TF/s (fp32-equivalent)\n", f1 ? "fc1p" : "fc2p", ms,
           fl / ms / 1e9);
    GemmEpi e0 = f1 ? gelu : badd;
    if (f1) e0.act = 0;
    gemm_x6(TILE_256x256, A, B, D, M, P, K, K, P, P, 0, 0, 0, 1, e0, ws, wsb, 0);
    std::vector<float> h1((size_t)M * P), h2((size_t)M * P);
    hipMemcpy(h1.data(), C, h1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), D, h2.size() * 4, hipMemcpyDeviceToHost);
    double dmax = 0, vmax = 0;
    for (size_t i = 0; i < h1.size(); ++i) {
      dmax = std::max(dmax, (double)std::fabs(h1[i] - h2[i]));
      vmax = std::max(vmax, (double)std::fabs(h2[i]));
    }
    printf("x6p vs x6: max|diff| %.3e (max|C| %.3e)\n", dmax, vmax);
    hipFree(Bp);
  }
  if (hipGetLastError() != hipSuccess) { printf("launch error\n"); return 1; }
  if (only_tile >= 0) return 0;
  // accuracy: M=256 N=4100 (ragged) K=520 (ragged), plain epilogue
  {
    const int M = 256, N = 4100, K = 520;
    std::vector<float> ha((size_t)M * K), hb((size_t)K * N);
    for (auto& v : ha) v = 0.05f * frand(seed);
    for (auto& v : hb) v = frand(seed);
    float *dA, *dB, *dC;
    hipMalloc(&dA, ha.size() * 4);
    hipMalloc(&dB, hb.size() * 4);
    hipMalloc(&dC, (size_t)M * N * 4);
    hipMemcpy(dA, ha.data(), ha.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
    std::vector<double> ref((size_t)M * N, 0.0), mag((size_t)M * N, 0.0);
    for (int m = 0; m < M; ++m)
      for (int k = 0; k < K; ++k) {
        const double a = ha[(size_t)m * K + k];
        for (int n = 0; n < N; ++n) {
          ref[(size_t)m * N + n] += a * hb[(size_t)k * N + n];
          mag[(size_t)m * N + n] += std::fabs(a * hb[(size_t)k * N + n]);
        }
      }
    std::vector<float> hc((size_t)M * N);
    GemmEpi none;
    for (int mode = 0; mode < 5; ++mode) {
      hipMemset(dC, 0, (size_t)M * N * 4);
      int rc;
      if (mode == 0)
        rc = gemm_uniform(TILE_128x128, dA, dB, dC, M, N, K, K, N, N, 0, 0, 0, 1, none, 0);
      else
        rc = gemm_x6(mode == 1 ? TILE_128x128 : mode == 2 ? TILE_256x128 : mode == 3 ? TILE_128x256 : TILE_256x256, dA, dB,
                     dC, M, N, K, K, N, N, 0, 0, 0, 1, none, ws, wsb, 0);
      hipMemcpy(hc.data(), dC, hc.size() * 4, hipMemcpyDeviceToHost);
      double emax = 0, erel = 0;
      for (size_t i = 0; i < hc.size(); ++i) {
        const double e = std::fabs(hc[i] - ref[i]);
        emax = std::max(emax, e);
        erel = std::max(erel, e / mag[i]);
      }
      printf("accuracy %s rc=%d: max|err| %.3e  max|err|/sum|ab| %.3e\n",
             mode == 0 ? "f32 " : mode == 1 ? "x6/128x128" : mode == 2 ? "x6/256x128" : mode == 3 ? "x6/128x256" : "x6/256x256",
             rc, emax, erel);
    }
  }
  return 0;
}
