// fp32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact fp32 fma chain, the
// chip's fp32 matrix peak).  Used for every dense contraction of the block:
//   * per-m Legendre contractions of the forward / inverse SHT (descriptor mode),
//   * the non-linear spectral MLP layers (complex GEMMs real-ified),
//   * the 1x1 convolutions (inner skip, MLP fc1/fc2) with fused epilogues.
// C[M,N] = A[M,K]·B[K,N], all row-major fp32.  Block tile BM×BN×16, 4 waves in
// a 2×2 arrangement, each wave owning (BM/2)×(BN/2) as 32×32 MFMA tiles.
// LDS is double buffered with one barrier per K-tile; A is staged k-major
// (transposed) so both MFMA operands are read as conflict-free ds_read_b32.
#include <cstdlib>
#include <string>

#include "gemm_common.h"

namespace msfno {

// WGM x (4 / WGM) waves: 2 x 2 (default) or 4 x 1 (the 32-column tiles: ragged
// narrow Legendre problems waste less padding)
template <int BM, int BN, int BK, bool VEC, int EPI, int WGM = 2>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int MT = WM / 32, NT = WN / 32;
  constexpr int LDA_S = BM + 2;  // staging-write conflict-free (see header)
  constexpr int LDB_S = BN;
  constexpr int A_LD = BM * BK / 1024;  // float4 staging loads per thread
  constexpr int B_LD = (BN * BK + 1023) / 1024;
  constexpr int B_N4 = BN * BK / 4;  // float4 of a B tile (< 256 for BN = 32: some threads idle)
  // one LDS array: the double-buffered A/B staging, reused by the epilogue as a
  // 64-row x (BN + 8) row-major image of the accumulators
  constexpr int CS_LD = BN + 8;
  constexpr int STAGE = 2 * BK * LDA_S + 2 * BK * LDB_S;
  constexpr int EPI_FLOATS = 32 * WGM * CS_LD;  // gemm_epilogue's row-tile image
  constexpr int LDS_FLOATS = STAGE > EPI_FLOATS ? STAGE : EPI_FLOATS;
  // + the tile's BM bias values, staged once: read from global inside the
  // epilogue they were serialised behind the C stores (possible aliasing),
  // one L2 round trip per float4 stored
  constexpr bool HAS_BIAS = (EPI & EPI_BIAS) != 0;
  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS + (HAS_BIAS ? BM : 0)];
  float* const bias_s = lds + LDS_FLOATS;
  auto As = [&](int buf) { return lds + buf * (BK * LDA_S); };
  auto Bs = [&](int buf) { return lds + 2 * BK * LDA_S + buf * (BK * LDB_S); };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  // ---- tile -> problem mapping ----------------------------------------------
  const float* A = p.A;
  const float* B = p.B;
  float* C = p.C;
  int M = p.M, N = p.N, K = p.K, lda = p.lda, ldb = p.ldb, ldc = p.ldc;
  int tm, tn;
  const float* bias = p.bias;
  const float* addend = p.addend;
  int dflags = 0;
  if (p.descs) {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    int lo = 0, hi = p.ndesc - 1;
    while (lo < hi) {  // last desc with tile_start <= lin
      const int mid = (lo + hi + 1) >> 1;
      if (p.descs[mid].tile_start <= lin) lo = mid; else hi = mid - 1;
    }
    const GemmDesc d = p.descs[lo];
    A += d.offA; B += d.offB; C += d.offC;
    M = d.M; N = d.N; K = d.K; lda = d.lda; ldb = d.ldb; ldc = d.ldc;
    dflags = d.flags;
    const int local = lin - d.tile_start;
    tm = local % d.tiles_m;
    tn = local / d.tiles_m;
  } else {
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    tm = lin % p.tiles_m;
    tn = lin / p.tiles_m;
    const int z = blockIdx.z;
    A += z * p.sA; B += z * p.sB; C += z * p.sC;
    if (bias) bias += z * p.sBias;
    if (addend) addend += z * p.sD;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    for (int r = tid; r < BM; r += 256) bias_s[r] = M > 0 ? bias[min(m0 + r, M - 1)] : 0.f;
  }  // visible after the prologue barrier


  float4 ra[A_LD], rb[B_LD];

  // Branch-free staging: loads use clamped (always in-bounds) addresses and the
  // out-of-range elements are zeroed only when the registers are written to LDS
  // (after the MFMAs of the current tile), so hipcc neither predicates the loads
  // nor waits for them before the compute.  With VEC, rows are padded to a
  // multiple of 4 floats (ld % 4 == 0), so a float4 at k < K stays in its row.
  const int Mc = M > 0 ? M - 1 : 0, Kc = K > 0 ? K - 1 : 0, Nc = N > 0 ? N - 1 : 0;
  auto load_A = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int idx = tid + 256 * q;
      const int row = min(m0 + idx / (BK / 4), Mc);
      const int k = k0 + (idx % (BK / 4)) * 4;
      const float* src = A + (int64_t)row * lda;
      if (p.segA_w) {  // band exchange layout: k-tiles never straddle a block (seg_w % 16 == 0)
        const int blk = min(k, Kc) / p.segA_w;
        src += blk * (p.segA_stride - p.segA_w);
      }
      if constexpr (VEC) {
        ra[q] = *reinterpret_cast<const float4*>(src + min(k, Kc & ~3));
      } else {
        ra[q] = make_float4(src[min(k, Kc)], src[min(k + 1, Kc)], src[min(k + 2, Kc)],
                            src[min(k + 3, Kc)]);
      }
    }
  };
  auto load_B = [&](int kt, float4* dst) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int idx = tid + 256 * q;
      if (B_N4 % 256 != 0 && idx >= B_N4) continue;  // wave-uniform (B_N4 = 128)
      const int kr = min(k0 + idx / (BN / 4), Kc);
      const int col = n0 + (idx % (BN / 4)) * 4;
      const float* src = B + (int64_t)kr * ldb;
      if constexpr (VEC) {
        dst[q] = *reinterpret_cast<const float4*>(src + min(col, Nc & ~3));
      } else {
        dst[q] = make_float4(src[min(col, Nc)], src[min(col + 1, Nc)], src[min(col + 2, Nc)],
                             src[min(col + 3, Nc)]);
      }
    }
  };
  auto store_A = [&](int buf, int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < A_LD; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx / (BK / 4);
      const int k = (idx % (BK / 4)) * 4;
      const bool rok = m0 + row < M;
      const int kg = k0 + k;
      float* dst = As(buf) + k * LDA_S + row;
      dst[0] = (rok && kg + 0 < K) ? ra[q].x : 0.f;
      dst[LDA_S] = (rok && kg + 1 < K) ? ra[q].y : 0.f;
      dst[2 * LDA_S] = (rok && kg + 2 < K) ? ra[q].z : 0.f;
      dst[3 * LDA_S] = (rok && kg + 3 < K) ? ra[q].w : 0.f;
    }
  };
  auto store_B = [&](int buf, int kt, const float4* src) {
    const int k0 = kt * BK;
#pragma unroll
    for (int q = 0; q < B_LD; ++q) {
      const int idx = tid + 256 * q;
      if (B_N4 % 256 != 0 && idx >= B_N4) continue;
      const int kr = idx / (BN / 4);
      const int col = (idx % (BN / 4)) * 4;
      const bool kok = k0 + kr < K;
      const int cg = n0 + col;
      float4 v = src[q];
      v.x = (kok && cg + 0 < N) ? v.x : 0.f;
      v.y = (kok && cg + 1 < N) ? v.y : 0.f;
      v.z = (kok && cg + 2 < N) ? v.z : 0.f;
      v.w = (kok && cg + 3 < N) ? v.w : 0.f;
      *reinterpret_cast<float4*>(Bs(buf) + kr * LDB_S + col) = v;
    }
  };

  const int half = lane >> 5;
  floatx16 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int l32 = lane & 31;
  // the MFMAs of one staged k-tile; per_kk(kk) runs after each MFMA group
  auto mfma_tile = [&](int buf, auto&& per_kk) {
    const float* as = As(buf);
    const float* bs = Bs(buf);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int k = 2 * kk + half;
      float a[MT], b[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) a[i] = as[k * LDA_S + wm * WM + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = bs[k * LDB_S + wn * WN + j * 32 + l32];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      per_kk(kk);
    }
  };

  if constexpr ((EPI & EPI_GELU_B) == 0) {
    if (nk > 0) {
      load_A(0);
      load_B(0, rb);
      store_A(0, 0);
      store_B(0, 0, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        load_A(kt + 1);
        load_B(kt + 1, rb);
      }
      mfma_tile(cur, [](int) {});
      if (kt + 1 < nk) {
        store_A(cur ^ 1, kt + 1);
        store_B(cur ^ 1, kt + 1, rb);
      }
      __syncthreads();
    }
  } else {
    // GELU(erf) of B (the MLP hidden layer) while it is staged: the next tile's
    // registers are transformed after the first MFMA groups of the current tile
    // (measured: spreading the GELUs over all groups with B loaded two tiles
    // ahead was slower, 3.50 vs 2.91 ms on fc2).
    constexpr int NE = B_LD * 4;
    auto gelu_all = [&]() {
#pragma unroll
      for (int q = 0; q < B_LD; ++q) {
        rb[q].x = gelu_erf(rb[q].x); rb[q].y = gelu_erf(rb[q].y);
        rb[q].z = gelu_erf(rb[q].z); rb[q].w = gelu_erf(rb[q].w);
      }
    };
    (void)NE;
    if (nk > 0) {
      load_A(0);
      load_B(0, rb);
      gelu_all();
      store_A(0, 0);
      store_B(0, 0, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) {
        load_A(kt + 1);
        load_B(kt + 1, rb);
      }
      mfma_tile(cur, [&](int kk) {
        if (kk == BK / 2 - 3 && more) gelu_all();
      });
      if (more) {
        store_A(cur ^ 1, kt + 1);
        store_B(cur ^ 1, kt + 1, rb);
      }
      __syncthreads();
    }
  }

  gemm_epilogue<BM, BN, EPI, WGM, WGN>(p, acc, lds, bias_s, C, addend, M, N, ldc, m0, n0, dflags);
}

GemmTile role_tile(GemmRole r, GemmTile dflt) {
  static int table[ROLE_COUNT];
  static bool init = false;
  if (!init) {
    for (int& t : table) t = -1;
    if (const char* e = getenv("MSFNO_TILES")) {
      static const char* names[ROLE_COUNT] = {"skip", "fc1", "fc2", "spec", "leg", "legi"};
      std::string spec(e);
      size_t pos = 0;
      while (pos < spec.size()) {
        size_t end = spec.find(',', pos);
        if (end == std::string::npos) end = spec.size();
        const std::string kv = spec.substr(pos, end - pos);
        const size_t eq = kv.find('=');
        if (eq != std::string::npos)
          for (int i = 0; i < ROLE_COUNT; ++i)
            if (kv.substr(0, eq) == names[i]) table[i] = atoi(kv.c_str() + eq + 1);
        pos = end + 1;
      }
    }
    init = true;
  }
  const int t = table[r];
  return (t >= 0 && t <= TILE_128x32) ? (GemmTile)t : dflt;
}

void gemm_tile_dims(GemmTile tile, int* bm, int* bn) {
  switch (tile) {
    case TILE_128x128: *bm = 128; *bn = 128; break;
    case TILE_128x64: *bm = 128; *bn = 64; break;
    case TILE_256x64: *bm = 256; *bn = 64; break;
    case TILE_256x128: *bm = 256; *bn = 128; break;
    case TILE_128x256: *bm = 128; *bn = 256; break;
    case TILE_256x256: *bm = 256; *bn = 256; break;
    case TILE_256x32: *bm = 256; *bn = 32; break;
    case TILE_128x32: *bm = 128; *bn = 32; break;
    default: *bm = 64; *bn = 64; break;
  }
}

static GemmParams make_params(const float* A, const float* B, float* C, const GemmEpi& e) {
  GemmParams p{};
  p.A = A; p.B = B; p.C = C;
  p.bias = e.bias; p.addend = e.addend;
  p.sBias = e.sBias; p.sD = e.sD;
  p.ldd = e.ldd; p.act = e.act; p.relu_period = e.relu_period; p.relu_rows = e.relu_rows;
  p.rowscale = e.rowscale;
  p.rs_C = e.rs_C;
  p.segA_w = e.segA_w; p.segA_stride = e.segA_stride;
  p.segC_w = e.segC_w; p.segC_stride = e.segC_stride;
  return p;
}

template <int BM, int BN, int BK, int EPI, int WGM = 2>
static void launch_e(const GemmParams& p, dim3 grid, hipStream_t s) {
  if (p.vecA && p.vecB)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, true, EPI, WGM>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, false, EPI, WGM>), grid, dim3(256), 0, s, p);
}



static int epi_code(const GemmParams& p) {
  return (p.bias ? EPI_BIAS : 0) | (p.addend ? EPI_ADD : 0) | (p.act == 1 ? EPI_GELU : 0) |
         (p.relu_period ? EPI_RELU : 0) |
         (p.rowscale ? EPI_ROWSCALE : 0) | (p.act == 2 ? EPI_GELU_B : 0);
}

// the 32-column tiles (4 x 1 waves): the Legendre descriptor GEMMs only (no epilogue
// or the forward row scale)
template <int BM, int BN, int BK>
static int launch_narrow(const GemmParams& p, dim3 grid, hipStream_t s) {
  switch (epi_code(p)) {
    case 0: launch_e<BM, BN, BK, 0, 4>(p, grid, s); break;
    case EPI_ROWSCALE: launch_e<BM, BN, BK, EPI_ROWSCALE, 4>(p, grid, s); break;
    default:
      set_error("gemm: 32-column tiles take no epilogue");
      return MSFNO_EUNSUPPORTED;
  }
  return MSFNO_OK;
}

// the epilogue combinations the block uses (anything else is rejected)
template <int BM, int BN, int BK>
static int launch(const GemmParams& p, dim3 grid, hipStream_t s) {
  switch (epi_code(p)) {
    case 0: launch_e<BM, BN, BK, 0>(p, grid, s); break;
    case EPI_RELU: launch_e<BM, BN, BK, EPI_RELU>(p, grid, s); break;
    case EPI_ROWSCALE: launch_e<BM, BN, BK, EPI_ROWSCALE>(p, grid, s); break;
    case EPI_BIAS: launch_e<BM, BN, BK, EPI_BIAS>(p, grid, s); break;
    case EPI_BIAS | EPI_GELU: launch_e<BM, BN, BK, EPI_BIAS | EPI_GELU>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD: launch_e<BM, BN, BK, EPI_BIAS | EPI_ADD>(p, grid, s); break;
    case EPI_GELU_B | EPI_BIAS: launch_e<BM, BN, BK, EPI_GELU_B | EPI_BIAS>(p, grid, s); break;
    case EPI_GELU_B | EPI_BIAS | EPI_ADD:
      launch_e<BM, BN, BK, EPI_GELU_B | EPI_BIAS | EPI_ADD>(p, grid, s); break;
    case EPI_ADD: launch_e<BM, BN, BK, EPI_ADD>(p, grid, s); break;
    case EPI_BIAS | EPI_ADD | EPI_GELU:  // decoder fc1 over the big-skip concatenation
      launch_e<BM, BN, BK, EPI_BIAS | EPI_ADD | EPI_GELU>(p, grid, s); break;
    default:
      set_error("gemm: unsupported epilogue combination");
      return MSFNO_EUNSUPPORTED;
  }
  return MSFNO_OK;
}

#ifndef MSFNO_GEMM_BK
#define MSFNO_GEMM_BK 16
#endif

static int dispatch(GemmTile tile, const GemmParams& p, dim3 grid, hipStream_t s) {
  int rc;
  switch (tile) {
    case TILE_128x128: rc = launch<128, 128, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_128x64: rc = launch<128, 64, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_256x64: rc = launch<256, 64, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_256x128: rc = launch<256, 128, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_128x256: rc = launch<128, 256, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_256x32: rc = launch_narrow<256, 32, MSFNO_GEMM_BK>(p, grid, s); break;
    case TILE_128x32: rc = launch_narrow<128, 32, MSFNO_GEMM_BK>(p, grid, s); break;
    default: rc = launch<64, 64, MSFNO_GEMM_BK>(p, grid, s); break;
  }
  if (rc != MSFNO_OK) return rc;
  return launch_check("gemm_f32");
}

static bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

int gemm_uniform(GemmTile tile, const float* A, const float* B, float* C, int M, int N, int K,
                 int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int batch,
                 const GemmEpi& epi, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return MSFNO_OK;
  if (tile == TILE_256x256) tile = TILE_128x256;  // no fp32 instance
  int bm, bn;
  gemm_tile_dims(tile, &bm, &bn);
  GemmParams p = make_params(A, B, C, epi);
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC;
  p.tiles_m = (int)cdiv(M, bm);
  p.tiles_n = (int)cdiv(N, bn);
  p.vecA = (lda % 4 == 0) && (sA % 4 == 0) && aligned16(A);
  p.vecB = (ldb % 4 == 0) && (sB % 4 == 0) && aligned16(B);
  p.vecC = (ldc % 4 == 0) && (sC % 4 == 0) && aligned16(C) &&
           (!epi.addend || ((epi.ldd % 4 == 0) && (epi.sD % 4 == 0) && aligned16(epi.addend)));
  MSFNO_REQUIRE(batch <= 65535, MSFNO_EINVAL, "gemm: batch too large");
  dim3 grid(p.tiles_m * p.tiles_n, 1, batch);
  return dispatch(tile, p, grid, s);
}

int gemm_desc(GemmTile tile, const float* A, const float* B, float* C, const GemmDesc* descs,
              int ndesc, int total_tiles, const GemmEpi& epi, hipStream_t s) {
  if (total_tiles <= 0) return MSFNO_OK;
  MSFNO_REQUIRE(tile != TILE_256x256, MSFNO_EINVAL, "gemm_desc: no fp32 256x256 instance");
  GemmParams p = make_params(A, B, C, epi);
  p.descs = descs;
  p.ndesc = ndesc;
  // descriptor problems are laid out with lda/ldb/offsets that are multiples of 4
  p.vecA = aligned16(A);
  p.vecB = aligned16(B);
  p.vecC = aligned16(C) && !epi.addend;
  return dispatch(tile, p, dim3(total_tiles), s);
}

}  // namespace msfno
