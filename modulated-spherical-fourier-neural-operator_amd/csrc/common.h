// Internal helpers shared by the libmsfno translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <map>
#include <vector>

#include "../../include/msfno.h"

namespace msfno {

void set_error(const std::string& msg);

struct Status {
  int code = MSFNO_OK;
};

#define MSFNO_CHECK_HIP(expr)                                                       \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      ::msfno::set_error(std::string("HIP error '") + hipGetErrorString(_e) +       \
                         "' at " + __FILE__ + ":" + std::to_string(__LINE__) +      \
                         " in " #expr);                                             \
      return MSFNO_EHIP;                                                            \
    }                                                                               \
  } while (0)

#define MSFNO_REQUIRE(cond, code, msg)          \
  do {                                          \
    if (!(cond)) {                              \
      ::msfno::set_error(msg);                  \
      return (code);                            \
    }                                           \
  } while (0)

#define MSFNO_TRY(expr)              \
  do {                               \
    int _rc = (expr);                \
    if (_rc != MSFNO_OK) return _rc; \
  } while (0)

inline int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e));
    return MSFNO_EHIP;
  }
  return MSFNO_OK;
}

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// Spectral ("S") layout, m-major packed triangle, parity split:
//   row r = (b*2 + ri)*C + c ;  for j = l - m (l in [m, lmax)):
//     j even -> column off[m] + j/2           (Le_m = ceil(L_m/2) columns)
//     j odd  -> column off[m] + Lpe_m + j/2   (Lo_m = floor(L_m/2) columns)
//   with Lpe_m = round_up(Le_m, 4), Lp_m = Lpe_m + round_up(Lo_m, 4); pads are 0.
// The split matches the equatorial symmetry P_l^m(-x) = (-1)^(l-m) P_l^m(x)
// that halves the Legendre work on symmetric grids (see msfno_sht_plan_s::sym).
// ---------------------------------------------------------------------------
__host__ __device__ inline int64_t spec_col(const int* off, const int* Lpe, int m, int l) {
  const int j = l - m;
  return off[m] + ((j & 1) ? Lpe[m] : 0) + (j >> 1);
}

struct SpecLayout {
  int lmax = 0, mmax = 0;
  int mact = 0;                 // number of m with lmax - m > 0
  std::vector<int> L, Lp, off;  // per m (size mmax)
  std::vector<int> Lpe;         // per m: padded even-parity block width
  int64_t T = 0;                // number of (l,m) with l>=m (tril count)
  int64_t Tp = 0;               // total padded columns
  int64_t ldT = 0;              // row stride of S buffers (multiple of 4)
  // mask (size mmax, optional): keep only the m with mask[m] != 0 (latitude-band
  // sharding: the m-set owned by one rank); the others get L = Lp = 0
  void build(int lmax_, int mmax_, const std::vector<char>* mask = nullptr);
  int64_t col(int m, int l) const { return spec_col(off.data(), Lpe.data(), m, l); }
};

// ---------------------------------------------------------------------------
// FFT plan part (longitude transform of length nlon)
// ---------------------------------------------------------------------------
constexpr int kMaxRadices = 24;
struct FFTPlan {
  int N = 0;         // nlon
  int H = 0;         // complex length actually transformed (N/2 if packed)
  int packed = 0;    // real-input packing (N even)
  int inplace = 1;   // all passes fit the in-register in-place scheme
  int codelet = 0;   // compiled fixed-size FFT (0 = generic runtime-radix path)
  int nrad = 0;
  int radices[kMaxRadices] = {0};
  float2* twH = nullptr;  // e^{-2πi t/H}, t < H      (device)
  float2* twN = nullptr;  // e^{-2πi k/N}, k <= N/2   (device)
};
int fft_plan_build(FFTPlan& p, int N);

// latitude geometry of a plan passed to kernels by value
struct LatGeom {
  int sym;        // equatorially symmetric parity-split slabs
  int nlat, nh;   // nh = nlat / 2 (pairs k, nlat-1-k for k < nh; centre row if odd)
  int Ke, Ko;     // nlat - nh, nh
  int ldke;       // column of Xa in a slab row
  int ldk;        // slab row stride
};
void fft_plan_free(FFTPlan& p);

// ---------------------------------------------------------------------------
// Batched GEMM descriptors (per-m Legendre problems)
// ---------------------------------------------------------------------------
struct GemmDesc {
  int64_t offA, offB, offC;
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n;
  int tile_start;
  int flags;  // bit 0: apply GemmEpi::rowscale (Legendre-forward m >= 1)
  int64_t offBx, offBs;  // x3h Legendre: the problem's table image / column scales
};

struct GemmEpi {
  const float* bias = nullptr;      // per row (batch stride sBias)
  const float* addend = nullptr;    // matrix, ld = ldd (batch stride sD)
  int64_t sBias = 0, sD = 0;
  int ldd = 0;
  int act = 0;                      // 0 none, 1 GELU(erf) on C, 2 GELU(erf) on B while staged
  int relu_period = 0, relu_rows = 0;  // ReLU rows where (row % period) < relu_rows
  const float* rowscale = nullptr;  // per-(b,c) factor for rows r=(b,ri,c); C = rs_C
  int rs_C = 0;
  // x6 engine only: operands in the bf16x3 plane format (three exact bf16 terms
  // per fp32 value, plane stride in elements; batch stride / ld as for fp32).
  // b_planes replaces B; c_planes receives C (the fp32 C pointer is unused)
  const unsigned short* b_planes = nullptr;
  int64_t b_plane_stride = 0;
  unsigned short* c_planes = nullptr;
  int64_t c_plane_stride = 0;
  // gemm_x6p only: A already split into its image ([3][KT][Mp][16], e.g. by
  // launch_spec_weights_x6p); the fp32 A pointer and the workspace are unused
  const unsigned short* a_planes = nullptr;
  // fp32 descriptor GEMM only (band plans, common.h msfno_sht_plan_s): A's K index
  // (segA) / C's column index (segC) is split into blocks of seg_w columns, block
  // q at q * seg_stride floats from the operand base (0: contiguous)
  int segA_w = 0, segC_w = 0;
  int64_t segA_stride = 0, segC_stride = 0;
  // gemm_x6 with fp32 B only: B rows k >= b2_k come from b2 (row k - b2_k, ld b2_ld,
  // batch stride b2_stride): the K concatenation [B ; b2] without materialising it
  const float* b2 = nullptr;
  int b2_k = 0, b2_ld = 0;
  int64_t b2_stride = 0;
};

enum GemmTile {
  TILE_128x128 = 0, TILE_128x64 = 1, TILE_64x64 = 2, TILE_256x64 = 3, TILE_256x128 = 4,
  TILE_128x256 = 5, TILE_256x256 = 6,  // 256x256: gemm_x6 only
  TILE_256x32 = 7, TILE_128x32 = 8      // fp32 descriptor (Legendre) GEMMs only
};
// GEMM role -> tile (defaults chosen by measurement); MSFNO_TILES
// ("skip=4,fc1=1,...", values = GemmTile) overrides them for A/B experiments
enum GemmRole { ROLE_SKIP = 0, ROLE_FC1, ROLE_FC2, ROLE_SPEC, ROLE_LEG, ROLE_LEGI, ROLE_COUNT };
GemmTile role_tile(GemmRole r, GemmTile dflt);

// C[M,N] = A[M,K] · B[K,N] (+ epilogue), row-major, fp32 MFMA.
// Uniform batched mode: batch index = grid.z, operand batch strides sA/sB/sC.
int gemm_uniform(GemmTile tile, const float* A, const float* B, float* C, int M, int N, int K,
                 int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int batch,
                 const GemmEpi& epi, hipStream_t s);
// Descriptor mode: per-problem dims/offsets from `descs` (device), tiles laid out 1-D.
int gemm_desc(GemmTile tile, const float* A, const float* B, float* C, const GemmDesc* descs,
              int ndesc, int total_tiles, const GemmEpi& epi, hipStream_t s);
void gemm_tile_dims(GemmTile tile, int* bm, int* bn);
// fp32-accurate GEMM on the bf16 matrix cores (gemm_x6.hip): same contract as
// gemm_uniform (no GELU-on-B / rowscale epilogues); ws >= gemm_x6_workspace
// holds A split into bf16 terms (written by this call, stream-ordered)
size_t gemm_x6_workspace(int M, int K, int batch);
int gemm_x6(GemmTile tile, const float* A, const float* B, float* C, int M, int N, int K, int lda,
            int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int batch, const GemmEpi& epi,
            void* ws, size_t ws_bytes, hipStream_t s);
int launch_split_a(const float* A, unsigned short* Ax, int M, int K, int lda, int64_t sA,
                   int batch, hipStream_t s);
// the same GEMM on the x3h engine (two fp16 terms, three MFMAs; gemm_x6.hip): B rows
// scaled by the powers of two bscale[z * K + k] while staged (every |scaled| < 2^14),
// A re-imaged per batch into ws (>= gemm_x3_workspace); bias-only epilogue
// x3h Legendre descriptor GEMM (legendre_x3.hip): tiles X3D_BM x x3d_bn(), k-tile X3D_BK
constexpr int X3D_BM = 128, X3D_BK = 32;
int x3d_bn(int inverse);
// register-resident variant (legendre_x3r): every problem K <= X3R_KMAX, N <= X3R_NMAX
constexpr int X3R_KMAX = 192, X3R_NMAX = 1024;
// register-B forward variant (legendre_x3f): K <= X3F_KMAX, X3F_RB rows x 64 columns per tile
constexpr int X3F_KMAX = 384, X3F_RB = 256;
int launch_legendre_x3_image(const float* table, const GemmDesc* descs, int ndesc,
                             unsigned short* img, float* invs, hipStream_t s);
int legendre_x3(const float* A, const unsigned short* img, const float* invs, float* C,
                const GemmDesc* descs, const int* tile_desc, int ndesc, int tiles, int bn,
                const GemmEpi& e, hipStream_t s);
int legendre_x3f(const unsigned short* Ap, const float* isr,
                 const unsigned short* img, const float* invs, float* C, const GemmDesc* descs,
                 const int* tile_desc, int ndesc, int tiles, hipStream_t s, int segA_w = 0,
                 int64_t segA_stride = 0);
int legendre_x3r(const float* A, const unsigned short* img, const float* invs, float* C,
                 const GemmDesc* descs, const int* tile_desc, int ndesc, int tiles,
                 const GemmEpi& e, hipStream_t s);
size_t gemm_x3_workspace(int M, int K, int batch);
int gemm_x3(const float* A, int lda, const float* bscale, const float* B, float* C, int M, int N,
            int K, int ldb, int ldc, int64_t sB, int64_t sC, int batch, const GemmEpi& epi,
            void* ws, size_t ws_bytes, hipStream_t s);
// x6 GEMM with B (and optionally C) in the bf16x3 plane format (gemm_x6p.hip):
// epi.b_planes required (ldb, sB, b_plane_stride % 8 == 0, 16-B aligned); A fp32
// is split per call into ws (>= gemm_x6p_workspace(M, K, sA == 0 ? 1 : batch))
size_t gemm_x6p_workspace(int M, int K, int batch_a);
// the A image of gemm_x6p (16-deep k-tiles) split once into ws, for a sequence of
// gemm_x6p calls that pass it as epi.a_planes (e.g. pixel-chunked MLPs)
int gemm_x6p_split_a(const float* A, int M, int K, int lda, int64_t sA, int batch, void* ws,
                     size_t ws_bytes, hipStream_t s);
int gemm_x6p(const float* A, float* C, int M, int N, int K, int lda, int ldb, int ldc,
             int64_t sA, int64_t sB, int64_t sC, int batch, const GemmEpi& epi, void* ws,
             size_t ws_bytes, hipStream_t s);
// all spectral-MLP weights of a block -> x6p A images in one launch: fill w, ci,
// co, out (each >= gemm_x6p_workspace(2 co, 2 ci, 1) bytes) and nlayers, then
// spec_weights_x6p_layout (fills start[], returns the bytes the images need)
struct SpecWeightsX6p {
  const float* w[9];
  unsigned short* out[9];
  int ci[9], co[9];
  int64_t start[10];  // pair offsets of each layer in the flattened index space
  int nlayers;
  // x3h 3M images (gemm_x6c.hip, NP = 2): per layer {weight scale tau, epilogue
  // multiplier} (2 floats per layer, device; spec_scales_x3h_kernel)
  float* scl = nullptr;
};
size_t spec_weights_x6p_layout(SpecWeightsX6p& a);
int launch_spec_weights_x6p(const SpecWeightsX6p& a, hipStream_t s);
// spectral-MLP layer as a Gauss 3M complex GEMM on the x6 engine (gemm_x6c.hip);
// activations in "3M planes" [b][re, im, re+im][plane][rows][ld]
size_t gemm_x6c_weight_bytes(int co, int ci);
size_t spec_weights_3m_layout(SpecWeightsX6p& a);
int launch_spec_weights_3m(const SpecWeightsX6p& a, hipStream_t s);
int launch_split3m(const float* S, unsigned short* X, int B, int C, int N, int ldS, int ldx,
                   hipStream_t s);
int gemm_x6c_f32b(const unsigned short* Aw, int co, int ci, const float* Sin, int ldSin, int N,
                  unsigned short* Y, int ldy, float* Sout, int ldSout, bool relu, int B,
                  hipStream_t s, bool tiled_out = false);
int64_t x6c_tiled_elems(int rows, int N);
int gemm_x6c(const unsigned short* Aw, int co, int ci, const unsigned short* X, int N, int ldx,
             unsigned short* Y, float* S, int ldS, bool relu, int B, hipStream_t s, int lay = 0);
// the same chain on the x3h engine (two fp16 terms, three MFMAs per product; tiled
// hidden activations of 6 planes).  Scaling (all powers of two): the weights of layer
// l by a.scl[2l] (spec_scales_x3h_kernel), layer 0's input column (b, n) by
// cs[b * ldcs + n] (launch_spec_colscale: its max |Re|, |Im| into [2^13, 2^14)),
// the hidden layers' outputs by a.scl[2l + 1]; the output layer undoes everything
// (a.scl[2L + 1] and the inverse column scales cs[B * ldcs + ...]).
int launch_spec_weights_3m_x3h(const SpecWeightsX6p& a, hipStream_t s);
int launch_spec_colscale(const float* S, int B, int C, int N, int ldS, float* cs, int ldcs,
                         hipStream_t s);
int64_t x3c_tiled_elems(int rows, int N);
int gemm_x3c(const unsigned short* Aw, int co, int ci, const float* Sin, int ldSin,
             const unsigned short* X, int N, unsigned short* Y, float* Sout, int ldSout,
             bool relu, const float* lscale, const float* colscale, int64_t cs_b, int B,
             hipStream_t s);
// fp32 x[z][r][c] (ld ldx, batch stride sx) -> bf16x3 planes xp[z][plane][r][c]
int launch_split_planes(const float* x, unsigned short* xp, int rows, int cols, int ldx,
                        int64_t sx, int ldp, int64_t pstride, int64_t sxp, int batch,
                        hipStream_t s);
// dense 1x1-conv GEMMs of the block / MLP: gemm_x6 unless MSFNO_GEMM=f32 (or no
// workspace / a GELU-on-B or rowscale epilogue), else the fp32 MFMA kernel on
// role_tile(role, f32_tile).  batch_a = 1 when sA == 0, else batch.
bool gemm_use_x6();
size_t gemm_dense_workspace(int M, int K, int batch_a);
int gemm_dense(GemmRole role, GemmTile f32_tile, const float* A, const float* B, float* C, int M,
               int N, int K, int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC,
               int batch, const GemmEpi& epi, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace msfno

struct msfno_sht_plan_s {
  int nlat, nlon, lmax, mmax, inverse;
  int ldk;                       // slab row stride (>= round_up(nlat,4), fits both layouts)
  msfno::SpecLayout spec;
  msfno::FFTPlan fft;
  float* table = nullptr;        // device, plan GEMM layout
  int64_t table_elems = 0;
  std::vector<int64_t> tab_off;  // per m offsets into table
  int64_t* d_tab_off = nullptr;  // device copies of the per-m metadata
  int* d_Lp = nullptr;
  int* d_off = nullptr;          // S-layout column offsets off[m]
  // m-set plans (latitude-band sharding): global tril index (torch.tril_indices(lmax,
  // mmax) order) -> position among the plan's own modes (ascending global order),
  // -1 for modes of other ranks; null for full plans.  lin_modes: the inverse map.
  int* d_tril_local = nullptr;
  std::vector<long long> lin_modes;
  // full plans: S column of every tril mode n (torch.tril_indices order), and the S
  // columns no mode maps to (block pads): the tiled S <-> tril re-layouts of the linear
  // filter (spec_tril_tiled_kernel, zero_spec_pads_kernel)
  int* d_tcol = nullptr;
  int* d_tpad = nullptr;
  int npad = 0;
  int table_loaded = 0;
  // equatorial symmetry: the grid is symmetric (table[m][l][nlat-1-k] =
  // (-1)^(l-m) table[m][l][k], checked at load).  Then the Legendre GEMMs run
  // over the northern half + equator only, on Xs = X_k + X_{n-1-k} (even l-m,
  // K = Ke) and Xa = X_k - X_{n-1-k} (odd, K = Ko): half the flops.  Slab rows
  // hold [Xs (Ke) | pad | Xa (Ko) | pad] (Xs at column 0, Xa at column ldke).
  int sym = 0;
  int nh = 0, Ke = 0, Ko = 0, ldke = 0;
  int* d_Lpe = nullptr;
  // Xt / Yt slab of each m (-1: m not in this plan's m-set); full plans: slab[m] = m
  std::vector<int> slab;
  int nslab = 0;
  // cached Legendre GEMM descriptors for a given row count R
  int desc_R = -1;
  msfno::GemmDesc* d_desc = nullptr;
  int ndesc = 0, desc_tiles = 0;
  // x3h Legendre (legendre_x3.hip): descriptor cache, the table image (two fp16
  // planes per problem, column-scaled) and the inverse column scales
  // descriptor sets per row count R (the band pipeline's uneven sub-batches alternate
  // R): built once each, freed with the plan; the fields below are the set of the
  // last R used
  struct DescSet {
    msfno::GemmDesc* d = nullptr;
    int* tile = nullptr;
    int n = 0, tiles = 0, res = 0;
  };
  std::map<int, DescSet> desc_sets, desc3_sets, desc3f_sets;
  int desc3_R = -1;
  msfno::GemmDesc* d_desc3 = nullptr;
  int* d_tile3 = nullptr;  // tile -> descriptor index
  int ndesc3 = 0, desc3_tiles = 0;
  unsigned short* tab3 = nullptr;
  float* tab3s = nullptr;
  int64_t tab3_elems = 0, tab3s_elems = 0;
  int tab3_valid = 0;
  int desc3_res = 0;  // inverse problems on legendre_x3r (one tile per 128 rows)
  // forward problems on legendre_x3f (tiles X3F_RB x 64; the image of desc3)
  int desc3f_R = -1;
  msfno::GemmDesc* d_desc3f = nullptr;
  int* d_tile3f = nullptr;
  int ndesc3f = 0, desc3f_tiles = 0;
  // Latitude-band plans (band.cpp): the Legendre GEMMs read / write the all-to-all
  // buffers directly.  Their slabs are [src or dst rank p][slab][R][band_ld] blocks:
  // a K (forward) or N (inverse) column k' = p * seg + j lies in rank p's block.
  //   symmetric:  band_ld = 2W, Xs / E at [0, W), Xa / O at [W, 2W), seg = W,
  //               kmap[k'] = the folded (northern) latitude of j in p's band;
  //   general:    band_ld = 2W, the rank's local rows at [0, 2W), seg = 2W,
  //               kmap[k'] = the latitude of p's local row j;
  // kmap = -1 on pads (zeros in the buffers and in the table).  band_world = 0:
  // not a band plan.
  int band_world = 0, band_W = 0;
  std::vector<int> kmap_sym, kmap_gen;  // world * W and world * 2W entries
  int* d_kmap = nullptr;                // device copy of the one in use
  int band_seg() const { return sym ? band_W : 2 * band_W; }
  int band_K() const { return band_world * band_seg(); }
  int64_t table_cap = 0;         // floats allocated for `table`
  msfno::LatGeom geom() const { return {sym, nlat, nh, Ke, Ko, ldke, ldk}; }
};
