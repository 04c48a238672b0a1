// Internal launcher declarations (host-callable, stream-ordered).
#pragma once
#include "common.h"

namespace msfno {

// ---- fft.hip ----------------------------------------------------------------
// x (rows, N) fp32 -> out (rows, mmax) complex, scaled by `scale`; optional
// per-row (mean, M2) over the N inputs.
// planes (optional, LDS-DMA path only): the input rows are also written as bf16x3
// planes in the C2RPlanes layout below (the inner-skip GEMM's B operand)
int launch_fft_r2c_rows(const FFTPlan& f, const float* x, float2* out, float2* rowstats,
                        int64_t rows, int mmax, float scale, hipStream_t s,
                        const struct C2RPlanes* planes = nullptr);
// in (rows, mmax) complex (Hermitian half spectrum, zero beyond mmax) -> x (rows, N);
// act: 0 none, 1 GELU; optional per-row (mean, M2) of the outputs.
// addsrc (may alias x): x = act(addsrc + irfft(in))  (the block's skip branch)
int launch_fft_c2r_rows(const FFTPlan& f, const float2* in, float* x, const float* addsrc,
                        float2* rowstats, int64_t rows, int mmax, int act, hipStream_t s,
                        const struct C2RPlanes* planes = nullptr);
// optional bf16x3 plane output of launch_fft_c2r_rows / _r2c_rows (the next GEMM's B
// operand, gemm_x6p): rows are (b*C + c)*nlat + lat, written to
// xp[b][plane][c][lat*N + n] with plane stride C*nlat*N; x (fp32) is not written
struct C2RPlanes {
  unsigned short* xp;
  int C, nlat;
};
bool fft_c2r_planes_supported(const FFTPlan& f, int mmax);
bool fft_r2c_planes_supported(const FFTPlan& f, int mmax);

// fused FFT + transpose (block path); only for plans with a compiled codelet
bool fft_tile_supported(const FFTPlan& f);
// x (B*C, nlat, N) -> Xt (mmax, R=2BC, ldk) raw spectrum·scale (+ per-row (mean, M2))
int launch_fft_r2c_tile(const FFTPlan& f, const float* x, float* Xt, float2* rowstats, int B,
                        int C, int nlat, int mmax, int ldk, float scale, hipStream_t s);
// Yt (mmax, R, ldk) -> out (B*C, nlat, N), GELU if act, optional output row stats
int launch_fft_c2r_tile(const FFTPlan& f, const float* Yt, float* out, float2* rowstats, int B,
                        int C, int nlat, int mmax, int mact, int ldk, int act, hipStream_t s);
// m = 0 slice of Xt: v -> scale[bc]·v + 2π·shift[bc] (real rows), scale[bc]·v (imag rows)
int launch_dc_fixup(float* Xt, int B, int C, int nlat, int ldk, const float* nscale,
                    const float* nshift, hipStream_t s);

// ---- spectral.hip ------------------------------------------------------------
// Xn (BC, nlat, mmax) complex -> Xt (mmax, R=2BC, ldk); per-bc affine of the
// spatial field folded in: m>0 -> s·X, m=0 -> s·X + 2π·t (real part).
// slab (device, optional, size mmax): Xt slab of each m (-1 = skip); default slab = m.
int launch_transpose_fwd(const float2* Xn, float* Xt, int B, int C, int nlat, int mmax, int ldk,
                         const float* nscale, const float* nshift, hipStream_t s,
                         const int* slab = nullptr, int kpad = 0);
// Yt (mmax, R, ldk) -> Yn (BC, nlat, mmax); m >= mact written as 0.
int launch_transpose_inv(const float* Yt, float2* Yn, int B, int C, int nlat, int mmax, int mact,
                         int ldk, hipStream_t s, const int* slab = nullptr);
// Combine per-(bc) partial (mean, M2) statistics (np partials, each over `cnt`
// elements except the last over `cnt_last`) and produce the affine that
// implements InstanceNorm (+ optional FiLM): y = scale·x + shift.  xscale (or null):
// per (b,c) the power of two 2^(14 - e), |mean| + sqrt(M2) = f 2^e (f in [0.5, 1)),
// under which every element of the channel scales below 2^14 in magnitude
// (|x - mean| <= sqrt(sum (x - mean)^2)): the x3h skip GEMM's B-row scales
int launch_chan_affine(const float2* partials, int64_t np, int64_t cnt, int64_t cnt_last,
                       int B, int C, const float* w, const float* b, float eps,
                       const float* gamma, const float* beta, float film_scale, float* scale,
                       float* shift, hipStream_t s, float* xscale = nullptr,
                       float* lsig = nullptr, float* abound = nullptr);
// abound (or null): per (b,c) |scale| sqrt(M2) + |scale mean + shift| (x 1.001), a bound of
// |scale x + shift| over the channel (|x - mean| <= sqrt(M2)): the fused MLP's x3h range
// latitude-band sharding helpers (band.cpp)
// rowstats (BC, np) (mean, M2) over cnt each -> out (BC, 3) fp64 {n, mean, M2}; xscale
// (or null): the local x3h skip B-row scales as in launch_chan_affine
int launch_stats_partial(const float2* rowstats, int64_t np, int64_t cnt, int64_t BC, double* out,
                         hipStream_t s, float* xscale = nullptr);
// parts (nparts, BC, 3) fp64 -> InstanceNorm (+FiLM) per-(b,c) affine
int launch_chan_affine_parts(const double* parts, int nparts, int B, int C, const float* w,
                             const float* b, float eps, const float* gamma, const float* beta,
                             float film_scale, float* scale, float* shift, hipStream_t s,
                             float* xscale = nullptr, float* abound = nullptr,
                             float* lsig = nullptr);
// the all-to-all buffers are the Legendre GEMMs' own operands: [p][slab][R][2W]
// blocks (common.h msfno_sht_plan_s band fields).  g: the rank's local rows as a
// small symmetric grid (Ke = its band, nh = the band rows that have a mirror row,
// stored after the band, ascending), ldke = W, ldk = 2W.  pack: Xn (local rows)
// -> send (slab perm[m], norm0 affine, fold, zero pads); unpack: recv -> Yn.
int launch_band_pack(const float2* Xn, float* send, int B, int C, const LatGeom& g, int mmax,
                     const float* nscale, const float* nshift, const int* perm, int W,
                     hipStream_t s);
int launch_band_unpack(const float* recv, float2* Yn, int B, int C, const LatGeom& g, int mmax,
                       int mact, const int* perm, hipStream_t s);
// W' [b] = W·diag(scale[b]),  b'[b] = bias + W·shift[b]
int launch_fold_affine(const float* W, const float* bias, const float* scale, const float* shift,
                       float* Wf, float* bf, int B, int O, int I, hipStream_t s);
// out[bc][p] = act(scale[bc]·x[bc][p] + shift[bc] + addend[bc][p]) with optional stats
int launch_affine_rows(const float* x, const float* scale, const float* shift,
                       const float* addend, float* out, int64_t BC, int64_t P, int act,
                       float2* stats, int stats_ld, hipStream_t s);
// ---- mlp_fused.hip: the block MLP with the hidden activation on-chip ----------
// out = W2·GELU(W1·(scale ⊙ x1 + shift) + b1) + b2 (+ resid), C = 256, H = 512 only
bool mlp_fused_supported(int C, int H);
size_t mlp_fused_image_bytes();
// W1 (H x C), W2 (C x H) fp32 -> the kernel's bf16x3 weight image (mlp_fused_image_bytes)
int launch_mlp_fused_images(const float* W1, const float* b1, const float* W2,
                            unsigned short* img, hipStream_t s);
// abound: [B][C] bound of |scale ⊙ x1 + shift| (chan_affine), the x3h range scalars
int launch_mlp_fused(const float* x1, const float* scale, const float* shift, const float* abound,
                     const float* resid, float* out, const unsigned short* img, const float* b1,
                     const float* b2, int B, int64_t P, hipStream_t s);
// mlp_fused_h.hip: the MLP on the x3h engine (fp32 as two fp16 terms, three fp16
// MFMAs per product, row-scaled weights); default (MSFNO_ENGINE=x6 selects the x6 engine)
bool mlp_fused_h_env();
// mlp_gen_h.hip: the standalone MLP (network encoder / decoder) fused on the x3h engine,
// per-pixel range scales; widths (Cin + Cin2, Cout) of the instantiated kernels only
bool mlp_gen_h_supported(int Ct, int H, int Cout);
size_t mlp_gen_h_workspace(int Ct, int H, int Cout);
// xa, xt (both or neither): [B][Cin] per-channel affine applied to x first (a deferred
// norm / FiLM of the producing block).  cache (or null): mlp_gen_h_workspace bytes holding
// the prepared weight image across calls, rebuilt only when cache_valid is 0 (ws is then
// unused)
int launch_mlp_gen_h(const float* x, const float* xa, const float* xt, const float* x2, int Cin,
                     int Cin2, const float* W1,
                     const float* b1, const float* W2, const float* b2, int H, int Cout,
                     const float* addend, int64_t add_bstride, float* out, int B, int64_t P,
                     void* ws, size_t ws_bytes, hipStream_t s, void* cache = nullptr,
                     int cache_valid = 0);
// inner skip at C = 256 on the mlp_fused_h tiling (x3h): out = Ws·x + bs, x scaled by the
// power-of-two channel scales xs (|xs x| < 2^14), or per pixel in-kernel when xs is null;
// ws >= skip_h_workspace(B)
bool skip_h_env();
size_t skip_h_workspace(int B);
// side_share: the persistent kernel's workgroups per CU when it runs on the block's side
// stream beside the SHT (0: the default for a kernel that runs alone)
int launch_skip_h(const float* W, const float* xs, const float* x, float* out, const float* bias,
                  int B, int64_t P, void* ws, size_t ws_bytes, hipStream_t s,
                  bool side = false);
// xs[r] = the power of two 2^(14 - e) with max_p |x[r][p]| = f 2^e (rows of P values): the
// x3h B-row scales of a 1x1 conv whose input carries no norm statistics
int launch_chan_pow2_scale(const float* x, int64_t rows, int64_t P, float* xs, hipStream_t s);
size_t mlp_fused_h_image_bytes();
int launch_mlp_fused_h_images(const float* W1, const float* b1, const float* W2,
                              unsigned short* img, hipStream_t s);
int launch_mlp_fused_h(const float* x1, const float* scale, const float* shift,
                       const float* abound, const float* resid, float* out,
                       const unsigned short* img, const float* b1, const float* b2, int B,
                       int64_t P, hipStream_t s);
// ---- cgemm.hip -----------------------------------------------------------------
// complex (Ci,Co,2) weight -> Ar, Ai (Co x Ci) row-major (Ar[o][i] = Re w[i][o])
int launch_split_complex_weight(const float* w, float* Ar, float* Ai, int Ci, int Co,
                                hipStream_t s);
// Y = W.X complex per column (3M scheme), X/Y rows [b][re|im][ci|co] in the S layout;
// relu: ComplexReLU(real) on the output; tile 0: 128x64, 1: 64x128, 2: 128x128
int gemm_c3m(const float* Ar, const float* Ai, const float* X, float* Y, int co, int ci, int N,
             int ldx, int ldy, int64_t sX, int64_t sY, int B, bool relu, int tile, hipStream_t s);
// complex (Ci,Co,2) weight -> real (2Co x 2Ci) block matrix [[Wr^T,-Wi^T],[Wi^T,Wr^T]]
int launch_expand_complex_weight(const float* w, float* Wexp, int Ci, int Co, hipStream_t s);
// (mmax,lmax,nlat) reference table -> plan GEMM layout (general or symmetric)
int launch_relayout_table(const msfno_sht_plan_s& p, const float* table, hipStream_t s);
// FiLM backward (film_bwd.hip)
int launch_transpose_mat(const float* A, int rows, int cols, int lda, float* AT, hipStream_t s);
int launch_gelu_grad_mul(float* dh, const float* pre, int64_t n, hipStream_t s);
int launch_film_grad_reduce(const float* du, const float* x1, const float* an, const float* tn,
                            float scale, int BC, int64_t P, float* dgamma, float* dbeta,
                            hipStream_t s);
// full block backward (block_bwd.cpp): per-row InstanceNorm moments and affine,
// InstanceNorm backward (with the FiLM factor 1 + gamma s and up to two addends),
// ComplexReLU(real) mask, complex conjugate transposes, tril <-> dense spectra, fill
int launch_row_moments(const float* x, int64_t rows, int C, int64_t P, const float* w,
                       const float* b, float eps, float* mean, float* rstd, float* scale,
                       float* shift, hipStream_t s);
int launch_inorm_backward(const float* x, const float* mean, const float* rstd, const float* w,
                          const float* gamma, float film_scale, const float* g, const float* add1,
                          const float* add2, float* dx, int64_t rows, int C, int64_t P,
                          hipStream_t s);
int launch_relu_real_mask(float* dh, const float* h, int64_t n, hipStream_t s);
int launch_conj_swap01(const float* w, int I, int K, int64_t T, float* wt, hipStream_t s);
int launch_tril_map(const float* src, float* dst, int64_t rows, int lmax, int mmax, int64_t T,
                    bool gather, hipStream_t s);
int launch_fill(float* p, int64_t n, float v, hipStream_t s);
// sc = (1 + gamma s) an, sh = (1 + gamma s) tn + beta s (n = B*C)
int launch_film_affine(const float* an, const float* tn, const float* gamma, const float* beta,
                       float film_scale, float* sc, float* sh, int64_t n, hipStream_t s);
// parameter gradients (param_bwd.hip): C[m * ldc + n * cs] = sum_b sum_k A_b[m][k] B'_b[n][k]
// (B' by mode: B, per-(b, n) affine sc B + sh, GELU(B), complex pairs (re, im) -> (im, -re))
enum { WGRAD_PLAIN = 0, WGRAD_AFFINE = 1, WGRAD_GELU = 2, WGRAD_CSWAP = 3 };
size_t wgrad_nt_workspace(int M, int N, int64_t K, int batch);
int launch_wgrad_nt(const float* A, int64_t lda, int64_t sA, const float* B, int64_t ldb,
                    int64_t sB, int M, int N, int64_t K, int batch, int mode, const float* bsc,
                    const float* bsh, float* C, int64_t ldc, int cs, void* ws, size_t ws_bytes,
                    hipStream_t s);
// dw[k][i][t] = sum_b g[b][k][t] conj(a[b][i][t]) (complex, the linear filter's weights)
int launch_lin_wgrad(const float* g, const float* a, float* dw, int B, int Co, int Ci, int64_t T,
                     hipStream_t s);
// InstanceNorm affine gradients (x null: the bias / row-sum gradient db only)
size_t norm_param_grad_workspace(int B, int C);
int launch_norm_param_grad(const float* g, const float* x, const float* mean, const float* rstd,
                           const float* gamma, float film_scale, int B, int C, int64_t P,
                           float* dw, float* db, void* ws, hipStream_t s);
// *d_flag |= 1 unless table[m][l][nlat-1-k] = (-1)^(l-m) table[m][l][k] (rel. 1e-5)
int launch_check_symmetry(const float* table, int mmax, int lmax, int nlat, int* d_flag,
                          hipStream_t s);
// symmetric plans: transposes that fold / unfold the hemispheres (common.h LatGeom)
int launch_transpose_fwd_sym(const float2* Xn, float* Xt, int B, int C, const LatGeom& g, int mmax,
                             const float* nscale, const float* nshift, hipStream_t s);
int launch_transpose_inv_sym(const float* Yt, float2* Yn, int B, int C, const LatGeom& g, int mmax,
                             int mact, hipStream_t s);
// x3h planes (legendre_x3f's A): the folded slab as fp16 pairs interleaved per 8 k
// ([m][R][ldk / 8][plane][8]), scaled per channel by lsig (chan_affine; 1 / sigma -> isr[R])
int launch_transpose_fwd_sym_h(const float2* Xn, unsigned short* Xp, int B, int C,
                               const LatGeom& g, int mmax, const float* nscale,
                               const float* nshift, const float* lsig, float* isr,
                               hipStream_t s);
int launch_band_pack_h(const float2* Xn, unsigned short* send, int B, int C, const LatGeom& g,
                       int mmax, const float* nscale, const float* nshift, const float* lsig,
                       float* isr, const int* perm, int W, hipStream_t s);
// S layout <-> reference (bc, lmax, mmax) complex dense
int launch_spec_to_ref(const msfno_sht_plan_s& p, const float* S, float2* out, int B, int C,
                       const int* d_off, hipStream_t s);
int launch_ref_to_spec(const msfno_sht_plan_s& p, const float2* in, float* S, int B, int C,
                       const int* d_off, hipStream_t s);
// S layout <-> tril (B,C,T,2) (torch.tril_indices(lmax,mmax) order, layers.py:368)
int launch_spec_to_tril(const msfno_sht_plan_s& p, const float* S, float* xt, int B, int C,
                        hipStream_t s);
int launch_tril_to_spec(const msfno_sht_plan_s& p, const float* yt, float* S, int B, int C,
                        hipStream_t s);
// compl_contract_fwd_c: a (B,Ci,T,2), w (Co,Ci,T,2) -> y (B,Co,T,2)
int launch_compl_contract(const float* a, const float* w, float* y, int B, int Ci, int Co,
                          int64_t T, hipStream_t s);
// compl_mul2d_fwd_c reference layout (standalone op)
int launch_compl_mul2d(const float* a, const float* w, float* y, int B, int Ci, int Co,
                       int64_t XY, int relu_real, hipStream_t s);

}  // namespace msfno
