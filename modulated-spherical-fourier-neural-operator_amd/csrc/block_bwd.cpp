// Full backward of the SFNO block with the SFNO weights frozen:
// dL/dx (and dL/dgamma, dL/dbeta) of FourierNeuralOperatorBlock[_Filmed].forward
// (MSFNO/Models/sfno/sfnonet.py:221-251, 359-393) for dout = dL/d(out).  MSFNO's
// fine-tuning modes --film-layers k (main.py:1083-1087) and --repeat-film
// (main.py:1133-1136) run several filmed blocks with autograd (sfnonet.py:838-844), so
// the gradient reaches the FiLM modulation of every block only through the dx of the
// blocks after it.
//
// The forward is recomputed (the reference's checkpoint(blk, ...)) in the reference's
// own layouts, keeping what the backward needs: the norm statistics, the spectral
// hidden activations (ComplexReLU masks), x1 and the MLP pre-activations.  The adjoint
// chain, last stage first:
//   MLP:      du = W1^T (GELU'(pre) * W2^T dout)               (absent: du = dout)
//   FiLM:     dgamma = s sum du xhat1, dbeta = s sum du
//   norm1:    dx1 = InstanceNorm backward of (1 + gamma s) du
//   (linear filter: dx1 *= GELU'(x1 before the GELU))
//   ISHT^T:   dZ = a forward SHT on the output grid whose table is pct c_m N / 2pi
//             (the adjoint of irfft(norm="forward") weights bin m by c_m = 2 except the DC
//             and Nyquist bins), plan `fwd_adj`
//   filter:   non-linear: dh = dZ wout^H, then per layer l (last first) the ReLU(real)
//             mask of the forward's activation and dh = dh w_l^H (compl_mul2d on the
//             conjugate-transposed weights); linear: the per-mode contraction on the
//             conjugate-swapped weight (Ci, Co, T), gathered / scattered over the tril modes
//   SHT^T:    dxhat0 = an inverse SHT on the input grid whose table is weights d_m 2pi / N
//             (rfft's adjoint: d_m = 1/2 except the DC and Nyquist bins), plan `inv_adj`
//   norm0:    dx = InstanceNorm backward of dxhat0 (+ dout through the identity outer skip)
//   skip:     dx += Ws^T dx1 (linear inner skip) or dx1 (identity inner skip)
// The caller builds the two adjoint plans once (msfno_amd: the block's adjoint transforms).
#include <cmath>

#include "block.h"

namespace msfno {

namespace {

struct BwdBufs {
  // forward recompute
  float *mean0, *rstd0, *sc0, *sh0, *mean1, *rstd1, *an1, *tn1, *sc1, *sh1, *ones, *zeros;
  float *xh0, *A, *Z, *F, *x1pre, *x1;
  float* h[8];
  // MLP backward
  float *du, *W1f, *b1f, *pre, *dh, *W2T, *W1T;
  void *wsa, *wsb, *wsc;
  size_t wsa_b, wsb_b, wsc_b;
  // spectral backward
  float *dx1, *dZ, *da, *db, *dA, *dxh0, *dxt, *WsT, *wadj;
  int64_t wadj_off[9];
  float *a_t, *y_t;  // linear filter: tril-gathered spectra
  void *sws, *skws, *skws2;
  size_t sws_b, skws_b;
  // parameter gradients (msfno_block_backward_params)
  void *wg, *nrows;
  size_t wg_b;
};

int64_t tril_count(int lmax, int mmax) {
  int64_t T = 0;
  for (int l = 0; l < lmax; ++l) T += std::min(l + 1, mmax);
  return T;
}

void carve_bwd(Carve& cv, BwdBufs& r, const msfno_block_desc* d, msfno_sht_plan_t f,
               msfno_sht_plan_t g, msfno_sht_plan_t fa, msfno_sht_plan_t ga, int B,
               bool params = false) {
  const int64_t C = d->C, BC = (int64_t)B * C;
  const int64_t Pi = (int64_t)f->nlat * f->nlon, Po = (int64_t)g->nlat * g->nlon;
  const int64_t XY = (int64_t)f->lmax * f->mmax;
  const bool lin = d->filter_type == MSFNO_FILTER_LINEAR;
  const int64_t Hs = lin ? C : d->spec_hidden, L = lin ? 0 : d->spectral_layers;
  for (float** p : {&r.mean0, &r.rstd0, &r.sc0, &r.sh0, &r.mean1, &r.rstd1, &r.an1, &r.tn1,
                    &r.sc1, &r.sh1, &r.ones, &r.zeros})
    *p = cv.take<float>(BC);
  r.xh0 = cv.take<float>(BC * Pi);
  r.A = cv.take<float>(BC * XY * 2);
  for (int l = 0; l < 8; ++l) r.h[l] = l < L ? cv.take<float>((int64_t)B * Hs * XY * 2) : nullptr;
  r.Z = cv.take<float>(BC * XY * 2);
  r.F = cv.take<float>(BC * Po);
  r.x1pre = cv.take<float>(BC * Po);
  r.x1 = lin ? cv.take<float>(BC * Po) : r.x1pre;
  r.du = r.W1f = r.b1f = r.pre = r.dh = r.W2T = r.W1T = nullptr;
  r.wsa = r.wsb = r.wsc = nullptr;
  r.wsa_b = r.wsb_b = r.wsc_b = 0;
  if (d->has_mlp) {
    const int64_t Hd = d->mlp_hidden;
    r.du = cv.take<float>(BC * Po);
    r.W1f = cv.take<float>((int64_t)B * Hd * C);
    r.b1f = cv.take<float>((int64_t)B * Hd);
    r.pre = cv.take<float>((int64_t)B * Hd * Po);
    r.dh = cv.take<float>((int64_t)B * Hd * Po);
    r.W2T = cv.take<float>(Hd * C);
    r.W1T = cv.take<float>(C * Hd);
    if ((r.wsa_b = gemm_dense_workspace((int)Hd, (int)C, B))) r.wsa = cv.take<char>(r.wsa_b);
    if ((r.wsb_b = gemm_dense_workspace((int)Hd, (int)C, 1))) r.wsb = cv.take<char>(r.wsb_b);
    if ((r.wsc_b = gemm_dense_workspace((int)C, (int)Hd, 1))) r.wsc = cv.take<char>(r.wsc_b);
  }
  r.dx1 = cv.take<float>(BC * Po);
  r.dZ = cv.take<float>(BC * XY * 2);
  const int64_t hw = std::max<int64_t>(Hs, C);
  r.da = cv.take<float>((int64_t)B * hw * XY * 2);
  r.db = cv.take<float>((int64_t)B * hw * XY * 2);
  r.dA = cv.take<float>(BC * XY * 2);
  r.dxh0 = cv.take<float>(BC * Pi);
  r.dxt = cv.take<float>(BC * Pi);
  r.WsT = d->inner_skip == MSFNO_SKIP_LINEAR ? cv.take<float>(C * C) : nullptr;
  // conjugate-transposed filter weights
  int64_t woff = 0;
  if (lin) {
    woff = C * C * tril_count(f->lmax, f->mmax) * 2;
  } else {
    for (int l = 0; l <= L; ++l) {
      r.wadj_off[l] = woff;
      const int64_t ci = l == 0 ? C : Hs, co = l == L ? C : Hs;
      woff += ci * co * 2;
    }
  }
  r.wadj = cv.take<float>(woff);
  r.a_t = r.y_t = nullptr;
  if (lin) {
    const int64_t T = tril_count(f->lmax, f->mmax);
    r.a_t = cv.take<float>(BC * T * 2);
    r.y_t = cv.take<float>(BC * T * 2);
  }
  r.sws_b = 0;
  for (msfno_sht_plan_t p : {f, g, fa, ga})
    r.sws_b = std::max(r.sws_b, msfno_sht_workspace_size(p, (int)BC));
  r.sws = cv.take<char>(r.sws_b);
  r.skws_b = gemm_dense_workspace((int)C, (int)C, 1);
  r.skws = r.skws_b ? cv.take<char>(r.skws_b) : nullptr;
  r.skws2 = r.skws_b ? cv.take<char>(r.skws_b) : nullptr;
  r.wg = r.nrows = nullptr;
  r.wg_b = 0;
  if (params) {
    // the largest weight-gradient GEMM: 1x1 convs over the output grid's pixels, the
    // spectral layers over 2 lmax mmax real columns
    const int64_t hd = d->has_mlp ? d->mlp_hidden : 0, wide = std::max<int64_t>({C, Hs, hd});
    r.wg_b = std::max(wgrad_nt_workspace((int)wide, (int)wide, Po, B),
                      wgrad_nt_workspace((int)wide, (int)wide, 2 * XY, B));
    r.wg = cv.take<char>(r.wg_b);
    r.nrows = cv.take<char>(norm_param_grad_workspace(B, (int)wide));
  }
}

int check_adjoint(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                  msfno_sht_plan_t fa, msfno_sht_plan_t ga) {
  MSFNO_TRY(check_pair(d, f, g));
  MSFNO_REQUIRE(fa && ga && !fa->inverse && ga->inverse, MSFNO_EINVAL,
                "block backward: fwd_adj must be a forward plan, inv_adj an inverse plan");
  MSFNO_REQUIRE(fa->nlat == g->nlat && fa->nlon == g->nlon && ga->nlat == f->nlat &&
                    ga->nlon == f->nlon,
                MSFNO_EINVAL, "block backward: adjoint plans must sit on the swapped grids");
  MSFNO_REQUIRE(fa->lmax == f->lmax && fa->mmax == f->mmax && ga->lmax == f->lmax &&
                    ga->mmax == f->mmax && g->lmax == f->lmax && g->mmax == f->mmax,
                MSFNO_EINVAL, "block backward: the four plans must share lmax / mmax");
  MSFNO_REQUIRE(fa->table_loaded && ga->table_loaded, MSFNO_EINVAL,
                "block backward: adjoint plan tables not loaded");
  MSFNO_REQUIRE(d->outer_skip != MSFNO_SKIP_LINEAR, MSFNO_EUNSUPPORTED,
                "outer_skip='linear' is not supported by the fused block");
  MSFNO_REQUIRE(d->filter_type == MSFNO_FILTER_LINEAR ||
                    (d->spectral_layers >= 0 && d->spectral_layers <= 8 && d->spec_wout),
                MSFNO_EINVAL, "block backward: bad spectral filter");
  return MSFNO_OK;
}

}  // namespace

}  // namespace msfno

extern "C" {

size_t msfno_block_backward_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t f,
                                           msfno_sht_plan_t g, msfno_sht_plan_t fa,
                                           msfno_sht_plan_t ga, int B) {
  using namespace msfno;
  if (B <= 0 || check_adjoint(d, f, g, fa, ga) != MSFNO_OK) return 0;
  Carve cv;
  BwdBufs r;
  carve_bwd(cv, r, d, f, g, fa, ga, B);
  return cv.off;
}

int msfno_block_backward_hidden_offsets(const msfno_block_desc* d, msfno_sht_plan_t f,
                                        msfno_sht_plan_t g, msfno_sht_plan_t fa,
                                        msfno_sht_plan_t ga, int B, size_t* offsets, int n,
                                        int* nlayers) {
  using namespace msfno;
  MSFNO_TRY(check_adjoint(d, f, g, fa, ga));
  MSFNO_REQUIRE(B > 0 && nlayers && (n == 0 || offsets), MSFNO_EINVAL,
                "hidden offsets: bad arguments");
  // carve against a non-null base so take() hands out addresses; subtract it again
  static char anchor alignas(256)[256];
  Carve cv;
  cv.base = anchor;
  BwdBufs r;
  carve_bwd(cv, r, d, f, g, fa, ga, B);
  const int L = d->filter_type == MSFNO_FILTER_LINEAR ? 0 : d->spectral_layers;
  for (int l = 0; l < L && l < n; ++l) offsets[l] = (size_t)((char*)r.h[l] - anchor);
  *nlayers = L;
  return MSFNO_OK;
}

size_t msfno_block_backward_params_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t f,
                                                  msfno_sht_plan_t g, msfno_sht_plan_t fa,
                                                  msfno_sht_plan_t ga, int B) {
  using namespace msfno;
  if (B <= 0 || check_adjoint(d, f, g, fa, ga) != MSFNO_OK) return 0;
  Carve cv;
  BwdBufs r;
  carve_bwd(cv, r, d, f, g, fa, ga, B, true);
  return cv.off;
}

int msfno_block_backward(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                         msfno_sht_plan_t fa, msfno_sht_plan_t ga, const float* x,
                         const float* gamma, const float* beta, float film_scale,
                         const float* dout, float* dx, float* dgamma, float* dbeta, int B,
                         void* ws, size_t ws_bytes, void* stream) {
  return msfno_block_backward_params(d, f, g, fa, ga, x, gamma, beta, film_scale, dout, dx,
                                     dgamma, dbeta, nullptr, B, ws, ws_bytes, stream);
}

int msfno_block_backward_params(const msfno_block_desc* d, msfno_sht_plan_t f,
                                msfno_sht_plan_t g, msfno_sht_plan_t fa, msfno_sht_plan_t ga,
                                const float* x, const float* gamma, const float* beta,
                                float film_scale, const float* dout, float* dx, float* dgamma,
                                float* dbeta, const msfno_block_param_grads* pg, int B, void* ws,
                                size_t ws_bytes, void* stream) {
  using namespace msfno;
  MSFNO_TRY(check_adjoint(d, f, g, fa, ga));
  MSFNO_REQUIRE(x && dout && B > 0, MSFNO_EINVAL, "block backward: missing tensors");
  MSFNO_REQUIRE((gamma == nullptr) == (beta == nullptr) &&
                    (dgamma == nullptr) == (dbeta == nullptr) && (!dgamma || gamma),
                MSFNO_EINVAL, "block backward: gamma / beta / dgamma / dbeta mismatch");
  MSFNO_REQUIRE(ws_bytes >= (pg ? msfno_block_backward_params_workspace_size(d, f, g, fa, ga, B)
                                 : msfno_block_backward_workspace_size(d, f, g, fa, ga, B)),
                MSFNO_EWORKSPACE, "workspace too small");
  const bool resample = f->nlat != g->nlat || f->nlon != g->nlon;
  MSFNO_REQUIRE(!resample || (d->inner_skip == MSFNO_SKIP_NONE && d->outer_skip == MSFNO_SKIP_NONE),
                MSFNO_EINVAL, "skips require equal input and output grids");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  BwdBufs r;
  carve_bwd(cv, r, d, f, g, fa, ga, B, pg != nullptr);
  const int C = d->C;
  const int64_t BC = (int64_t)B * C;
  const int64_t Pi = (int64_t)f->nlat * f->nlon, Po = (int64_t)g->nlat * g->nlon;
  const int lmax = f->lmax, mmax = f->mmax;
  const int64_t XY = (int64_t)lmax * mmax;
  const bool lin = d->filter_type == MSFNO_FILTER_LINEAR;
  const int Hs = lin ? C : d->spec_hidden, L = lin ? 0 : d->spectral_layers;
  MSFNO_REQUIRE(Pi < (1LL << 31) && Po < (1LL << 31), MSFNO_EINVAL, "block backward: grid too large");

  // ---- forward recompute -----------------------------------------------------------
  MSFNO_TRY(launch_fill(r.ones, BC, 1.f, s));
  MSFNO_TRY(launch_fill(r.zeros, BC, 0.f, s));
  // norm0: xhat0 = sc0 x + sh0
  MSFNO_TRY(launch_row_moments(x, BC, C, Pi, d->norm0_w, d->norm0_b, d->norm_eps, r.mean0,
                               r.rstd0, r.sc0, r.sh0, s));
  MSFNO_TRY(launch_affine_rows(x, r.sc0, r.sh0, nullptr, r.xh0, BC, Pi, 0, nullptr, 0, s));
  // filter (reference layouts: SHT -> (BC, lmax, mmax) complex)
  MSFNO_TRY(msfno_sht_forward(f, r.xh0, r.A, (int)BC, r.sws, r.sws_b, s));
  if (lin) {
    const int64_t T = tril_count(lmax, mmax);
    MSFNO_REQUIRE(d->lin_w, MSFNO_EINVAL, "missing linear filter weight");
    MSFNO_TRY(launch_tril_map(r.A, r.a_t, BC, lmax, mmax, T, true, s));
    MSFNO_TRY(launch_compl_contract(r.a_t, d->lin_w, r.y_t, B, C, C, T, s));
    MSFNO_TRY(launch_tril_map(r.y_t, r.Z, BC, lmax, mmax, T, false, s));
  } else {
    const float* hin = r.A;
    for (int l = 0; l < L; ++l) {
      MSFNO_REQUIRE(d->spec_w[l], MSFNO_EINVAL, "missing spectral weight");
      MSFNO_TRY(launch_compl_mul2d(hin, d->spec_w[l], r.h[l], B, l == 0 ? C : Hs, Hs, XY, 1, s));
      hin = r.h[l];
    }
    MSFNO_TRY(launch_compl_mul2d(hin, d->spec_wout, r.Z, B, L == 0 ? C : Hs, C, XY, 0, s));
  }
  MSFNO_TRY(msfno_sht_inverse(g, r.Z, r.F, (int)BC, r.sws, r.sws_b, s));
  // inner skip: x1pre = F + Ws x + bs  |  F + x  |  F
  if (d->inner_skip == MSFNO_SKIP_LINEAR) {
    MSFNO_REQUIRE(d->skip_w, MSFNO_EINVAL, "missing inner_skip weight");
    GemmEpi e;
    e.bias = d->skip_b;
    e.addend = r.F;
    e.sD = (int64_t)C * Po;
    e.ldd = (int)Po;
    MSFNO_TRY(gemm_dense(ROLE_SKIP, TILE_128x256, d->skip_w, x, r.x1pre, C, (int)Po, C, C,
                         (int)Po, (int)Po, 0, (int64_t)C * Pi, (int64_t)C * Po, B, e, r.skws,
                         r.skws_b, s));
  } else {
    const float* add = d->inner_skip == MSFNO_SKIP_IDENTITY ? x : nullptr;
    MSFNO_TRY(launch_affine_rows(r.F, r.ones, r.zeros, add, r.x1pre, BC, Po, 0, nullptr, 0, s));
  }
  if (lin)  // GELU after the skip (sfnonet.py:373-374, linear filter only)
    MSFNO_TRY(launch_affine_rows(r.x1pre, r.ones, r.zeros, nullptr, r.x1, BC, Po, 1, nullptr, 0, s));
  // norm1: xhat1 = an1 x1 + tn1;  u = (1 + gamma s) xhat1 + beta s = sc1 x1 + sh1
  MSFNO_TRY(launch_row_moments(r.x1, BC, C, Po, d->norm1_w, d->norm1_b, d->norm_eps, r.mean1,
                               r.rstd1, r.an1, r.tn1, s));

  // ---- MLP backward: du -------------------------------------------------------------
  const float* du = dout;
  if (d->has_mlp) {
    MSFNO_REQUIRE(d->fc1_w && d->fc2_w, MSFNO_EINVAL, "missing MLP weights");
    const int Hd = d->mlp_hidden;
    const int Pi2 = (int)Po;
    if (gamma) {
      // sc1 = (1 + gamma s) an1, sh1 = (1 + gamma s) tn1 + beta s: the FiLM'd affine
      MSFNO_TRY(launch_film_affine(r.an1, r.tn1, gamma, beta, film_scale, r.sc1, r.sh1, BC, s));
    } else {
      MSFNO_CHECK_HIP(hipMemcpyAsync(r.sc1, r.an1, BC * 4, hipMemcpyDeviceToDevice, s));
      MSFNO_CHECK_HIP(hipMemcpyAsync(r.sh1, r.tn1, BC * 4, hipMemcpyDeviceToDevice, s));
    }
    // pre = W1 (sc1 x1 + sh1) + b1 = (W1 diag(sc1)) x1 + (b1 + W1 sh1) per batch
    MSFNO_TRY(launch_fold_affine(d->fc1_w, d->fc1_b, r.sc1, r.sh1, r.W1f, r.b1f, B, Hd, C, s));
    GemmEpi e1;
    e1.bias = r.b1f;
    e1.sBias = Hd;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, r.W1f, r.x1, r.pre, Hd, Pi2, C, C, Pi2, Pi2,
                         (int64_t)Hd * C, (int64_t)C * Po, (int64_t)Hd * Po, B, e1, r.wsa,
                         r.wsa_b, s));
    MSFNO_TRY(launch_transpose_mat(d->fc2_w, C, Hd, Hd, r.W2T, s));
    GemmEpi e0;
    MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, r.W2T, dout, r.dh, Hd, Pi2, C, C, Pi2, Pi2, 0,
                         (int64_t)C * Po, (int64_t)Hd * Po, B, e0, r.wsb, r.wsb_b, s));
    MSFNO_TRY(launch_gelu_grad_mul(r.dh, r.pre, (int64_t)B * Hd * Po, s));
    MSFNO_TRY(launch_transpose_mat(d->fc1_w, Hd, C, C, r.W1T, s));
    MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, r.W1T, r.dh, r.du, C, Pi2, Hd, Hd, Pi2, Pi2, 0,
                         (int64_t)Hd * Po, (int64_t)C * Po, B, e0, r.wsc, r.wsc_b, s));
    du = r.du;
    if (pg) {
      // fc2: dW2 = dout GELU(pre)^T, db2 = sum dout;  fc1: dW1 = dpre u^T with the MLP input
      // u = sc1 x1 + sh1 (norm1 + FiLM), db1 = sum dpre   (layers.py:161-168)
      if (pg->fc2_w)
        MSFNO_TRY(launch_wgrad_nt(dout, Po, (int64_t)C * Po, r.pre, Po, (int64_t)Hd * Po, C, Hd, Po,
                                  B, WGRAD_GELU, nullptr, nullptr, pg->fc2_w, Hd, 1, r.wg, r.wg_b,
                                  s));
      if (pg->fc2_b)
        MSFNO_TRY(launch_norm_param_grad(dout, nullptr, nullptr, nullptr, nullptr, 0.f, B, C, Po,
                                         nullptr, pg->fc2_b, r.nrows, s));
      if (pg->fc1_w)
        MSFNO_TRY(launch_wgrad_nt(r.dh, Po, (int64_t)Hd * Po, r.x1, Po, (int64_t)C * Po, Hd, C, Po,
                                  B, WGRAD_AFFINE, r.sc1, r.sh1, pg->fc1_w, C, 1, r.wg, r.wg_b,
                                  s));
      if (pg->fc1_b)
        MSFNO_TRY(launch_norm_param_grad(r.dh, nullptr, nullptr, nullptr, nullptr, 0.f, B, Hd, Po,
                                         nullptr, pg->fc1_b, r.nrows, s));
    }
  }
  // norm1 affine: dw1 = sum_b (1 + gamma s) sum_p du xhat1, db1 = sum_b (1 + gamma s) sum_p du
  if (pg && (pg->norm1_w || pg->norm1_b))
    MSFNO_TRY(launch_norm_param_grad(du, r.x1, r.mean1, r.rstd1, gamma, film_scale, B, C, Po,
                                     pg->norm1_w, pg->norm1_b, r.nrows, s));
  // ---- FiLM: dgamma = s sum du xhat1, dbeta = s sum du -------------------------------
  if (dgamma) MSFNO_TRY(launch_film_grad_reduce(du, r.x1, r.an1, r.tn1, film_scale, (int)BC, Po,
                                                dgamma, dbeta, s));
  bool spec_params = false;
  if (pg) {
    spec_params = pg->norm0_w || pg->norm0_b || pg->spec_wout || pg->lin_w || pg->skip_w ||
                  pg->skip_b;
    for (int l = 0; l < 8; ++l) spec_params = spec_params || pg->spec_w[l];
  }
  if (!dx && !spec_params) return MSFNO_OK;

  // ---- norm1 (and FiLM) backward: dx1 ------------------------------------------------
  MSFNO_TRY(launch_inorm_backward(r.x1, r.mean1, r.rstd1, d->norm1_w, gamma, film_scale, du,
                                  nullptr, nullptr, r.dx1, BC, C, Po, s));
  if (lin) MSFNO_TRY(launch_gelu_grad_mul(r.dx1, r.x1pre, BC * Po, s));
  // inner skip: x1pre = F + Ws x + bs -> dWs = dx1pre x^T, dbs = sum dx1pre (sfnonet.py:366-371)
  if (pg && d->inner_skip == MSFNO_SKIP_LINEAR) {
    if (pg->skip_w)
      MSFNO_TRY(launch_wgrad_nt(r.dx1, Po, (int64_t)C * Po, x, Pi, (int64_t)C * Pi, C, C, Po, B,
                                WGRAD_PLAIN, nullptr, nullptr, pg->skip_w, C, 1, r.wg, r.wg_b, s));
    if (pg->skip_b)
      MSFNO_TRY(launch_norm_param_grad(r.dx1, nullptr, nullptr, nullptr, nullptr, 0.f, B, C, Po,
                                       nullptr, pg->skip_b, r.nrows, s));
  }
  // ---- ISHT^T, filter^T, SHT^T --------------------------------------------------------
  MSFNO_TRY(msfno_sht_forward(fa, r.dx1, r.dZ, (int)BC, r.sws, r.sws_b, s));
  if (lin) {
    const int64_t T = tril_count(lmax, mmax);
    MSFNO_TRY(launch_conj_swap01(d->lin_w, C, C, T, r.wadj, s));  // (Co, Ci, T) -> (Ci, Co, T)
    MSFNO_TRY(launch_tril_map(r.dZ, r.y_t, BC, lmax, mmax, T, true, s));
    // dw[k][i][t] = sum_b dy[b][k][t] conj(a[b][i][t]) (before a_t is reused below)
    if (pg && pg->lin_w) MSFNO_TRY(launch_lin_wgrad(r.y_t, r.a_t, pg->lin_w, B, C, C, T, s));
    MSFNO_TRY(launch_compl_contract(r.y_t, r.wadj, r.a_t, B, C, C, T, s));
    MSFNO_TRY(launch_tril_map(r.a_t, r.dA, BC, lmax, mmax, T, false, s));
  } else {
    // w (Ci, Co, 2) -> w^H as compl_mul2d's (Co, Ci, 2) weight
    for (int l = 0; l <= L; ++l) {
      const int ci = l == 0 ? C : Hs, co = l == L ? C : Hs;
      MSFNO_TRY(launch_conj_swap01(l == L ? d->spec_wout : d->spec_w[l], ci, co, 1,
                                   r.wadj + r.wadj_off[l], s));
    }
    const float* g_in = r.dZ;
    float* bufs[2] = {r.da, r.db};
    for (int l = L; l >= 0; --l) {
      // dh_l = dh_{l+1} w_l^H, then the mask of the forward's activation h_{l-1}
      const int ci = l == 0 ? C : Hs, co = l == L ? C : Hs;
      // dW_l[i][o] = sum_n conj(in_l[i][n]) g_l[o][n]: real part on (re, im) rows, imaginary
      // part against the pair-swapped gradient (layers.py:604-620, complex autograd)
      float* dwl = pg ? (l == L ? pg->spec_wout : pg->spec_w[l]) : nullptr;
      if (dwl) {
        const float* in = l == 0 ? r.A : r.h[l - 1];
        for (int part = 0; part < 2; ++part)
          MSFNO_TRY(launch_wgrad_nt(in, 2 * XY, (int64_t)ci * 2 * XY, g_in, 2 * XY,
                                    (int64_t)co * 2 * XY, ci, co, 2 * XY, B,
                                    part ? WGRAD_CSWAP : WGRAD_PLAIN, nullptr, nullptr, dwl + part,
                                    2 * co, 2, r.wg, r.wg_b, s));
      }
      float* out = l == 0 ? r.dA : bufs[l & 1];
      MSFNO_TRY(launch_compl_mul2d(g_in, r.wadj + r.wadj_off[l], out, B, co, ci, XY, 0, s));
      if (l > 0) MSFNO_TRY(launch_relu_real_mask(out, r.h[l - 1], (int64_t)B * Hs * XY, s));
      g_in = out;
    }
  }
  MSFNO_TRY(msfno_sht_inverse(ga, r.dA, r.dxh0, (int)BC, r.sws, r.sws_b, s));
  // norm0 affine: dw0 = sum dxhat0_out n0, db0 = sum dxhat0_out (sfnonet.py:363)
  if (pg && (pg->norm0_w || pg->norm0_b))
    MSFNO_TRY(launch_norm_param_grad(r.dxh0, x, r.mean0, r.rstd0, nullptr, 0.f, B, C, Pi,
                                     pg->norm0_w, pg->norm0_b, r.nrows, s));
  if (!dx) return MSFNO_OK;
  // ---- norm0 backward (+ dout through the identity outer skip, + dx1 through an identity
  // inner skip), then the linear inner skip's Ws^T dx1 --------------------------------------
  const float* add1 = d->outer_skip == MSFNO_SKIP_IDENTITY ? dout : nullptr;
  const float* add2 = d->inner_skip == MSFNO_SKIP_IDENTITY ? r.dx1 : nullptr;
  const bool skip_lin = d->inner_skip == MSFNO_SKIP_LINEAR;
  MSFNO_TRY(launch_inorm_backward(x, r.mean0, r.rstd0, d->norm0_w, nullptr, 0.f, r.dxh0, add1,
                                  add2, skip_lin ? r.dxt : dx, BC, C, Pi, s));
  if (skip_lin) {
    MSFNO_TRY(launch_transpose_mat(d->skip_w, C, C, C, r.WsT, s));
    GemmEpi e;
    e.addend = r.dxt;
    e.sD = (int64_t)C * Pi;
    e.ldd = (int)Pi;
    MSFNO_TRY(gemm_dense(ROLE_SKIP, TILE_128x256, r.WsT, r.dx1, dx, C, (int)Pi, C, C, (int)Pi,
                         (int)Pi, 0, (int64_t)C * Po, (int64_t)C * Pi, B, e, r.skws2, r.skws_b,
                         s));
  }
  return MSFNO_OK;
}

}  // extern "C"
