/*
 * msfno.h — C-ABI of libmsfno.so, the MI355X (gfx950) implementation of the
 * SFNO-Block forward hot path of Slusny/Modulated-Spherical-Fourier-Neural-Operator.
 *
 * The reference path is pure Python/PyTorch (no FFI).  Every entry point below
 * replaces one stock-torch / torch-harmonics call of the reference; the
 * replaced interface is cited on each declaration (paths relative to the
 * reference repo).  The Python host layer (msfno_amd/, ctypes) mirrors the
 * reference module API on top of these functions.
 *
 * Conventions
 *   - Plain pointers + sizes; every device pointer is caller-owned (PyTorch
 *     tensors); the library owns only plans (tables, twiddles, descriptors).
 *   - All work is stream-ordered on the hipStream_t passed as `stream`
 *     (void*); no call synchronises the device, allocates device memory or
 *     copies to the host, except *_plan_create/_load_* (one-time setup).
 *   - Return value: 0 = ok, otherwise an MSFNO_E* code; msfno_last_error()
 *     returns a thread-local message.  The Python layer re-raises the
 *     reference's exception types (NotImplementedError / ValueError /
 *     AssertionError) from these codes.
 *   - fp32 arithmetic throughout (complex64 in spectral space), as the
 *     reference runs its transforms with autocast disabled
 *     (MSFNO/Models/sfno/layers.py:403-422, 627-637).
 */
#ifndef MSFNO_H
#define MSFNO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSFNO_OK 0
#define MSFNO_EINVAL 1         /* bad argument / shape   -> ValueError / AssertionError */
#define MSFNO_EUNSUPPORTED 2   /* unsupported config    -> NotImplementedError        */
#define MSFNO_EHIP 3           /* HIP runtime failure   -> RuntimeError               */
#define MSFNO_EWORKSPACE 4     /* workspace too small    -> ValueError                 */

#define MSFNO_GRID_EQUIANGULAR 0
#define MSFNO_GRID_LEGENDRE_GAUSS 1

typedef struct msfno_sht_plan_s* msfno_sht_plan_t;

const char* msfno_last_error(void);
int msfno_abi_version(void);

/* ---------------------------------------------------------------------------
 * Host-side plan math (fp64).  Replaces torch_harmonics.quadrature
 * (used at MSFNO/Models/losses.py:90,129) and torch_harmonics.legendre as
 * used by RealSHT/InverseRealSHT.__init__ (constructed at
 * MSFNO/Models/sfno/sfnonet.py:537-548).
 * ------------------------------------------------------------------------- */
/* nodes ascending in [-1,1] (cos of colatitude, before the north->south flip) */
int msfno_quadrature(int nlat, int grid, double* nodes, double* weights);
/* table (mmax, lmax, nlat) float64, colatitudes north->south:
 *   inverse == 0 : P̄_l^m(cos θ_k) · w_k   (RealSHT.weights)
 *   inverse == 1 : P̄_l^m(cos θ_k)         (InverseRealSHT.pct)
 * orthonormal ("ortho") normalisation, Condon–Shortley phase if csphase. */
int msfno_legendre_table(int mmax, int lmax, int nlat, int grid, int inverse, int csphase,
                         double* table);

/* ---------------------------------------------------------------------------
 * SHT plans.  One plan per transform object (RealSHT / InverseRealSHT).
 * ------------------------------------------------------------------------- */
int msfno_sht_plan_create(int nlat, int nlon, int lmax, int mmax, int inverse,
                          msfno_sht_plan_t* plan);
int msfno_sht_plan_destroy(msfno_sht_plan_t plan);
/* Copy + re-lay-out the module's table (mmax,lmax,nlat) fp32 device buffer
 * (RealSHT.weights incl. the ×1e5 of sfnonet.py:552/554, or
 * InverseRealSHT.pct incl. the ÷1e5 of :553/:555) into the plan's GEMM layout. */
int msfno_sht_plan_load_table(msfno_sht_plan_t plan, const float* table, void* stream);

/* RealSHT.forward  (torch_harmonics RealSHT; called at layers.py:405,629):
 *   x (bc, nlat, nlon) fp32  ->  out (bc, lmax, mmax) complex64 interleaved */
size_t msfno_sht_workspace_size(msfno_sht_plan_t plan, int bc);
int msfno_sht_forward(msfno_sht_plan_t plan, const float* x, float* out, int bc,
                      void* ws, size_t ws_bytes, void* stream);
/* InverseRealSHT.forward (called at layers.py:421,638):
 *   in (bc, lmax, mmax) complex64 -> x (bc, nlat, nlon) fp32 */
int msfno_sht_inverse(msfno_sht_plan_t plan, const float* in, float* x, int bc,
                      void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Contractions (MSFNO/Models/sfno/contractions.py)
 * ------------------------------------------------------------------------- */
/* compl_contract_fwd_c  (contractions.py:37-41, einsum "bin,kin->bkn"):
 *   a (B,Ci,T,2), w (Co,Ci,T,2) -> y (B,Co,T,2)   [linear filter, layers.py:410-413] */
int msfno_compl_contract_fwd_c(const float* a, const float* w, float* y, int B, int Ci,
                               int Co, int T, void* stream);
/* compl_mul2d_fwd_c (contractions.py:132-137, einsum "bixy,io->boxy"):
 *   a (B,Ci,XY,2), w (Ci,Co,2) -> y (B,Co,XY,2); relu_real != 0 fuses
 *   ComplexReLU(mode="real") (activations.py:42-46) */
int msfno_compl_mul2d_fwd_c(const float* a, const float* w, float* y, int B, int Ci, int Co,
                            long long XY, int relu_real, void* stream);

/* 1x1 convolution, the block's inner skip as a standalone op (nn.Conv2d(C, C, 1) at
 * sfnonet.py:304-307, applied at :366-371):  out[b] = W x[b] + bias (per pixel)
 *   w (Cout, Cin, 1, 1), bias (Cout) or NULL, x (B, Cin, P), out (B, Cout, P); fp32 in and
 *   out, computed on the x3h engine (fp32 as two fp16 terms, three MFMAs per product)
 *   under per-(b, channel) power-of-two scales from max |x| (as accurate as fp32). */
size_t msfno_conv1x1_workspace_size(int B, int Cin, int Cout);
int msfno_conv1x1(const float* w, const float* bias, const float* x, float* out, int B, int Cin,
                  int Cout, long long P, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Fused SFNO-Block forward.
 * Replaces FourierNeuralOperatorBlock.forward (sfnonet.py:221-251) and
 * FourierNeuralOperatorBlock_Filmed.forward (sfnonet.py:359-393) including
 * SpectralFilterLayer (:56-133), SpectralAttentionS2 (layers.py:536-639) /
 * SpectralConvS2 (layers.py:336-427), InstanceNorm2d ×2, FiLM (:689-697) and
 * MLP (layers.py:145-178).
 * ------------------------------------------------------------------------- */
#define MSFNO_FILTER_NONLINEAR 0
#define MSFNO_FILTER_LINEAR 1
#define MSFNO_SKIP_NONE 0
#define MSFNO_SKIP_LINEAR 1
#define MSFNO_SKIP_IDENTITY 2

typedef struct msfno_block_desc {
  int C;                    /* embed_dim_sfno                                       */
  int filter_type;          /* MSFNO_FILTER_*                                       */
  int inner_skip;           /* MSFNO_SKIP_*   (sfnonet.py:304-307)                  */
  int outer_skip;           /* MSFNO_SKIP_NONE / _IDENTITY (sfnonet.py:333-336)      */
  int has_mlp;              /* mlp_mode != "none" (sfnonet.py:323)                  */
  int mlp_hidden;           /* int(C*mlp_ratio)                                      */
  int spectral_layers;      /* non-linear: number of hidden complex layers (w.0..)  */
  int spec_hidden;          /* non-linear: int(hidden_size_factor*C)               */
  float norm_eps;           /* InstanceNorm2d eps (1e-6, sfnonet.py:494)            */
  const float* norm0_w; const float* norm0_b;       /* (C)                          */
  const float* norm1_w; const float* norm1_b;       /* (C)                          */
  const float* spec_w[8];   /* non-linear: w.l  (Cin_l, Cout_l, 2)                  */
  const float* spec_wout;   /* non-linear: wout (spec_hidden, C, 2)                 */
  const float* lin_w;       /* linear: w (C, C, T, 2), T = #tril(lmax,mmax)         */
  const float* skip_w; const float* skip_b;         /* inner_skip (C,C,1,1), (C)    */
  const float* fc1_w; const float* fc1_b;           /* mlp.fwd.0 (H,C,1,1), (H)     */
  const float* fc2_w; const float* fc2_b;           /* mlp.fwd.2 (C,H,1,1), (C)     */
  /* Prepared-weight cache (optional).  The kernels consume the weights as bf16x3
   * "images" (the spectral-MLP 3M A images, the fused block MLP's slice image).
   * wcache: device buffer of msfno_block_wcache_size(d) bytes owned by the caller
   * (one per module), or NULL: the images are rebuilt in the workspace on every
   * call.  wcache_valid = 1: wcache already holds the images of the current weight
   * values (the call skips the preparation); 0: the call rebuilds them into
   * wcache.  The caller tracks weight changes (the Python mirror keys it on the
   * parameters' (data_ptr, _version)). */
  void* wcache;
  int wcache_valid;
} msfno_block_desc;

size_t msfno_block_wcache_size(const msfno_block_desc* d);

size_t msfno_block_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                  msfno_sht_plan_t inv, int B);
/* x (B,C,nlat_in,nlon_in) -> out (B,C,nlat_out,nlon_out).  gamma/beta (B,C) may
 * be NULL (unfilmed block); FiLM is (1+γ·scale)·x + β·scale after norm1. */
int msfno_block_forward(const msfno_block_desc* d, msfno_sht_plan_t fwd, msfno_sht_plan_t inv,
                        const float* x, const float* gamma, const float* beta, float film_scale,
                        float* out, int B, void* ws, size_t ws_bytes, void* stream);
/* The same block stopped before its output affine (blocks without MLP and outer skip:
 * the network's last block, sfnonet.py:838-846): x1_out (B,C,nlat_out,nlon_out) gets the
 * block's pre-norm1 state and affine_out (2*B*C) the per-(b,c) norm1 (+ FiLM) affine as
 * [scale (B*C)][shift (B*C)]; out = scale * x1 + shift.  The network hands both to
 * msfno_mlp_forward_affine (the decoder), so the affine pass over the full grid is
 * folded into the decoder's input loads.  Workspace: msfno_block_workspace_size. */
int msfno_block_forward_deferred(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                 msfno_sht_plan_t inv, const float* x, const float* gamma,
                                 const float* beta, float film_scale, float* x1_out,
                                 float* affine_out, int B, void* ws, size_t ws_bytes,
                                 void* stream);
/* FourierNeuralOperatorBlock_Filmed.global_conv(x, residual) (sfnonet.py:341-356): the
 * block up to norm1 -- norm0(x) -> filter -> + inner_skip(residual) (+ GELU for the
 * linear filter) -> norm1 -- without FiLM, MLP or outer skip.  residual may be NULL
 * (= x).  x, residual (B,C,nlat_in,nlon_in) -> out (B,C,nlat_out,nlon_out).
 * Workspace: msfno_block_workspace_size. */
int msfno_block_global_conv(const msfno_block_desc* d, msfno_sht_plan_t fwd, msfno_sht_plan_t inv,
                            const float* x, const float* residual, float* out, int B, void* ws,
                            size_t ws_bytes, void* stream);
/* SpectralFilterLayer.forward alone (sfnonet.py:132-133): SHT -> filter -> ISHT,
 * no norms.  x (B,C,nlat_in,nlon_in) -> y (B,C,nlat_out,nlon_out). */
int msfno_filter_forward(const msfno_block_desc* d, msfno_sht_plan_t fwd, msfno_sht_plan_t inv,
                         const float* x, float* y, int B, void* ws, size_t ws_bytes,
                         void* stream);

/* ---------------------------------------------------------------------------
 * Channel MLP (MSFNO/Models/sfno/layers.py:145-178, MLP.forward) as used by the
 * network encoder and decoder (sfnonet.py:513-523, 617-629, forward :667-686):
 *   out = W2 · GELU(W1 · [x ; x2] + b1) (+ b2) (+ addend)
 * x (B, Cin, P) and the optional second input x2 (B, Cin2, P) are the two halves
 * of the channel concatenation torch.cat((x, residual), dim=1) of the big skip
 * (sfnonet.py:680-681), consumed without materialising it; fc1_w is
 * (Hid, Cin + Cin2).  addend (optional) is added to the output with batch
 * stride add_bstride (0 broadcasts it: the encoder's pos_embed, :674).
 * ------------------------------------------------------------------------- */
typedef struct msfno_mlp_desc {
  int Cin, Cin2, Hid, Cout;
  const float* fc1_w; const float* fc1_b;   /* (Hid, Cin+Cin2, 1, 1), (Hid)  */
  const float* fc2_w; const float* fc2_b;   /* (Cout, Hid, 1, 1), (Cout) or NULL */
  /* Prepared-weight cache of the fused widths (as msfno_block_desc.wcache): NULL, or a
   * device buffer of msfno_mlp_wcache_size(d) bytes owned by the caller (one per
   * module) holding the x3h weight image; wcache_valid = 1 skips its preparation. */
  void* wcache;
  int wcache_valid;
} msfno_mlp_desc;

size_t msfno_mlp_wcache_size(const msfno_mlp_desc* d);
size_t msfno_mlp_workspace_size(const msfno_mlp_desc* d, int B, long long P);
/* 1 when the widths (Cin + Cin2, Hid, Cout) have the one-launch fused x3h kernel
 * (the encoder 73 -> 256 -> 256 and decoder 329 -> 256 -> 73 of the reference config). */
int msfno_mlp_fused_supported(const msfno_mlp_desc* d);
/* msfno_mlp_forward with x replaced by x_scale[b][c] * x + x_shift[b][c] (c < Cin; the
 * affine_out of msfno_block_forward_deferred); fused widths only (MSFNO_EUNSUPPORTED
 * otherwise).  Workspace: msfno_mlp_workspace_size. */
int msfno_mlp_forward_affine(const msfno_mlp_desc* d, const float* x, const float* x_scale,
                             const float* x_shift, const float* x2, const float* addend,
                             long long add_bstride, float* out, int B, long long P, void* ws,
                             size_t ws_bytes, void* stream);
int msfno_mlp_forward(const msfno_mlp_desc* d, const float* x, const float* x2,
                      const float* addend, long long add_bstride, float* out, int B,
                      long long P, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * FiLM backward.  MSFNO fine-tunes only its FiLM
 * generator: the filmed blocks and the decoder run with autograd, every SFNO
 * weight is frozen (MSFNO/Models/sfno/sfnonet.py:787-860, the training loop of
 * MSFNO/main.py).  These entry points give the gradients autograd would
 * compute there.
 *
 * msfno_block_film_backward replaces the backward of
 * FourierNeuralOperatorBlock_Filmed.forward(x, gamma, beta, scale)
 * (sfnonet.py:359-393) with respect to gamma and beta: given dout = dL/d(out),
 *   dgamma[b,c] = scale * sum_p du[b,c,p] * xhat[b,c,p],
 *   dbeta[b,c]  = scale * sum_p du[b,c,p],
 * with xhat = norm1(x1) (InstanceNorm-1 output), u = (1 + gamma scale) xhat +
 * beta scale, du = dL/du (through the channel MLP when the block has one; the
 * identity outer skip does not depend on u).  The forward up to x1 is recomputed
 * (as the reference's checkpoint(blk, ...)).  dL/dx is not produced: with the
 * reference default film_layers = 1 the filmed block is the last one and
 * nothing before it takes gradients.
 * ------------------------------------------------------------------------- */
size_t msfno_block_film_backward_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                                msfno_sht_plan_t inv, int B);
int msfno_block_film_backward(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                              msfno_sht_plan_t inv, const float* x, const float* gamma,
                              const float* beta, float film_scale, const float* dout,
                              float* dgamma, float* dbeta, int B, void* ws, size_t ws_bytes,
                              void* stream);

/* Full backward of the block, SFNO weights frozen: dx = dL/dx (and dgamma / dbeta for a
 * filmed block) for dout = dL/d(out) of msfno_block_forward -- what --film-layers k
 * (main.py:1083-1087) and --repeat-film (main.py:1133-1136) need, whose filmed blocks
 * run back to back with autograd (sfnonet.py:838-844).  The forward is recomputed.  Two
 * adjoint transform plans (built once by the caller):
 *   fwd_adj: a FORWARD plan on inv's grid, table pct[m,l,k] c_m nlon_out / (2 pi) with
 *            c_m = 1 for m = 0 and m = nlon_out / 2, else 2   (the adjoint of inv);
 *   inv_adj: an INVERSE plan on fwd's grid, table weights[m,l,k] d_m (2 pi) / nlon_in with
 *            d_m = 1 for m = 0 and m = nlon_in / 2, else 1/2  (the adjoint of fwd).
 * dx (B,C,nlat_in,nlon_in), dgamma / dbeta (B,C) may each be NULL; gamma / beta NULL for an
 * unfilmed block. */
size_t msfno_block_backward_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                           msfno_sht_plan_t inv, msfno_sht_plan_t fwd_adj,
                                           msfno_sht_plan_t inv_adj, int B);
int msfno_block_backward(const msfno_block_desc* d, msfno_sht_plan_t fwd, msfno_sht_plan_t inv,
                         msfno_sht_plan_t fwd_adj, msfno_sht_plan_t inv_adj, const float* x,
                         const float* gamma, const float* beta, float film_scale,
                         const float* dout, float* dx, float* dgamma, float* dbeta, int B,
                         void* ws, size_t ws_bytes, void* stream);
/* Parameter gradients of the block (the reference's --retrain-film, main.py:958-960: the
 * decoder and the last film_layers blocks train, MSFNO/Models/sfno/model.py:922-923,
 * 1016-1019).  Device fp32 outputs, each laid out as the parameter it is the gradient of;
 * NULL = not wanted.  Written (not accumulated). */
typedef struct msfno_block_param_grads {
  float* norm0_w;      /* (C)                     norm0.weight */
  float* norm0_b;      /* (C)                     norm0.bias */
  float* spec_w[8];    /* (Ci, Co, 2)             filter_layer.filter.w.l (non-linear) */
  float* spec_wout;    /* (spec_hidden, C, 2)     filter_layer.filter.wout */
  float* lin_w;        /* (C, C, T, 2)            filter_layer.filter.w (linear) */
  float* skip_w;       /* (C, C)                  inner_skip.weight */
  float* skip_b;       /* (C)                     inner_skip.bias */
  float* norm1_w;      /* (C)                     norm1.weight */
  float* norm1_b;      /* (C)                     norm1.bias */
  float* fc1_w;        /* (mlp_hidden, C)         mlp.fwd.0.weight */
  float* fc1_b;        /* (mlp_hidden)            mlp.fwd.0.bias */
  float* fc2_w;        /* (C, mlp_hidden)         mlp.fwd.2.weight */
  float* fc2_b;        /* (C)                     mlp.fwd.2.bias */
} msfno_block_param_grads;

/* msfno_block_backward plus the parameter gradients `pg` asks for (NULL pg: exactly
 * msfno_block_backward).  Weight gradients reduce over pixels or spectral modes in fp32
 * chunks combined in fp64. */
size_t msfno_block_backward_params_workspace_size(const msfno_block_desc* d,
                                                  msfno_sht_plan_t fwd, msfno_sht_plan_t inv,
                                                  msfno_sht_plan_t fwd_adj,
                                                  msfno_sht_plan_t inv_adj, int B);
int msfno_block_backward_params(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                msfno_sht_plan_t inv, msfno_sht_plan_t fwd_adj,
                                msfno_sht_plan_t inv_adj, const float* x, const float* gamma,
                                const float* beta, float film_scale, const float* dout, float* dx,
                                float* dgamma, float* dbeta, const msfno_block_param_grads* pg,
                                int B, void* ws, size_t ws_bytes, void* stream);

/* Introspection of msfno_block_backward's workspace: the byte offsets of the recomputed
 * non-linear filter's hidden activations h_l = ComplexReLU(...) (B, spec_hidden, lmax,
 * mmax) complex, l < spectral_layers, whose ReLU(real) masks the backward applies.  Writes
 * at most n offsets and the number of hidden layers (0 for the linear filter) to *nlayers.
 * Lets a test compare the masks the GPU actually used with an oracle's. */
int msfno_block_backward_hidden_offsets(const msfno_block_desc* d, msfno_sht_plan_t fwd,
                                        msfno_sht_plan_t inv, msfno_sht_plan_t fwd_adj,
                                        msfno_sht_plan_t inv_adj, int B, size_t* offsets, int n,
                                        int* nlayers);

/* Backward of the channel MLP (layers.py:145-178) to its first input, weights
 * frozen: the decoder over cat(x, residual) (sfnonet.py:679-686) when the loss
 * gradient dy = dL/dy reaches it.
 *   dx = W1[:, :Cin]^T (GELU'(W1 [x ; x2] + b1) * (W2^T dy))
 * (dL/dx2 is not produced: x2 is the network input.) */
/* The same backward with the second input's and the parameter gradients (the decoder
 * under --retrain-film; a plain network in training, whose big skip x2 is the network
 * input):  dx2 = W1[:, Cin:]^T dpre,  dW1 = dpre [x ; x2]^T, db1 = sum dpre,
 * dW2 = dy GELU(pre)^T, db2 = sum dy (summed over the batch and the P pixels).  dx, dx2
 * and each gradient output may be NULL. */
size_t msfno_mlp_backward_params_workspace_size(const msfno_mlp_desc* d, int B, long long P);
int msfno_mlp_backward_params(const msfno_mlp_desc* d, const float* x, const float* x2,
                              const float* dy, float* dx, float* dx2, float* dfc1_w,
                              float* dfc1_b, float* dfc2_w, float* dfc2_b, int B, long long P,
                              void* ws, size_t ws_bytes, void* stream);
size_t msfno_mlp_backward_input_workspace_size(const msfno_mlp_desc* d, int B, long long P);
int msfno_mlp_backward_input(const msfno_mlp_desc* d, const float* x, const float* x2,
                             const float* dy, float* dx, int B, long long P, void* ws,
                             size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Latitude-band sharded SFNO-Block (multi-GPU form of
 * msfno_block_forward).  The reference runs one block per process on the whole
 * field (DDP = replicas, MSFNO/main.py:1153); this splits ONE field batch over
 * `world` ranks.  row_start (world + 1 entries) partitions the northern half of
 * the grid, rows [0, nlat - nlat/2) (the equator row of an odd grid included):
 * rank r owns the band [row_start[r], row_start[r+1]) and the mirror rows
 * nlat-1-k of its band rows k < nlat/2, for every pointwise / FFT / 1x1-conv /
 * MLP stage (msfno_band_local_rows lists them: the band ascending, then the
 * mirrors ascending), and the zonal wavenumbers {m : m_owner[m] == r} for the
 * Legendre transforms and the spectral filter.  Owning mirror pairs keeps the
 * hemisphere fold of the symmetric Legendre transform local, and the exchange
 * buffers are the Legendre GEMMs' own operands (no re-layout pass).
 * The caller (Python, torch.distributed over RCCL) performs the collectives
 * between the stages; the library never communicates:
 *
 *   stage 0  x_local -> inner-skip GEMM (side stream), FFT rows    -> stats_local
 *   [all_gather stats_local -> stats_all]              (norm0, B*C*3 doubles)
 *   stage 1  norm0 affine, pack spectra by owner of m     -> send
 *   [all_to_all send -> recv, counts from msfno_band_exchange_counts(phase 0)]
 *   stage 2  recv -> Legendre fwd -> filter -> Legendre inv -> send
 *   [all_to_all send -> recv, phase 1]
 *   stage 3  recv -> inverse FFT rows + skip (+GELU)       -> stats_local
 *   [all_gather stats_local -> stats_all]              (norm1)
 *   stage 4  norm1 (+FiLM) -> MLP (+outer skip)            -> out_local
 *
 * Resampling blocks (different input and output grids, sfnonet.py:573-614: the
 * first block 721x1440 -> 120x240 and the last one back) take a second row
 * partition for the output grid (msfno_band_plan_create2); skips then must be
 * absent, as in the reference.  Both filters: the linear filter's per-mode
 * weight is sharded with the m-set (msfno_band_linear_modes), so each rank
 * streams only its modes' slice.  At most 64 ranks.
 *
 * Several sub-batches of one forward may be in flight between stage 0 and
 * stage 3 at once (their exchanges overlapping each other's compute): give each
 * a distinct io.slot (0..63), its own workspace and its own exchange buffers.
 * ------------------------------------------------------------------------- */
typedef struct msfno_band_plan_s* msfno_band_plan_t;

/* Default partition (host only, no GPU): balanced bands of the northern half and
 * a zig-zag (snake) assignment of m = 0..mact-1 that balances both the count of
 * m and the Legendre/filter work sum(lmax - m) per rank; m >= lmax -> -1. */
int msfno_band_partition(int world, int nlat, int lmax, int mmax, int* row_start, int* m_owner);
/* all-to-all element counts (floats) per peer for `rank` (host only):
 * phase 0 (spectra rows->m), phase 1 (m->rows); R = 2*B*C.  Every exchanged slab
 * row holds 2W floats, W = the widest band rounded up to 16. */
int msfno_band_exchange_counts(int world, int rank, int nlat, int mmax, const int* row_start,
                               const int* m_owner, int R, int phase, long long* send_counts,
                               long long* recv_counts);
/* The global latitude rows of `rank`'s local rows, in local order (rows may be
 * NULL to query *count = band rows + mirror rows). */
int msfno_band_local_rows(int world, int rank, int nlat, const int* row_start, int* rows,
                          int* count);
int msfno_band_plan_create(int nlat, int nlon, int lmax, int mmax, int world, int rank,
                           const int* row_start, const int* m_owner, msfno_band_plan_t* plan);
/* Resampling form: rows of the input grid (nlat_in x nlon_in, the forward
 * transform's) in row_in, of the output grid (the inverse transform's) in row_out. */
int msfno_band_plan_create2(int nlat_in, int nlon_in, int nlat_out, int nlon_out, int lmax,
                            int mmax, int world, int rank, const int* row_in, const int* row_out,
                            const int* m_owner, msfno_band_plan_t* plan);
/* all-to-all counts (floats per peer) of this plan's rank, phase 0 / 1, R = 2*B*C */
int msfno_band_plan_exchange_counts(msfno_band_plan_t plan, int R, int phase,
                                    long long* send_counts, long long* recv_counts);
/* Linear filter (SpectralConvS2, layers.py:336-427): the global tril indices
 * (torch.tril_indices(lmax, mmax) order, layers.py:368) of this rank's modes, in
 * ascending order; *count = their number T_r (modes may be NULL to query it).
 * The descriptor's lin_w for msfno_band_block_stage is then w[:, :, modes, :],
 * i.e. (C, C, T_r, 2) — the rank's share of the 34 GB weight at lmax 360. */
int msfno_band_linear_modes(msfno_band_plan_t plan, long long* modes, long long* count);
int msfno_band_plan_destroy(msfno_band_plan_t plan);
/* full reference tables (mmax,lmax,nlat) fp32 device buffers (RealSHT.weights,
 * InverseRealSHT.pct incl. the 1e5 rescale); only this rank's m-set is kept */
int msfno_band_plan_load_tables(msfno_band_plan_t plan, const float* fwd_table,
                                const float* inv_table, void* stream);

typedef struct msfno_band_io {
  const float* x;           /* (B, C, rows_local, nlon), msfno_band_local_rows  */
  const float* gamma;       /* (B, C) or NULL                                   */
  const float* beta;        /* (B, C) or NULL                                   */
  float film_scale;
  float* out;               /* (B, C, rows_local, nlon)                         */
  float* send;              /* exchange buffers, >= max over phases of the sum  */
  float* recv;              /*   of the send / recv counts (floats)             */
  double* stats_local;      /* (B*C, 3) {n, mean, M2}                           */
  const double* stats_all;  /* (world, B*C, 3), the all_gather of stats_local   */
  int slot;                 /* in-flight sub-batch index 0..63 (inner-skip join) */
} msfno_band_io;

size_t msfno_band_workspace_size(const msfno_block_desc* d, msfno_band_plan_t plan, int B);
/* Run one stage (0..4) on `stream`.  ws must be the same buffer for all five
 * stages of one forward. */
int msfno_band_block_stage(const msfno_block_desc* d, msfno_band_plan_t plan, int stage,
                           const msfno_band_io* io, int B, void* ws, size_t ws_bytes,
                           void* stream);

/* ---------------------------------------------------------------------------
 * Instrumentation (not a reference interface): per-stage device time of the
 * fused block measured with hipEvents recorded on the caller's stream between
 * stages.  Used by bench.py to time the dominant kernel inside the timed region.
 * ------------------------------------------------------------------------- */
#define MSFNO_PROF_NSTAGES 32
int msfno_profile_enable(int on);
/* mark the start of `stage` on `stream` (bench: the wait on a collective) */
int msfno_profile_mark(int stage, void* stream);
/* synchronises on the recorded events, adds per-stage milliseconds / launch
 * counts since the last collect into total_ms[stage] / counts[stage] (arrays of
 * MSFNO_PROF_NSTAGES), and clears the recorded marks */
int msfno_profile_collect(double* total_ms, int* counts);
const char* msfno_profile_stage_name(int stage);

#ifdef __cplusplus
}
#endif
#endif /* MSFNO_H */
