// Internal block-orchestration helpers shared by api.cpp (single-GPU block)
// and band.cpp (latitude-band sharded block).  Not part of the C-ABI.
#pragma once
#include <memory>
#include "kernels.h"

namespace msfno {

// stage profiler (hipEvents; msfno_profile_*)
enum Stage {
  ST_FFT_FWD = 0, ST_NORM0, ST_TRANSPOSE_FWD, ST_LEG_FWD, ST_SPEC_PREP, ST_SPEC_L0, ST_SPEC_L1,
  ST_SPEC_L2, ST_SPEC_L3, ST_SPEC_OUT, ST_LIN_GATHER, ST_LIN_CONTRACT, ST_LIN_SCATTER, ST_LEG_INV,
  ST_TRANSPOSE_INV, ST_FFT_INV, ST_SKIP, ST_NORM1, ST_FC1, ST_FC2, ST_OUT_AFFINE, ST_BAND_PACK,
  ST_BAND_EXCHANGE, ST_MLP_FUSED, ST_MLP_GEN, ST_END
};
void prof(int stage, hipStream_t s);

// workspace carving: deterministic 256-B aligned sub-allocations of one buffer
struct Carve {
  size_t off = 0;
  char* base = nullptr;
  template <typename T>
  T* take(size_t count) {
    const size_t o = off;
    off = (size_t)round_up((int64_t)(off + count * sizeof(T)), 256);
    return base ? reinterpret_cast<T*>(base + o) : nullptr;
  }
};

// per-device side stream for the inner-skip GEMM (fork/join through events).  Handed out
// reference-counted: a context evicted from side_ctx's per-caller LRU map stays alive
// (its events undestroyed) until the last call holding it has finished with it
struct SideCtx {
  hipStream_t side = nullptr;  // (pooled per device, never destroyed)
  hipEvent_t fork = nullptr, join = nullptr;
  SideCtx() = default;
  SideCtx(const SideCtx&) = delete;
  SideCtx& operator=(const SideCtx&) = delete;
  ~SideCtx() {
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
  }
};
int side_ctx(std::shared_ptr<SideCtx>* out, hipStream_t caller);

// split-A workspaces of the dense GEMMs (gemm_dense): one per call site, the
// skip GEMM runs on the side stream concurrently with the spectral path
struct DenseWs {
  void *skip = nullptr, *fc1 = nullptr, *fc2 = nullptr;
  size_t skip_b = 0, fc1_b = 0, fc2_b = 0;
  void* spec[9] = {};     // real-ified spectral MLP layers (x6 engine only)
  size_t spec_b[9] = {};
};
void carve_dense_ws(Carve& cv, DenseWs& w, const msfno_block_desc* d, int B);
void carve_spec_ws(Carve& cv, DenseWs& w, const msfno_block_desc* d);
bool spec_use_x6();
int64_t spec_hidden_floats(int B, int64_t Hs, const SpecLayout& L);

struct BlockBufs {
  float2* Xn; float* Xt; float2* rs0; float* sc0; float* sh0;
  float* Sa; float* Sb; float* Sc; float* Wexp[9];
  float* xt; float* yt;
  float* Yt; float2* Yn; float* x1;
  float2* st1; float* sc1; float* sh1;
  float* ab1 = nullptr;  // norm1 output bound per (b, c) (chan_affine abound; fused x3h MLP)
  float* W1f; float* b1f; float* h;
  unsigned short* x1p;  // x1 as bf16x3 planes for fc1 (x6 engine), else null
  unsigned short* mfimg;  // fused MLP weight image (mlp_fused), else null
  float* cs;  // x3h spectral MLP: per-(b, column) input scale and its inverse [2][B][ld]
  float* xs = nullptr;  // x3h inner skip: per-(b, c) power-of-two scale of x (B-row scales)
  float* lsig = nullptr;  // legendre_x3f: per-(b, c) slab scale sigma (chan_affine)
  float* isr = nullptr;  // legendre_x3f: 1 / sigma per slab row (R)
  DenseWs dw;
};

void carve_block(Carve& cv, BlockBufs& b, const msfno_block_desc* d, const msfno_sht_plan_s* f,
                 const msfno_sht_plan_s* g, int B, bool with_norms);
int check_pair(const msfno_block_desc* d, const msfno_sht_plan_s* f, const msfno_sht_plan_s* g);
int ensure_desc(msfno_sht_plan_s* p, int R, int other_ld, int64_t ldT, hipStream_t s = nullptr);
int transpose_fwd_plan(const msfno_sht_plan_s* p, const float2* Xn, float* Xt, int B, int C,
                       const float* nscale, const float* nshift, hipStream_t s);
int transpose_inv_plan(const msfno_sht_plan_s* p, const float* Yt, float2* Yn, int B, int C,
                       hipStream_t s);
int legendre_fwd(msfno_sht_plan_s* f, const float* Xt, float* S, int R, hipStream_t s,
                 const float* rowscale = nullptr, int C = 0);
int legendre_inv(msfno_sht_plan_s* g, const float* S, float* Yt, int R, hipStream_t s);
// spectral filter on S (f->spec layout) in b.Sa (in place)
bool x3f_usable(msfno_sht_plan_s* f);
int legendre_fwd_x3f(msfno_sht_plan_s* f, const unsigned short* Xp, const float* isr, float* S,
                     int R, hipStream_t s);
int run_filter(const msfno_block_desc* d, msfno_sht_plan_s* f, msfno_sht_plan_s* g,
               const BlockBufs& b, int B, hipStream_t s);
bool use_fft_tile(const msfno_sht_plan_s* p);
bool use_c3m();
int c3m_tile();
void set_table_offsets(msfno_sht_plan_s* p, int sym);
// channel MLP with norm1/FiLM folded into (W1f, b1f): out = W2·GELU(W1f·x1 + b1f) + b2 (+resid)
int run_mlp(const msfno_block_desc* d, const float* W1f, const float* b1f, const float* x1,
            float* h, float* out, const float* resid, int B, int64_t P, const DenseWs& dw,
            hipStream_t s, const unsigned short* x1p = nullptr);
bool mlp_h_planes(bool have_ws);
// prepared-weight cache (msfno_block_desc.wcache): the fused MLP image inside it (or
// null), and whether the cached images are current (the preparation is skipped)
unsigned short* wcache_mfimg(const msfno_block_desc* d);
bool wcache_ready(const msfno_block_desc* d);
// the block MLP as one fused kernel (mlp_fused.hip): x6 engine, C 256, H 512, fc1 bias,
// P % 4 == 0 (16-B rows for the kernel's LDS-DMA tile staging)
bool mlp_fused(const msfno_block_desc* d, int64_t P);
// x1p buffer needed: x1 planes from the irfft, or x planes from the rfft for the skip GEMM
bool x1p_buffer(const msfno_block_desc* d, const msfno_sht_plan_s* g);
// MLP stage of the block on x1 (fp32, or planes x1p when x1_planes): norm1/FiLM affine
// (sc1, sh1) applied in the fused kernel, or folded into (W1f, b1f) for run_mlp
int run_block_mlp(const msfno_block_desc* d, const float* x1, const unsigned short* x1p,
                  const float* sc1, const float* sh1, const float* ab1, float* W1f, float* b1f, float* h,
                  unsigned short* mfimg, float* out, const float* resid, int B, int64_t P,
                  const DenseWs& dw, hipStream_t s);
int64_t mlp_chunk(int64_t P);
int64_t mlp_h_floats(int B, int64_t Hd, int64_t P);
bool x1_planes(const msfno_block_desc* d, const msfno_sht_plan_s* g);
bool skip_planes(const msfno_block_desc* d, const msfno_sht_plan_s* f, const BlockBufs& b);
// the inner-skip GEMM on the x3h engine (gemm_x3), forked after the norm0 statistics
bool skip_x3(const msfno_block_desc* d);
// plan construction (mask: optional m-set, see SpecLayout::build)
int plan_create(int nlat, int nlon, int lmax, int mmax, int inverse,
                const std::vector<char>* mask, msfno_sht_plan_s** out);

}  // namespace msfno
