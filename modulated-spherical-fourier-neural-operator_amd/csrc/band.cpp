// Latitude-band sharded SFNO-Block: plans, exchange layout and
// the five per-rank stages between which the caller runs the collectives
// (include/msfno.h, "Latitude-band sharded SFNO-Block").
//
// Ownership.  row_start partitions the northern half [0, Ke) of the grid (Ke =
// nlat - nlat/2, the equator row included); rank r owns its band [a, b) and the
// mirror rows nlat-1-k of the band rows k < nlat/2.  Its local rows are the band
// ascending, then the mirrors ascending, so local row H-1-i is the mirror of local
// row i: the hemisphere fold of the symmetric Legendre transform is local.
//
// Exchange layout.  Every slab row has 2W floats (W = the widest band rounded up
// to 16): [Xs | Xa] folded on a symmetric plan, the local rows on a general one,
// zero padded.  Slabs leave stage 1 ordered by (owner of m, m), so the block for
// each peer is contiguous, and the receiver's buffer [source p][slab][R][2W] is
// read by the forward Legendre GEMM directly (its K index runs over the source
// blocks, common.h msfno_sht_plan_s band fields); the inverse GEMM writes the
// phase-1 send buffer [destination p][slab][R][2W] the same way.  No re-layout
// pass between the FFTs and the Legendre GEMMs beyond the one transpose each way
// that the unsharded block has too.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "block.h"

using namespace msfno;

struct msfno_band_plan_s {
  // input grid (stages 0-1) and output grid (stages 3-4); equal except for the
  // resampling blocks of a network (sfnonet.py:573-614: block 0 721x1440 -> 120x240,
  // the last block back)
  int nlat_in = 0, nlon_in = 0, nlat_out = 0, nlon_out = 0;
  int lmax = 0, mmax = 0, world = 0, rank = 0;
  std::vector<int> row_in, row_out;  // world + 1 band boundaries (northern half) on each grid
  int W_in = 0, W_out = 0;           // exchange slab rows hold 2W floats
  std::vector<int> owner;            // per m, -1: no coefficients (m >= lmax)
  std::vector<int> nm_of;            // per rank: number of owned m
  int rows_in = 0, rows_out = 0;     // local latitude rows (band + mirrors)
  int nm = 0;                        // local m count
  int mact = 0;                      // global count of m with lmax - m > 0
  msfno_sht_plan_s* fwd = nullptr;
  msfno_sht_plan_s* inv = nullptr;
  int* d_perm = nullptr;
  // inner-skip join events, one per in-flight sub-batch slot (msfno_band_io.slot):
  // several sub-batches of one forward can be between stage 0 and stage 3 at once
  std::vector<hipEvent_t> join;
  bool same_grid() const { return nlat_in == nlat_out && nlon_in == nlon_out; }
};

namespace {

struct BandRows {
  int a, b, bw, np, H;  // band [a, b), bw = b - a, np mirrored rows, H = bw + np
};
BandRows band_rows(int nlat, const int* rs, int r) {
  BandRows o;
  o.a = rs[r];
  o.b = rs[r + 1];
  o.bw = o.b - o.a;
  o.np = std::max(0, std::min(o.b, nlat / 2) - o.a);
  o.H = o.bw + o.np;
  return o;
}
int band_width(int world, const int* rs) {
  int w = 1;
  for (int r = 0; r < world; ++r) w = std::max(w, rs[r + 1] - rs[r]);
  return (int)round_up(w, 16);
}
// global latitude of local row i of rank r
int band_global_row(int nlat, const BandRows& o, int i) {
  return i < o.bw ? o.a + i : nlat - (o.a + o.np) + (i - o.bw);
}
// this rank's local rows as a small symmetric grid for the pack / unpack transposes
LatGeom band_geom(const msfno_sht_plan_s* sp, const BandRows& o, int W) {
  return LatGeom{sp->sym, o.H, o.np, o.bw, o.np, W, 2 * W};
}
// exchange-column -> latitude maps of a band plan (common.h msfno_sht_plan_s)
void set_band_maps(msfno_sht_plan_s* sp, int world, const int* rs, int W) {
  sp->band_world = world;
  sp->band_W = W;
  sp->kmap_sym.assign((size_t)world * W, -1);
  sp->kmap_gen.assign((size_t)world * 2 * W, -1);
  for (int p = 0; p < world; ++p) {
    const BandRows o = band_rows(sp->nlat, rs, p);
    for (int j = 0; j < o.bw; ++j) sp->kmap_sym[(size_t)p * W + j] = o.a + j;
    for (int i = 0; i < o.H; ++i)
      sp->kmap_gen[(size_t)p * 2 * W + i] = band_global_row(sp->nlat, o, i);
  }
}

}  // namespace

namespace {

int validate_rows(int world, int nlat, const int* row_start) {
  MSFNO_REQUIRE(row_start, MSFNO_EINVAL, "null row partition");
  MSFNO_REQUIRE(row_start[0] == 0 && row_start[world] == nlat - nlat / 2, MSFNO_EINVAL,
                "row_start must run from 0 to nlat - nlat/2 (the northern half and equator)");
  for (int r = 0; r < world; ++r)
    MSFNO_REQUIRE(row_start[r + 1] > row_start[r], MSFNO_EINVAL,
                  "every rank needs at least one latitude row");
  return MSFNO_OK;
}

int validate_partition(int world, int nlat, int lmax, int mmax, const int* row_start,
                       const int* m_owner) {
  MSFNO_REQUIRE(world >= 1 && world <= 64, MSFNO_EUNSUPPORTED, "band sharding needs 1..64 ranks");
  MSFNO_REQUIRE(row_start && m_owner, MSFNO_EINVAL, "null partition arrays");
  MSFNO_TRY(validate_rows(world, nlat, row_start));
  for (int m = 0; m < mmax; ++m) {
    const bool has = lmax - m > 0;
    MSFNO_REQUIRE(has ? (m_owner[m] >= 0 && m_owner[m] < world) : m_owner[m] == -1, MSFNO_EINVAL,
                  "m_owner must assign every m < lmax to a rank and m >= lmax to -1");
  }
  return MSFNO_OK;
}

// counts (floats) per peer: phase 0 sends my rows of q's m-set, phase 1 my m-set's
// slabs of q's rows; every slab row is 2W floats (W_in / W_out of the two grids)
void exchange_counts(int world, int rank, const std::vector<int>& nm, int W_in, int W_out,
                     long long R, int phase, long long* sc, long long* rc) {
  for (int q = 0; q < world; ++q) {
    if (phase == 0) {
      sc[q] = nm[q] * R * 2 * W_in;
      rc[q] = nm[rank] * R * 2 * W_in;
    } else {
      sc[q] = nm[rank] * R * 2 * W_out;
      rc[q] = nm[q] * R * 2 * W_out;
    }
  }
}

struct BandBufs {
  float2* Xn;   // (BC, max(rows_in, rows_out), mmax) spectra of local rows; reused as Yn
  float2* rs;   // (BC, max rows) row (mean, M2), norm0 then norm1
  float *sc0, *sh0, *sc1, *sh1, *ab1;
  BlockBufs fb; // filter buffers (Sa, Sb, Sc, Wexp / xt, yt) in the local spectral layout
  float* x1;    // (B, C, rows_out*nlon_out)
  float *W1f, *b1f, *h;
  // fb.x1p: (B, 3, C, P) bf16x3 planes (x6 engine with an MLP): x for the skip GEMM
  // (written by the rfft, same-grid blocks), then x1 for fc1 (written by the irfft)
};

void carve_band(Carve& cv, BandBufs& b, const msfno_block_desc* d, const msfno_band_plan_s* p,
                int B) {
  const int64_t C = d->C, BC = (int64_t)B * C, R = 2 * BC;
  const int64_t Pin = (int64_t)p->rows_in * p->nlon_in;
  const int64_t Pout = (int64_t)p->rows_out * p->nlon_out;
  const int64_t rmax = std::max(p->rows_in, p->rows_out);
  const SpecLayout& L = p->fwd->spec;
  b.Xn = cv.take<float2>(BC * rmax * p->mmax);
  b.rs = cv.take<float2>(BC * rmax);
  b.sc0 = cv.take<float>(BC);
  b.sh0 = cv.take<float>(BC);
  b.sc1 = cv.take<float>(BC);
  b.sh1 = cv.take<float>(BC);
  b.ab1 = cv.take<float>(BC);
  std::memset(&b.fb, 0, sizeof(b.fb));
  b.fb.Sa = cv.take<float>(R * L.ldT);
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) {
    const int64_t Hs = d->spec_hidden;
    b.fb.Sb = cv.take<float>(spec_hidden_floats(B, Hs, L));
    b.fb.Sc = cv.take<float>(spec_hidden_floats(B, Hs, L));
    b.fb.cs = cv.take<float>(2LL * B * round_up(L.Tp, 4));
    for (int l = 0; l <= d->spectral_layers && l < 9; ++l) {
      const int64_t ci = (l == 0) ? C : Hs;
      const int64_t co = (l == d->spectral_layers) ? C : Hs;
      b.fb.Wexp[l] = cv.take<float>(4 * ci * co);
    }
    if (d->wcache) {
      Carve wc;
      wc.base = static_cast<char*>(d->wcache);
      carve_spec_ws(wc, b.fb.dw, d);
    } else {
      carve_spec_ws(cv, b.fb.dw, d);
    }
  } else {
    b.fb.xt = cv.take<float>(std::max<int64_t>(BC * L.T * 2, 4));
    b.fb.yt = cv.take<float>(std::max<int64_t>(BC * L.T * 2, 4));
  }
  b.x1 = cv.take<float>(BC * Pout);
  b.W1f = b.b1f = b.h = nullptr;
  if (mlp_fused(d, Pout)) {
    b.fb.mfimg = wcache_mfimg(d);
    if (!b.fb.mfimg) b.fb.mfimg = cv.take<unsigned short>(mlp_fused_image_bytes() / 2);
  } else if (d->has_mlp) {
    const int64_t Hd = d->mlp_hidden;
    b.W1f = cv.take<float>((int64_t)B * Hd * C);
    b.b1f = cv.take<float>((int64_t)B * Hd);
    b.h = cv.take<float>(mlp_h_floats(B, Hd, Pout));
  }
  b.fb.x1p = (x1p_buffer(d, p->inv) && Pout % 8 == 0)
                 ? cv.take<unsigned short>(BC * 3 * std::max(Pin, Pout))
                 : nullptr;
  b.fb.xs = skip_x3(d) ? cv.take<float>((int64_t)B * d->C) : nullptr;
  // forward Legendre on legendre_x3f: the exchange carries x3h pairs, the channel's
  // sigma (stage 1) and 1 / sigma per slab row (read in stage 2)
  b.fb.lsig = b.fb.isr = nullptr;
  if (x3f_usable(p->fwd)) {
    b.fb.lsig = cv.take<float>(BC);
    b.fb.isr = cv.take<float>(R);
  }
  carve_dense_ws(cv, b.fb.dw, d, B);
}

int check_band(const msfno_block_desc* d, const msfno_band_plan_s* p) {
  MSFNO_REQUIRE(d && p, MSFNO_EINVAL, "null descriptor or band plan");
  MSFNO_REQUIRE(p->fwd->table_loaded && p->inv->table_loaded, MSFNO_EINVAL,
                "band plan tables not loaded");
  MSFNO_REQUIRE(d->C > 0, MSFNO_EINVAL, "C must be > 0");
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) {
    MSFNO_REQUIRE(d->spectral_layers >= 1 && d->spectral_layers <= 8, MSFNO_EUNSUPPORTED,
                  "spectral_layers must be in [1, 8]");
    MSFNO_REQUIRE(d->spec_hidden > 0, MSFNO_EINVAL, "spec_hidden must be > 0");
  } else {
    MSFNO_REQUIRE(d->filter_type == MSFNO_FILTER_LINEAR, MSFNO_EUNSUPPORTED, "unknown filter_type");
  }
  MSFNO_REQUIRE(d->outer_skip != MSFNO_SKIP_LINEAR, MSFNO_EUNSUPPORTED,
                "outer_skip='linear' is not supported by the fused block");
  MSFNO_REQUIRE(p->same_grid() || (d->inner_skip == MSFNO_SKIP_NONE &&
                                   d->outer_skip == MSFNO_SKIP_NONE),
                MSFNO_EINVAL, "skip connections need equal input and output grids");
  return MSFNO_OK;
}

hipEvent_t slot_event(msfno_band_plan_s* p, int slot) {
  if (slot < 0 || slot >= 64) return nullptr;
  if ((int)p->join.size() <= slot) p->join.resize(slot + 1, nullptr);
  if (!p->join[slot] &&
      hipEventCreateWithFlags(&p->join[slot], hipEventDisableTiming) != hipSuccess)
    p->join[slot] = nullptr;
  return p->join[slot];
}

}  // namespace

extern "C" {

int msfno_band_partition(int world, int nlat, int lmax, int mmax, int* row_start, int* m_owner) {
  MSFNO_REQUIRE(world >= 1 && world <= 64, MSFNO_EUNSUPPORTED, "band sharding needs 1..64 ranks");
  const int ke = nlat - nlat / 2;
  MSFNO_REQUIRE(ke >= world, MSFNO_EINVAL,
                "need at least one northern latitude row per rank (nlat - nlat/2 >= world)");
  MSFNO_REQUIRE(lmax > 0 && mmax > 0 && row_start && m_owner, MSFNO_EINVAL, "bad partition args");
  // bands of the northern half (+ equator); the equator row (odd nlat) has no
  // mirror, so the last band takes the smaller share
  const int q = ke / world, rem = ke % world;
  row_start[0] = 0;
  for (int r = 0; r < world; ++r) row_start[r + 1] = row_start[r] + q + (r < rem ? 1 : 0);
  // snake over m ascending (work lmax - m descending): 0..W-1, W-1..0, ...
  for (int m = 0; m < mmax; ++m) {
    if (lmax - m <= 0) {
      m_owner[m] = -1;
      continue;
    }
    const int round = m / world, pos = m % world;
    m_owner[m] = (round & 1) ? world - 1 - pos : pos;
  }
  return MSFNO_OK;
}

int msfno_band_exchange_counts(int world, int rank, int nlat, int mmax, const int* row_start,
                               const int* m_owner, int R, int phase, long long* send_counts,
                               long long* recv_counts) {
  MSFNO_REQUIRE(rank >= 0 && rank < world && R > 0 && send_counts && recv_counts, MSFNO_EINVAL,
                "bad exchange-count arguments");
  MSFNO_REQUIRE(phase == 0 || phase == 1, MSFNO_EINVAL, "phase must be 0 or 1");
  int lmax_eff = 0;  // validate against the implied lmax (owners of -1 mark m >= lmax)
  for (int m = 0; m < mmax; ++m)
    if (m_owner && m_owner[m] >= 0) lmax_eff = m + 1;
  MSFNO_TRY(validate_partition(world, nlat, std::max(lmax_eff, 1), mmax, row_start, m_owner));
  std::vector<int> nm(world, 0);
  for (int m = 0; m < mmax; ++m)
    if (m_owner[m] >= 0) ++nm[m_owner[m]];
  const int W = band_width(world, row_start);
  exchange_counts(world, rank, nm, W, W, R, phase, send_counts, recv_counts);
  return MSFNO_OK;
}

int msfno_band_local_rows(int world, int rank, int nlat, const int* row_start, int* rows,
                          int* count) {
  MSFNO_REQUIRE(world >= 1 && world <= 64 && rank >= 0 && rank < world && count, MSFNO_EINVAL,
                "bad local-rows arguments");
  MSFNO_TRY(validate_rows(world, nlat, row_start));
  const BandRows o = band_rows(nlat, row_start, rank);
  *count = o.H;
  if (rows)
    for (int i = 0; i < o.H; ++i) rows[i] = band_global_row(nlat, o, i);
  return MSFNO_OK;
}

int msfno_band_plan_exchange_counts(msfno_band_plan_t p, int R, int phase, long long* send_counts,
                                    long long* recv_counts) {
  MSFNO_REQUIRE(p && R > 0 && send_counts && recv_counts, MSFNO_EINVAL,
                "bad exchange-count arguments");
  MSFNO_REQUIRE(phase == 0 || phase == 1, MSFNO_EINVAL, "phase must be 0 or 1");
  exchange_counts(p->world, p->rank, p->nm_of, p->W_in, p->W_out, R, phase, send_counts,
                  recv_counts);
  return MSFNO_OK;
}

int msfno_band_plan_destroy(msfno_band_plan_t p) {
  if (!p) return MSFNO_OK;
  msfno_sht_plan_destroy(p->fwd);
  msfno_sht_plan_destroy(p->inv);
  if (p->d_perm) (void)hipFree(p->d_perm);
  for (hipEvent_t e : p->join)
    if (e) (void)hipEventDestroy(e);
  delete p;
  return MSFNO_OK;
}

int msfno_band_plan_create2(int nlat_in, int nlon_in, int nlat_out, int nlon_out, int lmax,
                            int mmax, int world, int rank, const int* row_in, const int* row_out,
                            const int* m_owner, msfno_band_plan_t* plan) {
  MSFNO_REQUIRE(plan, MSFNO_EINVAL, "null plan pointer");
  MSFNO_REQUIRE(rank >= 0 && rank < world, MSFNO_EINVAL, "rank out of range");
  MSFNO_TRY(validate_partition(world, nlat_in, lmax, mmax, row_in, m_owner));
  MSFNO_TRY(validate_rows(world, nlat_out, row_out));
  auto* p = new msfno_band_plan_s();
  p->nlat_in = nlat_in; p->nlon_in = nlon_in; p->nlat_out = nlat_out; p->nlon_out = nlon_out;
  p->lmax = lmax; p->mmax = mmax;
  p->world = world; p->rank = rank;
  p->row_in.assign(row_in, row_in + world + 1);
  p->row_out.assign(row_out, row_out + world + 1);
  p->owner.assign(m_owner, m_owner + mmax);
  p->rows_in = band_rows(nlat_in, row_in, rank).H;
  p->rows_out = band_rows(nlat_out, row_out, rank).H;
  p->W_in = band_width(world, row_in);
  p->W_out = band_width(world, row_out);
  p->nm_of.assign(world, 0);
  std::vector<char> mask(mmax, 0);
  for (int m = 0; m < mmax; ++m) {
    if (m_owner[m] < 0) continue;
    p->mact = m + 1;
    ++p->nm_of[m_owner[m]];
    if (m_owner[m] == rank) mask[m] = 1;
  }
  p->nm = p->nm_of[rank];
  // slab order for the exchanges: by (owner, m)
  std::vector<int> perm(mmax, -1), start(world, 0);
  for (int q = 1; q < world; ++q) start[q] = start[q - 1] + p->nm_of[q - 1];
  for (int m = 0; m < mmax; ++m)
    if (m_owner[m] >= 0) perm[m] = start[m_owner[m]]++;
  int rc = plan_create(nlat_in, nlon_in, lmax, mmax, 0, &mask, &p->fwd);
  if (rc == MSFNO_OK) rc = plan_create(nlat_out, nlon_out, lmax, mmax, 1, &mask, &p->inv);
  if (rc != MSFNO_OK) {
    msfno_band_plan_destroy(p);
    return rc;
  }
  set_band_maps(p->fwd, world, row_in, p->W_in);
  set_band_maps(p->inv, world, row_out, p->W_out);
  hipError_t e = hipMalloc(&p->d_perm, mmax * sizeof(int));
  if (e == hipSuccess)
    e = hipMemcpy(p->d_perm, perm.data(), mmax * sizeof(int), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    set_error(std::string("band plan allocation failed: ") + hipGetErrorString(e));
    msfno_band_plan_destroy(p);
    return MSFNO_EHIP;
  }
  *plan = p;
  return MSFNO_OK;
}

int msfno_band_plan_create(int nlat, int nlon, int lmax, int mmax, int world, int rank,
                           const int* row_start, const int* m_owner, msfno_band_plan_t* plan) {
  return msfno_band_plan_create2(nlat, nlon, nlat, nlon, lmax, mmax, world, rank, row_start,
                                 row_start, m_owner, plan);
}

int msfno_band_plan_load_tables(msfno_band_plan_t p, const float* fwd_table,
                                const float* inv_table, void* stream) {
  MSFNO_REQUIRE(p && fwd_table && inv_table, MSFNO_EINVAL, "null band plan or table");
  MSFNO_TRY(msfno_sht_plan_load_table(p->fwd, fwd_table, stream));
  MSFNO_TRY(msfno_sht_plan_load_table(p->inv, inv_table, stream));
  return MSFNO_OK;
}

int msfno_band_linear_modes(msfno_band_plan_t p, long long* modes, long long* count) {
  MSFNO_REQUIRE(p && count, MSFNO_EINVAL, "null band plan or count");
  const auto& v = p->fwd->lin_modes;
  *count = (long long)v.size();
  if (modes && !v.empty()) std::memcpy(modes, v.data(), v.size() * sizeof(long long));
  return MSFNO_OK;
}

size_t msfno_band_workspace_size(const msfno_block_desc* d, msfno_band_plan_t p, int B) {
  if (!d || !p || B <= 0) return 0;
  Carve cv;
  BandBufs b;
  carve_band(cv, b, d, p, B);
  return cv.off;
}

int msfno_band_block_stage(const msfno_block_desc* d, msfno_band_plan_t p, int stage,
                           const msfno_band_io* io, int B, void* ws, size_t ws_bytes,
                           void* stream) {
  MSFNO_TRY(check_band(d, p));
  MSFNO_REQUIRE(io && B > 0, MSFNO_EINVAL, "null io or bad batch");
  MSFNO_REQUIRE(ws_bytes >= msfno_band_workspace_size(d, p, B), MSFNO_EWORKSPACE,
                "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  BandBufs b;
  carve_band(cv, b, d, p, B);
  const int64_t C = d->C, BC = (int64_t)B * C, R = 2 * BC;
  const int64_t Pout = (int64_t)p->rows_out * p->nlon_out;
  // the skip GEMM as in msfno_block_forward: on x planes written by the rfft (forked
  // after it) when the plane buffer exists, on fp32 x on the x3h engine (forked in
  // stage 1 once the global statistics give its scales: the unsharded block's scales,
  // so both round alike), else on fp32 x (forked first)
  const bool xpl = skip_planes(d, p->fwd, b.fb);
  const int64_t Pl = (int64_t)p->rows_in * p->nlon_in;
  auto launch_skip = [&]() -> int {
    std::shared_ptr<SideCtx> side;
    MSFNO_TRY(side_ctx(&side, s));
    hipStream_t ss = s;
    hipEvent_t join = side ? slot_event(p, io->slot) : nullptr;
    MSFNO_REQUIRE(!side || join, MSFNO_EHIP, "band slot event unavailable (slot must be 0..63)");
    if (side) {
      MSFNO_CHECK_HIP(hipEventRecord(side->fork, s));
      MSFNO_CHECK_HIP(hipStreamWaitEvent(side->side, side->fork, 0));
      ss = side->side;
    }
    prof(ST_SKIP, ss);
    GemmEpi e;
    e.bias = d->skip_b;
    // x3h: B-row scales from the global norm0 statistics (stage 1).  The pipelined
    // sub-batches put this side-stream skip beside other sub-batches' row FFTs: safe since
    // the FFT units carry no packed-FP32 op_sel:[0,1] forms
    if (b.fb.xs && C == 256 && skip_h_env()) {
      MSFNO_TRY(launch_skip_h(d->skip_w, b.fb.xs, io->x, b.x1, d->skip_b, B, Pl, b.fb.dw.skip,
                              b.fb.dw.skip_b, ss));
    } else if (b.fb.xs) {
      MSFNO_TRY(gemm_x3(d->skip_w, (int)C, b.fb.xs, io->x, b.x1, (int)C, (int)Pl, (int)C,
                        (int)Pl, (int)Pl, C * Pl, C * Pl, B, e, b.fb.dw.skip, b.fb.dw.skip_b,
                        ss));
    } else if (xpl) {
      e.b_planes = b.fb.x1p;
      e.b_plane_stride = C * Pl;
      MSFNO_TRY(gemm_x6p(d->skip_w, b.x1, (int)C, (int)Pl, (int)C, (int)C, (int)Pl, (int)Pl,
                         0, 3 * C * Pl, C * Pl, B, e, b.fb.dw.skip, b.fb.dw.skip_b, ss));
    } else {
      MSFNO_TRY(gemm_dense(ROLE_SKIP, TILE_128x256, d->skip_w, io->x, b.x1, (int)C, (int)Pl,
                           (int)C, (int)C, (int)Pl, (int)Pl, 0, C * Pl, C * Pl, B, e,
                           b.fb.dw.skip, b.fb.dw.skip_b, ss));
    }
    if (side) {
      prof(ST_END, ss);
      MSFNO_CHECK_HIP(hipEventRecord(join, ss));
    }
    return MSFNO_OK;
  };
  switch (stage) {
    case 0: {
      MSFNO_REQUIRE(io->x && io->stats_local, MSFNO_EINVAL, "stage 0 needs x and stats_local");
      if (d->inner_skip == MSFNO_SKIP_LINEAR) {
        MSFNO_REQUIRE(d->skip_w, MSFNO_EINVAL, "missing inner_skip weight");
        if (!xpl && !b.fb.xs) MSFNO_TRY(launch_skip());
      }
      prof(ST_FFT_FWD, s);
      const float scale = (float)(2.0 * M_PI / p->nlon_in);
      const C2RPlanes xp{b.fb.x1p, (int)C, p->rows_in};
      MSFNO_TRY(launch_fft_r2c_rows(p->fwd->fft, io->x, b.Xn, b.rs, BC * p->rows_in, p->mmax,
                                    scale, s, xpl ? &xp : nullptr));
      if (xpl) MSFNO_TRY(launch_skip());
      prof(ST_NORM0, s);
      MSFNO_TRY(launch_stats_partial(b.rs, p->rows_in, p->nlon_in, BC, io->stats_local, s));
      prof(ST_END, s);
      break;
    }
    case 1: {
      MSFNO_REQUIRE(io->stats_all && io->send, MSFNO_EINVAL, "stage 1 needs stats_all and send");
      prof(ST_NORM0, s);
      MSFNO_TRY(launch_chan_affine_parts(io->stats_all, p->world, B, (int)C, d->norm0_w,
                                         d->norm0_b, d->norm_eps, nullptr, nullptr, 0.f, b.sc0,
                                         b.sh0, s, b.fb.xs, nullptr, b.fb.lsig));
      if (b.fb.xs && d->inner_skip == MSFNO_SKIP_LINEAR) {
        MSFNO_REQUIRE(io->x && d->skip_w, MSFNO_EINVAL, "stage 1 needs x for the x3h skip");
        MSFNO_TRY(launch_skip());
      }
      prof(ST_BAND_PACK, s);
      const BandRows o = band_rows(p->nlat_in, p->row_in.data(), p->rank);
      if (b.fb.lsig)  // x3h pairs for legendre_x3f (every rank decides alike: plan geometry)
        MSFNO_TRY(launch_band_pack_h(b.Xn, reinterpret_cast<unsigned short*>(io->send), B,
                                     (int)C, band_geom(p->fwd, o, p->W_in), p->mmax, b.sc0,
                                     b.sh0, b.fb.lsig, b.fb.isr, p->d_perm, p->W_in, s));
      else
        MSFNO_TRY(launch_band_pack(b.Xn, io->send, B, (int)C, band_geom(p->fwd, o, p->W_in),
                                   p->mmax, b.sc0, b.sh0, p->d_perm, p->W_in, s));
      prof(ST_END, s);
      break;
    }
    case 2: {
      MSFNO_REQUIRE(io->send && io->recv, MSFNO_EINVAL, "stage 2 needs send and recv");
      if (p->nm == 0) break;  // this rank owns no zonal wavenumber
      // the GEMMs read the phase-0 receive buffer and write the phase-1 send buffer
      prof(ST_LEG_FWD, s);
      if (b.fb.isr)
        MSFNO_TRY(legendre_fwd_x3f(p->fwd, reinterpret_cast<const unsigned short*>(io->recv),
                                   b.fb.isr, b.fb.Sa, (int)R, s));
      else
        MSFNO_TRY(legendre_fwd(p->fwd, io->recv, b.fb.Sa, (int)R, s));
      MSFNO_TRY(run_filter(d, p->fwd, p->inv, b.fb, B, s));
      prof(ST_LEG_INV, s);
      MSFNO_TRY(legendre_inv(p->inv, b.fb.Sa, io->send, (int)R, s));
      prof(ST_END, s);
      break;
    }
    case 3: {
      MSFNO_REQUIRE(io->recv && io->stats_local, MSFNO_EINVAL, "stage 3 needs recv and stats_local");
      prof(ST_TRANSPOSE_INV, s);
      const BandRows o = band_rows(p->nlat_out, p->row_out.data(), p->rank);
      MSFNO_TRY(launch_band_unpack(io->recv, b.Xn, B, (int)C, band_geom(p->inv, o, p->W_out),
                                   p->mmax, p->mact, p->d_perm, s));
      const float* skip_src = nullptr;
      if (d->inner_skip == MSFNO_SKIP_LINEAR) {
        std::shared_ptr<SideCtx> side;
        MSFNO_TRY(side_ctx(&side, s));
        if (side) {
          hipEvent_t join = slot_event(p, io->slot);
          MSFNO_REQUIRE(join, MSFNO_EHIP, "band slot event unavailable (slot must be 0..63)");
          MSFNO_CHECK_HIP(hipStreamWaitEvent(s, join, 0));
        }
        skip_src = b.x1;
      } else if (d->inner_skip == MSFNO_SKIP_IDENTITY) {
        MSFNO_REQUIRE(io->x, MSFNO_EINVAL, "stage 3 needs x for the identity skip");
        skip_src = io->x;
      }
      prof(ST_FFT_INV, s);
      // with an MLP on the x6 engine the irfft writes x1 as planes (fc1's B operand)
      const C2RPlanes x1p{b.fb.x1p, (int)C, p->rows_out};
      MSFNO_TRY(launch_fft_c2r_rows(p->inv->fft, b.Xn, b.x1, skip_src, b.rs, BC * p->rows_out,
                                    p->mmax, d->filter_type == MSFNO_FILTER_LINEAR ? 1 : 0, s,
                                    (b.fb.x1p && x1_planes(d, p->inv)) ? &x1p : nullptr));
      prof(ST_NORM1, s);
      MSFNO_TRY(launch_stats_partial(b.rs, p->rows_out, p->nlon_out, BC, io->stats_local, s));
      prof(ST_END, s);
      break;
    }
    case 4: {
      MSFNO_REQUIRE(io->stats_all && io->out, MSFNO_EINVAL, "stage 4 needs stats_all and out");
      MSFNO_REQUIRE((io->gamma == nullptr) == (io->beta == nullptr), MSFNO_EINVAL,
                    "gamma and beta must both be given or both be NULL");
      prof(ST_NORM1, s);
      MSFNO_TRY(launch_chan_affine_parts(io->stats_all, p->world, B, (int)C, d->norm1_w,
                                         d->norm1_b, d->norm_eps, io->gamma, io->beta,
                                         io->film_scale, b.sc1, b.sh1, s, nullptr, b.ab1));
      const float* resid = d->outer_skip == MSFNO_SKIP_IDENTITY ? io->x : nullptr;
      MSFNO_REQUIRE(d->outer_skip != MSFNO_SKIP_IDENTITY || io->x, MSFNO_EINVAL,
                    "stage 4 needs x for the outer skip");
      if (d->has_mlp) {
        MSFNO_TRY(run_block_mlp(d, b.x1, x1_planes(d, p->inv) ? b.fb.x1p : nullptr, b.sc1, b.sh1,
                                b.ab1, b.W1f, b.b1f, b.h, b.fb.mfimg, io->out, resid, B, Pout, b.fb.dw,
                                s));
      } else {
        prof(ST_OUT_AFFINE, s);
        MSFNO_TRY(launch_affine_rows(b.x1, b.sc1, b.sh1, resid, io->out, BC, Pout, 0, nullptr, 0,
                                     s));
      }
      prof(ST_END, s);
      break;
    }
    default:
      set_error("band stage must be 0..4");
      return MSFNO_EINVAL;
  }
  return MSFNO_OK;
}

}  // extern "C"
