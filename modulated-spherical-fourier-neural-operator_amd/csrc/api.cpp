// libmsfno C-ABI: plans (fp64 host math + device tables), standalone SHT
// transforms, contractions and the fused SFNO-Block forward orchestration.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>

#include "block.h"

namespace msfno {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

void SpecLayout::build(int lmax_, int mmax_, const std::vector<char>* mask) {
  lmax = lmax_;
  mmax = mmax_;
  L.assign(mmax, 0);
  Lp.assign(mmax, 0);
  Lpe.assign(mmax, 0);
  off.assign(mmax, 0);
  T = Tp = 0;
  mact = 0;
  for (int m = 0; m < mmax; ++m) {
    const int l = (mask && !(*mask)[m]) ? 0 : std::max(lmax - m, 0);
    L[m] = l;
    Lpe[m] = (int)round_up((l + 1) / 2, 8);  // 8: 16-B bf16 chunks of the x6 Legendre GEMM
    Lp[m] = Lpe[m] + (int)round_up(l / 2, 8);
    off[m] = (int)Tp;
    T += l;
    Tp += Lp[m];
    if (l > 0) mact = m + 1;
  }
  ldT = round_up(std::max<int64_t>(Tp, 8), 8);
}

// ---------------------------------------------------------------------------
// host-side fp64 plan math ([TH] torch_harmonics.quadrature / .legendre)
// ---------------------------------------------------------------------------
static void gauss_legendre(int n, std::vector<double>& x, std::vector<double>& w) {
  x.assign(n, 0.0);
  w.assign(n, 0.0);
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5));
    double pp = 0.0;
    for (int it = 0; it < 100; ++it) {
      double p1 = 1.0, p2 = 0.0;
      for (int j = 1; j <= n; ++j) {
        const double p3 = p2;
        p2 = p1;
        p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
      }
      pp = n * (z * p1 - p2) / (z * z - 1.0);
      const double z1 = z;
      z = z1 - p1 / pp;
      if (std::fabs(z - z1) < 1e-16) break;
    }
    // recompute derivative at the converged root
    double p1 = 1.0, p2 = 0.0;
    for (int j = 1; j <= n; ++j) {
      const double p3 = p2;
      p2 = p1;
      p1 = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
    }
    pp = n * (z * p1 - p2) / (z * z - 1.0);
    x[n - 1 - i] = z;  // ascending
    w[n - 1 - i] = 2.0 / ((1.0 - z * z) * pp * pp);
  }
}

static void clenshaw_curtis(int n, std::vector<double>& x, std::vector<double>& w) {
  x.assign(n, 0.0);
  w.assign(n, 0.0);
  if (n == 2) {
    x[0] = -1.0; x[1] = 1.0;
    w[0] = w[1] = 1.0;
    return;
  }
  const int N = n - 1;
  for (int j = 0; j < n; ++j) {
    const double th = M_PI - (double)j * M_PI / N;  // cos(linspace(pi, 0, n))
    x[j] = std::cos(th);
    const double tj = (double)j * M_PI / N;
    double s = 0.0;
    for (int k = 1; k <= N / 2; ++k) {
      const double bk = (2 * k == N) ? 1.0 : 2.0;
      s += bk / (4.0 * k * k - 1.0) * std::cos(2.0 * k * tj);
    }
    const double cj = (j == 0 || j == N) ? 1.0 : 2.0;
    w[j] = cj / N * (1.0 - s);
  }
}

static int quadrature(int nlat, int grid, std::vector<double>& x, std::vector<double>& w) {
  if (grid == MSFNO_GRID_LEGENDRE_GAUSS) {
    MSFNO_REQUIRE(nlat >= 1, MSFNO_EINVAL, "nlat must be >= 1");
    gauss_legendre(nlat, x, w);
  } else if (grid == MSFNO_GRID_EQUIANGULAR) {
    MSFNO_REQUIRE(nlat >= 2, MSFNO_EINVAL, "equiangular grid needs nlat >= 2");
    clenshaw_curtis(nlat, x, w);
  } else {
    set_error("Unknown quadrature mode");
    return MSFNO_EUNSUPPORTED;
  }
  return MSFNO_OK;
}

// (-1)^m c_l^m P_l^m at cos(theta_k), same recurrence and operation order as [TH] legpoly
static int legendre_table(int mmax, int lmax, int nlat, int grid, int inverse, int csphase,
                          double* out) {
  std::vector<double> x, w;
  MSFNO_TRY(quadrature(nlat, grid, x, w));
  const int nmax = std::max(mmax, lmax);
  // k-independent recurrence coefficients (same expressions as [TH] legpoly)
  std::vector<double> ca((size_t)nmax * nmax, 0.0), cb((size_t)nmax * nmax, 0.0);
  for (int l = 2; l < nmax; ++l)
    for (int m = 0; m < l - 1; ++m) {
      ca[(size_t)m * nmax + l] = std::sqrt((2.0 * l - 1) / (l - m) * (2.0 * l + 1) / (l + m));
      cb[(size_t)m * nmax + l] = std::sqrt((double)(l + m - 1) / (l - m) * (2.0 * l + 1) /
                                           (2.0 * l - 3) * (l - m - 1) / (l + m));
    }
  std::vector<double> vdm((size_t)nmax * nmax);
  for (int k = 0; k < nlat; ++k) {
    // theta = flip(arccos(nodes)): colatitude index k uses node nlat-1-k
    const double xk = std::cos(std::acos(x[nlat - 1 - k]));
    std::fill(vdm.begin(), vdm.end(), 0.0);
    auto V = [&](int m, int l) -> double& { return vdm[(size_t)m * nmax + l]; };
    V(0, 0) = 1.0 / std::sqrt(4.0 * M_PI);  // ortho norm; inverse factor is 1 as well
    for (int l = 1; l < nmax; ++l) {
      V(l - 1, l) = std::sqrt(2.0 * l + 1) * xk * V(l - 1, l - 1);
      V(l, l) = std::sqrt((2.0 * l + 1) * (1 + xk) * (1 - xk) / 2.0 / l) * V(l - 1, l - 1);
    }
    for (int m = 0; m < nmax; ++m) {
      const double* a = &ca[(size_t)m * nmax];
      const double* b = &cb[(size_t)m * nmax];
      double* v = &vdm[(size_t)m * nmax];
      for (int l = m + 2; l < nmax; ++l) v[l] = xk * a[l] * v[l - 1] - b[l] * v[l - 2];
    }
    const double wk = inverse ? 1.0 : w[k];  // weights are symmetric (unflipped in [TH])
    for (int m = 0; m < mmax; ++m) {
      const double sgn = (csphase && (m & 1)) ? -1.0 : 1.0;
      for (int l = 0; l < lmax; ++l)
        out[((size_t)m * lmax + l) * nlat + k] = sgn * V(m, l) * wk;
    }
  }
  return MSFNO_OK;
}

// ---------------------------------------------------------------------------
// stage profiler (hipEvents on the caller's stream)
// ---------------------------------------------------------------------------
static const char* kStageNames[MSFNO_PROF_NSTAGES] = {
    "fft_fwd", "norm0_stats", "transpose_fwd", "legendre_fwd", "spectral_prep", "spectral_l0",
    "spectral_l1", "spectral_l2", "spectral_l3", "spectral_out", "linear_gather",
    "linear_contract", "linear_scatter", "legendre_inv", "transpose_inv", "fft_inv",
    "inner_skip", "norm1_film_fold", "mlp_fc1", "mlp_fc2", "out_affine", "band_pack",
    "band_exchange", "mlp_fused", "mlp_gen", "end"};

struct Profiler {
  bool on = false;
  struct Mark {
    int stage;
    hipStream_t stream;
    hipEvent_t ev;
  };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> pool;
  // a stage lasts from its mark to the next mark recorded on the same stream
  void mark(int stage, hipStream_t s) {
    if (!on) return;
    hipEvent_t e;
    if (!pool.empty()) {
      e = pool.back();
      pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
      return;
    }
    if (hipEventRecord(e, s) != hipSuccess) {
      pool.push_back(e);
      return;
    }
    marks.push_back({stage, s, e});
  }
};
static Profiler g_prof;
void prof(int stage, hipStream_t s) { g_prof.mark(stage, s); }

// ---------------------------------------------------------------------------
// per-device side stream: the inner-skip 1x1 conv (MFMA-bound, depends only on
// the block input) runs concurrently with the HBM-bound SHT stages (fork/join
// through events; capture-safe).  MSFNO_SIDE_STREAM=0 disables it.
// ---------------------------------------------------------------------------

// side stream at the lowest priority: the skip GEMM fills what the spectral path
// leaves (+1 % over equal priority, measured); MSFNO_SIDE_PRIO=normal|high for A/B.
// MSFNO_SIDE_CUSTRIDE=k (A/B): the side stream runs on every k-th CU only (a CU
// mask; k coprime with 8 spreads it over all XCDs), at normal priority.
static hipError_t create_side_stream(hipStream_t* s, int dev) {
  const char* pe = getenv("MSFNO_SIDE_PRIO");
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  const char* ce = getenv("MSFNO_SIDE_CUSTRIDE");
  const int custride = ce ? atoi(ce) : 0;
  if (e == hipSuccess && custride > 1) {
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e == hipSuccess) {
      const int ncu = prop.multiProcessorCount;
      std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; i += custride) mask[(size_t)i / 32] |= 1u << (i % 32);
      e = hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
    }
  } else if (e == hipSuccess) {
    if (pe && std::string(pe) == "normal")
      e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    else
      e = hipStreamCreateWithPriority(s, hipStreamNonBlocking,
                                      (pe && std::string(pe) == "high") ? greatest : least);
  }
  return e;
}

int side_ctx(std::shared_ptr<SideCtx>* out, hipStream_t caller) {
  // (read at every call: tests switch it inside one process)
  const char* se = getenv("MSFNO_SIDE_STREAM");
  const bool enabled = !(se && se[0] == '0');
  out->reset();
  if (!enabled) return MSFNO_OK;
  // no fork while the caller's stream is being captured into a HIP graph: the
  // captured fork/join made a 12-block network step 19.0 ms instead of 12.4 ms
  // (replayed, config 3, round 2) and still 8.16 vs 8.10 ms in round 5 (profiles/r05_b);
  // the graph runs the skip GEMM in line
  if (caller) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(caller, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return MSFNO_OK;
  }
  // one side stream per device (pooled: every caller stream of that device forks to
  // it) + one fork/join event pair per (device, caller stream).  The device comes
  // from the caller's stream (not the thread's current device); two caller streams
  // never share fork/join events.  The per-caller map is bounded (LRU, kMaxCallers):
  // the oldest pair is dropped from the map, and its events are destroyed when the
  // last holder releases it (HIP releases an event whose recorded work is still
  // pending once it completes)
  static std::mutex mu;
  static std::map<int, hipStream_t> side_of_dev;
  struct Entry {
    std::shared_ptr<SideCtx> c;
    uint64_t used = 0;
  };
  static std::map<std::pair<int, hipStream_t>, Entry> ctx;
  static uint64_t tick = 0;
  constexpr size_t kMaxCallers = 64;
  int dev = 0;
  if (caller) MSFNO_CHECK_HIP(hipStreamGetDevice(caller, &dev));
  else MSFNO_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = ctx.find({dev, caller});
  if (it == ctx.end() && ctx.size() >= kMaxCallers) {
    auto lru = ctx.begin();
    for (auto j = ctx.begin(); j != ctx.end(); ++j)
      if (j->second.used < lru->second.used) lru = j;
    ctx.erase(lru);
  }
  Entry& en = ctx[{dev, caller}];
  en.used = ++tick;
  if (!en.c) {
    auto c = std::make_shared<SideCtx>();
    int cur = 0;
    MSFNO_CHECK_HIP(hipGetDevice(&cur));
    if (cur != dev) MSFNO_CHECK_HIP(hipSetDevice(dev));
    hipError_t e = hipSuccess;
    hipStream_t& pooled = side_of_dev[dev];
    if (!pooled) e = create_side_stream(&pooled, dev);
    c->side = pooled;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join, hipEventDisableTiming);
    if (cur != dev) (void)hipSetDevice(cur);
    if (e != hipSuccess) {
      ctx.erase({dev, caller});
      set_error(std::string("side stream creation failed: ") + hipGetErrorString(e));
      return MSFNO_EHIP;
    }
    en.c = std::move(c);
  }
  *out = en.c;
  return MSFNO_OK;
}

// ---------------------------------------------------------------------------
// workspace carving
// ---------------------------------------------------------------------------

// Legendre GEMM tiles (descriptor layout and launch must agree)
static GemmTile leg_tile(int inverse) {
  return inverse ? role_tile(ROLE_LEGI, TILE_128x128) : role_tile(ROLE_LEG, TILE_128x64);
}

// the per-(m, parity) Legendre problems of a plan for R rows, in launch order:
// forward A = Xt slab (R x K), B = table, C = S (ld ldT); inverse A = S (ld ldT),
// B = table, C = Yt slab (R x N); symmetric plans: one even- and one odd-parity
// problem per m (tiles not set)
static void leg_problems(const msfno_sht_plan_s* p, int R, int64_t ldT,
                         const std::function<void(GemmDesc)>& push) {
  const SpecLayout& L = p->spec;
  const int ldko = (int)round_up(p->Ko, 4);
  for (int m = 0; m < L.mact; ++m) {
    if (L.L[m] == 0) continue;  // m outside a sharded plan's m-set
    const int64_t slab = (int64_t)p->slab[m] * R * p->ldk;
    const int lpe = L.Lpe[m], lpo = L.Lp[m] - L.Lpe[m];
    const int le = (L.L[m] + 1) / 2, lo = L.L[m] / 2;
    const int flags = (!p->inverse && m > 0) ? 1 : 0;  // m = 0 is normalised by dc_fixup
    GemmDesc g{};
    g.M = R;
    g.flags = flags;
    if (p->band_world) {
      // band plan: A (forward) / C (inverse) is the exchange buffer [p][slab][R][2W],
      // its K / N index the exchange columns (segmented in the launch, legendre_*)
      const int W = p->band_W, ld = 2 * W, Kb = p->band_K();
      const int64_t bs = (int64_t)p->slab[m] * R * ld;
      if (!p->sym) {
        if (!p->inverse) {
          g.N = L.Lp[m]; g.K = Kb; g.lda = ld; g.ldb = L.Lp[m]; g.ldc = (int)ldT;
          g.offA = bs; g.offB = p->tab_off[m]; g.offC = L.off[m];
        } else {
          g.N = Kb; g.K = L.Lp[m]; g.lda = (int)ldT; g.ldb = Kb; g.ldc = ld;
          g.offA = L.off[m]; g.offB = p->tab_off[m]; g.offC = bs;
        }
        push(g);
      } else if (!p->inverse) {
        GemmDesc e = g;  // even: Xs (R x Kb) . We (Kb x Lpe)
        e.N = lpe; e.K = Kb; e.lda = ld; e.ldb = lpe; e.ldc = (int)ldT;
        e.offA = bs; e.offB = p->tab_off[m]; e.offC = L.off[m];
        push(e);
        if (lo > 0) {
          GemmDesc o = g;  // odd: Xa (R x Kb) . Wo (Kb x Lpo)
          o.N = lpo; o.K = Kb; o.lda = ld; o.ldb = lpo; o.ldc = (int)ldT;
          o.offA = bs + W; o.offB = p->tab_off[m] + (int64_t)Kb * lpe; o.offC = L.off[m] + lpe;
          push(o);
        }
      } else {
        GemmDesc e = g;  // even: E (R x Kb) = S_e (R x Le) . Pe (Le x Kb)
        e.N = Kb; e.K = le; e.lda = (int)ldT; e.ldb = Kb; e.ldc = ld;
        e.offA = L.off[m]; e.offB = p->tab_off[m]; e.offC = bs;
        push(e);
        GemmDesc o = g;  // odd: O (R x Kb); K = 0 writes zeros (the receiver reads O)
        o.N = Kb; o.K = lo; o.lda = (int)ldT; o.ldb = Kb; o.ldc = ld;
        o.offA = L.off[m] + lpe; o.offB = p->tab_off[m] + (int64_t)lpe * Kb; o.offC = bs + W;
        push(o);
      }
      continue;
    }
    if (!p->sym) {
      if (!p->inverse) {
        g.N = L.Lp[m]; g.K = p->nlat;
        g.lda = p->ldk; g.ldb = L.Lp[m]; g.ldc = (int)ldT;
        g.offA = slab; g.offB = p->tab_off[m]; g.offC = L.off[m];
      } else {
        g.N = p->nlat; g.K = L.Lp[m];
        g.lda = (int)ldT; g.ldb = p->ldk; g.ldc = p->ldk;
        g.offA = L.off[m]; g.offB = p->tab_off[m]; g.offC = slab;
      }
      push(g);
      continue;
    }
    if (!p->inverse) {
      GemmDesc e = g;  // even: Xs (R x Ke) . We (Ke x Lpe)
      e.N = lpe; e.K = p->Ke; e.lda = p->ldk; e.ldb = lpe; e.ldc = (int)ldT;
      e.offA = slab; e.offB = p->tab_off[m]; e.offC = L.off[m];
      push(e);
      if (lo > 0) {
        GemmDesc o = g;  // odd: Xa (R x Ko) . Wo (Ko x Lpo)
        o.N = lpo; o.K = p->Ko; o.lda = p->ldk; o.ldb = lpo; o.ldc = (int)ldT;
        o.offA = slab + p->ldke; o.offB = p->tab_off[m] + (int64_t)p->Ke * lpe;
        o.offC = L.off[m] + lpe;
        push(o);
      }
    } else {
      GemmDesc e = g;  // even: E (R x Ke) = S_e (R x Le) . Pe (Le x Ke)
      e.N = p->Ke; e.K = le; e.lda = (int)ldT; e.ldb = p->ldke; e.ldc = p->ldk;
      e.offA = L.off[m]; e.offB = p->tab_off[m]; e.offC = slab;
      push(e);
      GemmDesc o = g;  // odd: O (R x Ko) = S_o (R x Lo) . Po (Lo x Ko)
      o.N = p->Ko; o.K = lo; o.lda = (int)ldT; o.ldb = ldko; o.ldc = p->ldk;
      o.offA = L.off[m] + lpe; o.offB = p->tab_off[m] + (int64_t)lpe * p->ldke;
      o.offC = slab + p->ldke;
      push(o);  // also for lo == 0 (K = 0 writes zeros): transpose_inv_sym reads O
    }
  }
}

// descriptor and image builds allocate and copy synchronously: refused while the
// stream is being captured into a HIP graph (run the call once before capturing)
static int require_not_capturing(hipStream_t s, const char* what) {
  if (!s) return MSFNO_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    set_error(std::string(what) + ": first use of this row count or table under HIP graph "
              "capture; run the call once before capturing");
    return MSFNO_EINVAL;
  }
  return MSFNO_OK;
}

// device copies of a descriptor list and its tile -> descriptor map
static int upload_descs(const std::vector<GemmDesc>& d, int tiles, bool tile_map,
                        msfno_sht_plan_s::DescSet* set) {
  MSFNO_CHECK_HIP(hipMalloc(&set->d, std::max<size_t>(1, d.size()) * sizeof(GemmDesc)));
  if (!d.empty())
    MSFNO_CHECK_HIP(hipMemcpy(set->d, d.data(), d.size() * sizeof(GemmDesc), hipMemcpyHostToDevice));
  if (tile_map) {
    std::vector<int> t2d((size_t)std::max(tiles, 1), 0);
    for (size_t i = 0; i < d.size(); ++i)
      for (int t = 0; t < d[i].tiles_m * d[i].tiles_n; ++t) t2d[d[i].tile_start + t] = (int)i;
    MSFNO_CHECK_HIP(hipMalloc(&set->tile, t2d.size() * sizeof(int)));
    MSFNO_CHECK_HIP(hipMemcpy(set->tile, t2d.data(), t2d.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  set->n = (int)d.size();
  set->tiles = tiles;
  return MSFNO_OK;
}

int ensure_desc(msfno_sht_plan_s* p, int R, int other_ld, int64_t ldT, hipStream_t s) {
  if (p->desc_R == R && p->d_desc) return MSFNO_OK;
  auto hit = p->desc_sets.find(R);
  if (hit != p->desc_sets.end()) {
    p->d_desc = hit->second.d;
    p->ndesc = hit->second.n;
    p->desc_tiles = hit->second.tiles;
    p->desc_R = R;
    return MSFNO_OK;
  }
  MSFNO_TRY(require_not_capturing(s, "Legendre descriptors"));
  int bm, bn;
  gemm_tile_dims(leg_tile(p->inverse), &bm, &bn);
  std::vector<GemmDesc> d;
  int tiles = 0;
  // MSFNO_LEG_COMPACT=1 (diagnostic timing only, wrong results): the S operand of every
  // problem as its own compact [R][N] block instead of columns of the [R][ldT] rows
  static const bool compact = [] {
    const char* e = getenv("MSFNO_LEG_COMPACT");
    return e && e[0] == '1';
  }();
  int64_t coff = 0;
  leg_problems(p, R, ldT, [&](GemmDesc g) {
    if (compact && !p->band_world) {
      if (!p->inverse) {
        g.ldc = (int)round_up(g.N, 4);
        g.offC = coff;
        coff += (int64_t)R * g.ldc;
      } else {
        g.lda = (int)round_up(std::max(g.K, 1), 4);
        g.offA = coff;
        coff += (int64_t)R * g.lda;
      }
    }
    g.tiles_m = (int)cdiv(g.M, bm);
    g.tiles_n = (int)cdiv(g.N, bn);
    if (g.tiles_m * g.tiles_n == 0) return;
    g.tile_start = tiles;
    tiles += g.tiles_m * g.tiles_n;
    d.push_back(g);
  });
  (void)other_ld;
  msfno_sht_plan_s::DescSet set;
  MSFNO_TRY(upload_descs(d, tiles, false, &set));
  p->desc_sets[R] = set;
  p->d_desc = set.d;
  p->ndesc = set.n;
  p->desc_tiles = set.tiles;
  p->desc_R = R;
  return MSFNO_OK;
}

// ---- x3h Legendre (legendre_x3.hip) -------------------------------------------------
// The same problems on the x3h engine: the table as a column-scaled two-plane fp16
// image ([plane][n][Kp] per problem, built on first use after a table load), A split
// in-kernel under per-(row, k-tile) scales.  Default with the x3h engine (side stream
// off, two interleaved pairs: forward 0.32 vs 0.39 ms, inverse 0.52 vs 0.55 ms for the
// fp32-MFMA descriptor GEMM); MSFNO_LEG_X3=0 keeps the fp32 GEMM.
bool leg_x3_enabled() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_LEG_X3");
    if (e) return e[0] == '1' && gemm_use_x6();
    return mlp_fused_h_env() && gemm_use_x6();
  }();
  return on;
}

// inverse problems on the register-resident kernel (legendre_x3r) when every problem
// fits it (K <= X3R_KMAX, N <= X3R_NMAX); MSFNO_LEG_X3R=0 keeps the tiled kernel
static bool x3r_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_LEG_X3R");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int build_tab3(msfno_sht_plan_s* p, int R, int64_t ldT, hipStream_t s);

static int ensure_desc3(msfno_sht_plan_s* p, int R, int64_t ldT, hipStream_t s) {
  if (p->desc3_R == R && p->d_desc3 && p->tab3_valid) return MSFNO_OK;
  auto hit = p->desc3_sets.find(R);
  if (hit != p->desc3_sets.end()) {
    p->d_desc3 = hit->second.d;
    p->d_tile3 = hit->second.tile;
    p->ndesc3 = hit->second.n;
    p->desc3_tiles = hit->second.tiles;
    p->desc3_res = hit->second.res;
    p->desc3_R = R;
    if (p->tab3_valid) return MSFNO_OK;
  }
  MSFNO_TRY(require_not_capturing(s, "x3h Legendre image"));
  if (hit != p->desc3_sets.end()) return build_tab3(p, R, ldT, s);
  bool res = p->inverse && x3r_env();
  if (res)
    leg_problems(p, R, ldT, [&](GemmDesc g) {
      if (g.K > X3R_KMAX || g.N > X3R_NMAX || g.N <= 0) res = false;
    });
  p->desc3_res = res ? 1 : 0;
  std::vector<GemmDesc> d;
  int tiles = 0;
  int64_t img = 0, sc = 0;
  leg_problems(p, R, ldT, [&](GemmDesc g) {
    g.tiles_m = (int)cdiv(g.M, X3D_BM);
    g.tiles_n = res ? 1 : (int)cdiv(g.N, x3d_bn(p->inverse));
    // every problem gets its image, also K = 0 ones (written as zeros)
    g.offBx = img;
    g.offBs = sc;
    img += 2LL * g.N * round_up(std::max(g.K, 1), X3D_BK);
    sc += g.N;
    if (g.tiles_m * g.tiles_n == 0) return;
    g.tile_start = tiles;
    tiles += g.tiles_m * g.tiles_n;
    d.push_back(g);
  });
  msfno_sht_plan_s::DescSet set;
  MSFNO_TRY(upload_descs(d, tiles, true, &set));
  set.res = p->desc3_res;
  p->desc3_sets[R] = set;
  p->d_desc3 = set.d;
  p->d_tile3 = set.tile;
  p->ndesc3 = set.n;
  p->desc3_tiles = set.tiles;
  p->desc3_R = R;
  (void)img;
  (void)sc;
  return build_tab3(p, R, ldT, s);
}

// the x3h table image and column scales (R-independent: every descriptor set gives the
// same image offsets), rebuilt after a table load
static int build_tab3(msfno_sht_plan_s* p, int R, int64_t ldT, hipStream_t s) {
  int64_t img = 0, sc = 0;
  leg_problems(p, R, ldT, [&](GemmDesc g) {
    img += 2LL * g.N * round_up(std::max(g.K, 1), X3D_BK);
    sc += g.N;
  });
  if (!p->tab3_valid || img > p->tab3_elems || sc > p->tab3s_elems) {
    if (img > p->tab3_elems) {
      if (p->tab3) MSFNO_CHECK_HIP(hipFree(p->tab3));
      p->tab3 = nullptr;
      MSFNO_CHECK_HIP(hipMalloc(&p->tab3, std::max<int64_t>(1, img) * sizeof(unsigned short)));
      p->tab3_elems = img;
    }
    if (sc > p->tab3s_elems) {
      if (p->tab3s) MSFNO_CHECK_HIP(hipFree(p->tab3s));
      p->tab3s = nullptr;
      MSFNO_CHECK_HIP(hipMalloc(&p->tab3s, std::max<int64_t>(1, sc) * sizeof(float)));
      p->tab3s_elems = sc;
    }
    MSFNO_TRY(launch_legendre_x3_image(p->table, p->d_desc3, p->ndesc3, p->tab3, p->tab3s, s));
    p->tab3_valid = 1;
  }
  return MSFNO_OK;
}

// forward problems on legendre_x3f: the image and column scales of desc3, tiles of
// X3F_RB rows x 64 columns (column blocks of one row block adjacent).  Default with the
// x3h Legendre on symmetric, unsharded blocks with norm0 (the slab planes need its
// per-channel bound); MSFNO_LEG_X3F=0 keeps legendre_x3 on the fp32 slab.
bool x3f_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_LEG_X3F");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool x3f_usable(msfno_sht_plan_s* f) {
  if (!x3f_env() || !leg_x3_enabled() || !f->sym || f->inverse) return false;
  if (f->band_world)  // the receive buffer, segmented by source rank (W % 8 == 0)
    return f->band_W % 8 == 0 && f->band_K() <= X3F_KMAX;
  if (f->nslab != f->mmax) return false;
  return f->Ke <= X3F_KMAX && f->Ko <= X3F_KMAX && f->ldke % 8 == 0 && f->ldk % 8 == 0 &&
         std::max(f->ldke, f->ldk - f->ldke) <= cdiv(f->Ke, 64) * 64;
}

static int ensure_desc3f(msfno_sht_plan_s* p, int R, int64_t ldT, hipStream_t s) {
  MSFNO_TRY(ensure_desc3(p, R, ldT, s));
  if (p->desc3f_R == R && p->d_desc3f) return MSFNO_OK;
  auto hit = p->desc3f_sets.find(R);
  if (hit != p->desc3f_sets.end()) {
    p->d_desc3f = hit->second.d;
    p->d_tile3f = hit->second.tile;
    p->ndesc3f = hit->second.n;
    p->desc3f_tiles = hit->second.tiles;
    p->desc3f_R = R;
    return MSFNO_OK;
  }
  MSFNO_TRY(require_not_capturing(s, "x3h forward Legendre descriptors"));
  std::vector<GemmDesc> d;
  int tiles = 0;
  int64_t img = 0, sc = 0;
  leg_problems(p, R, ldT, [&](GemmDesc g) {  // the offsets ensure_desc3 gave the image
    g.offBx = img;
    g.offBs = sc;
    img += 2LL * g.N * round_up(std::max(g.K, 1), X3D_BK);
    sc += g.N;
    g.tiles_m = (int)cdiv(g.M, X3F_RB);
    g.tiles_n = (int)cdiv(g.N, 64);
    if (g.tiles_m * g.tiles_n == 0 || g.K <= 0) return;
    g.tile_start = tiles;
    tiles += g.tiles_m * g.tiles_n;
    d.push_back(g);
  });
  msfno_sht_plan_s::DescSet set;
  MSFNO_TRY(upload_descs(d, tiles, true, &set));
  p->desc3f_sets[R] = set;
  p->d_desc3f = set.d;
  p->d_tile3f = set.tile;
  p->ndesc3f = set.n;
  p->desc3f_tiles = set.tiles;
  p->desc3f_R = R;
  return MSFNO_OK;
}

// forward Legendre on the slab planes of launch_transpose_fwd_sym_h (Xp: fp16 pairs
// interleaved per 8 k, isr: 1 / sigma per row) -> S
int legendre_fwd_x3f(msfno_sht_plan_s* f, const unsigned short* Xp, const float* isr, float* S,
                     int R, hipStream_t s) {
  MSFNO_TRY(ensure_desc3f(f, R, f->spec.ldT, s));
  const int segw = f->band_world ? f->band_seg() : 0;
  const int64_t segs = f->band_world ? (int64_t)f->nslab * R * 2 * f->band_W : 0;
  return legendre_x3f(Xp, isr, f->tab3, f->tab3s, S, f->d_desc3f, f->d_tile3f,
                      f->ndesc3f, f->desc3f_tiles, s, segw, segs);
}

// spectral MLP: Gauss 3M complex GEMM by default (MSFNO_SPEC_4M=1: the real-ified
// 4-multiplication GEMM, kept as an A/B switch); MSFNO_C3M_TILE picks its tile
bool use_c3m() {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("MSFNO_SPEC_4M");
    mode = (e && e[0] == '1') ? 0 : 1;
  }
  return mode == 1;
}

// spectral MLP on the x6 engine (real-ified 4-multiplication GEMM on the bf16
// matrix cores, fp32-accurate split) whenever the dense GEMMs use it;
// MSFNO_SPEC_X6=0 keeps the fp32 3M kernel for A/B
bool spec_use_x6() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SPEC_X6");
    return gemm_use_x6() && !(e && e[0] == '0');
  }();
  return on;
}

int c3m_tile() {
  static int t = -1;
  if (t < 0) {
    const char* e = getenv("MSFNO_C3M_TILE");
    t = e ? atoi(e) : 1;  // 64x128 measured best (in-block A/B)
  }
  return t;
}

// MSFNO_FFT_TILE=1 selects the fused FFT+transpose tile kernels instead of the
// row FFT + separate transpose kernels (measured slower on MI355X at 721x1440:
// DESIGN.md §5); kept as an A/B switch.
bool use_fft_tile(const msfno_sht_plan_s* p) {
  static int mode = -1;
  if (mode < 0) {
    const char* e = getenv("MSFNO_FFT_TILE");
    mode = (e && e[0] == '1') ? 1 : 0;
  }
  return mode == 1 && !p->sym && fft_tile_supported(p->fft);  // tile kernels: general layout
}

// Xn (BC, nlat, mmax) -> the plan's slab layout (hemispheres folded when symmetric)
int transpose_fwd_plan(const msfno_sht_plan_s* p, const float2* Xn, float* Xt, int B, int C,
                       const float* nscale, const float* nshift, hipStream_t s) {
  if (p->sym)
    return launch_transpose_fwd_sym(Xn, Xt, B, C, p->geom(), p->mmax, nscale, nshift, s);
  return launch_transpose_fwd(Xn, Xt, B, C, p->nlat, p->mmax, p->ldk, nscale, nshift, s);
}

int transpose_inv_plan(const msfno_sht_plan_s* p, const float* Yt, float2* Yn, int B, int C,
                       hipStream_t s) {
  if (p->sym) return launch_transpose_inv_sym(Yt, Yn, B, C, p->geom(), p->mmax, p->spec.mact, s);
  return launch_transpose_inv(Yt, Yn, B, C, p->nlat, p->mmax, p->spec.mact, p->ldk, s);
}

int legendre_fwd(msfno_sht_plan_s* f, const float* Xt, float* S, int R, hipStream_t s,
                 const float* rowscale, int C) {
  if (leg_x3_enabled() && !rowscale) {
    MSFNO_TRY(ensure_desc3(f, R, f->spec.ldT, s));
    GemmEpi e;
    if (f->band_world) {
      e.segA_w = f->band_seg();
      e.segA_stride = (int64_t)f->nslab * R * 2 * f->band_W;
    }
    return legendre_x3(Xt, f->tab3, f->tab3s, S, f->d_desc3, f->d_tile3, f->ndesc3,
                       f->desc3_tiles, x3d_bn(0), e, s);
  }
  MSFNO_TRY(ensure_desc(f, R, 0, f->spec.ldT, s));
  GemmEpi e;
  e.rowscale = rowscale;
  e.rs_C = C;
  if (f->band_world) {  // Xt is the phase-0 receive buffer: one block per source rank
    e.segA_w = f->band_seg();
    e.segA_stride = (int64_t)f->nslab * R * 2 * f->band_W;
  }
  return gemm_desc(leg_tile(0), Xt, f->table, S, f->d_desc, f->ndesc,
                   f->desc_tiles, e, s);
}

int legendre_inv(msfno_sht_plan_s* g, const float* S, float* Yt, int R, hipStream_t s) {
  if (leg_x3_enabled()) {
    MSFNO_TRY(ensure_desc3(g, R, g->spec.ldT, s));
    GemmEpi e;
    if (g->band_world) {
      e.segC_w = g->band_seg();
      e.segC_stride = (int64_t)g->nslab * R * 2 * g->band_W;
    }
    if (g->desc3_res)
      return legendre_x3r(S, g->tab3, g->tab3s, Yt, g->d_desc3, g->d_tile3, g->ndesc3,
                          g->desc3_tiles, e, s);
    return legendre_x3(S, g->tab3, g->tab3s, Yt, g->d_desc3, g->d_tile3, g->ndesc3,
                       g->desc3_tiles, x3d_bn(1), e, s);
  }
  MSFNO_TRY(ensure_desc(g, R, 0, g->spec.ldT, s));
  GemmEpi e;
  if (g->band_world) {  // Yt is the phase-1 send buffer: one block per destination rank
    e.segC_w = g->band_seg();
    e.segC_stride = (int64_t)g->nslab * R * 2 * g->band_W;
  }
  return gemm_desc(leg_tile(1), S, g->table, Yt, g->d_desc, g->ndesc,
                   g->desc_tiles, e, s);
}

// ---------------------------------------------------------------------------
// block workspace layout (shared by size query and forward)
// ---------------------------------------------------------------------------


void carve_block(Carve& cv, BlockBufs& b, const msfno_block_desc* d,
                        const msfno_sht_plan_s* f, const msfno_sht_plan_s* g, int B,
                        bool with_norms) {
  const int64_t C = d->C, BC = (int64_t)B * C, R = 2 * BC;
  const int64_t P = (int64_t)g->nlat * g->nlon;
  const SpecLayout& L = f->spec;
  b.Xn = cv.take<float2>(BC * f->nlat * f->mmax);
  b.Xt = cv.take<float>((int64_t)f->mmax * R * f->ldk);
  b.rs0 = cv.take<float2>(BC * f->nlat);
  b.sc0 = cv.take<float>(BC);
  b.sh0 = cv.take<float>(BC);
  b.Sa = cv.take<float>(R * L.ldT);
  b.Sb = b.Sc = nullptr;
  b.cs = nullptr;
  for (auto& w : b.Wexp) w = nullptr;
  b.dw = DenseWs{};
  b.xt = b.yt = nullptr;
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) {
    const int64_t Hs = d->spec_hidden;
    b.Sb = cv.take<float>(spec_hidden_floats(B, Hs, L));
    b.Sc = cv.take<float>(spec_hidden_floats(B, Hs, L));
    b.cs = cv.take<float>(2LL * B * round_up(L.Tp, 4));
    for (int l = 0; l <= d->spectral_layers; ++l) {
      const int64_t ci = (l == 0) ? C : Hs;
      const int64_t co = (l == d->spectral_layers) ? C : Hs;
      b.Wexp[l] = cv.take<float>(4 * ci * co);
    }
    if (d->wcache) {
      Carve wc;
      wc.base = static_cast<char*>(d->wcache);
      carve_spec_ws(wc, b.dw, d);
    } else {
      carve_spec_ws(cv, b.dw, d);
    }
  } else {
    // the gathered copies of the linear filter's input and output (tril order)
    b.xt = cv.take<float>(2 * BC * L.T);
    b.yt = cv.take<float>(2 * BC * L.T);
  }
  b.Yt = cv.take<float>((int64_t)g->mmax * R * g->ldk);
  b.Yn = cv.take<float2>(BC * g->nlat * g->mmax);
  b.x1 = nullptr;
  b.st1 = nullptr;
  b.sc1 = b.sh1 = b.W1f = b.b1f = b.h = nullptr;
  b.x1p = nullptr;
  b.mfimg = nullptr;
  if (!with_norms) return;
  b.x1 = cv.take<float>(BC * P);
  b.st1 = cv.take<float2>(BC * g->nlat);
  b.sc1 = cv.take<float>(BC);
  b.sh1 = cv.take<float>(BC);
  b.ab1 = cv.take<float>(BC);
  if (mlp_fused(d, P)) {
    b.mfimg = wcache_mfimg(d);
    if (!b.mfimg) b.mfimg = cv.take<unsigned short>(mlp_fused_image_bytes() / 2);
  } else if (d->has_mlp) {
    const int64_t Hd = d->mlp_hidden;
    b.W1f = cv.take<float>((int64_t)B * Hd * C);
    b.b1f = cv.take<float>((int64_t)B * Hd);
    b.h = cv.take<float>(mlp_h_floats(B, Hd, P));
  }
  b.x1p = x1p_buffer(d, g) ? cv.take<unsigned short>(BC * 3 * P) : nullptr;
  b.xs = skip_x3(d) ? cv.take<float>(BC) : nullptr;
  b.lsig = nullptr;
  b.isr = nullptr;
  if (x3f_env() && leg_x3_enabled()) {
    b.lsig = cv.take<float>(BC);
    b.isr = cv.take<float>(R);
  }
  carve_dense_ws(cv, b.dw, d, B);
}

void carve_dense_ws(Carve& cv, DenseWs& w, const msfno_block_desc* d, int B) {
  w.skip = w.fc1 = w.fc2 = nullptr;
  w.skip_b = w.fc1_b = w.fc2_b = 0;
  const int C = (int)d->C;
  if (d->inner_skip == MSFNO_SKIP_LINEAR &&
      (w.skip_b = std::max({gemm_dense_workspace(C, C, 1),
                            skip_x3(d) ? gemm_x3_workspace(C, C, B) : 0,
                            skip_x3(d) && C == 256 ? skip_h_workspace(B) : 0})))
    w.skip = cv.take<char>(w.skip_b);
  if (d->has_mlp) {
    const int Hd = (int)d->mlp_hidden;
    if ((w.fc1_b = gemm_dense_workspace(Hd, C, B))) w.fc1 = cv.take<char>(w.fc1_b);
    if ((w.fc2_b = gemm_dense_workspace(C, Hd, 1))) w.fc2 = cv.take<char>(w.fc2_b);
  }
}

// spectral MLP as Gauss 3M complex GEMMs on the x6 engine (gemm_x6c.hip);
// MSFNO_SPEC_3M=0 keeps the real-ified 4M x6p GEMMs for A/B
bool spec_use_3m() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SPEC_3M");
    return !(e && e[0] == '0');
  }();
  return on && spec_use_x6();
}

// spectral MLP on the x3h engine (gemm_x3c: fp32 as two fp16 terms, three fp16 MFMAs
// per product, power-of-two scaled operands) by default; MSFNO_ENGINE=x6 or
// MSFNO_SPEC_X3H=0 keep the x6 chain (A/B)
bool spec_use_x3h() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SPEC_X3H");
    if (e) return e[0] == '1';
    return mlp_fused_h_env();
  }();
  return on && spec_use_3m();
}

// floats to reserve for one spectral-MLP hidden buffer (B, 2 Hs, T): fp32, or
// bf16x3 planes with a row stride padded to 8 on the x6 engine
int64_t spec_hidden_floats(int B, int64_t Hs, const SpecLayout& L) {
  if (!spec_use_x6()) return (int64_t)B * 2 * Hs * L.ldT;
  const int64_t planes = spec_use_3m() ? 9 : 6;  // 3M: re, im, re+im; 4M: re/im rows
  return std::max<int64_t>({(int64_t)B * 2 * Hs * L.ldT,
                            cdiv((int64_t)B * planes * Hs * round_up(L.Tp, 8) * 2, 4),
                            cdiv((int64_t)B * x6c_tiled_elems((int)Hs, (int)L.Tp) * 2, 4)});
}

// prepared-weight cache layout (msfno_block_desc.wcache): the spectral images
// (carve_spec_ws order), then the fused MLP image
static size_t wcache_layout(const msfno_block_desc* d, unsigned short** mfimg) {
  Carve wc;
  wc.base = static_cast<char*>(d->wcache);
  DenseWs w;
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) carve_spec_ws(wc, w, d);
  unsigned short* m = nullptr;
  if (d->has_mlp && gemm_use_x6() && d->fc1_b && mlp_fused_supported((int)d->C, (int)d->mlp_hidden))
    m = wc.take<unsigned short>(mlp_fused_image_bytes() / 2);
  if (mfimg) *mfimg = m;
  return wc.off;
}

unsigned short* wcache_mfimg(const msfno_block_desc* d) {
  if (!d->wcache) return nullptr;
  unsigned short* m = nullptr;
  wcache_layout(d, &m);
  return m;
}

bool wcache_ready(const msfno_block_desc* d) { return d->wcache && d->wcache_valid; }

// split-A planes of the real-ified spectral MLP weights (x6 engine)
void carve_spec_ws(Carve& cv, DenseWs& w, const msfno_block_desc* d) {
  for (auto& p : w.spec) p = nullptr;
  for (auto& n : w.spec_b) n = 0;
  if (!spec_use_x6() || d->filter_type != MSFNO_FILTER_NONLINEAR) return;
  for (int l = 0; l <= d->spectral_layers && l < 9; ++l) {
    const int ci = (l == 0) ? (int)d->C : (int)d->spec_hidden;
    const int co = (l == d->spectral_layers) ? (int)d->C : (int)d->spec_hidden;
    w.spec_b[l] = std::max(gemm_dense_workspace(2 * co, 2 * ci, 1), gemm_x6c_weight_bytes(co, ci));
    if (w.spec_b[l]) w.spec[l] = cv.take<char>(w.spec_b[l]);
  }
}

int check_pair(const msfno_block_desc* d, const msfno_sht_plan_s* f,
                      const msfno_sht_plan_s* g) {
  MSFNO_REQUIRE(d && f && g, MSFNO_EINVAL, "null descriptor or plan");
  MSFNO_REQUIRE(!f->inverse && g->inverse, MSFNO_EINVAL,
                "forward plan must be a RealSHT plan and inverse an InverseRealSHT plan");
  MSFNO_REQUIRE(f->lmax == g->lmax && f->mmax == g->mmax, MSFNO_EINVAL,
                "inverse_transform lmax/mmax must equal forward_transform's (layers.py:364-365)");
  MSFNO_REQUIRE(f->table_loaded && g->table_loaded, MSFNO_EINVAL, "plan tables not loaded");
  MSFNO_REQUIRE(d->C > 0, MSFNO_EINVAL, "C must be > 0");
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) {
    MSFNO_REQUIRE(d->spectral_layers >= 1 && d->spectral_layers <= 8, MSFNO_EUNSUPPORTED,
                  "spectral_layers must be in [1, 8]");
    MSFNO_REQUIRE(d->spec_hidden > 0, MSFNO_EINVAL, "spec_hidden must be > 0");
  } else {
    MSFNO_REQUIRE(d->filter_type == MSFNO_FILTER_LINEAR, MSFNO_EUNSUPPORTED, "unknown filter_type");
  }
  return MSFNO_OK;
}

int run_filter(const msfno_block_desc* d, msfno_sht_plan_s* f, msfno_sht_plan_s* g,
                      const BlockBufs& b, int B, hipStream_t s) {
  const int64_t C = d->C;
  const SpecLayout& L = f->spec;
  if (d->filter_type == MSFNO_FILTER_NONLINEAR) {
    const int nl = d->spectral_layers;
    const int64_t Hs = d->spec_hidden;
    prof(ST_SPEC_PREP, s);
    const bool x6 = spec_use_x6() && b.dw.spec[0];
    const bool c3m = !x6 && use_c3m();
    if (x6 && spec_use_3m() && C <= Hs) {
      // Gauss 3M complex GEMMs (gemm_x6c.hip): weights Wr, Wi, Wr+Wi of all layers in
      // one launch; layer 0's input split into 3M planes in Sc (free until layer 1)
      SpecWeightsX6p sw{};
      sw.nlayers = nl + 1;
      for (int l = 0; l <= nl; ++l) {
        sw.w[l] = (l == nl) ? d->spec_wout : d->spec_w[l];
        MSFNO_REQUIRE(sw.w[l], MSFNO_EINVAL, "missing spectral weight");
        sw.ci[l] = (l == 0) ? (int)C : (int)Hs;
        sw.co[l] = (l == nl) ? (int)C : (int)Hs;
        sw.out[l] = static_cast<unsigned short*>(b.dw.spec[l]);
      }
      spec_weights_3m_layout(sw);
      if (spec_use_x3h() && b.cs && L.ldT % 4 == 0) {
        // x3h engine: two fp16 planes per value, three MFMAs per product; the layer
        // scales (2 floats per layer) live behind layer 0's A image (inside wcache when
        // the images are cached), the per-column input scales in b.cs
        const int64_t a0 = round_up(6LL * round_up(sw.co[0], 128) * round_up(sw.ci[0], 16) * 2, 256);
        MSFNO_REQUIRE((size_t)a0 + 2 * (nl + 1) * sizeof(float) <= b.dw.spec_b[0], MSFNO_EWORKSPACE,
                      "x3h spectral scales do not fit behind layer 0's image");
        sw.scl = reinterpret_cast<float*>(static_cast<char*>(b.dw.spec[0]) + a0);
        if (!wcache_ready(d)) MSFNO_TRY(launch_spec_weights_3m_x3h(sw, s));
        const int ldcs = (int)round_up(L.Tp, 4);
        MSFNO_TRY(launch_spec_colscale(b.Sa, B, (int)C, (int)L.Tp, (int)L.ldT, b.cs, ldcs, s));
        unsigned short* cur = nullptr;
        for (int l = 0; l <= nl; ++l) {
          prof(l == nl ? ST_SPEC_OUT : ST_SPEC_L0 + std::min(l, 3), s);
          unsigned short* out = l == nl ? nullptr
                                        : reinterpret_cast<unsigned short*>((l & 1) ? b.Sc : b.Sb);
          MSFNO_TRY(gemm_x3c(sw.out[l], sw.co[l], sw.ci[l], l == 0 ? b.Sa : nullptr, (int)L.ldT,
                             l == 0 ? nullptr : cur, (int)L.Tp, out, l == nl ? b.Sa : nullptr,
                             (int)L.ldT, l < nl, sw.scl + 2 * l + 1,
                             l == 0 ? b.cs : (l == nl ? b.cs + (int64_t)B * ldcs : nullptr), ldcs, B,
                             s));
          cur = out;
        }
        return MSFNO_OK;
      }
      if (!wcache_ready(d)) MSFNO_TRY(launch_spec_weights_3m(sw, s));
      const int ldTx = (int)round_up(L.Tp, 8);
      unsigned short* cur = reinterpret_cast<unsigned short*>(b.Sc);
      // layer 0 stages S fp32 and splits it in-kernel (no split3m pass, 0.1 ms less
      // per block at config 2); MSFNO_SPEC_L0F32=0 restores the separate split3m
      static const bool l0f32 = [] {
        const char* e = getenv("MSFNO_SPEC_L0F32");
        return !(e && e[0] == '0');
      }();
      const bool f32b = l0f32 && nl >= 1 && L.ldT % 4 == 0;
      // hidden activations in the tiled layout (gemm_x6c.hip; spectral MLP 8 % faster
      // at config 2); MSFNO_X6C_TILED=0: row layout [b][mat][plane][c][ld]
      static const bool tiled = [] {
        const char* e = getenv("MSFNO_X6C_TILED");
        return !(e && e[0] == '0');
      }();
      if (f32b && tiled) {
        for (int l = 0; l <= nl; ++l) {
          prof(l == nl ? ST_SPEC_OUT : ST_SPEC_L0 + std::min(l, 3), s);
          unsigned short* out = l == nl ? nullptr
                                        : reinterpret_cast<unsigned short*>((l & 1) ? b.Sc : b.Sb);
          if (l == 0)
            MSFNO_TRY(gemm_x6c_f32b(sw.out[0], sw.co[0], sw.ci[0], b.Sa, (int)L.ldT, (int)L.Tp, out,
                                    ldTx, nullptr, 0, true, B, s, true));
          else
            MSFNO_TRY(gemm_x6c(sw.out[l], sw.co[l], sw.ci[l], cur, (int)L.Tp, ldTx, out,
                               l == nl ? b.Sa : nullptr, (int)L.ldT, l < nl, B, s, l == nl ? 1 : 3));
          cur = out;
        }
        return MSFNO_OK;
      }
      if (!f32b) MSFNO_TRY(launch_split3m(b.Sa, cur, B, (int)C, (int)L.Tp, (int)L.ldT, ldTx, s));
      for (int l = 0; l <= nl; ++l) {
        prof(l == nl ? ST_SPEC_OUT : ST_SPEC_L0 + std::min(l, 3), s);
        unsigned short* out = l == nl ? nullptr
                                      : reinterpret_cast<unsigned short*>((l & 1) ? b.Sc : b.Sb);
        if (l == 0 && f32b)
          MSFNO_TRY(gemm_x6c_f32b(sw.out[0], sw.co[0], sw.ci[0], b.Sa, (int)L.ldT, (int)L.Tp, out,
                                  ldTx, nullptr, 0, true, B, s));
        else
          MSFNO_TRY(gemm_x6c(sw.out[l], sw.co[l], sw.ci[l], cur, (int)L.Tp, ldTx, out,
                             l == nl ? b.Sa : nullptr, (int)L.ldT, l < nl, B, s));
        cur = out;
      }
      return MSFNO_OK;
    }
    const bool split_l0 = x6 && C <= Hs;  // layer 0 input split into Sc (below)
    if (x6) {
      // every layer's real-ified weight straight into its x6p A image, one launch
      SpecWeightsX6p sw{};
      sw.nlayers = nl + 1;
      for (int l = 0; l <= nl; ++l) {
        sw.w[l] = (l == nl) ? d->spec_wout : d->spec_w[l];
        MSFNO_REQUIRE(sw.w[l], MSFNO_EINVAL, "missing spectral weight");
        sw.ci[l] = (l == 0) ? (int)C : (int)Hs;
        sw.co[l] = (l == nl) ? (int)C : (int)Hs;
        sw.out[l] = static_cast<unsigned short*>(b.dw.spec[l]);
      }
      spec_weights_x6p_layout(sw);
      if (!wcache_ready(d)) MSFNO_TRY(launch_spec_weights_x6p(sw, s));
    }
    for (int l = 0; l <= nl; ++l) {
      const int ci = (l == 0) ? (int)C : (int)Hs;
      const int co = (l == nl) ? (int)C : (int)Hs;
      const float* w = (l == nl) ? d->spec_wout : d->spec_w[l];
      MSFNO_REQUIRE(w, MSFNO_EINVAL, "missing spectral weight");
      if (x6 && (l > 0 || split_l0)) continue;  // prepared above
      if (c3m)
        MSFNO_TRY(launch_split_complex_weight(w, b.Wexp[l], b.Wexp[l] + (int64_t)ci * co, ci, co, s));
      else
        MSFNO_TRY(launch_expand_complex_weight(w, b.Wexp[l], ci, co, s));
    }
    const float* in = b.Sa;
    for (int l = 0; l <= nl; ++l) {
      const int ci = (l == 0) ? (int)C : (int)Hs;
      const int co = (l == nl) ? (int)C : (int)Hs;
      float* out = (l == nl) ? b.Sa : ((l & 1) ? b.Sc : b.Sb);
      prof(l == nl ? ST_SPEC_OUT : ST_SPEC_L0 + std::min(l, 3), s);
      if (x6) {
        // real-ified [[Wr, -Wi], [Wi, Wr]] GEMM on the x6 engine, ComplexReLU(real)
        // = ReLU on the real rows of each batch block, in the epilogue.  Hidden
        // activations travel as bf16x3 planes [b][plane][2 Hs][ldTx]: layer 0
        // splits its fp32 input in-kernel, later layers stage planes by LDS-DMA
        // (gemm_x6p), the output layer writes fp32 S for the inverse Legendre.
        const int64_t ldTx = round_up(L.Tp, 8);
        GemmEpi e;
        if (l < nl) {
          e.relu_period = 2 * co;
          e.relu_rows = co;
          e.c_planes = reinterpret_cast<unsigned short*>(out);
          e.c_plane_stride = 2LL * co * ldTx;
        }
        const int ldc = l < nl ? (int)ldTx : (int)L.ldT;
        const int64_t sC = l < nl ? 3 * 2LL * co * ldTx : 2LL * co * L.ldT;
        if (l > 0 || split_l0) e.a_planes = static_cast<const unsigned short*>(b.dw.spec[l]);
        if (l == 0 && split_l0) {  // Sc is free during layer 0
          // layer 0's fp32 input (the forward Legendre output) -> planes in Sc: one
          // streaming pass, then the LDS-DMA kernel (cheaper than splitting the
          // 2C x T operand once per M-tile inside the GEMM)
          unsigned short* inx = reinterpret_cast<unsigned short*>(b.Sc);
          MSFNO_TRY(launch_split_planes(in, inx, 2 * ci, (int)L.Tp, (int)L.ldT, 2LL * ci * L.ldT,
                                        (int)ldTx, 2LL * ci * ldTx, 3 * 2LL * ci * ldTx, B, s));
          e.b_planes = inx;
          e.b_plane_stride = 2LL * ci * ldTx;
          MSFNO_TRY(gemm_x6p(b.Wexp[l], out, 2 * co, (int)L.Tp, 2 * ci, 2 * ci, (int)ldTx, ldc, 0,
                             3 * 2LL * ci * ldTx, sC, B, e, b.dw.spec[l], b.dw.spec_b[l], s));
        } else if (l == 0) {
          MSFNO_TRY(gemm_dense(ROLE_SPEC, TILE_128x128, b.Wexp[l], in, out, 2 * co, (int)L.Tp,
                               2 * ci, 2 * ci, (int)L.ldT, ldc, 0, 2LL * ci * L.ldT, sC, B, e,
                               b.dw.spec[l], b.dw.spec_b[l], s));
        } else {
          e.b_planes = reinterpret_cast<const unsigned short*>(in);
          e.b_plane_stride = 2LL * ci * ldTx;
          MSFNO_TRY(gemm_x6p(b.Wexp[l], out, 2 * co, (int)L.Tp, 2 * ci, 2 * ci, (int)ldTx, ldc, 0,
                             3 * 2LL * ci * ldTx, sC, B, e, b.dw.spec[l], b.dw.spec_b[l], s));
        }
      } else if (c3m) {
        // Gauss 3-multiplication complex GEMM (cgemm.hip), ComplexReLU(real) fused
        MSFNO_TRY(gemm_c3m(b.Wexp[l], b.Wexp[l] + (int64_t)ci * co, in, out, co, ci, (int)L.Tp,
                           (int)L.ldT, (int)L.ldT, 2LL * ci * L.ldT, 2LL * co * L.ldT, B, l < nl,
                           c3m_tile(), s));
      } else {
        GemmEpi e;
        if (l < nl) {  // ComplexReLU(mode="real") on the real rows of each batch block
          e.relu_period = 2 * co;
          e.relu_rows = co;
        }
        MSFNO_TRY(gemm_uniform(role_tile(ROLE_SPEC, TILE_128x128), b.Wexp[l], in, out, 2 * co,
                               (int)L.Tp, 2 * ci, 2 * ci, (int)L.ldT, (int)L.ldT, 0,
                               2LL * ci * L.ldT, 2LL * co * L.ldT, B, e, s));
      }
      in = out;
    }
  } else {
    MSFNO_REQUIRE(d->lin_w, MSFNO_EINVAL, "missing linear spectral weight");
    prof(ST_LIN_GATHER, s);
    MSFNO_TRY(launch_spec_to_tril(*f, b.Sa, b.xt, B, (int)C, s));
    prof(ST_LIN_CONTRACT, s);
    MSFNO_TRY(launch_compl_contract(b.xt, d->lin_w, b.yt, B, (int)C, (int)C, L.T, s));
    prof(ST_LIN_SCATTER, s);
    MSFNO_TRY(launch_tril_to_spec(*f, b.yt, b.Sa, B, (int)C, s));
  }
  (void)g;
  return MSFNO_OK;
}

// x -> (FFT, norm0 folded) -> Legendre -> filter -> inverse Legendre -> Yn
// xplanes: the forward FFT also writes x as bf16x3 planes; after_fft runs once the
// forward FFT is enqueued (the block forks its inner-skip GEMM there)
int run_spectral(const msfno_block_desc* d, msfno_sht_plan_s* f, msfno_sht_plan_s* g,
                 const BlockBufs& b, const float* x, int B, bool norm0, hipStream_t s,
                 const C2RPlanes* xplanes = nullptr,
                 const std::function<int()>& after_fft = std::function<int()>(),
                 const std::function<int()>& after_norm0 = std::function<int()>(),
                 const std::function<int()>& after_leg = std::function<int()>(),
                 const std::function<int()>& before_inv = std::function<int()>()) {
  const int64_t C = d->C, BC = (int64_t)B * C, R = 2 * BC;
  prof(ST_FFT_FWD, s);
  const float scale = (float)(2.0 * M_PI / f->nlon);
  if (use_fft_tile(f)) {
    // fused FFT + transpose; norm0 applied afterwards (m = 0 fix-up + GEMM row scale)
    MSFNO_TRY(launch_fft_r2c_tile(f->fft, x, b.Xt, norm0 ? b.rs0 : nullptr, B, (int)C, f->nlat,
                                  f->mmax, f->ldk, scale, s));
    if (norm0) {
      prof(ST_NORM0, s);
      MSFNO_TRY(launch_chan_affine(b.rs0, f->nlat, f->nlon, f->nlon, B, (int)C, d->norm0_w,
                                   d->norm0_b, d->norm_eps, nullptr, nullptr, 0.f, b.sc0, b.sh0,
                                   s, b.xs));
      if (after_norm0) MSFNO_TRY(after_norm0());
      MSFNO_TRY(launch_dc_fixup(b.Xt, B, (int)C, f->nlat, f->ldk, b.sc0, b.sh0, s));
    }
    prof(ST_LEG_FWD, s);
    MSFNO_TRY(legendre_fwd(f, b.Xt, b.Sa, (int)R, s, norm0 ? b.sc0 : nullptr, (int)C));
  } else {
    MSFNO_TRY(launch_fft_r2c_rows(f->fft, x, b.Xn, norm0 ? b.rs0 : nullptr, BC * f->nlat, f->mmax,
                                  scale, s, xplanes));
    if (after_fft) MSFNO_TRY(after_fft());
    if (norm0) {
      prof(ST_NORM0, s);
      MSFNO_TRY(launch_chan_affine(b.rs0, f->nlat, f->nlon, f->nlon, B, (int)C, d->norm0_w,
                                   d->norm0_b, d->norm_eps, nullptr, nullptr, 0.f, b.sc0, b.sh0,
                                   s, b.xs, b.lsig));
      if (after_norm0) MSFNO_TRY(after_norm0());
    }
    prof(ST_TRANSPOSE_FWD, s);
    if (norm0 && b.lsig && b.isr && x3f_usable(f)) {
      // slab as x3h fp16 pairs in the Xt buffer (the fp32 bytes)
      unsigned short* Xp = reinterpret_cast<unsigned short*>(b.Xt);
      MSFNO_TRY(launch_transpose_fwd_sym_h(b.Xn, Xp, B, (int)C, f->geom(), f->mmax, b.sc0, b.sh0,
                                           b.lsig, b.isr, s));
      prof(ST_LEG_FWD, s);
      MSFNO_TRY(legendre_fwd_x3f(f, Xp, b.isr, b.Sa, (int)R, s));
    } else {
      MSFNO_TRY(transpose_fwd_plan(f, b.Xn, b.Xt, B, (int)C, norm0 ? b.sc0 : nullptr,
                                   norm0 ? b.sh0 : nullptr, s));
      prof(ST_LEG_FWD, s);
      MSFNO_TRY(legendre_fwd(f, b.Xt, b.Sa, (int)R, s));
    }
  }
  if (after_leg) MSFNO_TRY(after_leg());
  MSFNO_TRY(run_filter(d, f, g, b, B, s));
  if (before_inv) MSFNO_TRY(before_inv());
  prof(ST_LEG_INV, s);
  // (the linear filter on S writes its output to Sb)
  MSFNO_TRY(legendre_inv(g, b.Sa, b.Yt, (int)R, s));
  return MSFNO_OK;
}

// Yt -> spatial rows (fused transpose + irfft when enabled); out = act(addsrc + irfft)
int run_inverse_fft(msfno_sht_plan_s* g, const BlockBufs& b, int B, int C, float* out,
                           const float* addsrc, float2* rowstats, int act, hipStream_t s,
                           unsigned short* planes = nullptr) {
  const int64_t BC = (int64_t)B * C;
  if (use_fft_tile(g) && addsrc == nullptr) {
    prof(ST_FFT_INV, s);
    return launch_fft_c2r_tile(g->fft, b.Yt, out, rowstats, B, C, g->nlat, g->mmax,
                               g->spec.mact, g->ldk, act, s);
  }
  prof(ST_TRANSPOSE_INV, s);
  MSFNO_TRY(transpose_inv_plan(g, b.Yt, b.Yn, B, C, s));
  prof(ST_FFT_INV, s);
  if (planes) {
    const C2RPlanes pl{planes, C, g->nlat};
    return launch_fft_c2r_rows(g->fft, b.Yn, out, addsrc, rowstats, BC * g->nlat, g->mmax, act,
                               s, &pl);
  }
  return launch_fft_c2r_rows(g->fft, b.Yn, out, addsrc, rowstats, BC * g->nlat, g->mmax, act, s);
}


// per-m table offsets of the plan GEMM layout:
//   general:   fwd  W (nlat x Lp) columns in S order;  inv  P (Lp x ldk) rows in S order
//   symmetric: fwd  We (Ke x Lpe), Wo (Ko x Lpo);      inv  Pe (Lpe x ldke), Po (Lpo x ldko)
void set_table_offsets(msfno_sht_plan_s* p, int sym) {
  const SpecLayout& L = p->spec;
  p->tab_off.assign(p->mmax, 0);
  int64_t acc = 0;
  for (int m = 0; m < p->mmax; ++m) {
    p->tab_off[m] = acc;
    if (L.L[m] == 0) continue;
    const int64_t lpe = L.Lpe[m], lpo = L.Lp[m] - L.Lpe[m];
    if (p->band_world) {  // band plans: W / P blocks over the band_K() exchange columns
      acc += (int64_t)p->band_K() * L.Lp[m];
      continue;
    }
    if (!sym)
      acc += p->inverse ? (int64_t)L.Lp[m] * p->ldk : (int64_t)p->nlat * L.Lp[m];
    else
      acc += p->inverse ? lpe * p->ldke + lpo * round_up(p->Ko, 4)
                        : (int64_t)p->Ke * lpe + (int64_t)p->Ko * lpo;
  }
  p->table_elems = acc;
}

int plan_create(int nlat, int nlon, int lmax, int mmax, int inverse,
                const std::vector<char>* mask, msfno_sht_plan_s** plan) {
  MSFNO_REQUIRE(nlat > 0 && nlon > 1 && lmax > 0 && mmax > 0, MSFNO_EINVAL, "bad SHT dims");
  MSFNO_REQUIRE(mmax <= nlon / 2 + 1, MSFNO_EINVAL, "mmax must be <= nlon//2 + 1");
  MSFNO_REQUIRE(!mask || (int)mask->size() == mmax, MSFNO_EINVAL, "m-set mask must have mmax entries");
  auto* p = new msfno_sht_plan_s();
  p->nlat = nlat; p->nlon = nlon; p->lmax = lmax; p->mmax = mmax; p->inverse = inverse ? 1 : 0;
  p->nh = nlat / 2;
  p->Ke = nlat - p->nh;
  p->Ko = p->nh;
  // slab columns padded to 16: whole k-tiles of the x6 Legendre GEMM stay in a row
  p->ldke = (int)round_up(p->Ke, 16);
  p->ldk = (int)std::max<int64_t>(round_up(nlat, 16), p->ldke + round_up(p->Ko, 16));
  p->spec.build(lmax, mmax, mask);
  p->slab.assign(mmax, -1);
  for (int m = 0; m < mmax; ++m) {
    if (!mask) p->slab[m] = m;
    else if (p->spec.L[m] > 0) p->slab[m] = p->nslab++;
  }
  if (!mask) p->nslab = mmax;
  int rc = fft_plan_build(p->fft, nlon);
  if (rc != MSFNO_OK) { delete p; return rc; }
  // table sized for the general (non-symmetric) layout, the larger of the two
  set_table_offsets(p, 0);
  const int64_t acc = p->table_elems;
  p->table_cap = std::max<int64_t>(acc, 4);
  hipError_t e = hipMalloc(&p->table, p->table_cap * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&p->d_tab_off, mmax * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&p->d_Lp, mmax * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&p->d_off, mmax * sizeof(int));
  if (e == hipSuccess) e = hipMalloc(&p->d_Lpe, mmax * sizeof(int));
  if (e == hipSuccess) e = hipMemcpy(p->d_Lpe, p->spec.Lpe.data(), mmax * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_tab_off, p->tab_off.data(), mmax * sizeof(int64_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_Lp, p->spec.Lp.data(), mmax * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(p->d_off, p->spec.off.data(), mmax * sizeof(int), hipMemcpyHostToDevice);
  if (e == hipSuccess && mask) {
    // tril order: row l holds m = 0..min(l, mmax-1) (torch.tril_indices(lmax, mmax),
    // layers.py:368); keep the plan's own modes in ascending global order
    std::vector<int> loc;
    loc.reserve((size_t)lmax * std::min(lmax, mmax));
    for (int l = 0; l < lmax; ++l)
      for (int m = 0; m <= std::min(l, mmax - 1); ++m) {
        if ((*mask)[m]) {
          loc.push_back((int)p->lin_modes.size());
          p->lin_modes.push_back((long long)loc.size() - 1);
        } else {
          loc.push_back(-1);
        }
      }
    e = hipMalloc(&p->d_tril_local, std::max<size_t>(loc.size(), 1) * sizeof(int));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_tril_local, loc.data(), loc.size() * sizeof(int), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && !mask) {
    const SpecLayout& L = p->spec;
    std::vector<int> tcol;
    tcol.reserve((size_t)L.T);
    std::vector<char> used((size_t)L.Tp, 0);
    for (int l = 0; l < lmax; ++l)
      for (int m = 0; m <= std::min(l, mmax - 1); ++m) {
        const int64_t t = L.col(m, l);
        tcol.push_back((int)t);
        used[(size_t)t] = 1;
      }
    std::vector<int> pad;
    for (int64_t t = 0; t < L.Tp; ++t)
      if (!used[(size_t)t]) pad.push_back((int)t);
    p->npad = (int)pad.size();
    e = hipMalloc(&p->d_tcol, std::max<size_t>(tcol.size(), 1) * sizeof(int));
    if (e == hipSuccess)
      e = hipMemcpy(p->d_tcol, tcol.data(), tcol.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_tpad, std::max<size_t>(pad.size(), 1) * sizeof(int));
    if (e == hipSuccess && !pad.empty())
      e = hipMemcpy(p->d_tpad, pad.data(), pad.size() * sizeof(int), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    set_error(std::string("plan allocation failed: ") + hipGetErrorString(e));
    msfno_sht_plan_destroy(p);
    return MSFNO_EHIP;
  }
  *plan = p;
  return MSFNO_OK;
}

// channel MLP of the block (layers.py:145-178) on x1 (B, C, P) with norm1/FiLM
// already folded into (W1f, b1f):  out = W2·GELU(W1f·x1 + b1f) + b2 (+ resid).
// GELU(erf) in fc1's epilogue on 128x64 tiles, bias + outer skip in fc2's
// (measured cheapest split: DESIGN.md §8).
int run_mlp(const msfno_block_desc* d, const float* W1f, const float* b1f, const float* x1,
            float* h, float* out, const float* resid, int B, int64_t P, const DenseWs& dw,
            hipStream_t s, const unsigned short* x1p) {
  const int64_t C = d->C, Hd = d->mlp_hidden;
  // x6 engine: h travels as bf16x3 planes [B][3][Hd][ldh] (fc1 splits it once in its
  // epilogue, fc2 stages it without conversion)
  const bool planes = mlp_h_planes(dw.fc1 != nullptr && dw.fc2 != nullptr);
  const int64_t ldh = planes ? round_up(P, 8) : P;
  unsigned short* hx = planes ? reinterpret_cast<unsigned short*>(h) : nullptr;
  prof(ST_FC1, s);
  const int64_t chunk = mlp_chunk(P);
  if (planes && x1p && chunk > 0 && chunk < P) {
    // pixel chunks: fc1 writes a chunk of h (planes) that fc2 reads back while it is
    // still in the Infinity Cache; both weight images are split once
    MSFNO_TRY(gemm_x6p_split_a(W1f, (int)Hd, (int)C, (int)C, Hd * C, B, dw.fc1, dw.fc1_b, s));
    MSFNO_TRY(gemm_x6p_split_a(d->fc2_w, (int)C, (int)Hd, (int)Hd, 0, 1, dw.fc2, dw.fc2_b, s));
    const int64_t ldc = round_up(chunk, 8);
    for (int64_t p0 = 0; p0 < P; p0 += chunk) {
      const int pc = (int)std::min<int64_t>(chunk, P - p0);
      GemmEpi e1;
      e1.bias = b1f;
      e1.sBias = Hd;
      e1.act = 1;
      e1.a_planes = static_cast<const unsigned short*>(dw.fc1);
      e1.b_planes = x1p + p0;
      e1.b_plane_stride = C * P;
      e1.c_planes = hx;
      e1.c_plane_stride = Hd * ldc;
      MSFNO_TRY(gemm_x6p(W1f, h, (int)Hd, pc, (int)C, (int)C, (int)P, (int)ldc, Hd * C, 3 * C * P,
                         3 * Hd * ldc, B, e1, dw.fc1, dw.fc1_b, s));
      GemmEpi e2;
      e2.bias = d->fc2_b;
      if (resid) { e2.addend = resid + p0; e2.sD = C * P; e2.ldd = (int)P; }
      e2.a_planes = static_cast<const unsigned short*>(dw.fc2);
      e2.b_planes = hx;
      e2.b_plane_stride = Hd * ldc;
      MSFNO_TRY(gemm_x6p(d->fc2_w, out + p0, (int)C, pc, (int)Hd, (int)Hd, (int)ldc, (int)P, 0,
                         3 * Hd * ldc, C * P, B, e2, dw.fc2, dw.fc2_b, s));
    }
    return MSFNO_OK;
  }
  GemmEpi e1;
  e1.bias = b1f;
  e1.sBias = Hd;
  e1.act = 1;
  if (planes) { e1.c_planes = hx; e1.c_plane_stride = Hd * ldh; }
  if (planes && x1p) {
    // x1 arrives as planes from the inverse FFT: LDS-DMA GEMM (per-field folded W1)
    e1.b_planes = x1p;
    e1.b_plane_stride = C * P;
    MSFNO_TRY(gemm_x6p(W1f, h, (int)Hd, (int)P, (int)C, (int)C, (int)P, (int)ldh, Hd * C,
                       3 * C * P, 3 * Hd * ldh, B, e1, dw.fc1, dw.fc1_b, s));
  } else
  MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, W1f, x1, h, (int)Hd, (int)P, (int)C, (int)C,
                       (int)P, (int)ldh, Hd * C, C * P, (planes ? 3 : 1) * Hd * ldh, B, e1,
                       dw.fc1, dw.fc1_b, s));
  prof(ST_FC2, s);
  GemmEpi e2;
  e2.bias = d->fc2_b;
  if (resid) { e2.addend = resid; e2.sD = C * P; e2.ldd = (int)P; }
  if (planes) {
    e2.b_planes = hx;
    e2.b_plane_stride = Hd * ldh;
    return gemm_x6p(d->fc2_w, out, (int)C, (int)P, (int)Hd, (int)Hd, (int)ldh, (int)P, 0,
                    3 * Hd * ldh, C * P, B, e2, dw.fc2, dw.fc2_b, s);
  }
  return gemm_dense(ROLE_FC2, TILE_256x128, d->fc2_w, h, out, (int)C, (int)P, (int)Hd, (int)Hd,
                    (int)ldh, (int)P, 0, (planes ? 3 : 1) * Hd * ldh, C * P, B, e2, dw.fc2,
                    dw.fc2_b, s);
}

// the inner-skip GEMM reads fp32 x and splits it in-kernel (gemm_x6), forked before
// the forward FFT; MSFNO_SKIP_PLANES=1: x as bf16x3 planes written by the forward FFT
// (into the x1 plane buffer), the GEMM forked after it.  With the fused MLP the fp32
// form measured 2.8 % faster per block (rfft 0.70 -> 0.51 ms without the 1.6 GB of
// plane stores)
static bool skip_planes_env() {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SKIP_PLANES");
    return e && e[0] == '1';
  }();
  return on;
}

// the inner skip on the x3h engine by default (MSFNO_ENGINE=x6 or MSFNO_SKIP_X3H=0 keep x6)
bool skip_x3(const msfno_block_desc* d) {
  static const bool on = [] {
    const char* e = getenv("MSFNO_SKIP_X3H");
    if (e) return e[0] == '1';
    return mlp_fused_h_env();
  }();
  return on && gemm_use_x6() && !skip_planes_env() && d->inner_skip == MSFNO_SKIP_LINEAR;
}

bool skip_planes(const msfno_block_desc* d, const msfno_sht_plan_s* f, const BlockBufs& b) {
  return skip_planes_env() && b.x1p && b.dw.skip && d->inner_skip == MSFNO_SKIP_LINEAR &&
         !use_fft_tile(f) && fft_r2c_planes_supported(f->fft, f->mmax);
}

// pixels per fc1 -> fc2 chunk of the block MLP (MSFNO_MLP_CHUNK, multiple of 256;
// 0 = one pass over the field)
int64_t mlp_chunk(int64_t P) {
  static const int64_t c = [] {
    const char* e = getenv("MSFNO_MLP_CHUNK");
    return e ? (int64_t)atoll(e) / 256 * 256 : (int64_t)0;
  }();
  (void)P;
  return c;
}

// x1 (the MLP input) written by the inverse FFT as bf16x3 planes: x6 engine, an
// MLP, and an LDS-DMA inverse FFT whose rows tile the plane rows (P % 8 == 0);
// MSFNO_X1_PLANES=0 keeps fp32 x1 for A/B
bool x1_planes(const msfno_block_desc* d, const msfno_sht_plan_s* g) {
  static const bool on = [] {
    const char* e = getenv("MSFNO_X1_PLANES");
    return !(e && e[0] == '0');
  }();
  return on && d->has_mlp && mlp_h_planes(true) && !mlp_fused(d, (int64_t)g->nlat * g->nlon) &&
         ((int64_t)g->nlat * g->nlon) % 8 == 0 && fft_c2r_planes_supported(g->fft, g->mmax);
}

bool mlp_fused(const msfno_block_desc* d, int64_t P) {
  return d->has_mlp && gemm_use_x6() && d->fc1_b != nullptr && P % 4 == 0 && P >= 4 &&
         mlp_fused_supported((int)d->C, (int)d->mlp_hidden);
}

bool x1p_buffer(const msfno_block_desc* d, const msfno_sht_plan_s* g) {
  return x1_planes(d, g) ||
         (skip_planes_env() && mlp_fused(d, (int64_t)g->nlat * g->nlon) &&
          d->inner_skip == MSFNO_SKIP_LINEAR && mlp_h_planes(true));
}

int run_block_mlp(const msfno_block_desc* d, const float* x1, const unsigned short* x1p,
                  const float* sc1, const float* sh1, const float* ab1, float* W1f, float* b1f, float* h,
                  unsigned short* mfimg, float* out, const float* resid, int B, int64_t P,
                  const DenseWs& dw, hipStream_t s) {
  MSFNO_REQUIRE(d->fc1_w && d->fc2_w, MSFNO_EINVAL, "missing MLP weights");
  if (mfimg) {
    prof(ST_MLP_FUSED, s);
    if (!(wcache_ready(d) && mfimg == wcache_mfimg(d)))
      MSFNO_TRY(launch_mlp_fused_images(d->fc1_w, d->fc1_b, d->fc2_w, mfimg, s));
    return launch_mlp_fused(x1, sc1, sh1, ab1, resid, out, mfimg, d->fc1_b, d->fc2_b, B, P, s);
  }
  const int64_t C = d->C, Hd = d->mlp_hidden;
  MSFNO_TRY(launch_fold_affine(d->fc1_w, d->fc1_b, sc1, sh1, W1f, b1f, B, (int)Hd, (int)C, s));
  return run_mlp(d, W1f, b1f, x1, h, out, resid, B, P, dw, s, x1p);
}

// MLP hidden activation in the bf16x3 plane format (x6 engine; MSFNO_H_PLANES=0
// keeps it fp32 for A/B)
bool mlp_h_planes(bool have_ws) {
  static const bool on = [] {
    const char* e = getenv("MSFNO_H_PLANES");
    return gemm_use_x6() && !(e && e[0] == '0');
  }();
  return on && have_ws;
}

// floats to reserve for the MLP hidden activation h (B, Hd, P) in either format
int64_t mlp_h_floats(int B, int64_t Hd, int64_t P) {
  if (!mlp_h_planes(true)) return (int64_t)B * Hd * P;
  return cdiv((int64_t)B * 3 * Hd * round_up(P, 8) * 2, 4);
}
}  // namespace msfno

using namespace msfno;

extern "C" {

const char* msfno_last_error(void) { return g_last_error.c_str(); }
int msfno_abi_version(void) { return 6; }

int msfno_quadrature(int nlat, int grid, double* nodes, double* weights) {
  std::vector<double> x, w;
  MSFNO_TRY(quadrature(nlat, grid, x, w));
  std::memcpy(nodes, x.data(), nlat * sizeof(double));
  std::memcpy(weights, w.data(), nlat * sizeof(double));
  return MSFNO_OK;
}

int msfno_legendre_table(int mmax, int lmax, int nlat, int grid, int inverse, int csphase,
                         double* table) {
  MSFNO_REQUIRE(mmax > 0 && lmax > 0 && nlat > 0 && table, MSFNO_EINVAL, "bad table arguments");
  return legendre_table(mmax, lmax, nlat, grid, inverse, csphase, table);
}

int msfno_sht_plan_create(int nlat, int nlon, int lmax, int mmax, int inverse,
                          msfno_sht_plan_t* plan) {
  MSFNO_REQUIRE(plan, MSFNO_EINVAL, "null plan pointer");
  return plan_create(nlat, nlon, lmax, mmax, inverse, nullptr, plan);
}

int msfno_sht_plan_destroy(msfno_sht_plan_t p) {
  if (!p) return MSFNO_OK;
  fft_plan_free(p->fft);
  if (p->table) (void)hipFree(p->table);
  if (p->d_tab_off) (void)hipFree(p->d_tab_off);
  if (p->d_Lp) (void)hipFree(p->d_Lp);
  if (p->d_off) (void)hipFree(p->d_off);
  if (p->d_tril_local) (void)hipFree(p->d_tril_local);
  if (p->d_tcol) (void)hipFree(p->d_tcol);
  if (p->d_tpad) (void)hipFree(p->d_tpad);
  if (p->d_Lpe) (void)hipFree(p->d_Lpe);
  for (auto* sets : {&p->desc_sets, &p->desc3_sets, &p->desc3f_sets})
    for (auto& kv : *sets) {
      if (kv.second.d) (void)hipFree(kv.second.d);
      if (kv.second.tile) (void)hipFree(kv.second.tile);
    }
  if (p->tab3) (void)hipFree(p->tab3);
  if (p->tab3s) (void)hipFree(p->tab3s);
  if (p->d_kmap) (void)hipFree(p->d_kmap);
  delete p;
  return MSFNO_OK;
}

int msfno_sht_plan_load_table(msfno_sht_plan_t p, const float* table, void* stream) {
  MSFNO_REQUIRE(p && table, MSFNO_EINVAL, "null plan or table");
  hipStream_t s = (hipStream_t)stream;
  // one-time setup: detect the equatorial symmetry of this table (host sync)
  int sym = 0;
  if (!getenv("MSFNO_NO_SYM") && p->nlat >= 2) {
    int* d_flag = nullptr;
    MSFNO_CHECK_HIP(hipMalloc(&d_flag, sizeof(int)));
    int h_flag = 0;
    hipError_t e = hipMemsetAsync(d_flag, 0, sizeof(int), s);
    int rc = MSFNO_OK;
    if (e == hipSuccess) rc = launch_check_symmetry(table, p->mmax, p->lmax, p->nlat, d_flag, s);
    if (e == hipSuccess && rc == MSFNO_OK)
      e = hipMemcpyAsync(&h_flag, d_flag, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d_flag);
    MSFNO_TRY(rc);
    MSFNO_CHECK_HIP(e);
    sym = h_flag == 0;
  }
  p->sym = sym;
  set_table_offsets(p, sym);
  if (p->table_elems > p->table_cap) {  // band plans: the exchange layout can be larger
    MSFNO_CHECK_HIP(hipFree(p->table));
    p->table = nullptr;
    p->table_cap = p->table_elems;
    MSFNO_CHECK_HIP(hipMalloc(&p->table, p->table_cap * sizeof(float)));
  }
  if (p->band_world) {
    const std::vector<int>& km = sym ? p->kmap_sym : p->kmap_gen;
    if (!p->d_kmap)
      MSFNO_CHECK_HIP(hipMalloc(&p->d_kmap, p->kmap_gen.size() * sizeof(int)));
    MSFNO_CHECK_HIP(hipMemcpy(p->d_kmap, km.data(), km.size() * sizeof(int),
                              hipMemcpyHostToDevice));
  }
  MSFNO_CHECK_HIP(hipMemcpy(p->d_tab_off, p->tab_off.data(), p->mmax * sizeof(int64_t),
                            hipMemcpyHostToDevice));
  // descriptors depend on the layout (symmetric or not): every cached set goes
  MSFNO_CHECK_HIP(hipStreamSynchronize(s));
  for (auto* sets : {&p->desc_sets, &p->desc3_sets, &p->desc3f_sets}) {
    for (auto& kv : *sets) {
      if (kv.second.d) MSFNO_CHECK_HIP(hipFree(kv.second.d));
      if (kv.second.tile) MSFNO_CHECK_HIP(hipFree(kv.second.tile));
    }
    sets->clear();
  }
  p->d_desc = p->d_desc3 = p->d_desc3f = nullptr;
  p->d_tile3 = p->d_tile3f = nullptr;
  p->desc_R = -1;
  MSFNO_TRY(launch_relayout_table(*p, table, s));
  p->desc3_R = -1;
  p->desc3f_R = -1;
  p->tab3_valid = 0;  // the x3h image is rebuilt from the new table on first use
  p->table_loaded = 1;
  return MSFNO_OK;
}

size_t msfno_sht_workspace_size(msfno_sht_plan_t p, int bc) {
  if (!p) return 0;
  Carve cv;
  const int64_t R = 2LL * bc;
  cv.take<float2>((int64_t)bc * p->nlat * p->mmax);   // Xn / Yn
  cv.take<float>((int64_t)p->mmax * R * p->ldk);       // Xt / Yt
  cv.take<float>(R * p->spec.ldT);                     // S
  return cv.off;
}

int msfno_sht_forward(msfno_sht_plan_t p, const float* x, float* out, int bc, void* ws,
                      size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(p && !p->inverse, MSFNO_EINVAL, "msfno_sht_forward needs a forward plan");
  MSFNO_REQUIRE(p->table_loaded, MSFNO_EINVAL, "plan table not loaded");
  MSFNO_REQUIRE(ws_bytes >= msfno_sht_workspace_size(p, bc), MSFNO_EWORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  const int64_t R = 2LL * bc;
  float2* Xn = cv.take<float2>((int64_t)bc * p->nlat * p->mmax);
  float* Xt = cv.take<float>((int64_t)p->mmax * R * p->ldk);
  float* S = cv.take<float>(R * p->spec.ldT);
  const float scale = (float)(2.0 * M_PI / p->nlon);
  if (use_fft_tile(p)) {
    MSFNO_TRY(launch_fft_r2c_tile(p->fft, x, Xt, nullptr, 1, bc, p->nlat, p->mmax, p->ldk, scale, s));
  } else {
    MSFNO_TRY(launch_fft_r2c_rows(p->fft, x, Xn, nullptr, (int64_t)bc * p->nlat, p->mmax, scale, s));
    MSFNO_TRY(transpose_fwd_plan(p, Xn, Xt, 1, bc, nullptr, nullptr, s));
  }
  MSFNO_TRY(legendre_fwd(p, Xt, S, (int)R, s));
  MSFNO_TRY(launch_spec_to_ref(*p, S, reinterpret_cast<float2*>(out), 1, bc, p->d_off, s));
  return MSFNO_OK;
}

int msfno_sht_inverse(msfno_sht_plan_t p, const float* in, float* x, int bc, void* ws,
                      size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(p && p->inverse, MSFNO_EINVAL, "msfno_sht_inverse needs an inverse plan");
  MSFNO_REQUIRE(p->table_loaded, MSFNO_EINVAL, "plan table not loaded");
  MSFNO_REQUIRE(ws_bytes >= msfno_sht_workspace_size(p, bc), MSFNO_EWORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  const int64_t R = 2LL * bc;
  float2* Yn = cv.take<float2>((int64_t)bc * p->nlat * p->mmax);
  float* Yt = cv.take<float>((int64_t)p->mmax * R * p->ldk);
  float* S = cv.take<float>(R * p->spec.ldT);
  MSFNO_TRY(launch_ref_to_spec(*p, reinterpret_cast<const float2*>(in), S, 1, bc, p->d_off, s));
  MSFNO_TRY(legendre_inv(p, S, Yt, (int)R, s));
  if (use_fft_tile(p)) {
    MSFNO_TRY(launch_fft_c2r_tile(p->fft, Yt, x, nullptr, 1, bc, p->nlat, p->mmax, p->spec.mact,
                                  p->ldk, 0, s));
  } else {
    MSFNO_TRY(transpose_inv_plan(p, Yt, Yn, 1, bc, s));
    MSFNO_TRY(launch_fft_c2r_rows(p->fft, Yn, x, nullptr, nullptr, (int64_t)bc * p->nlat, p->mmax, 0, s));
  }
  return MSFNO_OK;
}

int msfno_compl_contract_fwd_c(const float* a, const float* w, float* y, int B, int Ci, int Co,
                               int T, void* stream) {
  MSFNO_REQUIRE(a && w && y && B > 0 && Ci > 0 && Co > 0 && T > 0, MSFNO_EINVAL,
                "bad compl_contract_fwd_c arguments");
  return launch_compl_contract(a, w, y, B, Ci, Co, T, (hipStream_t)stream);
}

int msfno_compl_mul2d_fwd_c(const float* a, const float* w, float* y, int B, int Ci, int Co,
                            long long XY, int relu_real, void* stream) {
  MSFNO_REQUIRE(a && w && y && B > 0 && Ci > 0 && Co > 0 && XY > 0, MSFNO_EINVAL,
                "bad compl_mul2d_fwd_c arguments");
  return launch_compl_mul2d(a, w, y, B, Ci, Co, XY, relu_real, (hipStream_t)stream);
}

// 1x1 convolution (the block's inner skip as a standalone op): x3h engine, B rows scaled
// per (b, channel) by the power of two below its max |x| (no norm statistics here)
size_t msfno_conv1x1_workspace_size(int B, int Cin, int Cout) {
  if (B <= 0 || Cin <= 0 || Cout <= 0) return 0;
  const size_t xs = round_up((int64_t)B * Cin * 4, 256);
  return xs + (Cin == 256 && Cout == 256 ? skip_h_workspace(B) : gemm_x3_workspace(Cout, Cin, B));
}

int msfno_conv1x1(const float* w, const float* bias, const float* x, float* out, int B, int Cin,
                  int Cout, long long P, void* ws, size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(w && x && out && ws && B > 0 && Cin > 0 && Cout > 0 && P > 0 && P < (1LL << 31),
                MSFNO_EINVAL, "bad conv1x1 arguments");
  MSFNO_REQUIRE(ws_bytes >= msfno_conv1x1_workspace_size(B, Cin, Cout), MSFNO_EWORKSPACE,
                "conv1x1: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  float* xs = static_cast<float*>(ws);
  const size_t xs_bytes = round_up((int64_t)B * Cin * 4, 256);
  void* rest = static_cast<char*>(ws) + xs_bytes;
  MSFNO_TRY(launch_chan_pow2_scale(x, (int64_t)B * Cin, P, xs, s));
  if (Cin == 256 && Cout == 256 && skip_h_env())
    return launch_skip_h(w, xs, x, out, bias, B, P, rest, ws_bytes - xs_bytes, s);
  GemmEpi e;
  e.bias = bias;
  return gemm_x3(w, Cin, xs, x, out, Cout, (int)P, Cin, (int)P, (int)P, (int64_t)Cin * P,
                 (int64_t)Cout * P, B, e, rest, ws_bytes - xs_bytes, s);
}

size_t msfno_block_wcache_size(const msfno_block_desc* d) {
  if (!d) return 0;
  msfno_block_desc t = *d;
  t.wcache = nullptr;
  return wcache_layout(&t, nullptr);
}

size_t msfno_block_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t f,
                                  msfno_sht_plan_t g, int B) {
  if (!d || !f || !g) return 0;
  Carve cv;
  BlockBufs b;
  carve_block(cv, b, d, f, g, B, true);
  return cv.off;
}

int msfno_filter_forward(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                         const float* x, float* y, int B, void* ws, size_t ws_bytes,
                         void* stream) {
  MSFNO_TRY(check_pair(d, f, g));
  MSFNO_REQUIRE(ws_bytes >= msfno_block_workspace_size(d, f, g, B), MSFNO_EWORKSPACE,
                "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  BlockBufs b;
  carve_block(cv, b, d, f, g, B, false);
  MSFNO_TRY(run_spectral(d, f, g, b, x, B, false, s));
  MSFNO_TRY(run_inverse_fft(g, b, B, d->C, y, nullptr, nullptr, 0, s));
  prof(ST_END, s);
  return MSFNO_OK;
}

}  // extern "C"

// x1_ext / aff_out (both or neither; blocks without MLP and outer skip): the block stops
// before its output affine, leaving x1 in x1_ext and the per-(b,c) norm1 (+ FiLM) affine
// in aff_out = [scale (B*C)][shift (B*C)] for the consumer to apply (the decoder MLP)
// skip_x (or null = x): the inner skip's input (global_conv's `residual`); norm_only: stop
// after norm1 (no FiLM, MLP or outer skip: FourierNeuralOperatorBlock_Filmed.global_conv)
static int block_forward_impl(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                              const float* x, const float* gamma, const float* beta,
                              float film_scale, float* out, float* x1_ext, float* aff_out, int B,
                              void* ws, size_t ws_bytes, void* stream,
                              const float* skip_x = nullptr, bool norm_only = false) {
  MSFNO_TRY(check_pair(d, f, g));
  MSFNO_REQUIRE(ws_bytes >= msfno_block_workspace_size(d, f, g, B), MSFNO_EWORKSPACE,
                "workspace too small");
  MSFNO_REQUIRE((gamma == nullptr) == (beta == nullptr), MSFNO_EINVAL,
                "gamma and beta must both be given or both be NULL");
  MSFNO_REQUIRE(d->outer_skip != MSFNO_SKIP_LINEAR, MSFNO_EUNSUPPORTED,
                "outer_skip='linear' is not supported by the fused block");
  const bool resample = (f->nlat != g->nlat) || (f->nlon != g->nlon);
  MSFNO_REQUIRE(!resample || (d->inner_skip == MSFNO_SKIP_NONE && d->outer_skip == MSFNO_SKIP_NONE),
                MSFNO_EINVAL, "skips require equal input and output grids");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  BlockBufs b;
  carve_block(cv, b, d, f, g, B, true);
  const int64_t C = d->C, BC = (int64_t)B * C;
  const int64_t P = (int64_t)g->nlat * g->nlon;
  const int act = d->filter_type == MSFNO_FILTER_LINEAR ? 1 : 0;  // GELU after skip (linear only)

  // ---- inner skip 1x1 conv (depends only on x): x1 = Ws·x + bs, on the side stream ----
  // With x6 planes the forward FFT also writes x as bf16x3 planes into the x1 plane
  // buffer (dead until the inverse FFT, which runs after the skip GEMM): the skip
  // GEMM is forked after the forward FFT and stages B by LDS-DMA (gemm_x6p) instead
  // of splitting fp32 x in-kernel.
  float* x1 = x1_ext ? x1_ext : b.x1;
  const float* sx = skip_x ? skip_x : x;
  std::shared_ptr<SideCtx> side;
  const bool xpl = skip_planes(d, f, b) && sx == x;  // the FFT writes planes of x
  const C2RPlanes xp{b.x1p, (int)C, f->nlat};
  auto launch_skip = [&]() -> int {
    hipStream_t ss = s;
    if (side) {  // fork
      MSFNO_CHECK_HIP(hipEventRecord(side->fork, s));
      MSFNO_CHECK_HIP(hipStreamWaitEvent(side->side, side->fork, 0));
      ss = side->side;
    }
    prof(ST_SKIP, ss);
    GemmEpi e;
    e.bias = d->skip_b;
    // a separate skip input has no norm0 statistics: its x3h B-row scales from its max
    if (b.xs && sx != x) MSFNO_TRY(launch_chan_pow2_scale(sx, (int64_t)B * C, P, b.xs, ss));
    if (b.xs && C == 256 && skip_h_env()) {
      // the quarter-CU side grid only where the skip is forked at the block start and
      // overlaps the whole SHT + spectral chain (non-linear filter); the other filters fork
      // it after the contraction (skip_late below), where it is on the critical path (1.80 vs 0.79 ms,
      // linear 85.9 vs 97.5 fields/s, profiles/r06_j)
      MSFNO_TRY(launch_skip_h(d->skip_w, b.xs, sx, x1, d->skip_b, B, P, b.dw.skip, b.dw.skip_b,
                              ss, side != nullptr && d->filter_type == MSFNO_FILTER_NONLINEAR));
    } else if (b.xs) {
      MSFNO_TRY(gemm_x3(d->skip_w, (int)C, b.xs, sx, x1, (int)C, (int)P, (int)C, (int)P, (int)P,
                        C * P, C * P, B, e, b.dw.skip, b.dw.skip_b, ss));
    } else if (xpl) {
      e.b_planes = b.x1p;
      e.b_plane_stride = C * P;
      MSFNO_TRY(gemm_x6p(d->skip_w, x1, (int)C, (int)P, (int)C, (int)C, (int)P, (int)P, 0,
                         3 * C * P, C * P, B, e, b.dw.skip, b.dw.skip_b, ss));
    } else {
      // sx: global_conv's skip input is the residual, not the filter input x
      MSFNO_TRY(gemm_dense(ROLE_SKIP, TILE_128x256, d->skip_w, sx, x1, (int)C, (int)P, (int)C,
                           (int)C, (int)P, (int)P, 0, C * P, C * P, B, e, b.dw.skip, b.dw.skip_b,
                           ss));
    }
    if (side) {
      prof(ST_END, ss);
      MSFNO_CHECK_HIP(hipEventRecord(side->join, ss));
    }
    return MSFNO_OK;
  };
  if (d->inner_skip == MSFNO_SKIP_LINEAR) {
    MSFNO_REQUIRE(d->skip_w, MSFNO_EINVAL, "missing inner_skip weight");
    MSFNO_TRY(side_ctx(&side, s));
    if (!xpl && !b.xs) MSFNO_TRY(launch_skip());
  }
  // The skip is forked after the norm0 statistics (x3h: its per-channel scales come from
  // them).  It slows whatever it overlaps by about its own length: forked after the forward
  // Legendre instead (overlapping only the MFMA-bound spectral layers) measured equal
  // (160.8 / 159.9 vs 160.7 / 159.9 fields/s, round 5).  The linear filter forks it after
  // the per-mode contraction, so its 2.1 GB do not share HBM with the 34 GB weight stream:
  // 94.0 / 94.2 vs 92.2 / 92.3 fields/s (profiles/r05_b)
  const bool skip_late = d->filter_type != MSFNO_FILTER_NONLINEAR;
  if (b.xs && skip_late)
    MSFNO_TRY(run_spectral(d, f, g, b, x, B, true, s, nullptr, std::function<int()>(),
                           std::function<int()>(), std::function<int()>(), launch_skip));
  else if (b.xs)
    MSFNO_TRY(run_spectral(d, f, g, b, x, B, true, s, nullptr, std::function<int()>(), launch_skip));
  else if (xpl)
    MSFNO_TRY(run_spectral(d, f, g, b, x, B, true, s, &xp, launch_skip));
  else
    MSFNO_TRY(run_spectral(d, f, g, b, x, B, true, s));
  if (side) MSFNO_CHECK_HIP(hipStreamWaitEvent(s, side->join, 0));  // join
  // ---- filter output + skip (+ GELU for the linear filter) -> x1, norm1 partials ---
  const float* skip_src = d->inner_skip == MSFNO_SKIP_LINEAR ? x1
                          : (d->inner_skip == MSFNO_SKIP_IDENTITY ? sx : nullptr);
  // irfft writes x1 as planes (the unfused MLP's fc1 operand; global_conv reads fp32 x1)
  unsigned short* x1p = !norm_only && x1_planes(d, g) ? b.x1p : nullptr;
  MSFNO_TRY(run_inverse_fft(g, b, B, (int)C, x1, skip_src, b.st1, act, s, x1p));
  const int64_t np = g->nlat, cnt = g->nlon, cnt_last = g->nlon;
  // ---- norm1 (+ FiLM) as a per-(b,c) affine --------------------------------------
  prof(ST_NORM1, s);
  MSFNO_TRY(launch_chan_affine(b.st1, np, cnt, cnt_last, B, (int)C, d->norm1_w, d->norm1_b,
                               d->norm_eps, gamma, beta, film_scale, b.sc1, b.sh1, s, nullptr,
                               nullptr, b.ab1));
  const float* resid = d->outer_skip == MSFNO_SKIP_IDENTITY ? x : nullptr;
  if (norm_only) {
    prof(ST_OUT_AFFINE, s);
    MSFNO_TRY(launch_affine_rows(x1, b.sc1, b.sh1, nullptr, out, BC, P, 0, nullptr, 0, s));
  } else if (aff_out) {
    MSFNO_CHECK_HIP(hipMemcpyAsync(aff_out, b.sc1, BC * sizeof(float), hipMemcpyDeviceToDevice, s));
    MSFNO_CHECK_HIP(
        hipMemcpyAsync(aff_out + BC, b.sh1, BC * sizeof(float), hipMemcpyDeviceToDevice, s));
  } else if (d->has_mlp) {
    MSFNO_TRY(run_block_mlp(d, x1, x1p, b.sc1, b.sh1, b.ab1, b.W1f, b.b1f, b.h, b.mfimg, out, resid, B,
                            P, b.dw, s));
  } else {
    prof(ST_OUT_AFFINE, s);
    MSFNO_TRY(launch_affine_rows(x1, b.sc1, b.sh1, resid, out, BC, P, 0, nullptr, 0, s));
  }
  prof(ST_END, s);
  return MSFNO_OK;
}

extern "C" {

int msfno_block_forward(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                        const float* x, const float* gamma, const float* beta, float film_scale,
                        float* out, int B, void* ws, size_t ws_bytes, void* stream) {
  return block_forward_impl(d, f, g, x, gamma, beta, film_scale, out, nullptr, nullptr, B, ws,
                            ws_bytes, stream);
}

int msfno_block_global_conv(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                            const float* x, const float* residual, float* out, int B, void* ws,
                            size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(x && out, MSFNO_EINVAL, "global_conv: missing tensors");
  return block_forward_impl(d, f, g, x, nullptr, nullptr, 0.f, out, nullptr, nullptr, B, ws,
                            ws_bytes, stream, residual, true);
}

int msfno_block_forward_deferred(const msfno_block_desc* d, msfno_sht_plan_t f,
                                 msfno_sht_plan_t g, const float* x, const float* gamma,
                                 const float* beta, float film_scale, float* x1_out,
                                 float* affine_out, int B, void* ws, size_t ws_bytes,
                                 void* stream) {
  MSFNO_REQUIRE(d && x1_out && affine_out, MSFNO_EINVAL, "block_forward_deferred: null output");
  MSFNO_REQUIRE(!d->has_mlp && d->outer_skip == MSFNO_SKIP_NONE, MSFNO_EUNSUPPORTED,
                "block_forward_deferred: blocks without MLP and outer skip only");
  return block_forward_impl(d, f, g, x, gamma, beta, film_scale, nullptr, x1_out, affine_out, B,
                            ws, ws_bytes, stream);
}

int msfno_profile_mark(int stage, void* stream) {
  MSFNO_REQUIRE(stage >= 0 && stage <= ST_END, MSFNO_EINVAL, "profile stage out of range");
  prof(stage, (hipStream_t)stream);
  return MSFNO_OK;
}

int msfno_profile_enable(int on) {
  g_prof.on = on != 0;
  return MSFNO_OK;
}

const char* msfno_profile_stage_name(int stage) {
  if (stage < 0 || stage >= MSFNO_PROF_NSTAGES || !kStageNames[stage]) return "";
  return kStageNames[stage];
}

int msfno_profile_collect(double* total_ms, int* counts) {
  auto& mk = g_prof.marks;
  for (auto& m : mk) MSFNO_CHECK_HIP(hipEventSynchronize(m.ev));
  for (size_t i = 0; i < mk.size(); ++i) {
    if (mk[i].stage == ST_END) continue;
    size_t j = i + 1;
    while (j < mk.size() && mk[j].stream != mk[i].stream) ++j;
    if (j == mk.size()) continue;
    float ms = 0.f;
    MSFNO_CHECK_HIP(hipEventElapsedTime(&ms, mk[i].ev, mk[j].ev));
    if (total_ms) total_ms[mk[i].stage] += ms;
    if (counts) counts[mk[i].stage] += 1;
  }
  for (auto& m : mk) g_prof.pool.push_back(m.ev);
  mk.clear();
  return MSFNO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// channel MLP (encoder / decoder of the network)
// ---------------------------------------------------------------------------
extern "C" {

size_t msfno_mlp_workspace_size(const msfno_mlp_desc* d, int B, long long P) {
  if (!d || B <= 0 || P <= 0) return 0;
  if (mlp_gen_h_supported(d->Cin + d->Cin2, d->Hid, d->Cout))
    return mlp_gen_h_workspace(d->Cin + d->Cin2, d->Hid, d->Cout);
  Carve cv;
  cv.take<float>(std::max<int64_t>((int64_t)B * d->Hid * P, mlp_h_floats(B, d->Hid, P)));  // h
  // first half of fc1 (two-GEMM concatenation on the fp32 engine only)
  if (d->Cin2 > 0 && !gemm_use_x6()) cv.take<float>((int64_t)B * d->Hid * P);
  cv.take<char>(gemm_dense_workspace(d->Hid, d->Cin + d->Cin2, 1));  // split fc1 weights
  if (d->Cin2 > 0) cv.take<char>(gemm_dense_workspace(d->Hid, d->Cin2, 1));
  cv.take<char>(gemm_dense_workspace(d->Cout, d->Hid, 1));  // split fc2 weights
  return cv.off;
}

int msfno_mlp_fused_supported(const msfno_mlp_desc* d) {
  return d && mlp_gen_h_supported(d->Cin + d->Cin2, d->Hid, d->Cout) ? 1 : 0;
}

size_t msfno_mlp_wcache_size(const msfno_mlp_desc* d) {
  return msfno_mlp_fused_supported(d) ? mlp_gen_h_workspace(d->Cin + d->Cin2, d->Hid, d->Cout) : 0;
}

int msfno_mlp_forward_affine(const msfno_mlp_desc* d, const float* x, const float* x_scale,
                             const float* x_shift, const float* x2, const float* addend,
                             long long add_bstride, float* out, int B, long long P, void* ws,
                             size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(d && x && x_scale && x_shift && out && d->fc1_w && d->fc1_b && d->fc2_w,
                MSFNO_EINVAL, "mlp_forward_affine: missing tensors");
  MSFNO_REQUIRE(msfno_mlp_fused_supported(d), MSFNO_EUNSUPPORTED,
                "mlp_forward_affine: widths without the fused x3h kernel");
  MSFNO_REQUIRE((d->Cin2 > 0) == (x2 != nullptr) && B > 0 && P > 0 &&
                    ws_bytes >= msfno_mlp_workspace_size(d, B, P),
                MSFNO_EINVAL, "mlp_forward_affine: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  prof(ST_MLP_GEN, s);
  MSFNO_TRY(launch_mlp_gen_h(x, x_scale, x_shift, x2, d->Cin, d->Cin2, d->fc1_w, d->fc1_b, d->fc2_w,
                             d->fc2_b, d->Hid, d->Cout, addend, add_bstride, out, B, P, ws,
                             ws_bytes, s, d->wcache, d->wcache_valid));
  prof(ST_END, s);
  return MSFNO_OK;
}

int msfno_mlp_forward(const msfno_mlp_desc* d, const float* x, const float* x2,
                      const float* addend, long long add_bstride, float* out, int B,
                      long long P, void* ws, size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(d && x && out && d->fc1_w && d->fc2_w && d->fc1_b, MSFNO_EINVAL,
                "mlp: missing tensors");
  MSFNO_REQUIRE(d->Cin > 0 && d->Hid > 0 && d->Cout > 0 && d->Cin2 >= 0 && B > 0 && P > 0,
                MSFNO_EINVAL, "mlp: bad sizes");
  MSFNO_REQUIRE((d->Cin2 > 0) == (x2 != nullptr), MSFNO_EINVAL,
                "mlp: x2 must be given exactly when Cin2 > 0");
  MSFNO_REQUIRE(P <= 0x7fffffff, MSFNO_EINVAL, "mlp: too many pixels");
  MSFNO_REQUIRE(ws_bytes >= msfno_mlp_workspace_size(d, B, P), MSFNO_EWORKSPACE,
                "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  if (mlp_gen_h_supported(d->Cin + d->Cin2, d->Hid, d->Cout)) {
    // one fused x3h launch, the hidden activation on-chip (mlp_gen_h.hip)
    prof(ST_MLP_GEN, s);
    MSFNO_TRY(launch_mlp_gen_h(x, nullptr, nullptr, x2, d->Cin, d->Cin2, d->fc1_w, d->fc1_b, d->fc2_w, d->fc2_b,
                               d->Hid, d->Cout, addend, add_bstride, out, B, P, ws, ws_bytes, s,
                               d->wcache, d->wcache_valid));
    prof(ST_END, s);
    return MSFNO_OK;
  }
  Carve cv;
  cv.base = (char*)ws;
  const int64_t Hd = d->Hid, Ct = d->Cin + d->Cin2;
  float* h = cv.take<float>(std::max<int64_t>((int64_t)B * Hd * P, mlp_h_floats(B, Hd, P)));
  float* t = (d->Cin2 > 0 && !gemm_use_x6()) ? cv.take<float>((int64_t)B * Hd * P) : nullptr;
  const size_t w1b = gemm_dense_workspace((int)Hd, (int)Ct, 1);
  void* w1 = cv.take<char>(w1b);
  const size_t w1b2 = d->Cin2 > 0 ? gemm_dense_workspace((int)Hd, d->Cin2, 1) : 0;
  void* w12 = d->Cin2 > 0 ? cv.take<char>(w1b2) : nullptr;
  const size_t w2b = gemm_dense_workspace(d->Cout, (int)Hd, 1);
  void* w2 = cv.take<char>(w2b);
  const int Pi = (int)P;
  // x6 engine: h travels as bf16x3 planes [B][3][Hd][ldh] (fc1's epilogue splits it
  // once); fc2 stages it by LDS-DMA (gemm_x6p) or, for Cout <= 128 (the decoder's
  // 256 -> 73), on the 128-row x6 tile with plane B
  const bool planes = mlp_h_planes(w1 != nullptr && w2 != nullptr);
  const int64_t ldh = planes ? round_up(P, 8) : P;
  unsigned short* hx = planes ? reinterpret_cast<unsigned short*>(h) : nullptr;
  prof(ST_FC1, s);
  if (d->Cin2 > 0 && gemm_use_x6()) {
    // fc1 over the concatenation [x ; x2] as one GEMM, K = Cin + Cin2: the B rows past
    // Cin are read from x2 in place (GemmEpi::b2)
    GemmEpi e1;
    e1.bias = d->fc1_b;
    e1.act = 1;
    e1.b2 = x2; e1.b2_k = d->Cin; e1.b2_ld = Pi; e1.b2_stride = (int64_t)d->Cin2 * P;
    if (planes) { e1.c_planes = hx; e1.c_plane_stride = Hd * ldh; }
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w, x, h, (int)Hd, Pi, (int)Ct, (int)Ct, Pi,
                         (int)ldh, 0, (int64_t)d->Cin * P, (planes ? 3 : 1) * Hd * ldh, B, e1, w1,
                         w1b, s));
  } else if (d->Cin2 > 0) {
    // fc1 over the concatenation [x ; x2]: t = W1[:, :Cin]·x, then h = GELU(W1[:, Cin:]·x2 + b1 + t)
    GemmEpi e0;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w, x, t, (int)Hd, Pi, d->Cin, (int)Ct, Pi,
                         Pi, 0, (int64_t)d->Cin * P, Hd * P, B, e0, w1, w1b, s));
    GemmEpi e1;
    e1.bias = d->fc1_b;
    e1.addend = t; e1.sD = Hd * P; e1.ldd = Pi;
    e1.act = 1;
    if (planes) { e1.c_planes = hx; e1.c_plane_stride = Hd * ldh; }
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w + d->Cin, x2, h, (int)Hd, Pi, d->Cin2,
                         (int)Ct, Pi, (int)ldh, 0, (int64_t)d->Cin2 * P,
                         (planes ? 3 : 1) * Hd * ldh, B, e1, w12, w1b2, s));
  } else {
    GemmEpi e1;
    e1.bias = d->fc1_b;
    e1.act = 1;
    if (planes) { e1.c_planes = hx; e1.c_plane_stride = Hd * ldh; }
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w, x, h, (int)Hd, Pi, d->Cin, d->Cin, Pi,
                         (int)ldh, 0, (int64_t)d->Cin * P, (planes ? 3 : 1) * Hd * ldh, B, e1, w1,
                         w1b, s));
  }
  prof(ST_FC2, s);
  GemmEpi e2;
  e2.bias = d->fc2_b;
  if (addend) { e2.addend = addend; e2.sD = add_bstride; e2.ldd = Pi; }
  if (planes) {
    e2.b_planes = hx;
    e2.b_plane_stride = Hd * ldh;
    if (d->Cout > 128) {
      MSFNO_TRY(gemm_x6p(d->fc2_w, out, d->Cout, Pi, (int)Hd, (int)Hd, (int)ldh, Pi, 0,
                         3 * Hd * ldh, (int64_t)d->Cout * P, B, e2, w2, w2b, s));
      prof(ST_END, s);
      return MSFNO_OK;
    }
  }
  const GemmTile t2 = d->Cout <= 128 ? TILE_128x128 : TILE_256x128;
  MSFNO_TRY(gemm_dense(ROLE_FC2, t2, d->fc2_w, h, out, d->Cout, Pi, (int)Hd, (int)Hd, (int)ldh, Pi,
                       0, (planes ? 3 : 1) * Hd * ldh, (int64_t)d->Cout * P, B, e2, w2, w2b, s));
  prof(ST_END, s);
  return MSFNO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FiLM backward: gradients of a loss with respect to the
// FiLM modulation (gamma, beta) of a filmed block and through the decoder, with
// every SFNO weight frozen, as MSFNO fine-tunes its FiLM generator
// (MSFNO/Models/sfno/sfnonet.py:787-860: blocks before the filmed ones run under
// no_grad; the filmed block and the decoder run with autograd).
// ---------------------------------------------------------------------------
namespace msfno {

struct FilmBwdBufs {
  BlockBufs b;
  float *an, *tn, *du, *pre, *dh, *W2T, *W1T;
  void *wsa, *wsb;
  size_t wsa_b, wsb_b;
};

static void carve_film_bwd(Carve& cv, FilmBwdBufs& r, const msfno_block_desc* d,
                           const msfno_sht_plan_s* f, const msfno_sht_plan_s* g, int B) {
  carve_block(cv, r.b, d, f, g, B, true);
  const int64_t C = d->C, BC = (int64_t)B * C, P = (int64_t)g->nlat * g->nlon;
  r.an = cv.take<float>(BC);
  r.tn = cv.take<float>(BC);
  r.du = r.pre = r.dh = r.W2T = r.W1T = nullptr;
  r.wsa = r.wsb = nullptr;
  r.wsa_b = r.wsb_b = 0;
  if (!d->has_mlp) return;
  const int64_t Hd = d->mlp_hidden;
  r.du = cv.take<float>(BC * P);
  r.pre = cv.take<float>((int64_t)B * Hd * P);
  r.dh = cv.take<float>((int64_t)B * Hd * P);
  r.W2T = cv.take<float>(Hd * C);
  r.W1T = cv.take<float>(C * Hd);
  if ((r.wsa_b = gemm_dense_workspace((int)Hd, (int)C, 1))) r.wsa = cv.take<char>(r.wsa_b);
  if ((r.wsb_b = gemm_dense_workspace((int)C, (int)Hd, 1))) r.wsb = cv.take<char>(r.wsb_b);
}

}  // namespace msfno

extern "C" {

size_t msfno_block_film_backward_workspace_size(const msfno_block_desc* d, msfno_sht_plan_t f,
                                                msfno_sht_plan_t g, int B) {
  if (check_pair(d, f, g) != MSFNO_OK || B <= 0) return 0;
  Carve cv;
  FilmBwdBufs r;
  carve_film_bwd(cv, r, d, f, g, B);
  return cv.off;
}

int msfno_block_film_backward(const msfno_block_desc* d, msfno_sht_plan_t f, msfno_sht_plan_t g,
                              const float* x, const float* gamma, const float* beta,
                              float film_scale, const float* dout, float* dgamma, float* dbeta,
                              int B, void* ws, size_t ws_bytes, void* stream) {
  MSFNO_TRY(check_pair(d, f, g));
  MSFNO_REQUIRE(x && gamma && beta && dout && dgamma && dbeta && B > 0, MSFNO_EINVAL,
                "film backward: missing tensors");
  MSFNO_REQUIRE(ws_bytes >= msfno_block_film_backward_workspace_size(d, f, g, B),
                MSFNO_EWORKSPACE, "workspace too small");
  MSFNO_REQUIRE(d->outer_skip != MSFNO_SKIP_LINEAR, MSFNO_EUNSUPPORTED,
                "outer_skip='linear' is not supported by the fused block");
  MSFNO_REQUIRE(f->nlat == g->nlat && f->nlon == g->nlon || d->inner_skip == MSFNO_SKIP_NONE,
                MSFNO_EINVAL, "skips require equal input and output grids");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  FilmBwdBufs r;
  carve_film_bwd(cv, r, d, f, g, B);
  BlockBufs& b = r.b;
  const int64_t C = d->C, BC = (int64_t)B * C;
  const int64_t P = (int64_t)g->nlat * g->nlon;
  const int act = d->filter_type == MSFNO_FILTER_LINEAR ? 1 : 0;
  // ---- recompute x1 (fp32) and its InstanceNorm-1 statistics (the forward's
  // checkpoint, as the reference's checkpoint(blk, ...) does) ----------------------
  float* x1 = b.x1;
  if (d->inner_skip == MSFNO_SKIP_LINEAR) {
    MSFNO_REQUIRE(d->skip_w, MSFNO_EINVAL, "missing inner_skip weight");
    GemmEpi e;
    e.bias = d->skip_b;
    MSFNO_TRY(gemm_dense(ROLE_SKIP, TILE_128x256, d->skip_w, x, x1, (int)C, (int)P, (int)C,
                         (int)C, (int)P, (int)P, 0, C * P, C * P, B, e, b.dw.skip, b.dw.skip_b, s));
  }
  MSFNO_TRY(run_spectral(d, f, g, b, x, B, true, s));
  const float* skip_src = d->inner_skip == MSFNO_SKIP_LINEAR ? x1
                          : (d->inner_skip == MSFNO_SKIP_IDENTITY ? x : nullptr);
  MSFNO_TRY(run_inverse_fft(g, b, B, (int)C, x1, skip_src, b.st1, act, s, nullptr));
  const int64_t np = g->nlat, cnt = g->nlon;
  // norm1 alone: xhat = an * x1 + tn; norm1 + FiLM: u = sc1 * x1 + sh1
  MSFNO_TRY(launch_chan_affine(b.st1, np, cnt, cnt, B, (int)C, d->norm1_w, d->norm1_b,
                               d->norm_eps, nullptr, nullptr, 0.f, r.an, r.tn, s));
  const float* du = dout;
  if (d->has_mlp) {
    // out = W2 GELU(W1 u + b1) + b2 (+ x):  du = W1^T (GELU'(pre) * W2^T dout)
    MSFNO_REQUIRE(d->fc1_w && d->fc2_w, MSFNO_EINVAL, "missing MLP weights");
    MSFNO_TRY(launch_chan_affine(b.st1, np, cnt, cnt, B, (int)C, d->norm1_w, d->norm1_b,
                                 d->norm_eps, gamma, beta, film_scale, b.sc1, b.sh1, s));
    const int64_t Hd = d->mlp_hidden;
    const int Pi = (int)P;
    MSFNO_TRY(launch_fold_affine(d->fc1_w, d->fc1_b, b.sc1, b.sh1, b.W1f, b.b1f, B, (int)Hd,
                                 (int)C, s));
    GemmEpi e1;  // pre-activation of fc1 (no GELU)
    e1.bias = b.b1f;
    e1.sBias = Hd;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, b.W1f, x1, r.pre, (int)Hd, Pi, (int)C, (int)C,
                         Pi, Pi, Hd * C, C * P, Hd * P, B, e1, b.dw.fc1, b.dw.fc1_b, s));
    MSFNO_TRY(launch_transpose_mat(d->fc2_w, (int)C, (int)Hd, (int)Hd, r.W2T, s));
    GemmEpi e0;
    MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, r.W2T, dout, r.dh, (int)Hd, Pi, (int)C, (int)C,
                         Pi, Pi, 0, C * P, Hd * P, B, e0, r.wsa, r.wsa_b, s));
    MSFNO_TRY(launch_gelu_grad_mul(r.dh, r.pre, (int64_t)B * Hd * P, s));
    MSFNO_TRY(launch_transpose_mat(d->fc1_w, (int)Hd, (int)C, (int)C, r.W1T, s));
    MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, r.W1T, r.dh, r.du, (int)C, Pi, (int)Hd, (int)Hd,
                         Pi, Pi, 0, Hd * P, C * P, B, e0, r.wsb, r.wsb_b, s));
    du = r.du;
  }
  // dgamma = s sum_p du xhat, dbeta = s sum_p du  (FiLM: (1 + gamma s) xhat + beta s)
  return launch_film_grad_reduce(du, x1, r.an, r.tn, film_scale, (int)BC, P, dgamma, dbeta, s);
}

size_t msfno_mlp_backward_input_workspace_size(const msfno_mlp_desc* d, int B, long long P) {
  if (!d || B <= 0 || P <= 0) return 0;
  Carve cv;
  cv.take<float>((int64_t)B * d->Hid * P);  // pre
  cv.take<float>((int64_t)B * d->Hid * P);  // t, then dh
  cv.take<float>((int64_t)d->Hid * d->Cout);  // W2^T
  cv.take<float>((int64_t)d->Cin * d->Hid);   // W1[:, :Cin]^T
  cv.take<char>(gemm_dense_workspace(d->Hid, d->Cin, 1));
  if (d->Cin2 > 0) cv.take<char>(gemm_dense_workspace(d->Hid, d->Cin2, 1));
  cv.take<char>(gemm_dense_workspace(d->Hid, d->Cout, 1));
  cv.take<char>(gemm_dense_workspace(d->Cin, d->Hid, 1));
  return cv.off;
}

size_t msfno_mlp_backward_params_workspace_size(const msfno_mlp_desc* d, int B, long long P) {
  using namespace msfno;
  const size_t base = msfno_mlp_backward_input_workspace_size(d, B, P);
  if (!base) return 0;
  const int wide = std::max({d->Cin, d->Cin2, d->Hid, d->Cout});
  return round_up((int64_t)base, 256) + round_up((int64_t)wgrad_nt_workspace(wide, wide, P, B), 256) +
         norm_param_grad_workspace(B, wide);
}

int msfno_mlp_backward_input(const msfno_mlp_desc* d, const float* x, const float* x2,
                             const float* dy, float* dx, int B, long long P, void* ws,
                             size_t ws_bytes, void* stream) {
  MSFNO_REQUIRE(dx, MSFNO_EINVAL, "mlp backward: missing tensors");
  return msfno_mlp_backward_params(d, x, x2, dy, dx, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   B, P, ws, ws_bytes, stream);
}

int msfno_mlp_backward_params(const msfno_mlp_desc* d, const float* x, const float* x2,
                              const float* dy, float* dx, float* dx2, float* dfc1_w,
                              float* dfc1_b, float* dfc2_w, float* dfc2_b, int B, long long P,
                              void* ws, size_t ws_bytes, void* stream) {
  const bool params = dfc1_w || dfc1_b || dfc2_w || dfc2_b || dx2;
  MSFNO_REQUIRE(d && x && dy && d->fc1_w && d->fc2_w && d->fc1_b, MSFNO_EINVAL,
                "mlp backward: missing tensors");
  MSFNO_REQUIRE(d->Cin > 0 && d->Hid > 0 && d->Cout > 0 && d->Cin2 >= 0 && B > 0 && P > 0 &&
                    P <= 0x7fffffff,
                MSFNO_EINVAL, "mlp backward: bad sizes");
  MSFNO_REQUIRE((d->Cin2 > 0) == (x2 != nullptr), MSFNO_EINVAL,
                "mlp backward: x2 must be given exactly when Cin2 > 0");
  MSFNO_REQUIRE(ws_bytes >= (params ? msfno_mlp_backward_params_workspace_size(d, B, P)
                                     : msfno_mlp_backward_input_workspace_size(d, B, P)),
                MSFNO_EWORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  Carve cv;
  cv.base = (char*)ws;
  const int64_t Hd = d->Hid, Ct = d->Cin + d->Cin2;
  const int Pi = (int)P;
  float* pre = cv.take<float>((int64_t)B * Hd * P);
  float* t = cv.take<float>((int64_t)B * Hd * P);
  float* W2T = cv.take<float>(Hd * d->Cout);
  float* W1T = cv.take<float>((int64_t)d->Cin * Hd);
  const size_t w1b = gemm_dense_workspace((int)Hd, d->Cin, 1);
  void* w1 = cv.take<char>(w1b);
  const size_t w1b2 = d->Cin2 > 0 ? gemm_dense_workspace((int)Hd, d->Cin2, 1) : 0;
  void* w12 = d->Cin2 > 0 ? cv.take<char>(w1b2) : nullptr;
  const size_t w2b = gemm_dense_workspace((int)Hd, d->Cout, 1);
  void* w2 = cv.take<char>(w2b);
  const size_t w3b = gemm_dense_workspace(d->Cin, (int)Hd, 1);
  void* w3 = cv.take<char>(w3b);
  // pre = W1 [x ; x2] + b1 (fc1 without its GELU)
  if (d->Cin2 > 0) {
    GemmEpi e0;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w, x, t, (int)Hd, Pi, d->Cin, (int)Ct, Pi,
                         Pi, 0, (int64_t)d->Cin * P, Hd * P, B, e0, w1, w1b, s));
    GemmEpi e1;
    e1.bias = d->fc1_b;
    e1.addend = t; e1.sD = Hd * P; e1.ldd = Pi;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w + d->Cin, x2, pre, (int)Hd, Pi, d->Cin2,
                         (int)Ct, Pi, Pi, 0, (int64_t)d->Cin2 * P, Hd * P, B, e1, w12, w1b2, s));
  } else {
    GemmEpi e1;
    e1.bias = d->fc1_b;
    MSFNO_TRY(gemm_dense(ROLE_FC1, TILE_128x256, d->fc1_w, x, pre, (int)Hd, Pi, d->Cin, d->Cin, Pi,
                         Pi, 0, (int64_t)d->Cin * P, Hd * P, B, e1, w1, w1b, s));
  }
  // dh = GELU'(pre) * W2^T dy ;  dx = W1[:, :Cin]^T dh
  MSFNO_TRY(launch_transpose_mat(d->fc2_w, d->Cout, (int)Hd, (int)Hd, W2T, s));
  GemmEpi e0;
  float* dh = t;
  MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, W2T, dy, dh, (int)Hd, Pi, d->Cout, d->Cout, Pi, Pi,
                       0, (int64_t)d->Cout * P, Hd * P, B, e0, w2, w2b, s));
  if (params) {
    // dW2 = dy GELU(pre)^T and db2 = sum dy, before dh overwrites pre's partner buffer
    void* wg = cv.take<char>(wgrad_nt_workspace(std::max({d->Cin, d->Cin2, d->Hid, d->Cout}),
                                                std::max({d->Cin, d->Cin2, d->Hid, d->Cout}), P, B));
    const size_t wg_b = wgrad_nt_workspace(std::max({d->Cin, d->Cin2, d->Hid, d->Cout}),
                                           std::max({d->Cin, d->Cin2, d->Hid, d->Cout}), P, B);
    void* nr = cv.take<char>(norm_param_grad_workspace(B, std::max({d->Cin, d->Cin2, d->Hid, d->Cout})));
    if (dfc2_w)
      MSFNO_TRY(launch_wgrad_nt(dy, P, (int64_t)d->Cout * P, pre, P, Hd * P, d->Cout, (int)Hd, P, B,
                                WGRAD_GELU, nullptr, nullptr, dfc2_w, Hd, 1, wg, wg_b, s));
    if (dfc2_b)
      MSFNO_TRY(launch_norm_param_grad(dy, nullptr, nullptr, nullptr, nullptr, 0.f, B, d->Cout, P,
                                       nullptr, dfc2_b, nr, s));
    MSFNO_TRY(launch_gelu_grad_mul(dh, pre, (int64_t)B * Hd * P, s));
    // dW1 = dpre [x ; x2]^T (columns Cin.. from x2), db1 = sum dpre
    if (dfc1_w) {
      MSFNO_TRY(launch_wgrad_nt(dh, P, Hd * P, x, P, (int64_t)d->Cin * P, (int)Hd, d->Cin, P, B,
                                WGRAD_PLAIN, nullptr, nullptr, dfc1_w, Ct, 1, wg, wg_b, s));
      if (d->Cin2 > 0)
        MSFNO_TRY(launch_wgrad_nt(dh, P, Hd * P, x2, P, (int64_t)d->Cin2 * P, (int)Hd, d->Cin2, P, B,
                                  WGRAD_PLAIN, nullptr, nullptr, dfc1_w + d->Cin, Ct, 1, wg, wg_b,
                                  s));
    }
    if (dfc1_b)
      MSFNO_TRY(launch_norm_param_grad(dh, nullptr, nullptr, nullptr, nullptr, 0.f, B, (int)Hd, P,
                                       nullptr, dfc1_b, nr, s));
  } else {
    MSFNO_TRY(launch_gelu_grad_mul(dh, pre, (int64_t)B * Hd * P, s));
  }
  if (dx2) {
    // dx2 = W1[:, Cin:]^T dpre (W1T holds the Cin2 x Hd transpose first, then dx's)
    MSFNO_REQUIRE(x2 && d->Cin2 > 0 && d->Cin2 <= d->Cin, MSFNO_EINVAL,
                  "mlp backward: dx2 needs x2 and Cin2 <= Cin");
    MSFNO_TRY(launch_transpose_mat(d->fc1_w + d->Cin, (int)Hd, d->Cin2, (int)Ct, W1T, s));
    MSFNO_TRY(gemm_dense(ROLE_FC2, TILE_256x128, W1T, dh, dx2, d->Cin2, Pi, (int)Hd, (int)Hd, Pi,
                         Pi, 0, Hd * P, (int64_t)d->Cin2 * P, B, e0, w3, w3b, s));
  }
  if (!dx) return MSFNO_OK;
  MSFNO_TRY(launch_transpose_mat(d->fc1_w, (int)Hd, d->Cin, (int)Ct, W1T, s));
  return gemm_dense(ROLE_FC2, TILE_256x128, W1T, dh, dx, d->Cin, Pi, (int)Hd, (int)Hd, Pi, Pi, 0,
                    Hd * P, (int64_t)d->Cin * P, B, e0, w3, w3b, s);
}

}  // extern "C"
