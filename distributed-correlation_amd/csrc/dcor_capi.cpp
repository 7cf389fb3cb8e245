// dcor_capi.cpp -- host side of the C-ABI declared in include/dcor.h.
//
// Validates arguments the way the reference's stopifnot() calls do, evaluates every
// data-independent scalar of the estimators once (R operation order, cited), and
// launches the gfx950 kernels.  There is no CPU compute path: without a visible
// device every compute entry fails with DCOR_ENODEV.
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dcor.h"
#include "dcor_engine.h"
#include "dcor_host.h"

using namespace dcor;

namespace dcor {
namespace host {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(DCOR_EHIP, "%s: %s", what, hipGetErrorString(e));
}


// The process that first reached the device.  A process forked from it afterwards (R's
// mclapply children) inherits no usable HIP state: every entry there fails with DCOR_EFORK
// before touching HIP.
std::atomic<int> g_owner_pid{0};

int fork_guard() {
  const int me = (int)getpid();
  int owner = g_owner_pid.load();
  if (owner == 0 && g_owner_pid.compare_exchange_strong(owner, me)) owner = me;
  if (owner != me)
    return fail(DCOR_EFORK, "the dcor engine was used in process %d before this process (%d) was "
                            "forked (mclapply?): HIP does not survive fork(); run the grid from the "
                            "parent with one dcor_grid_run call (R: dcor_grid)", owner, me);
  return DCOR_OK;
}

int need_device() {
  if (int st = fork_guard()) return st;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return fail(DCOR_ENODEV, "no HIP device visible: the dcor engine has no CPU path");
  }
  return DCOR_OK;
}

double r_min(double a, double b) { return (std::isnan(a) || std::isnan(b)) ? NAN : (a < b ? a : b); }
double r_max(double a, double b) { return (std::isnan(a) || std::isnan(b)) ? NAN : (a > b ? a : b); }

struct DevBuf {  // RAII device allocation for the host-pointer entry points
  void* p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t bytes) {
    const hipError_t e = hipMalloc(&p, bytes ? bytes : 8);
    if (e == hipSuccess) count_alloc();
    return e;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

template <class T>
int upload(DevBuf& b, const T* h, size_t count) {
  HIPCHK(b.alloc(sizeof(T) * count));
  if (h && count) HIPCHK(hipMemcpy(b.p, h, sizeof(T) * count, hipMemcpyHostToDevice));
  else if (count) HIPCHK(hipMemset(b.p, 0, sizeof(T) * count));
  return DCOR_OK;
}

// T with (double)w * 2^-32 < p  <=>  w < T for every uint32 w: T = ceil(p * 2^32) clamped
// to [0, 2^32] (p * 2^32 is exact).
uint64_t u32_threshold(double p) {
  if (!(p > 0)) return 0;
  const double t = std::ceil(p * 4294967296.0);
  return t >= 4294967296.0 ? (uint64_t)4294967296ull : (uint64_t)t;
}

// MixConst for sort(x)[ceiling(p*nsim)], p = 1 - alpha/2.
int make_mix(int64_t nsim, double alpha, MixConst& mx) {
  if (nsim < 1 || nsim > 2048) return fail(DCOR_EINVAL, "nsim must be in [1, 2048] (got %lld)", (long long)nsim);
  const double pos = std::ceil((1.0 - alpha / 2.0) * (double)nsim);
  mx.nsim = (int32_t)nsim;
  mx.pos = (pos >= 1 && pos <= (double)nsim) ? (int32_t)pos - 1 : -1;
  mx.P = 1;
  while (mx.P < mx.nsim) mx.P <<= 1;
  mx.pad = 0;
  return DCOR_OK;
}

// MASS::mvrnorm factor A = V diag(sqrt(ev)) of the 2x2 covariance (vert-cor.R:389-394).
void mvrnorm_factor(const double sigma[2], double rho, double A[4]) {
  const double s11 = sigma[0] * sigma[0];
  const double s12 = sigma[0] * sigma[1] * rho;
  const double s22 = sigma[1] * sigma[1];
  const double mid = (s11 + s22) / 2.0, hd = (s11 - s22) / 2.0;
  const double d = std::sqrt(hd * hd + s12 * s12);
  const double l1 = mid + d, l2 = mid - d;
  double v0, v1;
  if (s12 == 0.0) {
    if (s11 > s22) { v0 = 1.0; v1 = 0.0; } else { v0 = 0.0; v1 = 1.0; }
  } else {
    if (s11 >= s22) { v0 = l1 - s22; v1 = s12; } else { v0 = s12; v1 = l1 - s11; }
    const double nr = std::sqrt(v0 * v0 + v1 * v1);
    v0 /= nr; v1 /= nr;
    if (v1 < 0) { v0 = -v0; v1 = -v1; }
  }
  const double a1 = std::sqrt(l1 > 0 ? l1 : 0.0), a2 = std::sqrt(l2 > 0 ? l2 : 0.0);
  A[0] = v0 * a1; A[1] = -v1 * a2;
  A[2] = v1 * a1; A[3] = v0 * a2;
}

// MASS::mvrnorm's check: stop("'Sigma' is not positive definite") unless every eigenvalue
// ev >= -tol * |ev[1]| with tol = 1e-6 (ev decreasing).  False for |rho| > 1 (beyond tol).
bool mvrnorm_pd(const double sigma[2], double rho) {
  const double s11 = sigma[0] * sigma[0], s12 = sigma[0] * sigma[1] * rho, s22 = sigma[1] * sigma[1];
  const double mid = (s11 + s22) / 2.0, hd = (s11 - s22) / 2.0;
  const double d = std::sqrt(hd * hd + s12 * s12);
  const double l1 = mid + d, l2 = mid - d;
  return !std::isnan(l2) && l1 >= -1e-6 * std::fabs(l1) && l2 >= -1e-6 * std::fabs(l1);
}

int make_dgp(const dcor_cell& c, DgpConst& g) {
  std::memset(&g, 0, sizeof(g));
  g.dgp = c.dgp;
  if (c.dgp == DCOR_DGP_GAUSSIAN) {
    if (!mvrnorm_pd(c.sigma, c.rho))
      return fail(DCOR_EINVAL, "mvrnorm: 'Sigma' is not positive definite (|rho| > 1; MASS::mvrnorm, vert-cor.R:394)");
    double A[4];
    mvrnorm_factor(c.sigma, c.rho, A);
    g.mu0 = c.mu[0]; g.mu1 = c.mu[1];
    g.a00 = A[0]; g.a01 = A[1]; g.a10 = A[2]; g.a11 = A[3];
  } else if (c.dgp == DCOR_DGP_BERNOULLI) {
    if (!(std::fabs(c.rho) <= 1)) return fail(DCOR_EINVAL, "gen_bernoulli: |rho| <= 1 required (vert-cor.R:79)");
    const double p11 = 0.25 + c.rho / 4, p10 = 0.25 - c.rho / 4, p01 = p10;  // vert-cor.R:80-83
    g.thr0 = p01 / 0.5; g.thr1 = p11 / 0.5;
    g.T0 = u32_threshold(g.thr0); g.T1 = u32_threshold(g.thr1);
    g.T0_24 = (uint32_t)std::ceil(g.thr0 * 16777216.0);  // thr <= 1: exact scaling, <= 2^24
    g.T1_24 = (uint32_t)std::ceil(g.thr1 * 16777216.0);
  } else if (c.dgp == DCOR_DGP_BOUNDED_FACTOR) {
    g.cU = std::sqrt(3.0 * c.rho); g.cE = std::sqrt(3.0 * (1.0 - c.rho));  // ver-cor-subG.R:148-149
    g.cU2 = g.cU - -g.cU; g.cE2 = g.cE - -g.cE;
    // rho outside [0, 1]: R's sqrt gives NaN (a warning) and runif(n, NaN, NaN) NaN draws, so the
    // replicate's estimates are all NaN; the launch writes those without generating anything.
    g.nan_dgp = (std::isnan(g.cU) || std::isnan(g.cE)) ? 1 : 0;
  } else if (c.dgp == DCOR_DGP_MIX_GAUSSIAN) {
    if (!(c.mix_pi >= 0 && c.mix_pi <= 1)) return fail(DCOR_EINVAL, "gen_mix_gaussian: pi_mix in [0,1] required");
    if (!mvrnorm_pd(c.mix_sigma0, c.rho) || !mvrnorm_pd(c.mix_sigma1, c.rho))
      return fail(DCOR_EINVAL, "gen_mix_gaussian: mvrnorm 'Sigma' is not positive definite (|rho| > 1)");
    mvrnorm_factor(c.mix_sigma0, c.rho, g.xa[0]);   // ver-cor-subG.R:119-122
    mvrnorm_factor(c.mix_sigma1, c.rho, g.xa[1]);
    g.xmu[0][0] = c.mix_mu0[0]; g.xmu[0][1] = c.mix_mu0[1];
    g.xmu[1][0] = c.mix_mu1[0]; g.xmu[1][1] = c.mix_mu1[1];
    const double t = std::ceil(c.mix_pi * 16777216.0);  // exact: pi * 2^24
    g.T24 = t >= 16777216.0 ? 16777216u : (uint32_t)t;
  } else {
    return fail(DCOR_EINVAL, "unknown dgp %d", c.dgp);
  }
  return DCOR_OK;
}

int check_common(int64_t n, double eps1, double eps2, double alpha) {
  if (n < 1 || n > 0x7fffffffLL) return fail(DCOR_EINVAL, "n must be in [1, 2^31) (got %lld)", (long long)n);
  if (!(eps1 > 0) || !(eps2 > 0) || !std::isfinite(eps1) || !std::isfinite(eps2))
    return fail(DCOR_EINVAL, "eps1 > 0 and eps2 > 0 required (vert-cor.R:264)");
  // The reference never checks alpha: qnorm(1 - alpha/2) and mixquant's
  // sort(x)[ceiling((1 - alpha/2) nsim)] are evaluated as they come (alpha = 1: a zero-width
  // CI; alpha < 0: NaN).  alpha >= 2 makes the mixquant index < 1, where R's x[0] is
  // numeric(0) and run_sim_one's detail assignment fails, so it is refused here.
  if (std::isnan(alpha) || !(alpha < 2))
    return fail(DCOR_EINVAL, "alpha must be < 2 (R's mixquant index ceiling((1-alpha/2)*nsim) >= 1)");
  return DCOR_OK;
}

// ci_NI_signbatch + ci_INT_signflip scalars (vert-cor.R:204-317).
// allow_k0: INT-only single calls (ci_INT_signflip has no batch requirement).
int make_sign(int64_t n, double eps1, double eps2, double alpha, int normalise, int mode,
              int64_t nsim, bool allow_k0, SignConst& c) {
  std::memset(&c, 0, sizeof(c));
  if (int st = check_common(n, eps1, eps2, alpha)) return st;
  const double nd = (double)n;
  const double md = std::ceil(8.0 / (eps1 * eps2));                     // :207
  const double kd = std::floor(nd / md);                                 // :208
  if (!(kd >= 1) && !allow_k0)
    return fail(DCOR_EKLT1, "ci_NI_signbatch: k = floor(n/m) = %g < 1 (n=%lld, m=%g; vert-cor.R:209)", kd, (long long)n, md);
  if (md > 0x7fffffff) return fail(DCOR_EINVAL, "batch size m too large");
  c.n = n; c.m = (int32_t)md; c.k = kd >= 1 ? (int64_t)kd : 0;
  c.nd = nd; c.md = md; c.kd = kd;
  c.pieces = sign_pieces(c.m);
  {
    int e = 0;
    c.md_pow2 = (std::frexp(md, &e) == 0.5) ? 1 : 0;  // md = 2^(e-1): count / md == count * 2^(1-e)
    c.inv_md = c.md_pow2 ? std::ldexp(1.0, 1 - e) : 0.0;
  }
  c.normalise = normalise ? 1 : 0;
  const double L = std::sqrt(2.0 * std::log(nd));                        // :212
  c.L = L;
  c.s_mu_x = 2.0 * L / (nd * (eps1 / 2));                                // :335-336
  c.s_m2_x = 2.0 * (L * L) / (nd * (eps1 / 2));                          // :339-340
  c.s_mu_y = 2.0 * L / (nd * (eps2 / 2));
  c.s_m2_y = 2.0 * (L * L) / (nd * (eps2 / 2));
  c.bx = 2.0 / (md * eps1);                                              // :230
  c.by = 2.0 / (md * eps2);                                              // :231
  c.inv_k = 1.0 / kd;                                                    // :234
  c.crit = dcor_qnorm(1.0 - alpha / 2.0);                                // :242
  c.sqrt_k = std::sqrt(kd);
  c.sender_is_X = (eps1 >= eps2) ? 1 : 0;                                // :275
  const double eps_s = c.sender_is_X ? eps1 : eps2, eps_r = c.sender_is_X ? eps2 : eps1;
  const double es = std::exp(eps_s);
  c.pflip = es / (es + 1.0);                                             // :174
  c.flipT = u32_threshold(c.pflip);
  {
    const double t = std::ceil(c.pflip * 16777216.0);  // exact scaling
    c.flipT24 = t >= 16777216.0 ? 16777216u : (t > 0 ? (uint32_t)t : 0u);
  }
  c.scale_Z = 2.0 * (es + 1.0) / (nd * (es - 1.0) * eps_r);              // :186-187
  c.coefZ = (es + 1.0) / (nd * (es - 1.0));                              // :190-191
  const double q = (es - 1.0) / (es + 1.0);
  c.q2 = q * q;                                                          // :284
  c.ratio = (es + 1.0) / (es - 1.0);                                     // :289
  c.inv_sqrt_n = 1.0 / std::sqrt(nd);
  c.eps_r = eps_r;
  c.w_laplace = (2.0 / (nd * eps_r)) * c.ratio * std::log(1.0 / alpha);  // :305-308
  int md_ = mode;
  if (md_ == DCOR_MODE_AUTO) md_ = (std::sqrt(nd) * eps_r > 0.5) ? DCOR_MODE_NORMAL : DCOR_MODE_LAPLACE;  // :294-296
  else if (md_ != DCOR_MODE_NORMAL && md_ != DCOR_MODE_LAPLACE) return fail(DCOR_EINVAL, "ci_mode must be auto/normal/laplace");
  c.mode_normal = (md_ == DCOR_MODE_NORMAL) ? 1 : 0;
  if (int st = make_mix(nsim, alpha, c.mix)) return st;
  return DCOR_OK;
}

// correlation_NI_subG + ci_INT_subG scalars (ver-cor-subG.R:25-108; HRS variant
// real-data-sims.R:115-147,176-252 when hrs).
int make_subg(int64_t n, double eps1, double eps2, double eta1, double eta2, double alpha,
              int hrs, double lam_x, double lam_y, double lam_s, double lam_o, double lam_r,
              double delta, int64_t nsim, SubgConst& c, double* lo_out, double* crit_sqrt2_s) {
  std::memset(&c, 0, sizeof(c));
  if (int st = check_common(n, eps1, eps2, alpha)) return st;
  if (hrs && n < 2) return fail(DCOR_EINVAL, "n >= 2 required (real-data-sims.R:121)");
  const double nd = (double)n;
  c.n = n; c.nd = nd;
  c.l1 = (hrs && !std::isnan(lam_x)) ? lam_x : dcor_lambda_n(nd, eta1);  // :30 / rds:123
  c.l2 = (hrs && !std::isnan(lam_y)) ? lam_y : dcor_lambda_n(nd, eta2);
  double md = std::ceil(8.0 / (eps1 * eps2));                            // :37
  if (md > nd) md = nd;
  double kd = std::floor(nd / md);                                       // :38
  if (hrs) {
    if (kd < 2) { kd = 2; md = std::floor(nd / kd); }                    // rds:130
  } else if (!(kd >= 1)) {
    return fail(DCOR_EKLT1, "correlation_NI_subG: k < 1 (ver-cor-subG.R:38)");
  }
  c.m = (int32_t)md; c.k = (int64_t)kd; c.md = md; c.kd = kd;
  {
    int e = 0;
    c.md_pow2 = (std::frexp(md, &e) == 0.5) ? 1 : 0;
    c.inv_md = c.md_pow2 ? std::ldexp(1.0, 1 - e) : 0.0;
  }
  c.bx = 2.0 * c.l1 / (md * eps1);                                       // :48
  c.by = 2.0 * c.l2 / (md * eps2);                                       // :49
  c.m_over_k = md / kd;                                                  // :51
  c.crit = dcor_qnorm(1.0 - alpha / 2.0);                                // :57
  c.sqrt_k = std::sqrt(kd);
  c.sender_is_X = (eps1 >= eps2) ? 1 : 0;                                // :76
  const double eps_s = c.sender_is_X ? eps1 : eps2, eps_r = c.sender_is_X ? eps2 : eps1;
  const double eta_s = c.sender_is_X ? eta1 : eta2, eta_r = c.sender_is_X ? eta2 : eta1;
  double lo_ = NAN;
  if (!hrs) {
    double lam[2];
    dcor_lambda_int_n(nd, eta_s, eta_r, eps_s, lam);                     // :83-85
    c.ls = lam[0]; c.lr = lam[1];
  } else {
    const double dl = std::isnan(delta) ? 1.0 / nd : delta;              // rds:199
    double ls = lam_s;
    lo_ = lam_o;
    if (std::isnan(ls) || std::isnan(lo_)) {                             // rds:202-208
      double lam[2];
      dcor_lambda_int_n(nd, eta_s, eta_r, eps_s, lam);
      if (std::isnan(ls)) ls = lam[0];
      if (std::isnan(lo_)) lo_ = dcor_lambda_n(nd, c.sender_is_X ? eta2 : eta1);
    }
    double lr = lam_r;
    if (std::isnan(lr)) lr = dcor_lambda_receiver_from_noise(ls, lo_, eps_s, dl);  // rds:211-218
    c.ls = ls; c.lr = lr;
  }
  c.bs = 2.0 * c.ls / (eps_s);                                           // :89
  c.s_central = 2.0 * c.lr / (nd * eps_r);                               // :91
  c.sn2x2 = 2.0 * (c.s_central * c.s_central);                           // :99
  c.sqrt_n = std::sqrt(nd);
  c.eps_r = eps_r;
  if (lo_out) *lo_out = lo_;
  if (crit_sqrt2_s) *crit_sqrt2_s = c.crit * std::sqrt(2.0) * (2.0 * c.lr / (nd * eps_r));  // rds:238
  if (int st = make_mix(nsim, alpha, c.mix)) return st;
  return DCOR_OK;
}

// Library-owned device state of one (host thread, device): the scratch arenas (the one-pass
// sign kernel's code slabs, the batched grid's tables and partials, the R-stream buffers), the
// auxiliary stream with the fork/join events of the two-stream chunk pipeline, and a pinned
// staging buffer for the grid tables.  One per calling thread and device, so two host threads
// never share scratch or streams; every context is registered for dcor_shutdown(), and the grid's
// worker threads release theirs when they finish.
std::mutex g_ctx_mu;
std::vector<Ctx*> g_ctxs;            // every live context (guarded by g_ctx_mu)
// Bytes held by every live context's arenas (dcor_device_bytes): updated where an arena grows or
// is freed, so a reader needs no access to another thread's context.
std::atomic<int64_t> g_device_bytes{0};
std::atomic<uint64_t> g_ctx_gen{1};  // bumped by dcor_shutdown: older thread caches are stale
struct ThreadCtx { Ctx* c[64] = {}; uint64_t gen = 0; };
thread_local ThreadCtx t_ctx;

void ctx_free(Ctx* c) {
  if (c->pipe.s) {
    (void)hipStreamSynchronize(c->pipe.s);
    (void)hipStreamSynchronize(c->pipe.s2);
    (void)hipStreamDestroy(c->pipe.s);
    (void)hipStreamDestroy(c->pipe.s2);
    for (hipEvent_t e : {c->pipe.fork, c->pipe.join, c->pipe.entry, c->pipe.end[0], c->pipe.end[1]})
      (void)hipEventDestroy(e);
  }
  for (Pinned* b : {&c->stage[0], &c->stage[1], &c->hrec, &c->hacc}) {
    if (b->done) { (void)hipEventSynchronize(b->done); (void)hipEventDestroy(b->done); }
    if (b->p) (void)hipHostFree(b->p);
  }
  if (c->work) { (void)hipStreamSynchronize(c->work); (void)hipStreamDestroy(c->work); }
  for (Arena* a : {&c->codes, &c->rs, &c->grid, &c->gpart, &c->out, &c->rsj})
    if (a->p) {
      (void)hipFree(a->p);
      g_device_bytes.fetch_sub((int64_t)a->bytes);
    }
  delete c;
}

int ctx_get(Ctx** out) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return fail(DCOR_EINVAL, "device id out of range");
  const uint64_t gen = g_ctx_gen.load();
  if (t_ctx.gen != gen) { t_ctx = ThreadCtx(); t_ctx.gen = gen; }
  if (!t_ctx.c[dev]) {
    Ctx* c = new Ctx();
    c->dev = dev;
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    g_ctxs.push_back(c);
    t_ctx.c[dev] = c;
  }
  *out = t_ctx.c[dev];
  return DCOR_OK;
}

void ctx_release_thread() {
  if (t_ctx.gen != g_ctx_gen.load()) { t_ctx = ThreadCtx(); return; }
  for (Ctx*& c : t_ctx.c) {
    if (!c) continue;
    {
      std::lock_guard<std::mutex> lk(g_ctx_mu);
      g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), c), g_ctxs.end());
    }
    ctx_free(c);
    c = nullptr;
  }
}

int pipe_get(Pipe** out) {
  Ctx* c = nullptr;
  if (int st = ctx_get(&c)) return st;
  Pipe& p = c->pipe;
  if (!p.s) {
    HIPCHK(hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&p.s2, hipStreamNonBlocking));
    for (hipEvent_t* e : {&p.fork, &p.join, &p.entry, &p.end[0], &p.end[1]})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  *out = &p;
  return DCOR_OK;
}

std::atomic<int64_t> g_alloc_count{0};
void count_alloc() { g_alloc_count.fetch_add(1); }

int arena_grow(Arena& a, size_t bytes, void** out) {
  if (a.bytes < bytes) {
    // the old block may still be read by work queued earlier: wait for the device
    if (a.p) {
      HIPCHK(hipDeviceSynchronize());
      HIPCHK(hipFree(a.p));
      g_device_bytes.fetch_sub((int64_t)a.bytes);
      a.p = nullptr;
      a.bytes = 0;
    }
    if (hipMalloc(&a.p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      a.p = nullptr;
      return fail(DCOR_ENOMEM, "scratch arena: cannot allocate %zu bytes", bytes);
    }
    count_alloc();
    a.bytes = bytes;
    g_device_bytes.fetch_add((int64_t)bytes);
  }
  *out = a.p;
  return DCOR_OK;
}

int pinned_grow(Pinned& b, size_t bytes, void** out) {
  if (!b.done) HIPCHK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
  HIPCHK(hipEventSynchronize(b.done));   // a never-recorded event is complete
  if (b.bytes < bytes) {
    if (b.p) HIPCHK(hipHostFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    if (hipHostMalloc(&b.p, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      b.p = nullptr;
      return fail(DCOR_ENOMEM, "pinned staging: cannot allocate %zu bytes", bytes);
    }
    count_alloc();
    b.bytes = bytes;
  }
  *out = b.p;
  return DCOR_OK;
}

int codes_arena(Ctx* c, size_t bytes, void** out) {
  c->pipe.sig = 0;
  return arena_grow(c->codes, bytes, out);
}

int arena_get(size_t bytes, void** out) {
  Ctx* c = nullptr;
  if (int st = ctx_get(&c)) return st;
  return codes_arena(c, bytes, out);
}

int rs_arena_get(size_t bytes, void** out) {
  Ctx* c = nullptr;
  if (int st = ctx_get(&c)) return st;
  return arena_grow(c->rs, bytes, out);
}

// The first n jump polynomials of the R-stream jump path on this device, as launch_rsj takes
// them: per polynomial the list of its set bits (host table: mt_segment_polys, computed once per
// process; uploaded when the device copy is short).
int rsj_polys(int n, const uint32_t** poff, const uint32_t** pidx) {
  Ctx* c = nullptr;
  if (int st = ctx_get(&c)) return st;
  if (c->rsj_npoly < n) {
    std::vector<uint64_t> table;
    int words = 0;
    if (int st = mt_segment_polys(RSJ_L, n, table, &words)) return st;
    if (words != RSJ_PW) return fail(DCOR_EINVAL, "jump polynomial width %d", words);
    const size_t head = (size_t)(n + 1 + 3) / 4 * 4;
    std::vector<uint32_t> buf(head, 0u);
    std::vector<uint16_t> idx;
    for (int s = 0; s < n; ++s) {
      buf[(size_t)s] = (uint32_t)(buf.size() - head);
      idx.clear();
      for (int w = 0; w < RSJ_PW; ++w)
        for (uint64_t b = table[(size_t)s * RSJ_PW + w]; b; b &= b - 1)
          idx.push_back((uint16_t)(64 * w + __builtin_ctzll(b)));
      while (idx.size() % 8) idx.push_back((uint16_t)RSJ_PAD);
      for (size_t i = 0; i < idx.size(); i += 2) buf.push_back((uint32_t)idx[i] | ((uint32_t)idx[i + 1] << 16));
    }
    buf[(size_t)n] = (uint32_t)(buf.size() - head);
    void* d = nullptr;
    if (int st = arena_grow(c->rsj, buf.size() * 4, &d)) return st;
    HIPCHK(hipMemcpy(d, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
    c->rsj_npoly = n;
  }
  *poff = (const uint32_t*)c->rsj.p;
  *pidx = *poff + (size_t)(c->rsj_npoly + 1 + 3) / 4 * 4;
  return DCOR_OK;
}

// Monotone code map of clip(v): base + [0, 2R) -> [0, levels).  Only affects speed (how many
// samples tie a threshold's code), never results.
void code_map(double center, double R, double levels, double* base, double* inv) {
  if (!(R > 0) || !std::isfinite(R)) R = 1.0;
  if (!std::isfinite(center)) center = 0.0;
  *base = center - R;
  *inv = levels / (2.0 * R);
}

// E[clip(X, -L, L)] for X ~ N(m, s^2): the centre of a Gaussian cell's code window.
static double clipped_normal_mean(double m, double s, double L) {
  if (!(s > 0) || !std::isfinite(s)) return r_min(r_max(m, -L), L);
  const double a = (-L - m) / s, b = (L - m) / s;
  auto Phi = [](double t) { return 0.5 * std::erfc(-t / std::sqrt(2.0)); };
  auto phi = [](double t) { return std::exp(-0.5 * t * t) / std::sqrt(2.0 * M_PI); };
  return m * (Phi(b) - Phi(a)) + s * (phi(a) - phi(b)) + L * (1.0 - Phi(b)) - L * Phi(a);
}

// Every data-independent constant of one fused cell (R operation order) and the kernel family
// that runs it.  The status is the one the reference raises for the cell (stopifnot, k < 1).
int prepare_cell(const dcor_cell& c, CellPlan& p) {
  std::memset(&p, 0, sizeof(p));
  DgpConst g;
  if (int st = make_dgp(c, g)) return st;
  p.dgp = c.dgp;
  p.nan_dgp = g.nan_dgp != 0;
  const char* var = dcor::variant("DCOR_SIGN_KERNEL");
  const bool force_regen = var && std::strcmp(var, "regen") == 0;
  if (c.family == DCOR_FAMILY_SIGN) {
    SignConst& k = p.sign;
    if (int st = make_sign(c.n, c.eps1, c.eps2, c.alpha, c.normalise, c.ci_mode, c.nsim, false, k)) return st;
    k.g = g;
    k.k0 = (uint32_t)c.seed; k.k1 = (uint32_t)(c.seed >> 32);
    // code windows centred on the DGP's location (speed only)
    double cx = 0.0, cy = 0.0, rx = 1.0, ry = 1.0;
    if (c.dgp == DCOR_DGP_GAUSSIAN) {
      // The private centres are mean(clip(x)) + Laplace(s_mu) (vert-cor.R:335-336): within
      // 7 sd(mean) + 24 noise scales of E[clip(x)] but with probability below 1e-9 per replicate
      // (sd(mean) <= sd(x) / sqrt(n)).  A window that narrow spends the 128 code levels where the
      // thresholds fall, so few samples tie one (each tie batch is recomputed exactly in pass 2);
      // samples outside it clamp to the end codes, still decided exactly while the thresholds lie
      // inside -- and when one does not, its end code ties every clamped sample, and those batches
      // are recomputed too: exact, only slower.  (Round 4 used 12 sd + 40 scales with 2^15 levels;
      // at 128 levels the narrower window takes 40 % of the ties off.)  DCOR_CODE_WINDOW=wide: the
      // round-3 window, 2 sd of the sample around mu.
      const double sx = std::sqrt(g.a00 * g.a00 + g.a01 * g.a01);
      const double sy = std::sqrt(g.a10 * g.a10 + g.a11 * g.a11);
      const char* wv = dcor::variant("DCOR_CODE_WINDOW");
      if (wv && std::strcmp(wv, "wide") == 0) {
        cx = r_min(r_max(c.mu[0], -k.L), k.L); cy = r_min(r_max(c.mu[1], -k.L), k.L);
        rx = 2.0 * sx;
        ry = 2.0 * sy;
      } else {
        // DCOR_CODE_WINDOW=<a>,<b> (A/B runs): a sd(mean) + b noise scales instead of 7, 24
        double wa = 7.0, wb = 24.0;
        if (wv) {
          double a2 = 0, b2 = 0;
          if (std::sscanf(wv, "%lf,%lf", &a2, &b2) == 2 && a2 > 0 && b2 > 0) { wa = a2; wb = b2; }
        }
        const double rn = 1.0 / std::sqrt((double)c.n);
        cx = clipped_normal_mean(c.mu[0], sx, k.L);
        cy = clipped_normal_mean(c.mu[1], sy, k.L);
        rx = r_min(2.0 * sx, wa * sx * rn + wb * k.s_mu_x);
        ry = r_min(2.0 * sy, wa * sy * rn + wb * k.s_mu_y);
      }
    } else if (c.dgp == DCOR_DGP_BERNOULLI) {
      cx = cy = 0.5; rx = ry = 1.0;
    } else if (c.dgp == DCOR_DGP_MIX_GAUSSIAN) {
      cx = cy = 0.0; rx = ry = 1.0;       // clipped to [-1, 1]
    } else {
      cx = cy = 0.0; rx = ry = 2.0;
    }
    // the window onto t in [0, 1], whose unorm16 (t 65535, rounded) >> 9 is the 7-bit record code
    code_map(cx, rx, 65535.0, &k.cbase_x, &k.cinv_x);
    code_map(cy, ry, 65535.0, &k.cbase_y, &k.cinv_y);
    // code16_pair's unorm16 maps t in [0, 1] to [0, 65535]: the fp32 map is the code map / 65535
    k.cinv_xf = (float)(k.cinv_x / 65535.0); k.cnb_xf = (float)(-k.cbase_x * k.cinv_x / 65535.0);
    k.cinv_yf = (float)(k.cinv_y / 65535.0); k.cnb_yf = (float)(-k.cbase_y * k.cinv_y / 65535.0);
    if (c.dgp == DCOR_DGP_BERNOULLI && !force_regen)
      p.kind = c.n <= GRID_BERN_W_NMAX ? GK_SIGN_BERN_W : GK_SIGN_BERN;
    else if (force_regen || !c.normalise)
      p.kind = GK_SIGN_REGEN;
    else
      p.kind = c.n <= SIGN_W_NMAX ? GK_SIGN_CODES_W : GK_SIGN_CODES;
    p.vpl32 = k.mix.nsim > 1024 ? 1 : 0;
  } else if (c.family == DCOR_FAMILY_SUBG) {
    SubgConst& k = p.subg;
    if (int st = make_subg(c.n, c.eps1, c.eps2, c.eta1, c.eta2, c.alpha, 0, NAN, NAN, NAN, NAN,
                           NAN, NAN, c.nsim, k, nullptr, nullptr)) return st;
    k.g = g;
    k.k0 = (uint32_t)c.seed; k.k1 = (uint32_t)(c.seed >> 32);
    p.kind = c.n <= SUBG_W_NMAX ? GK_SUBG_W : GK_SUBG;
    p.vpl32 = k.mix.nsim > 1024 ? 1 : 0;
  } else {
    return fail(DCOR_EINVAL, "unknown family %d", c.family);
  }
  return DCOR_OK;
}

}  // namespace host

// ------------------------------------------------------------------ implementation switches
// The A/B and test switches of the kernels and launchers, set only through dcor_set_variant.
// Each one selects a kernel variant, a launch plan or a test hook; none is read from the
// environment, so a stray variable in a user's shell cannot move a replicate's bits.
namespace {
const char* const kVariantNames[] = {
    "DCOR_SIGN_KERNEL",      // "regen": the regenerate-everything sign kernel
    "DCOR_CODE_WINDOW",      // "wide" or "a,b": the sign records' code window
    "DCOR_SIGN_PIPELINE",    // "0": sign chunks on one stream
    "DCOR_SIGN_XCALL",       // "0": no overlap of back-to-back sign calls
    "DCOR_SIGN_P2E",         // "0": small cells' pass 2 and epilogue as two kernels
    "DCOR_EPILOGUE",         // "block" (sign) / "wave" (premat): epilogue kernel form
    "DCOR_HRS_FUSED_L2",     // "1": a coded panel through the uncoded fused HRS kernel
    "DCOR_HRS_WPE",          // "4": fused HRS kernel at 4 waves per SIMD
    "DCOR_PREMAT_PIPELINE",  // "1": two-stream premat halves
    "DCOR_DICT_VARIANT",     // 0-3: coded-panel kernel shape
    "DCOR_L2_VARIANT",       // 0-3: L2-gather kernel shape
    "DCOR_TILED",            // "0": no tiled kernel (L2 gathers)
    "DCOR_TILED_VARIANT",    // 0/1: 512- or 1024-thread tiled kernel
    "DCOR_TILED_INT",        // 0/1/2: where the tiled path's INT sums run
    "DCOR_GRID_CHUNK_ITEMS", // grid planner caps (memory-bound tests)
    "DCOR_GRID_SLAB_MB",
    "DCOR_GRID_MIN_CHUNKS",
    "DCOR_GRID_REC_MB",
    "DCOR_RS_JUMP",          // R-stream: 0 never / 1 always the jump path
    "DCOR_RS_BUDGET_MB",
    "DCOR_RS_MAX_CHUNK",     // test hook: short R-stream chunks
    "DCOR_RSJ_TIGHT",        // test hook: a jump budget every mixquant chunk overruns
};
constexpr int kNVariants = (int)(sizeof(kVariantNames) / sizeof(kVariantNames[0]));
std::mutex g_var_mu;
std::string g_var_val[kNVariants];
bool g_var_set[kNVariants] = {};

int variant_index(const char* name) {
  for (int i = 0; i < kNVariants; ++i)
    if (std::strcmp(name, kVariantNames[i]) == 0) return i;
  return -1;
}
}  // namespace

const char* variant(const char* name) {
  const int i = variant_index(name);
  if (i < 0) return nullptr;
  thread_local std::string copy[kNVariants];
  std::lock_guard<std::mutex> lk(g_var_mu);
  if (!g_var_set[i]) return nullptr;
  copy[i] = g_var_val[i];
  return copy[i].c_str();
}
}  // namespace dcor

using namespace dcor::host;

// ===================================================================== ABI
extern "C" {

const char* dcor_version(void) { return "dcor-mi355x 0.1.0 (gfx950)"; }

int dcor_set_variant(const char* name, const char* value) {
  std::lock_guard<std::mutex> lk(dcor::g_var_mu);
  if (name == nullptr) {
    for (int i = 0; i < dcor::kNVariants; ++i) { dcor::g_var_set[i] = false; dcor::g_var_val[i].clear(); }
    return DCOR_OK;
  }
  const int i = dcor::variant_index(name);
  if (i < 0) return fail(DCOR_EINVAL, "unknown implementation switch %s", name);
  dcor::g_var_set[i] = value != nullptr;
  dcor::g_var_val[i] = value ? value : "";
  return DCOR_OK;
}

int dcor_get_variant(const char* name, char* buf, size_t len) {
  if (name == nullptr || dcor::variant_index(name) < 0) {
    fail(DCOR_EINVAL, "unknown implementation switch %s", name ? name : "(null)");
    return -1;
  }
  const char* v = dcor::variant(name);
  if (buf && len) {
    std::strncpy(buf, v ? v : "", len - 1);
    buf[len - 1] = 0;
  }
  return v != nullptr;
}

int dcor_last_error(char* buf, size_t len) {
  if (buf && len) {
    std::strncpy(buf, g_err, len - 1);
    buf[len - 1] = 0;
  }
  return (int)std::strlen(g_err);
}

int dcor_device_count(void) {
  if (fork_guard()) return 0;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return 0; }
  return n;
}

double dcor_lambda_n(double n, double eta) {  // ver-cor-subG.R:1
  return r_min(2.0 * eta * std::sqrt(std::log(n)), 2.0 * std::sqrt(3.0));
}

void dcor_lambda_int_n(double n, double eta_s, double eta_r, double eps_s, double out[2]) {
  out[0] = r_min(2.0 * eta_s * std::sqrt(std::log(n)), 2.0 * std::sqrt(3.0));  // ver-cor-subG.R:4
  out[1] = 5.0 * r_max(eta_r, 1.0) * r_min(std::log(n), 6.0) / (r_min(eps_s, 1.0));  // :5
}

double dcor_lambda_receiver_from_noise(double lam_s, double lam_o, double eps_s, double delta) {
  const double b_s = 2.0 * lam_s / eps_s;  // real-data-sims.R:172
  return (lam_s + b_s * std::log(1.0 / delta)) * lam_o;
}

double dcor_lambda_from_priv(double lo, double hi, double mean, double sd, double eps_sd) {
  const double sig = r_max(sd, eps_sd);  // real-data-sims.R:104
  return r_max(std::fabs((lo - mean) / sig), std::fabs((hi - mean) / sig));
}

double dcor_qnorm(double p) {
  // R's qnorm(p, 0, 1) (qnorm.c: Wichura's AS241, lower tail, log.p = FALSE), same operation
  // order, so crit = qnorm(1 - alpha/2) is R's double.
  if (std::isnan(p) || p < 0 || p > 1) return NAN;
  if (p == 0) return -INFINITY;
  if (p == 1) return INFINITY;
  const double q = p - 0.5;
  double r, val;
  if (std::fabs(q) <= .425) {
    r = .180625 - q * q;
    return q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r +
                     67265.770927008700853) * r + 45921.953931549871457) * r +
                   13731.693765509461125) * r + 1971.5909503065514427) * r +
                 133.14166789178437745) * r + 3.387132872796366608) /
           (((((((r * 5226.495278852545925 + 28729.085735721942674) * r +
                 39307.89580009271061) * r + 21213.794301586595867) * r +
               5394.1960214247511077) * r + 687.1870074920579083) * r +
             42.313330701600911252) * r + 1.);
  }
  r = std::sqrt(-std::log((q > 0) ? (0.5 - p + 0.5) : p));
  if (r <= 5.) {
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r +
                .24178072517745061177) * r + 1.27045825245236838258) * r +
              3.64784832476320460504) * r + 5.7694972214606914055) * r +
            4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r +
                .0151986665636164571966) * r + .14810397642748007459) * r +
              .68976733498510000455) * r + 1.6763848301838038494) * r +
            2.05319162663775882187) * r + 1.);
  } else {
    r += -5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r +
                .0012426609473880784386) * r + .026532189526576123093) * r +
              .29656057182850489123) * r + 1.7848265399172913358) * r +
            5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r +
                1.8463183175100546818e-5) * r + 7.868691311456132591e-4) * r +
              .0148753612908506148525) * r + .13692988092273580531) * r +
            .59983220655588793769) * r + 1.);
  }
  return (q < 0.0) ? -val : val;
}

int dcor_batch_geometry(int64_t n, double eps1, double eps2, int family, int hrs, int64_t km[2]) {
  const double nd = (double)n;
  double md = std::ceil(8.0 / (eps1 * eps2));
  if (family == DCOR_FAMILY_SUBG && md > nd) md = nd;
  double kd = std::floor(nd / md);
  if (family == DCOR_FAMILY_SUBG && hrs && kd < 2) { kd = 2; md = std::floor(nd / kd); }
  km[0] = (int64_t)kd; km[1] = (int64_t)md;
  if (!(kd >= 1)) return fail(DCOR_EKLT1, "k = floor(n/m) < 1");
  return DCOR_OK;
}

// The one-pass sign path's replicate chunks: two slabs (two-stream chunk pipeline), each within a
// budget of >= 512 MiB and >= 2048 replicates' records, <= 4 GiB; equal chunks (no small tail
// launch).  At the headline's n that is four chunks of 2048 per 8192 replicates (round 2: chunks of
// 512-1024 measured 3-8 % slower, 4096 the same).  dcor_sim_launch and dcor_sim_chunking (bench.py's
// live ceilings) share it.
static void codes_chunking(int64_t n, int64_t rep_count, int64_t* chunk, int64_t* nchunks) {
  const size_t per_rep = (size_t)sign_rec_words(n) * sizeof(uint32_t);
  size_t budget = (size_t)512 << 20;
  if (budget < 2048 * per_rep) budget = 2048 * per_rep;
  if (budget > ((size_t)4 << 30)) budget = (size_t)4 << 30;
  int64_t maxchunk = (int64_t)(budget / per_rep);
  if (maxchunk < 1) maxchunk = 1;
  int64_t nch = (rep_count + maxchunk - 1) / maxchunk;
  if (nch == 1 && rep_count >= 512) nch = 2;  // two chunks at least: pass 2 of one beside pass 1 of the other
  *nchunks = nch;
  *chunk = nch > 0 ? (rep_count + nch - 1) / nch : 0;
}

int dcor_sim_launch(const dcor_cell* cell, int64_t rep_begin, int64_t rep_count,
                    dcor_rep_out* d_out, void* stream) {
  if (!cell || (rep_count > 0 && !d_out)) return fail(DCOR_EINVAL, "null argument");
  if (rep_begin < 0 || rep_count < 0 || rep_begin + rep_count > 0xffffffffLL)
    return fail(DCOR_EINVAL, "replicate range must lie in [0, 2^32)");
  if (rep_count > 0x7fffffffLL) return fail(DCOR_EINVAL, "rep_count too large for one launch");
  if (int st = need_device()) return st;
  const dcor_cell& c = *cell;
  CellPlan cp;
  if (int st = prepare_cell(c, cp)) return st;
  if (cp.nan_dgp) {  // every estimate NaN (see make_dgp); the estimators' own checks applied
    if (rep_count > 0)
      HIPCHK(hipMemsetAsync(d_out, 0xFF, sizeof(dcor_rep_out) * (size_t)rep_count, (hipStream_t)stream));
    return DCOR_OK;
  }
  int rc;
  if (cp.kind == GK_SUBG || cp.kind == GK_SUBG_W) {
    SubgConst k = cp.subg;
    k.rep_begin = rep_begin;
    rc = launch_subg_fused(k, rep_count, d_out, stream);
  } else {
    SignConst k = cp.sign;
    k.rep_begin = rep_begin;
    if ((cp.kind == GK_SIGN_BERN_W || cp.kind == GK_SIGN_BERN) && rep_count > 0) {
      // two-valued samples: bit-plane kernel (normalise = TRUE or FALSE)
      const size_t per_rep = (size_t)3 * 4 * (size_t)((c.n + 255) / 256) * sizeof(uint64_t) + 64;
      size_t budget = (size_t)1 << 30;
      if (budget < 2048 * per_rep) budget = 2048 * per_rep;
      int64_t chunk = (int64_t)(budget / per_rep);
      if (chunk < 1) chunk = 1;
      if (chunk > rep_count) chunk = rep_count;
      const size_t plane_bytes = ((size_t)chunk * (per_rep - 64) + 255) / 256 * 256;
      void* scratch = nullptr;
      if (int st = arena_get(plane_bytes + (size_t)chunk * 64, &scratch)) return st;  // clears pipe.sig
      rc = launch_sign_bern(k, rep_count, chunk, (uint64_t*)scratch,
                            (SignPartial*)((char*)scratch + plane_bytes), d_out, stream);
    } else if ((cp.kind != GK_SIGN_CODES && cp.kind != GK_SIGN_CODES_W) || rep_count == 0) {
      rc = launch_sign_fused(k, rep_count, d_out, stream);
    } else {
      const size_t per_rep = (size_t)sign_item_words(c.n, c.dgp) * sizeof(uint32_t);   // u16 records
      int64_t chunk = 0, nch = 0;
      codes_chunking(c.n, rep_count, &chunk, &nch);
      const size_t slab_b = ((size_t)chunk * per_rep + 255) / 256 * 256 + 256;  // + pass 2's over-read
      const size_t sums_b = ((size_t)chunk * (8 * sizeof(double) + 48) + 255) / 256 * 256;
      const int nbuf = nch > 1 ? 2 : 1;
      Ctx* cx = nullptr;
      if (int st = ctx_get(&cx)) return st;
      // the layout of the arena's last user, if that was this path (any other user cleared it)
      const uint64_t prev_sig = cx->pipe.sig;
      void* scratch = nullptr;
      if (int st = arena_get(nbuf * (slab_b + sums_b), &scratch)) return st;
      CodesBufs bf;
      char* base = (char*)scratch;
      for (int b = 0; b < 2; ++b) {
        const int bb = b < nbuf ? b : 0;
        bf.slab[b] = (uint32_t*)(base + bb * slab_b);
        bf.sums[b] = (double*)(base + nbuf * slab_b + bb * sums_b);
      }
      bf.lib[0] = bf.lib[1] = bf.ev_entry = bf.ev_end[0] = bf.ev_end[1] = nullptr;
      bf.cross = false;
      const char* pv = dcor::variant("DCOR_SIGN_PIPELINE");
      Pipe* pp = nullptr;
      if (int st = pipe_get(&pp)) return st;
      if (nbuf == 2 && !(pv && std::strcmp(pv, "0") == 0)) {
        bf.lib[0] = pp->s2; bf.lib[1] = pp->s;
        bf.ev_entry = pp->entry; bf.ev_end[0] = pp->end[0]; bf.ev_end[1] = pp->end[1];
        // calls of the same layout back to back: the next call's first chunks may start while
        // the previous call's last chunk finishes (DCOR_SIGN_XCALL=0 orders every call after the
        // caller's stream)
        const uint64_t sig = ((uint64_t)(uintptr_t)scratch * 1000003u) ^ ((uint64_t)slab_b * 31u) ^
                             ((uint64_t)sums_b << 1) ^ 1u;
        const char* xv = dcor::variant("DCOR_SIGN_XCALL");
        bf.cross = sig == prev_sig && !(xv && std::strcmp(xv, "0") == 0);
        pp->sig = sig;
      } else {
        pp->sig = 0;
      }
      rc = launch_sign_fused_codes(k, rep_count, chunk, bf, d_out, stream);
    }
  }
  if (rc) return hip_fail((hipError_t)rc, "sim kernel launch");
  return DCOR_OK;
}

int dcor_sim_chunking(const dcor_cell* cell, int64_t rep_count, int64_t* chunk, int64_t* nchunks) {
  if (!cell || !chunk || !nchunks || rep_count < 0) return fail(DCOR_EINVAL, "sim_chunking: bad arguments");
  CellPlan cp;
  if (int st = prepare_cell(*cell, cp)) return st;
  if ((cp.kind != GK_SIGN_CODES && cp.kind != GK_SIGN_CODES_W) || cp.nan_dgp || rep_count == 0) {
    *chunk = rep_count;
    *nchunks = rep_count > 0 ? 1 : 0;
    return DCOR_OK;
  }
  codes_chunking(cell->n, rep_count, chunk, nchunks);
  return DCOR_OK;
}

int dcor_diag_sign_pass(const dcor_cell* cell, int64_t rep_begin, int64_t reps, int which, void* stream) {
  if (!cell || reps < 1 || reps > 65535 || rep_begin < 0 || rep_begin + reps > 0xffffffffLL)
    return fail(DCOR_EINVAL, "diag_sign_pass: bad arguments");
  if ((which < 1 || which > 3) && (which < 11 || which > 15))
    return fail(DCOR_EINVAL, "diag_sign_pass: which must be 1-3 or 11-15");
  if (int st = need_device()) return st;
  CellPlan cp;
  if (int st = prepare_cell(*cell, cp)) return st;
  // a small cell (wave kernels) runs here in the workgroup kernels: the same records and tie
  // batches per replicate, results equal to the wave kernels' up to the order of the compensated
  // sums (passes 1-3 only; the ceilings are the headline's)
  if ((cp.kind != GK_SIGN_CODES && !(cp.kind == GK_SIGN_CODES_W && which <= 3)) || cp.nan_dgp)
    return fail(DCOR_EINVAL, "diag_sign_pass: the cell does not run the one-pass sign kernels");
  if (which > 10 && (cp.dgp != DCOR_DGP_GAUSSIAN || cp.sign.m != 8))
    return fail(DCOR_EINVAL, "diag_sign_pass: the ceilings run the Gaussian DGP at m = 8");
  SignConst k = cp.sign;
  k.rep_begin = rep_begin;
  const size_t slab_b = ((size_t)reps * sign_item_words(cell->n, cell->dgp) * sizeof(uint32_t) + 255) / 256 * 256 + 256;  // + pass 2's over-read
  const size_t sums_b = ((size_t)reps * SIGN_SUMS * sizeof(double) + 255) / 256 * 256;
  const size_t part_b = ((size_t)reps * SIGN_PARTIAL_BYTES + 255) / 256 * 256;
  void* scratch = nullptr;
  if (int st = arena_get(slab_b + sums_b + part_b + (size_t)reps * sizeof(dcor_rep_out), &scratch)) return st;
  char* b = (char*)scratch;
  const int rc = launch_sign_diag(k, reps, which, (uint32_t*)b, (double*)(b + slab_b), b + slab_b + sums_b,
                                  (dcor_rep_out*)(b + slab_b + sums_b + part_b), stream);
  if (rc) return hip_fail((hipError_t)rc, "diag_sign_pass launch");
  return DCOR_OK;
}

int dcor_diag_sign_ties(const dcor_cell* cell, int64_t rep_begin, int64_t reps, int64_t* h_ties) {
  if (!h_ties) return fail(DCOR_EINVAL, "diag_sign_ties: null output");
  if (int st = dcor_diag_sign_pass(cell, rep_begin, reps, 1, nullptr)) return st;
  if (int st = dcor_diag_sign_pass(cell, rep_begin, reps, 2, nullptr)) return st;
  void* scratch = nullptr;
  if (int st = arena_get(0, &scratch)) return st;   // the same arena dcor_diag_sign_pass used
  const size_t slab_b = ((size_t)reps * sign_item_words(cell->n, cell->dgp) * sizeof(uint32_t) + 255) / 256 * 256 + 256;  // + pass 2's over-read
  const size_t sums_b = ((size_t)reps * SIGN_SUMS * sizeof(double) + 255) / 256 * 256;
  std::vector<long long> part((size_t)reps * SIGN_PARTIAL_BYTES / sizeof(long long));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(part.data(), (char*)scratch + slab_b + sums_b, (size_t)reps * SIGN_PARTIAL_BYTES,
                   hipMemcpyDeviceToHost));
  const size_t words = SIGN_PARTIAL_BYTES / sizeof(long long);
  for (int64_t r = 0; r < reps; ++r) h_ties[r] = part[(size_t)r * words + words - 1] >> 8;
  return DCOR_OK;
}

int dcor_accumulate_launch(const dcor_rep_out* d_out, int64_t count, double rho,
                           dcor_accum* d_acc, void* stream) {
  if (!d_acc || (count > 0 && !d_out) || count < 0) return fail(DCOR_EINVAL, "bad accumulate arguments");
  if (int st = need_device()) return st;
  const int rc = launch_accumulate(d_out, count, rho, d_acc, stream);
  if (rc) return hip_fail((hipError_t)rc, "accumulate launch");
  return DCOR_OK;
}

static void dd_add_host(double* a, const double* b) {  // a += b (double-double)
  auto two_sum = [](double x, double y, double& s, double& e) {
    s = x + y;
    const double bb = s - x;
    e = (x - (s - bb)) + (y - bb);
  };
  double s, e, t, f;
  two_sum(a[0], b[0], s, e);
  two_sum(a[1], b[1], t, f);
  e += t;
  double s2, e2;
  two_sum(s, e, s2, e2);
  e2 += f;
  two_sum(s2, e2, a[0], a[1]);
}

void dcor_accum_merge(dcor_accum* dst, const dcor_accum* src) {
  dst->n += src->n; dst->n_cover += src->n_cover; dst->n_cover_na += src->n_cover_na;
  dst->n_na_est += src->n_na_est; dst->n_na_ci += src->n_na_ci;
  dd_add_host(dst->est, src->est); dd_add_host(dst->est2, src->est2);
  dd_add_host(dst->se2, src->se2); dd_add_host(dst->len, src->len);
  dd_add_host(dst->lo, src->lo); dd_add_host(dst->hi, src->hi);
}

void dcor_accum_finalize(const dcor_accum* a, double rho, dcor_summary* out) {
  // vert-cor.R:422-430: mse = mean(se2), bias = mean(est) - rho, var = var(est),
  // coverage = mean(cover), ci_length = mean(up - lo); NA propagates like R's mean/var.
  const double n = (double)a->n;
  const long double est = (long double)a->est[0] + a->est[1];
  const long double est2 = (long double)a->est2[0] + a->est2[1];
  const bool nae = a->n_na_est > 0, nac = a->n_na_ci > 0;
  out->mse = nae || a->n == 0 ? NAN : (double)(((long double)a->se2[0] + a->se2[1]) / n);
  out->bias = nae || a->n == 0 ? NAN : (double)(est / n) - rho;
  out->var = (nae || a->n < 2) ? NAN : (double)((est2 - est * est / n) / (n - 1));
  out->coverage = (a->n_cover_na > 0 || a->n == 0) ? NAN : (double)a->n_cover / n;
  out->ci_length = nac || a->n == 0 ? NAN : (double)(((long double)a->len[0] + a->len[1]) / n);
}

int dcor_premat_sign_launch(const dcor_premat_sign* d, dcor_rep_out* d_out, void* stream) {
  if (!d || !d_out || d->reps < 0) return fail(DCOR_EINVAL, "null argument");
  if (!d->X || !d->Y || !d->lap_ni_sc || !d->lap_ni_x || !d->lap_ni_y || !d->lap_int_sc ||
      !d->flips || !d->lap_z || !d->mix_z || !d->mix_l)
    return fail(DCOR_EINVAL, "premat_sign: every input array is required");
  if (int st = need_device()) return st;
  PrematSignConst p;
  std::memset(&p, 0, sizeof(p));
  if (int st = make_sign(d->n, d->eps1, d->eps2, d->alpha, d->normalise, d->ci_mode, d->nsim,
                         false, p.s)) return st;
  p.X = d->X; p.Y = d->Y; p.xy_stride = d->xy_stride;
  p.lap_ni_sc = d->lap_ni_sc; p.lap_ni_x = d->lap_ni_x; p.lap_ni_y = d->lap_ni_y;
  p.lap_int_sc = d->lap_int_sc; p.flips = d->flips; p.flip_words = (d->n + 31) / 32;
  p.lap_z = d->lap_z; p.mix_z = d->mix_z; p.mix_l = d->mix_l;
  const int rc = launch_premat_sign(p, d->reps, d_out, stream);
  if (rc) return hip_fail((hipError_t)rc, "premat_sign launch");
  return DCOR_OK;
}

static int premat_subg_const(const dcor_premat_subg* d, PrematSubgConst& p) {
  std::memset(&p, 0, sizeof(p));
  if (int st = make_subg(d->n, d->eps1, d->eps2, d->eta1, d->eta2, d->alpha, d->hrs, d->lam_x,
                         d->lam_y, d->lam_s, d->lam_o, d->lam_r, d->delta, d->nsim, p.s, &p.lo_,
                         &p.crit_sqrt2_s)) return st;
  p.hrs = d->hrs ? 1 : 0;
  // element-aligned arrays (the streaming kernels read 16 B at a time from the first 16-B
  // boundary of each row)
  const uintptr_t mis8 = ((uintptr_t)d->X | (uintptr_t)d->Y | (uintptr_t)d->lap_ni_x |
                          (uintptr_t)d->lap_ni_y | (uintptr_t)d->lap_local |
                          (uintptr_t)d->lap_central | (uintptr_t)d->mix_z | (uintptr_t)d->mix_l) & 7;
  if (mis8 || ((uintptr_t)d->perm & 3))
    return fail(DCOR_EINVAL, "premat_subg: arrays must be aligned to their element size");
  p.X = d->X; p.Y = d->Y; p.xy_stride = d->xy_stride; p.perm = d->perm;
  p.lap_ni_x = d->lap_ni_x; p.lap_ni_y = d->lap_ni_y; p.lap_local = d->lap_local;
  p.lap_central = d->lap_central; p.mix_z = d->mix_z; p.mix_l = d->mix_l;
  return DCOR_OK;
}

}  // extern "C" (reopened below)

struct dcor_panel {
  const double* X;
  const double* Y;
  int64_t n;
  void* buf;          // codes (n u16, 256-B padded) | 512 dictionary doubles | ok flag
  size_t codes_b;
  void* stream;
  int coded;          // host copy of the device flag (read once at create)
  uint16_t* codes() const { return (uint16_t*)buf; }
  double* dict() const { return (double*)((char*)buf + codes_b); }
  int* ok() const { return (int*)((char*)buf + codes_b + 512 * sizeof(double)); }
};

static int premat_subg_run(const dcor_premat_subg* d, const dcor_panel* panel, dcor_rep_out* d_out,
                           void* stream, void* scratch = nullptr, size_t scratch_b = 0);

// The Philox noise of HRS replicates materialised in HBM (the dcor_perm_launch /
// dcor_draws_launch sites of the fused kernel's contract, all seven arrays from one
// launch_hrs_noise), then the pre-materialised panel kernels: the pipeline of dcor.hrs.hrs_replicates(rng='philox', mode='premat'), natively.
// hrs_noise_per: bytes of one replicate's noise; hrs_premat_chunks runs d->reps replicates in
// chunks of cr over the caller's stream-ordered buffer of per * cr bytes.
static size_t hrs_al(size_t b) { return (b + 255) & ~(size_t)255; }

static int hrs_noise_geometry(const dcor_premat_subg* d, int64_t* k, int64_t* m, size_t* per) {
  int64_t km[2];
  if (int st = dcor_batch_geometry(d->n, d->eps1, d->eps2, DCOR_FAMILY_SUBG, 1, km)) return st;
  *k = km[0]; *m = km[1];
  *per = hrs_al((size_t)km[0] * km[1] * 4) + 2 * hrs_al((size_t)km[0] * 8) +
         hrs_al((size_t)d->n * 8) + 256 + 2 * hrs_al((size_t)d->nsim * 8);
  return DCOR_OK;
}

static int hrs_premat_chunks(const dcor_premat_subg* d, const dcor_panel* panel, uint64_t seed_ni,
                             uint64_t seed_int, int64_t rep_begin, dcor_rep_out* d_out, char* buf,
                             int64_t cr, int64_t k, int64_t m, void* stream,
                             void* scratch = nullptr, size_t scratch_b = 0) {
  const int64_t n = d->n, ns = d->nsim;
  int32_t* perm = (int32_t*)buf;
  double* lx = (double*)(buf + hrs_al((size_t)cr * k * m * 4));
  double* ly = lx + (hrs_al((size_t)cr * k * 8) / 8);
  double* ll = ly + (hrs_al((size_t)cr * k * 8) / 8);
  double* lc = ll + (hrs_al((size_t)cr * n * 8) / 8);
  double* mz = lc + (hrs_al((size_t)cr * 8) / 8);
  double* ml = mz + (hrs_al((size_t)cr * ns * 8) / 8);
  for (int64_t r0 = 0; r0 < d->reps; r0 += cr) {
    const int64_t nr = d->reps - r0 < cr ? d->reps - r0 : cr;
    const HrsNoise j{seed_ni, seed_int, rep_begin + r0, n, k, k * m, ns, perm, lx, ly, ll, lc, mz, ml};
    if (int rc = launch_hrs_noise(j, nr, stream)) return hip_fail((hipError_t)rc, "hrs noise launch");
    dcor_premat_subg q = *d;
    q.reps = nr;
    q.perm = perm; q.lap_ni_x = lx; q.lap_ni_y = ly; q.lap_local = ll; q.lap_central = lc;
    q.mix_z = mz; q.mix_l = ml;
    if (int e = premat_subg_run(&q, panel, d_out + r0, stream, scratch, scratch_b)) return e;
  }
  return DCOR_OK;
}

// chunk of replicates whose noise fits `budget` bytes, capped at `cap`
static int64_t hrs_chunk(size_t per, int64_t reps, size_t budget, int64_t cap) {
  int64_t cr = (int64_t)(budget / per);
  if (cr < 1) cr = 1;
  if (cr > cap) cr = cap;
  return cr > reps ? reps : cr;
}

// dcor_hrs_fused_launch on an uncoded panel too large for the LDS index row (n > 65536): the
// same Philox streams materialised per chunk, then the pre-materialised panel kernels --
// replicate r equals the fused kernel's replicate r within the compensated sums' rounding, as
// for any panel.
static int hrs_fused_materialised(const dcor_premat_subg* d, const dcor_panel* panel,
                                  uint64_t seed_ni, uint64_t seed_int, int64_t rep_begin,
                                  dcor_rep_out* d_out, void* stream) {
  int64_t k, m;
  size_t per;
  if (int st = hrs_noise_geometry(d, &k, &m, &per)) return st;
  const int64_t cr = hrs_chunk(per, d->reps, (size_t)1 << 30, 65535);
  if (cr == 0) return DCOR_OK;
  char* buf = nullptr;
  const hipStream_t st = (hipStream_t)stream;
  if (hipMallocAsync((void**)&buf, per * (size_t)cr, st) != hipSuccess) {
    (void)hipGetLastError();
    return fail(DCOR_ENOMEM, "hrs_fused: cannot allocate %zu noise bytes", per * (size_t)cr);
  }
  count_alloc();
  const int e = hrs_premat_chunks(d, panel, seed_ni, seed_int, rep_begin, d_out, buf, cr, k, m, stream);
  (void)hipFreeAsync(buf, st);
  return e;
}

extern "C" {

int dcor_panel_create(const double* d_X, const double* d_Y, int64_t n, void* stream,
                      dcor_panel** out) {
  if (!d_X || !d_Y || !out || n < 1) return fail(DCOR_EINVAL, "panel_create: bad arguments");
  if (int st = need_device()) return st;
  *out = nullptr;
  dcor_panel* pn = new dcor_panel();
  pn->X = d_X; pn->Y = d_Y; pn->n = n; pn->stream = stream;
  pn->codes_b = ((size_t)n * 2 + 255) & ~(size_t)255;
  if (hipMalloc(&pn->buf, pn->codes_b + 512 * sizeof(double) + 256) != hipSuccess) {
    (void)hipGetLastError();
    delete pn;
    return fail(DCOR_ENOMEM, "panel_create: cannot allocate the coded panel");
  }
  count_alloc();
  int rc = 0;
  if (n <= DCOR_DICT_NMAX && premat_dict_lds_bytes(n) <= 150 * 1024)
    rc = launch_panel_dict(d_X, d_Y, n, pn->codes(), pn->dict(), pn->ok(), stream);
  else
    rc = (int)hipMemsetAsync(pn->ok(), 0, sizeof(int), (hipStream_t)stream);
  if (!rc) rc = (int)hipMemcpyAsync(&pn->coded, pn->ok(), sizeof(int), hipMemcpyDeviceToHost,
                                     (hipStream_t)stream);
  if (!rc) rc = (int)hipStreamSynchronize((hipStream_t)stream);
  if (rc) {
    (void)hipFree(pn->buf);
    delete pn;
    return hip_fail((hipError_t)rc, "panel_create");
  }
  *out = pn;
  return DCOR_OK;
}

int dcor_panel_coded(const dcor_panel* pn, int* coded) {
  if (!pn || !coded) return fail(DCOR_EINVAL, "panel_coded: null argument");
  *coded = pn->coded;
  return DCOR_OK;
}

int dcor_panel_destroy(dcor_panel* pn) {
  if (!pn) return DCOR_OK;
  (void)hipStreamSynchronize((hipStream_t)pn->stream);
  const hipError_t e = hipFree(pn->buf);
  delete pn;
  return e == hipSuccess ? DCOR_OK : hip_fail(e, "panel_destroy");
}

int dcor_premat_subg_panel_launch(const dcor_premat_subg* d, const dcor_panel* panel,
                                  dcor_rep_out* d_out, void* stream) {
  if (!panel) return fail(DCOR_EINVAL, "premat_subg_panel: null panel");
  if (!d || d->X != panel->X || d->Y != panel->Y || d->xy_stride != 0 || d->n != panel->n)
    return fail(DCOR_EINVAL, "premat_subg_panel: X, Y, n must be the panel's and xy_stride 0");
  return premat_subg_run(d, panel, d_out, stream);
}

int dcor_premat_subg_launch(const dcor_premat_subg* d, dcor_rep_out* d_out, void* stream) {
  return premat_subg_run(d, nullptr, d_out, stream);
}

int dcor_hrs_fused_launch(const dcor_premat_subg* d, const dcor_panel* panel, uint64_t seed_ni,
                          uint64_t seed_int, int64_t rep_begin, dcor_rep_out* d_out, void* stream) {
  if (!d || !panel || d->reps < 0 || (d->reps > 0 && !d_out))
    return fail(DCOR_EINVAL, "hrs_fused: null argument");
  if (d->X != panel->X || d->Y != panel->Y || d->xy_stride != 0 || d->n != panel->n)
    return fail(DCOR_EINVAL, "hrs_fused: X, Y, n must be the panel's and xy_stride 0");
  if (!d->hrs) return fail(DCOR_EINVAL, "hrs_fused: the HRS variant only (hrs = 1)");
  if (rep_begin < 0 || rep_begin + d->reps > 0xffffffffLL)
    return fail(DCOR_EINVAL, "hrs_fused: replicate range exceeds 2^32");
  if (int st = need_device()) return st;
  PrematSubgConst p;
  if (int st = premat_subg_const(d, p)) return st;
  // DCOR_HRS_FUSED_L2=1 runs a coded panel through the uncoded kernel (A/B and the tests'
  // bit-identity check of the two kernels)
  const bool force_l2 = [] {
    const char* e = dcor::variant("DCOR_HRS_FUSED_L2");
    return e && std::strcmp(e, "1") == 0;
  }();
  const bool coded = panel->coded && !force_l2;
  if (!coded && d->n > DCOR_DICT_NMAX)
    return hrs_fused_materialised(d, panel, seed_ni, seed_int, rep_begin, d_out, stream);
  p.perm = nullptr; p.lap_ni_x = p.lap_ni_y = p.lap_local = p.lap_central = nullptr;
  p.mix_z = p.mix_l = nullptr;
  if (coded) {
    p.dict_codes = panel->codes(); p.dict_vals = panel->dict(); p.dict_ok = panel->ok();
    p.dict_built = 2;
  } else {
    p.dict_codes = nullptr; p.dict_vals = nullptr; p.dict_ok = nullptr;
  }
  if (d->reps == 0) return DCOR_OK;
  const size_t part_b = ((size_t)d->reps * 80 + 255) & ~(size_t)255;
  const size_t pack_b = coded ? 0 : (size_t)d->n * 32;  // xyc | soc (uncoded kernel)
  const size_t bytes = part_b + pack_b;
  void* part = nullptr;
  if (hipMallocAsync(&part, bytes, (hipStream_t)stream) != hipSuccess) {
    (void)hipGetLastError();
    return fail(DCOR_ENOMEM, "hrs_fused: cannot allocate %zu scratch bytes", bytes);
  }
  count_alloc();
  if (!coded) {
    p.xyc = (const double2*)((char*)part + part_b);
    p.soc = p.xyc + d->n;
  }
  const int rc = launch_hrs_fused(p, seed_ni, seed_int, rep_begin, d->reps, part, d_out, stream);
  (void)hipFreeAsync(part, (hipStream_t)stream);
  if (rc) return hip_fail((hipError_t)rc, "hrs_fused launch");
  return DCOR_OK;
}

int dcor_hrs_sweep_launch(const dcor_premat_subg* base, const dcor_panel* panel,
                          const dcor_hrs_segment* segs, int64_t nseg, dcor_rep_out* d_out,
                          void* stream) {
  if (!base || !panel || nseg < 0 || (nseg > 0 && (!segs || !d_out)))
    return fail(DCOR_EINVAL, "hrs_sweep: null argument");
  if (base->X != panel->X || base->Y != panel->Y || base->xy_stride != 0 || base->n != panel->n)
    return fail(DCOR_EINVAL, "hrs_sweep: X, Y, n must be the panel's and xy_stride 0");
  if (!base->hrs) return fail(DCOR_EINVAL, "hrs_sweep: the HRS variant only (hrs = 1)");
  if (!(base->delta > 0.0)) return fail(DCOR_EINVAL, "hrs_sweep: delta must be positive");
  // every segment's constants and geometry first: nothing is enqueued for an invalid sweep
  struct SegPlan {
    dcor_premat_subg q;
    int64_t k, m, cr;
  };
  std::vector<SegPlan> plan((size_t)nseg);
  size_t need = 0;
  int64_t cap = 0;
  // noise of up to 8192 replicates per launch chain (C5's 8192 x 420 KB: 3.4 GB), at most 4 GB
  const size_t budget = (size_t)4 << 30;
  for (int64_t i = 0; i < nseg; ++i) {
    const dcor_hrs_segment& g = segs[i];
    if (g.reps < 0 || g.rep_begin < 0 || g.out_row < 0 || !(g.eps > 0.0))
      return fail(DCOR_EINVAL, "hrs_sweep: segment %lld: need eps > 0, reps, rep_begin, out_row >= 0",
                  (long long)i);
    if (g.rep_begin + g.reps > 0xffffffffLL)
      return fail(DCOR_EINVAL, "hrs_sweep: segment %lld: replicate range exceeds 2^32", (long long)i);
    SegPlan& sp = plan[(size_t)i];
    dcor_premat_subg& q = sp.q;
    q = *base;
    q.reps = g.reps;
    q.eps1 = q.eps2 = g.eps;
    q.eta1 = q.eta2 = 1.0;
    q.lam_r = dcor_lambda_receiver_from_noise(base->lam_s, base->lam_o, g.eps, base->delta);
    PrematSubgConst pc;   // the launch constants' own checks, here rather than mid-sweep
    if (int st = premat_subg_const(&q, pc)) return st;
    size_t per;
    if (int st = hrs_noise_geometry(&q, &sp.k, &sp.m, &per)) return st;
    sp.cr = hrs_chunk(per, g.reps, budget, 8192);
    need = std::max(need, per * (size_t)sp.cr);
    cap = std::max(cap, sp.cr);
  }
  if (need == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  // the premat launches' partials (80 B per replicate slice) and packed panel (uncoded: 32 B
  // per sample) follow the noise: one allocation per call, reused launch after launch in
  // stream order
  const size_t scr_b = hrs_al((size_t)cap * 80 * DCOR_DICT_SLICES) + hrs_al((size_t)base->n * 32);
  char* buf = nullptr;
  const hipStream_t st = (hipStream_t)stream;
  if (hipMallocAsync((void**)&buf, need + scr_b, st) != hipSuccess) {
    (void)hipGetLastError();
    return fail(DCOR_ENOMEM, "hrs_sweep: cannot allocate %zu noise bytes", need + scr_b);
  }
  count_alloc();
  int e = DCOR_OK;
  for (int64_t i = 0; i < nseg && !e; ++i) {
    const dcor_hrs_segment& g = segs[i];
    const SegPlan& sp = plan[(size_t)i];
    if (g.reps == 0) continue;
    e = hrs_premat_chunks(&sp.q, panel, g.seed_ni, g.seed_int, g.rep_begin, d_out + g.out_row, buf,
                          sp.cr, sp.k, sp.m, stream, buf + need, scr_b);
  }
  (void)hipFreeAsync(buf, st);
  return e;
}

}  // extern "C" (reopened below)

static int premat_subg_run(const dcor_premat_subg* d, const dcor_panel* panel, dcor_rep_out* d_out,
                           void* stream, void* scratch, size_t scratch_b) {
  if (!d || !d_out || d->reps < 0) return fail(DCOR_EINVAL, "null argument");
  if (!d->X || !d->Y || !d->lap_ni_x || !d->lap_ni_y || !d->lap_local || !d->lap_central ||
      !d->mix_z || !d->mix_l)
    return fail(DCOR_EINVAL, "premat_subg: every input array except perm is required");
  if (int st = need_device()) return st;
  PrematSubgConst p;
  if (int st = premat_subg_const(d, p)) return st;
  // stream-ordered scratch for the stream -> epilogue partials: safe under concurrent
  // launches on different streams.
  // HRS over one shared panel: the packed clipped panel (2 x n x 16 B) follows the partials.
  // a prepared panel's path is known on the host: launch only the kernel that does the work
  const bool pack = p.hrs && p.perm && p.xy_stride == 0 && !(panel != nullptr && panel->coded);
  // Shared panel + random batches: try the dictionary-coded LDS kernel first (the device
  // decides; the packed L2-gather kernel is the fallback).
  const bool dict = p.perm && p.xy_stride == 0 && p.s.n <= DCOR_DICT_NMAX &&
                    premat_dict_lds_bytes(p.s.n) <= 150 * 1024 && panel == nullptr;
  // partials: 80 B per replicate slice (a prepared coded panel slices each replicate)
  const int64_t pslots = (panel != nullptr && panel->coded) ? DCOR_DICT_SLICES : 1;
  const size_t part_b = ((size_t)d->reps * 80 * pslots + 255) & ~(size_t)255;
  const size_t pack_b = pack ? (size_t)p.s.n * 32 : 0;
  const size_t codes_b = dict ? (((size_t)p.s.n * 2 + 255) & ~(size_t)255) : 0;
  const size_t dict_b = dict ? 2 * 256 * sizeof(double) + 256 : 0;
  const size_t bytes = part_b + pack_b + codes_b + dict_b;
  // a caller's stream-ordered scratch (the sweep's) when it is large enough: no per-launch
  // pool allocation, whose cross-stream reuse would order one stream's launches after another's
  const bool own = !(scratch != nullptr && scratch_b >= bytes);
  void* part = own ? nullptr : scratch;
  if (own) {
    if (hipMallocAsync(&part, bytes, (hipStream_t)stream) != hipSuccess) {
      (void)hipGetLastError();
      return fail(DCOR_ENOMEM, "premat sub-G: cannot allocate %zu scratch bytes", bytes);
    }
    count_alloc();
  }
  if (pack) {
    p.xyc = (const double2*)((char*)part + part_b);
    p.soc = p.xyc + p.s.n;
  }
  if (dict) {
    char* q = (char*)part + part_b + pack_b;
    p.dict_codes = (uint16_t*)q;
    p.dict_vals = (double*)(q + codes_b);
    p.dict_ok = (int*)(q + codes_b + 2 * 256 * sizeof(double));
  } else if (panel != nullptr && p.perm && panel->coded) {
    p.dict_codes = panel->codes();
    p.dict_vals = panel->dict();
    p.dict_ok = panel->ok();
    p.dict_built = 2;  // built and known coded: no L2-gather launch
  }
  int rc = 0;
  const char* pv = dcor::variant("DCOR_PREMAT_PIPELINE");
  if (panel != nullptr && panel->coded && p.perm && d->reps >= 4096 && pv && std::strcmp(pv, "1") == 0) {
    // DCOR_PREMAT_PIPELINE=1: two replicate halves, the first half's mixquant epilogue on the
    // auxiliary stream beside the second half's streaming kernel.  Off by default: the
    // streaming kernel already reads at ~5.8 TB/s, and the epilogue's workgroups beside it
    // cost more than they hide (r01 A/B: 12.5e6 piped vs 13.0e6 serial replicates/s).
    Pipe* pp = nullptr;
    if (int st = pipe_get(&pp)) {
      if (own) (void)hipFreeAsync(part, (hipStream_t)stream);
      return st;
    }
    const int64_t half = d->reps / 2;
    for (int h = 0; h < 2 && !rc; ++h) {
      const int64_t r0 = h ? half : 0, nr = h ? d->reps - half : half;
      PrematSubgConst q = p;
      const int64_t km = p.s.k * p.s.m, n = p.s.n, ns = p.s.mix.nsim;
      q.perm = p.perm + r0 * km;
      q.lap_ni_x = p.lap_ni_x + r0 * p.s.k;
      q.lap_ni_y = p.lap_ni_y + r0 * p.s.k;
      q.lap_local = p.lap_local + r0 * n;
      q.lap_central = p.lap_central + r0;
      q.mix_z = p.mix_z + r0 * ns;
      q.mix_l = p.mix_l + r0 * ns;
      rc = launch_premat_subg(q, nr, (char*)part + r0 * 80 * pslots, d_out + r0, stream, h ? nullptr : pp->s,
                              pp->fork);
    }
    if (!rc && hipEventRecord(pp->join, pp->s) != hipSuccess) rc = (int)hipGetLastError();
    if (!rc && hipStreamWaitEvent((hipStream_t)stream, pp->join, 0) != hipSuccess) rc = (int)hipGetLastError();
  } else {
    // the tiled path's INT kernel may run on the auxiliary stream (DCOR_TILED_INT=2)
    Pipe* pp = nullptr;
    const char* iv = dcor::variant("DCOR_TILED_INT");
    if (iv && std::strcmp(iv, "2") == 0 && pipe_get(&pp) != 0) pp = nullptr;
    rc = launch_premat_subg(p, d->reps, part, d_out, stream, nullptr, nullptr, pp ? pp->s : nullptr,
                            pp ? pp->fork : nullptr, pp ? pp->join : nullptr);
  }
  if (own) (void)hipFreeAsync(part, (hipStream_t)stream);
  if (rc) return hip_fail((hipError_t)rc, "premat_subg launch");
  return DCOR_OK;
}

extern "C" {

int dcor_panel_dict_probe(const double* d_X, const double* d_Y, int64_t n, int* ok) {
  if (!d_X || !d_Y || !ok || n < 1) return fail(DCOR_EINVAL, "panel_dict_probe: bad arguments");
  if (int st = need_device()) return st;
  *ok = 0;
  if (n > DCOR_DICT_NMAX) return DCOR_OK;
  DevBuf buf;
  const size_t codes_b = ((size_t)n * 2 + 255) & ~(size_t)255;
  HIPCHK(buf.alloc(codes_b + 512 * sizeof(double) + 256));
  char* q = (char*)buf.p;
  int* d_ok = (int*)(q + codes_b + 512 * sizeof(double));
  const int rc = launch_panel_dict(d_X, d_Y, n, (uint16_t*)q, (double*)(q + codes_b), d_ok, nullptr);
  if (rc) return hip_fail((hipError_t)rc, "panel_dict launch");
  HIPCHK(hipMemcpy(ok, d_ok, sizeof(int), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

// ------------------------------------------- single-call host-pointer forms
static int run_premat_sign_1(const double* X, const double* Y, int64_t n, double eps1,
                             double eps2, double alpha, int normalise, int mode, bool int_only,
                             const double* lap_ni_sc, const double* lap_x, const double* lap_y,
                             const double* lap_int_sc, const uint8_t* flips, double lap_z,
                             const double* mix_z, const double* mix_l, int64_t nsim,
                             dcor_rep_out* res) {
  if (!X || !Y) return fail(DCOR_EINVAL, "X and Y are required");
  if (int st = need_device()) return st;
  PrematSignConst p;
  std::memset(&p, 0, sizeof(p));
  if (int st = make_sign(n, eps1, eps2, alpha, normalise, mode, nsim > 0 ? nsim : 1, int_only, p.s)) return st;
  const int64_t k = p.s.k;
  std::vector<uint32_t> fw((size_t)((n + 31) / 32), 0u);
  if (flips)
    for (int64_t i = 0; i < n; ++i) if (flips[i]) fw[(size_t)(i >> 5)] |= (1u << (i & 31));
  DevBuf bX, bY, bnsc, blx, bly, bisc, bfl, bz, bmz, bml, bout;
  if (int st = upload(bX, X, (size_t)n)) return st;
  if (int st = upload(bY, Y, (size_t)n)) return st;
  if (int st = upload(bnsc, lap_ni_sc, 4)) return st;
  if (int st = upload(blx, lap_x, (size_t)k)) return st;
  if (int st = upload(bly, lap_y, (size_t)k)) return st;
  if (int st = upload(bisc, lap_int_sc, 4)) return st;
  if (int st = upload(bfl, fw.data(), fw.size())) return st;
  if (int st = upload(bz, &lap_z, 1)) return st;
  const size_t ns = (size_t)p.s.mix.nsim;
  if (int st = upload(bmz, mix_z, mix_z ? ns : ns)) return st;
  if (int st = upload(bml, mix_l, ns)) return st;
  HIPCHK(bout.alloc(sizeof(dcor_rep_out)));
  p.X = bX.as<double>(); p.Y = bY.as<double>(); p.xy_stride = 0;
  p.lap_ni_sc = bnsc.as<double>(); p.lap_ni_x = blx.as<double>(); p.lap_ni_y = bly.as<double>();
  p.lap_int_sc = bisc.as<double>(); p.flips = bfl.as<uint32_t>(); p.flip_words = (n + 31) / 32;
  p.lap_z = bz.as<double>(); p.mix_z = bmz.as<double>(); p.mix_l = bml.as<double>();
  const int rc = launch_premat_sign(p, 1, bout.as<dcor_rep_out>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "premat_sign launch");
  HIPCHK(hipMemcpy(res, bout.p, sizeof(dcor_rep_out), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_ci_ni_signbatch(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                         double alpha, int normalise, const double lap_sc[4],
                         const double* lap_x, const double* lap_y, double out[3]) {
  if (!out || !lap_x || !lap_y || (normalise && !lap_sc)) return fail(DCOR_EINVAL, "null argument");
  dcor_rep_out r;
  if (int st = run_premat_sign_1(X, Y, n, eps1, eps2, alpha, normalise, DCOR_MODE_LAPLACE, false,
                                 lap_sc, lap_x, lap_y, lap_sc, nullptr, 0.0, nullptr, nullptr, 1, &r))
    return st;
  out[0] = r.ni_hat; out[1] = r.ni_lo; out[2] = r.ni_hi;
  return DCOR_OK;
}

int dcor_ci_int_signflip(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                         double alpha, int mode, int normalise, const double lap_sc[4],
                         const uint8_t* flips, double lap_z, const double* mix_z,
                         const double* mix_l, int64_t nsim, double out[3]) {
  if (!out || !flips || (normalise && !lap_sc)) return fail(DCOR_EINVAL, "null argument");
  dcor_rep_out r;
  if (int st = run_premat_sign_1(X, Y, n, eps1, eps2, alpha, normalise, mode, true, lap_sc,
                                 nullptr, nullptr, lap_sc, flips, lap_z, mix_z, mix_l, nsim, &r))
    return st;
  out[0] = r.int_hat; out[1] = r.int_lo; out[2] = r.int_hi;
  return DCOR_OK;
}

static int run_premat_subg_1(const double* X, const double* Y, int64_t n, double eps1,
                             double eps2, double eta1, double eta2, double alpha, int hrs,
                             double lam_x, double lam_y, double lam_s, double lam_o,
                             double lam_r, double delta, const int32_t* perm,
                             const double* lap_x, const double* lap_y, const double* lap_local,
                             double lap_central, const double* mix_z, const double* mix_l,
                             int64_t nsim, dcor_rep_out* res) {
  if (!X || !Y) return fail(DCOR_EINVAL, "X and Y are required");
  if (int st = need_device()) return st;
  dcor_premat_subg d;
  std::memset(&d, 0, sizeof(d));
  d.n = n; d.reps = 1; d.eps1 = eps1; d.eps2 = eps2; d.eta1 = eta1; d.eta2 = eta2; d.alpha = alpha;
  d.hrs = hrs; d.lam_x = lam_x; d.lam_y = lam_y; d.lam_s = lam_s; d.lam_o = lam_o;
  d.lam_r = lam_r; d.delta = delta; d.nsim = nsim > 0 ? nsim : 1;
  PrematSubgConst p;
  if (int st = premat_subg_const(&d, p)) return st;
  const int64_t k = p.s.k, m = p.s.m;
  DevBuf bX, bY, bp, blx, bly, bll, bc, bmz, bml, bout;
  if (int st = upload(bX, X, (size_t)n)) return st;
  if (int st = upload(bY, Y, (size_t)n)) return st;
  if (perm) { if (int st = upload(bp, perm, (size_t)(k * m))) return st; }
  if (int st = upload(blx, lap_x, (size_t)k)) return st;
  if (int st = upload(bly, lap_y, (size_t)k)) return st;
  if (int st = upload(bll, lap_local, (size_t)n)) return st;
  if (int st = upload(bc, &lap_central, 1)) return st;
  const size_t ns = (size_t)p.s.mix.nsim;
  if (int st = upload(bmz, mix_z, ns)) return st;
  if (int st = upload(bml, mix_l, ns)) return st;
  HIPCHK(bout.alloc(sizeof(dcor_rep_out)));
  p.X = bX.as<double>(); p.Y = bY.as<double>(); p.xy_stride = 0;
  p.perm = perm ? bp.as<int32_t>() : nullptr;
  p.lap_ni_x = blx.as<double>(); p.lap_ni_y = bly.as<double>(); p.lap_local = bll.as<double>();
  p.lap_central = bc.as<double>(); p.mix_z = bmz.as<double>(); p.mix_l = bml.as<double>();
  DevBuf bpart;
  HIPCHK(bpart.alloc(80));
  const int rc = launch_premat_subg(p, 1, bpart.p, bout.as<dcor_rep_out>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "premat_subg launch");
  HIPCHK(hipMemcpy(res, bout.p, sizeof(dcor_rep_out), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_correlation_ni_subg(const double* X, const double* Y, int64_t n, double eps1,
                             double eps2, double eta1, double eta2, double alpha, int hrs,
                             double lam_x, double lam_y, const int32_t* perm,
                             const double* lap_x, const double* lap_y, double out[3]) {
  if (!out || !lap_x || !lap_y) return fail(DCOR_EINVAL, "null argument");
  dcor_rep_out r;
  if (int st = run_premat_subg_1(X, Y, n, eps1, eps2, eta1, eta2, alpha, hrs, lam_x, lam_y, NAN,
                                 NAN, NAN, NAN, perm, lap_x, lap_y, nullptr, 0.0, nullptr,
                                 nullptr, 1, &r)) return st;
  out[0] = r.ni_hat; out[1] = r.ni_lo; out[2] = r.ni_hi;
  return DCOR_OK;
}

int dcor_ci_int_subg(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                     double eta1, double eta2, double alpha, int hrs, double lam_s,
                     double lam_o, double lam_r, double delta, const double* lap_local,
                     double lap_central, const double* mix_z, const double* mix_l,
                     int64_t nsim, double out[3]) {
  if (!out || !lap_local || !mix_z || !mix_l) return fail(DCOR_EINVAL, "null argument");
  dcor_rep_out r;
  if (int st = run_premat_subg_1(X, Y, n, eps1, eps2, eta1, eta2, alpha, hrs, NAN, NAN, lam_s,
                                 lam_o, lam_r, delta, nullptr, nullptr, nullptr, lap_local,
                                 lap_central, mix_z, mix_l, nsim, &r)) return st;
  out[0] = r.int_hat; out[1] = r.int_lo; out[2] = r.int_hi;
  return DCOR_OK;
}

int dcor_mixquant(const double* z, const double* l, int64_t nsim, double c, double p,
                  double* out) {
  if (!z || !l || !out) return fail(DCOR_EINVAL, "null argument");
  if (nsim < 1 || nsim > 2048) return fail(DCOR_EINVAL, "nsim must be in [1, 2048]");
  if (int st = need_device()) return st;
  const double pos = std::ceil(p * (double)nsim);  // ceiling(p*nsim)
  const int32_t ip = (pos >= 1 && pos <= (double)nsim) ? (int32_t)pos - 1 : -1;
  DevBuf bz, bl, bo;
  if (int st = upload(bz, z, (size_t)nsim)) return st;
  if (int st = upload(bl, l, (size_t)nsim)) return st;
  HIPCHK(bo.alloc(sizeof(double)));
  const int rc = launch_mixquant(bz.as<double>(), bl.as<double>(), (int32_t)nsim, c, ip,
                                 bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "mixquant launch");
  HIPCHK(hipMemcpy(out, bo.p, sizeof(double), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_priv_standardize(const double* v, int64_t n, double eps_norm, double L_raw,
                          const double lap[2], double* out) {
  if (!v || !lap || !out || n < 1) return fail(DCOR_EINVAL, "bad argument");
  if (int st = need_device()) return st;
  const double nd = (double)n;
  const double s_mu = 2.0 * L_raw / (nd * (eps_norm / 2));           // vert-cor.R:336
  const double s_m2 = 2.0 * (L_raw * L_raw) / (nd * (eps_norm / 2));  // vert-cor.R:340
  DevBuf bv, bl, bo;
  if (int st = upload(bv, v, (size_t)n)) return st;
  if (int st = upload(bl, lap, 2)) return st;
  HIPCHK(bo.alloc(sizeof(double) * (size_t)n));
  const int rc = launch_priv_standardize(bv.as<double>(), n, L_raw, s_mu, s_m2, bl.as<double>(),
                                         bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "priv_standardize launch");
  HIPCHK(hipMemcpy(out, bo.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_dp_sd(const double* x, int64_t n, double lo, double hi, double eps1, double eps2,
               const double lap[2], double out[2]) {
  if (!x || !lap || !out || n < 1) return fail(DCOR_EINVAL, "bad argument");
  if (int st = need_device()) return st;
  const double nd = (double)n;
  const double s_mu = (hi - lo) / (nd * eps1);                // real-data-sims.R:69
  const double s_m2 = (hi * hi - lo * lo) / (nd * eps2);      // real-data-sims.R:80
  DevBuf bx, bl, bo;
  if (int st = upload(bx, x, (size_t)n)) return st;
  if (int st = upload(bl, lap, 2)) return st;
  HIPCHK(bo.alloc(sizeof(double) * 2));
  const int rc = launch_dp_sd(bx.as<double>(), n, lo, hi, s_mu, s_m2, bl.as<double>(),
                              bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "dp_sd launch");
  HIPCHK(hipMemcpy(out, bo.p, sizeof(double) * 2, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_perm_launch(uint64_t seed, int site, int64_t rep_begin, int64_t reps, int64_t n,
                     int64_t count, int32_t* d_out, void* stream) {
  if (n < 1 || n > 0x7fffffffLL || count < 0 || count > n || reps < 0 || reps > 65535 ||
      (reps * count > 0 && !d_out))
    return fail(DCOR_EINVAL, "bad perm arguments (need 0 <= count <= n < 2^31, reps <= 65535)");
  if (rep_begin < 0 || rep_begin + reps > 0xffffffffLL) return fail(DCOR_EINVAL, "rep range");
  if (int st = need_device()) return st;
  const int rc = launch_perm((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)site, rep_begin,
                             reps, n, count, d_out, stream);
  if (rc) return hip_fail((hipError_t)rc, "perm launch");
  return DCOR_OK;
}

int64_t dcor_alloc_count(void) { return g_alloc_count.load(); }

int64_t dcor_device_bytes(void) { return g_device_bytes.load(); }

int dcor_shutdown(void) {
  const int owner = g_owner_pid.load();
  if (owner != 0 && owner != (int)getpid()) {
    grid_workers_stop(true);
    // A forked child: the inherited contexts' streams, events and allocations belong to the
    // parent's HIP runtime.  Forget them without a single HIP call (their host memory is the
    // child's copy; nothing is freed twice) and report the fork.
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    g_ctxs.clear();
    g_ctx_gen.fetch_add(1);
    g_device_bytes.store(0);
    return fork_guard();
  }
  grid_workers_stop(false);   // idle workers first: their contexts are freed below
  std::vector<Ctx*> all;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    all.swap(g_ctxs);
    g_ctx_gen.fetch_add(1);
  }
  for (Ctx* c : all) ctx_free(c);
  return DCOR_OK;
}

int dcor_dgp_launch(const dcor_cell* cell, int64_t rep_begin, int64_t reps, double* d_X,
                    double* d_Y, void* stream) {
  if (!cell || reps < 0 || cell->n < 1 || cell->n > 0x7fffffffLL || (reps > 0 && (!d_X || !d_Y)))
    return fail(DCOR_EINVAL, "bad dgp arguments");
  if (reps > 65535) return fail(DCOR_EINVAL, "dgp: at most 65535 replicates per launch");
  if (rep_begin < 0 || rep_begin + reps > 0xffffffffLL) return fail(DCOR_EINVAL, "dgp: replicate range exceeds 2^32");
  DgpConst g;
  if (int st = make_dgp(*cell, g)) return st;
  if (int st = need_device()) return st;
  const int rc = launch_dgp(g, (uint32_t)cell->seed, (uint32_t)(cell->seed >> 32), rep_begin, reps,
                            cell->n, d_X, d_Y, stream);
  if (rc) return hip_fail((hipError_t)rc, "dgp launch");
  return DCOR_OK;
}

int dcor_draws_launch(int kind, uint64_t seed, int site, int64_t rep_begin, int64_t reps,
                      int64_t count, double* d_out, void* stream) {
  if (kind < 0 || kind > 2 || reps < 0 || count < 0 || (reps * count > 0 && !d_out))
    return fail(DCOR_EINVAL, "bad draws arguments");
  if (reps > 65535) return fail(DCOR_EINVAL, "draws: at most 65535 replicates per launch");
  if (rep_begin < 0 || rep_begin + reps > 0xffffffffLL || count > 0x7fffffffLL)
    return fail(DCOR_EINVAL, "draws: need rep_begin + reps <= 2^32 and count < 2^31");
  if (int st = need_device()) return st;
  const int rc = launch_draws(kind, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)site,
                              rep_begin, reps, count, d_out, stream);
  if (rc) return hip_fail((hipError_t)rc, "draws launch");
  return DCOR_OK;
}

}  // extern "C"

// ======================================================= R-stream mode (f4) ===
// Replicates consume R's own streams (set.seed(cell.seed), then SURVEY.md Appendix A's draw
// order), so dcor_rstream_grid_run returns run_sim_one's per-seed numbers.  Kernels:
// dcor_rstream.hip; estimators: the pre-materialised kernels (dcor_premat.hip).
namespace {

// set.seed(seed): RNG_Init's scrambling, 625 words, word 0 (the position) set to 624
void rs_seed(int32_t seed, RsState& s) {
  std::memset(&s, 0, sizeof(s));
  uint32_t x = (uint32_t)seed;
  for (int j = 0; j < 50; ++j) x = 69069u * x + 1u;
  x = 69069u * x + 1u;
  for (int j = 0; j < 624; ++j) { x = 69069u * x + 1u; s.mt[j] = x; }
  s.mti = 624;
}

// MASS::mvrnorm's factor V diag(sqrt(ev)): eigen(Sigma, symmetric = TRUE) is LAPACK dsyevr;
// for 2x2 dsytrd is the identity and dstemr's n = 2 branch calls dlaev2 (eigenvector
// (cs, sn) of the larger root, (-sn, cs) of the smaller); R reverses to decreasing order.
// The product with diag() follows dgemm: C = 0; C += D(l, j) * V(i, l).
void rs_mvrnorm_factor(const double sigma[2], double rho, double A[4]) {
  const double a = sigma[0] * sigma[0], b = sigma[0] * sigma[1] * rho, c = sigma[1] * sigma[1];
  const double sm = a + c, df = a - c, adf = std::fabs(df), tb = b + b, ab = std::fabs(tb);
  const double acmx = (std::fabs(a) > std::fabs(c)) ? a : c, acmn = (std::fabs(a) > std::fabs(c)) ? c : a;
  double rt;
  if (adf > ab) { const double t = ab / adf; rt = adf * std::sqrt(1.0 + t * t); }
  else if (adf < ab) { const double t = adf / ab; rt = ab * std::sqrt(1.0 + t * t); }
  else rt = ab * std::sqrt(2.0);
  double rt1, rt2;
  int sgn1;
  if (sm < 0.0) { rt1 = 0.5 * (sm - rt); sgn1 = -1; rt2 = (acmx / rt1) * acmn - (b / rt1) * b; }
  else if (sm > 0.0) { rt1 = 0.5 * (sm + rt); sgn1 = 1; rt2 = (acmx / rt1) * acmn - (b / rt1) * b; }
  else { rt1 = 0.5 * rt; rt2 = -0.5 * rt; sgn1 = 1; }
  double cs;
  int sgn2;
  if (df >= 0.0) { cs = df + rt; sgn2 = 1; } else { cs = df - rt; sgn2 = -1; }
  double cs1, sn1;
  if (std::fabs(cs) > ab) {
    const double ct = -tb / cs;
    sn1 = 1.0 / std::sqrt(1.0 + ct * ct);
    cs1 = ct * sn1;
  } else if (ab == 0.0) {
    cs1 = 1.0; sn1 = 0.0;
  } else {
    const double tn = -cs / tb;
    cs1 = 1.0 / std::sqrt(1.0 + tn * tn);
    sn1 = tn * cs1;
  }
  if (sgn1 == sgn2) { const double tn = cs1; cs1 = -sn1; sn1 = tn; }
  bool swap = false;
  if (rt1 < rt2) { std::swap(rt1, rt2); swap = true; }
  // R's columns: 1 = eigenvector of rt1, 2 = of rt2
  const double V11 = swap ? -sn1 : cs1, V21 = swap ? cs1 : sn1;
  const double V12 = swap ? cs1 : -sn1, V22 = swap ? sn1 : cs1;
  const double d0 = std::sqrt(std::fmax(rt1, 0.0)), d1 = std::sqrt(std::fmax(rt2, 0.0));
  A[0] = (0.0 + d0 * V11) + 0.0 * V12;
  A[1] = (0.0 + 0.0 * V11) + d1 * V12;
  A[2] = (0.0 + d0 * V21) + 0.0 * V22;
  A[3] = (0.0 + 0.0 * V21) + d1 * V22;
}

struct RsPlan {
  RsCell c;
  int64_t rep_max;       // words per replicate, upper bound (exp_rand takes <= 17 words)
  int64_t jrep;          // words per replicate the jump path budgets (exp_rand: 2 words per draw
                         // and a margin; the mean is 1.69, sd 1.09)
  size_t per_rep;        // device bytes per replicate in flight
};

int rs_plan(const dcor_cell& cell, RsPlan& p) {
  std::memset(&p, 0, sizeof(p));
  RsCell& c = p.c;
  const int64_t n = cell.n;
  if (n < 1 || !(cell.eps1 > 0) || !(cell.eps2 > 0) || cell.nsim < 1)
    return fail(DCOR_EINVAL, "rstream: bad n / eps / nsim");
  if (cell.family != DCOR_FAMILY_SIGN && cell.family != DCOR_FAMILY_SUBG)
    return fail(DCOR_EINVAL, "rstream: bad family");
  if (cell.dgp != DCOR_DGP_GAUSSIAN && cell.dgp != DCOR_DGP_BERNOULLI &&
      cell.dgp != DCOR_DGP_BOUNDED_FACTOR && cell.dgp != DCOR_DGP_MIX_GAUSSIAN)
    return fail(DCOR_EINVAL, "rstream: bad dgp");
  if (cell.dgp == DCOR_DGP_MIX_GAUSSIAN && (n > RS_MIX_NMAX || !(cell.mix_pi >= 0.0 && cell.mix_pi <= 1.0)))
    return fail(DCOR_EINVAL, "rstream: gen_mix_gaussian needs n <= %d and 0 <= pi_mix <= 1", RS_MIX_NMAX);
  if (cell.seed > 0x7fffffffull) return fail(DCOR_EINVAL, "rstream: set.seed takes a 32-bit integer");
  if ((cell.dgp == DCOR_DGP_GAUSSIAN && !mvrnorm_pd(cell.sigma, cell.rho)) ||
      (cell.dgp == DCOR_DGP_MIX_GAUSSIAN &&
       (!mvrnorm_pd(cell.mix_sigma0, cell.rho) || !mvrnorm_pd(cell.mix_sigma1, cell.rho))))
    return fail(DCOR_EINVAL, "rstream: mvrnorm 'Sigma' is not positive definite (|rho| > 1)");
  if (cell.dgp == DCOR_DGP_BERNOULLI && !(std::fabs(cell.rho) <= 1))
    return fail(DCOR_EINVAL, "rstream: gen_bernoulli needs |rho| <= 1 (vert-cor.R:79)");
  if (int st = check_common(n, cell.eps1, cell.eps2, cell.alpha)) return st;
  c.n = n; c.nsim = cell.nsim; c.family = cell.family; c.dgp = cell.dgp;
  const bool subg = cell.family == DCOR_FAMILY_SUBG;
  c.normalise = (!subg && cell.normalise) ? 1 : 0;
  double m = std::ceil(8.0 / (cell.eps1 * cell.eps2));
  if (subg && m > (double)n) m = (double)n;
  const double kd = std::floor((double)n / m);
  if (!(kd >= 1)) return fail(DCOR_EKLT1, "Need at least one full batch (k < 1)");
  c.k = (int64_t)kd;
  if (subg) {
    c.has_mix = 1;
  } else {
    const double eps_r = (cell.eps1 >= cell.eps2) ? cell.eps2 : cell.eps1;
    int mode = cell.ci_mode;
    if (mode == DCOR_MODE_AUTO) mode = (std::sqrt((double)n) * eps_r > 0.5) ? DCOR_MODE_NORMAL : DCOR_MODE_LAPLACE;
    c.has_mix = (mode == DCOR_MODE_NORMAL) ? 1 : 0;
  }
  // DGP (vert-cor.R:78-98,389-394; ver-cor-subG.R:113-154)
  int64_t shuffle_words = 0;
  if (cell.dgp == DCOR_DGP_MIX_GAUSSIAN) {
    // labels rbinom(n, 1, pi) (n words unless pi is 0 or 1), 2n normals (4n words), then
    // sample.int(n): R_unif_index's rejection takes < 2 attempts per draw on average; the
    // buffer allows 4x that (the walker stops, flagged, rather than overrun it)
    const double pp = cell.mix_pi;
    if (pp == 0.0 || pp == 1.0) { c.lab_on = 0; c.lab_const = (pp == 1.0); }
    else { c.lab_on = 1; c.lab_q = 1. - std::fmin(pp, 1. - pp); c.lab_inv = (pp > 0.5) ? 1 : 0; }
    c.shuffle = 1;
    c.dgp_words = (c.lab_on ? n : 0) + 4 * n;
    c.pre_a = c.dgp_words;
    const int64_t wpa = (n > 32768) ? 2 : 1;   // words per attempt (16 bits each)
    shuffle_words = 8 * wpa * n + 4096;
    rs_mvrnorm_factor(cell.mix_sigma0, cell.rho, c.mA0);
    rs_mvrnorm_factor(cell.mix_sigma1, cell.rho, c.mA1);
    c.mmu0[0] = cell.mix_mu0[0]; c.mmu0[1] = cell.mix_mu0[1];
    c.mmu1[0] = cell.mix_mu1[0]; c.mmu1[1] = cell.mix_mu1[1];
  } else if (cell.dgp == DCOR_DGP_GAUSSIAN) {
    c.dgp_words = 4 * n;
    rs_mvrnorm_factor(cell.sigma, cell.rho, c.A);
    c.mu[0] = cell.mu[0]; c.mu[1] = cell.mu[1];
  } else if (cell.dgp == DCOR_DGP_BERNOULLI) {
    c.dgp_words = 2 * n;
    const double p11 = 0.25 + cell.rho / 4, p10 = 0.25 - cell.rho / 4, p01 = p10;
    c.bern_t0 = p01 / 0.5; c.bern_t1 = p11 / 0.5;
  } else {
    c.cU = std::sqrt(3 * cell.rho); c.cE = std::sqrt(3 * (1 - cell.rho));
    // runif(n, a, b): non-finite bounds give NaN, a == b gives a, neither draws
    c.u_draw = (std::isfinite(c.cU) && -c.cU != c.cU) ? 1 : 0;
    c.e_draw = (std::isfinite(c.cE) && -c.cE != c.cE) ? 1 : 0;
    c.u_const = std::isfinite(c.cU) ? -c.cU : NAN;
    c.e_const = std::isfinite(c.cE) ? -c.cE : NAN;
    c.dgp_words = (c.u_draw + 2 * c.e_draw) * n;
  }
  int64_t pre = c.dgp_words;
  if (!subg) {
    const double eps_s = (cell.eps1 >= cell.eps2) ? cell.eps1 : cell.eps2;
    const double pp = std::exp(eps_s) / (std::exp(eps_s) + 1);          // vert-cor.R:174
    if (pp == 0.0 || pp == 1.0) { c.flip_on = 0; c.flip_const = (pp == 1.0); }
    else {
      const double pm = std::fmin(pp, 1. - pp);
      c.flip_on = 1; c.flip_q = 1. - pm; c.flip_inv = (pp > 0.5) ? 1 : 0;
    }
    pre += 2 * (c.normalise ? 4 : 0) + 2 * c.k + (c.flip_on ? n : 0) + 1;
  } else {
    pre += 2 * c.k + n + 1;
  }
  if (c.has_mix) pre += 2 * c.nsim;
  c.pre = pre;
  p.rep_max = pre + shuffle_words + (c.has_mix ? 18 * c.nsim : 0);
  c.jpost = c.has_mix ? c.nsim : 0;
  p.jrep = pre + (c.has_mix ? c.nsim + 2 * c.nsim + 64 + 8 * (int64_t)std::ceil(std::sqrt((double)c.nsim)) : 0);
  if (dcor::variant("DCOR_RSJ_TIGHT"))   // test hook: a budget every mixquant chunk overruns
    p.jrep = pre + (c.has_mix ? c.nsim + c.nsim : 0);
  p.rep_max = std::max(p.rep_max, p.jrep);
  const int64_t fw = (n + 31) / 32;
  p.per_rep = (size_t)p.rep_max * 4 + (size_t)c.nsim * 8 * 3 + (size_t)n * 16 + 64 +
              (size_t)c.k * 16 + (size_t)fw * 4 + (subg ? (size_t)n * 8 : 0) + 8 + 16 +
              (c.shuffle ? (size_t)n * 4 + 8 : 0) + sizeof(dcor_rep_out) + 256;
  return DCOR_OK;
}

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// Carve cell c's buffers for rc replicates out of `base` (advanced).
void rs_carve(RsPlan& p, int32_t rc, char*& base) {
  RsCell& c = p.c;
  auto take = [&](size_t bytes) { char* q = base; base += al256(bytes); return (void*)q; };
  const int64_t n = c.n, k = c.k, nsim = c.nsim, fw = (n + 31) / 32;
  c.words = (uint32_t*)take(((size_t)rc * p.rep_max + 2 * 624 + 64) * 4);
  c.rep_off = (int64_t*)take((size_t)rc * 8);
  c.exp_end = (int64_t*)take((size_t)rc * 8);
  c.expv = (double*)take((size_t)rc * nsim * 8);
  c.X = (double*)take((size_t)rc * n * 8);
  c.Y = (double*)take((size_t)rc * n * 8);
  c.lap_nsc = (double*)take((size_t)rc * 32);
  c.lap_isc = (double*)take((size_t)rc * 32);
  c.lap_x = (double*)take((size_t)rc * k * 8);
  c.lap_y = (double*)take((size_t)rc * k * 8);
  c.flips = (uint32_t*)take((size_t)rc * fw * 4);
  c.lap_local = (c.family == DCOR_FAMILY_SUBG) ? (double*)take((size_t)rc * n * 8) : nullptr;
  c.lap_scalar = (double*)take((size_t)rc * 8);
  c.mix_z = (double*)take((size_t)rc * nsim * 8);
  c.mix_l = (double*)take((size_t)rc * nsim * 8);
  c.shuf = c.shuffle ? (int32_t*)take((size_t)rc * n * 4) : nullptr;
  c.shuf_end = c.shuffle ? (int64_t*)take((size_t)rc * 8) : nullptr;
  c.words_cap = (int64_t)rc * p.rep_max + 2 * 624 + 64;
}

size_t rs_cell_bytes(const RsPlan& p, int32_t rc) {
  const RsCell& c = p.c;
  const int64_t n = c.n, k = c.k, nsim = c.nsim, fw = (n + 31) / 32;
  return al256(((size_t)rc * p.rep_max + 2 * 624 + 64) * 4) + 2 * al256((size_t)rc * 8) +
         al256((size_t)rc * nsim * 8) + 2 * al256((size_t)rc * n * 8) + 2 * al256((size_t)rc * 32) +
         2 * al256((size_t)rc * k * 8) + al256((size_t)rc * fw * 4) +
         ((c.family == DCOR_FAMILY_SUBG) ? al256((size_t)rc * n * 8) : 0) + al256((size_t)rc * 8) +
         2 * al256((size_t)rc * nsim * 8) +
         (c.shuffle ? al256((size_t)rc * n * 4) + al256((size_t)rc * 8) : 0);
}

// The estimators over one chunk of materialised replicates of one cell.
int rs_estimate(const dcor_cell& cell, const RsCell& c, int64_t reps, dcor_rep_out* d_out) {
  if (cell.family == DCOR_FAMILY_SIGN) {
    dcor_premat_sign d;
    std::memset(&d, 0, sizeof(d));
    d.n = c.n; d.reps = reps; d.eps1 = cell.eps1; d.eps2 = cell.eps2; d.alpha = cell.alpha;
    d.normalise = cell.normalise; d.ci_mode = cell.ci_mode; d.nsim = c.nsim;
    d.X = c.X; d.Y = c.Y; d.xy_stride = c.n;
    d.lap_ni_sc = c.lap_nsc; d.lap_ni_x = c.lap_x; d.lap_ni_y = c.lap_y; d.lap_int_sc = c.lap_isc;
    d.flips = c.flips; d.lap_z = c.lap_scalar; d.mix_z = c.mix_z; d.mix_l = c.mix_l;
    return dcor_premat_sign_launch(&d, d_out, nullptr);
  }
  dcor_premat_subg d;
  std::memset(&d, 0, sizeof(d));
  d.n = c.n; d.reps = reps; d.eps1 = cell.eps1; d.eps2 = cell.eps2; d.eta1 = cell.eta1;
  d.eta2 = cell.eta2; d.alpha = cell.alpha; d.hrs = 0;
  d.lam_x = d.lam_y = d.lam_s = d.lam_o = d.lam_r = d.delta = NAN;
  d.nsim = c.nsim; d.X = c.X; d.Y = c.Y; d.xy_stride = c.n; d.perm = nullptr;
  d.lap_ni_x = c.lap_x; d.lap_ni_y = c.lap_y; d.lap_local = c.lap_local;
  d.lap_central = c.lap_scalar; d.mix_z = c.mix_z; d.mix_l = c.mix_l;
  return dcor_premat_subg_launch(&d, d_out, nullptr);
}

struct View {  // a typed window into the R-stream arena
  void* p;
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// The jump path's tables for a chunk of rc replicates of cell p (launch_rsj): budget jN words,
// T levels 2^k <= nsim, G levels 2^k <= rc.
int rs_bits(int64_t v) { int b = 0; while (v) { ++b; v >>= 1; } return b; }
void rsj_dims(RsPlan& p, int64_t rc) {
  RsCell& c = p.c;
  c.jN = rc * p.jrep + 256;
  c.jlt = c.has_mix ? rs_bits(c.nsim) : 0;
  c.jlg = c.has_mix ? rs_bits(rc) : 0;
}
size_t rsj_cell_bytes(const RsPlan& p) {
  const RsCell& c = p.c;
  return al256((size_t)RSJ_L * 4) + al256((size_t)RSJ_TBYTES(c.jlt, c.jN + 1)) +
         al256((size_t)c.jlg * (size_t)(c.jN + 1) * 4) + 256;
}
// DCOR_RS_JUMP: 0 never, 1 whenever the batch allows it, unset: batches of at most 64 cells
// (below that k_rs_stream leaves CUs idle; above it its one-CU-per-cell walk is the cheaper).
// Cells with gen_mix_gaussian's sample.int rejection walk stay on k_rs_stream.
bool rsj_use(const std::vector<RsPlan>& plan, int i0, int nb) {
  for (int i = 0; i < nb; ++i)
    if (plan[(size_t)(i0 + i)].c.shuffle) return false;
  const char* e = dcor::variant("DCOR_RS_JUMP");
  if (e && *e) return std::atoi(e) != 0;
  return nb <= 64;
}

size_t rs_budget() {
  const char* e = dcor::variant("DCOR_RS_BUDGET_MB");
  const long mb = e ? std::atol(e) : 4096;
  return (size_t)(mb > 16 ? mb : 16) << 20;
}

}  // namespace

extern "C" {

int dcor_rstream_grid_run(const dcor_cell* cells, int ncells, int64_t B, dcor_accum* h_acc,
                          dcor_rep_out* h_detail) {
  if (!cells || ncells < 0 || B < 1 || !h_acc) return fail(DCOR_EINVAL, "bad grid arguments");
  if (int st = need_device()) return st;
  std::vector<RsPlan> plan((size_t)ncells);
  for (int i = 0; i < ncells; ++i)
    if (int st = rs_plan(cells[i], plan[(size_t)i])) return st;
  const size_t budget = rs_budget();
  int i0 = 0;
  while (i0 < ncells) {
    // a batch of cells whose streams run side by side (one wave each)
    size_t sum = 0;
    int nb = 0;
    const int64_t rc_min = std::min<int64_t>(B, 8);
    while (i0 + nb < ncells && nb < 65535) {
      const size_t add = plan[(size_t)(i0 + nb)].per_rep;
      if (nb > 0 && (sum + add) * (size_t)rc_min > budget) break;
      sum += add;
      ++nb;
    }
    int64_t rc = (int64_t)(budget / std::max<size_t>(sum, 1));
    rc = std::max<int64_t>(1, std::min<int64_t>({rc, B, (int64_t)(0x7fffffff / nb)}));
    if (const char* e = dcor::variant("DCOR_RS_MAX_CHUNK"))   // test hook: force short chunks
      rc = std::max<int64_t>(1, std::min<int64_t>(rc, std::atol(e)));
    bool jump = rsj_use(plan, i0, nb);
    size_t bytes = 0, jbytes = 0;
    for (;;) {
      bytes = jbytes = 0;
      bool fits32 = true;
      for (int i = 0; i < nb; ++i) {
        RsPlan& p = plan[(size_t)(i0 + i)];
        bytes += rs_cell_bytes(p, (int32_t)rc);
        if (jump) {
          rsj_dims(p, rc);
          jbytes += rsj_cell_bytes(p);
          fits32 = fits32 && p.c.jN < 0x7ffffff0ll;
        }
      }
      if ((fits32 && bytes + jbytes <= budget) || rc == 1) {
        if (!fits32) jump = false;
        break;
      }
      rc = (rc + 1) / 2;
    }
    if (!jump) jbytes = 0;
    // one library-owned arena (kept across calls): cell buffers | jump tables | states |
    // descriptors (and the fallback's) | replicate records | accumulators
    const size_t off_st = bytes + jbytes, off_cells = off_st + al256(sizeof(RsState) * (size_t)nb);
    const size_t off_sub = off_cells + al256(sizeof(RsCell) * (size_t)nb);
    const size_t off_out = off_sub + al256(sizeof(RsCell) * (size_t)nb);
    const size_t off_acc = off_out + al256(sizeof(dcor_rep_out) * (size_t)B * (size_t)nb);
    void* arena = nullptr;
    if (int st = rs_arena_get(off_acc + al256(sizeof(dcor_accum) * 2 * (size_t)nb), &arena))
      return st;
    const View buf{arena}, dst{(char*)arena + off_st}, dcells{(char*)arena + off_cells},
        dsub{(char*)arena + off_sub}, dout{(char*)arena + off_out}, acc{(char*)arena + off_acc};
    std::vector<RsState> hst((size_t)nb);
    std::vector<RsCell> hc((size_t)nb);
    char* base = buf.as<char>();
    int64_t max_pos = 0, max_exp = 0, need = 0;
    int max_lt = 0, max_lg = 0;
    for (int i = 0; i < nb; ++i) {
      rs_seed((int32_t)cells[i0 + i].seed, hst[(size_t)i]);
      RsPlan& p = plan[(size_t)(i0 + i)];
      rs_carve(p, (int32_t)rc, base);
      p.c.st = dst.as<RsState>() + i;
      hc[(size_t)i] = p.c;
    }
    const uint32_t *d_poff = nullptr, *d_pidx = nullptr;
    int nseg = 1;
    if (jump) {
      for (int i = 0; i < nb; ++i) {
        RsCell& c = hc[(size_t)i];
        c.raw = (uint32_t*)base;
        base += al256((size_t)RSJ_L * 4);
        c.tlift = (uint8_t*)base;
        base += al256((size_t)RSJ_TBYTES(c.jlt, c.jN + 1));
        c.glift = (int32_t*)base;
        base += al256((size_t)c.jlg * (size_t)(c.jN + 1) * 4);
        max_pos = std::max(max_pos, c.jN + 1);
        max_exp = std::max(max_exp, c.has_mix ? rc * c.nsim : 0);
        max_lt = std::max(max_lt, (int)c.jlt);
        max_lg = std::max(max_lg, (int)c.jlg);
        need = std::max(need, 624 + c.jN + 64 + 623);
      }
      int32_t* flags = (int32_t*)base;   // one flag per cell, read back in one copy
      base += al256((size_t)nb * 4);
      for (int i = 0; i < nb; ++i) hc[(size_t)i].jflag = flags + i;
      nseg = (int)((need + RSJ_L - 1) / RSJ_L);
      if (nseg > 1)
        if (int st = rsj_polys(nseg - 1, &d_poff, &d_pidx)) return st;
    }
    HIPCHK(hipMemcpy(dst.p, hst.data(), sizeof(RsState) * (size_t)nb, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dcells.p, hc.data(), sizeof(RsCell) * (size_t)nb, hipMemcpyHostToDevice));
    size_t mix_lds = 0;
    for (int i = 0; i < nb; ++i)
      if (hc[(size_t)i].shuffle) mix_lds = std::max(mix_lds, rs_mix_lds_bytes(hc[(size_t)i].n));
    std::vector<int32_t> hflag((size_t)nb);
    for (int64_t done = 0; done < B; done += rc) {
      const int32_t rcc = (int32_t)std::min<int64_t>(rc, B - done);
      int e = 0;
      if (jump) {
        e = launch_rsj(dcells.as<RsCell>(), nb, rcc, d_poff, d_pidx, nseg, max_pos, max_lt, max_lg, max_exp, nullptr);
        if (e) return hip_fail((hipError_t)e, "rstream jump launch");
        // a cell whose chunk ran past its word budget (never seen: the budget is ~10 sd above the
        // mean) kept its state; k_rs_stream walks it instead
        HIPCHK(hipMemcpy(hflag.data(), hc[0].jflag, 4 * (size_t)nb, hipMemcpyDeviceToHost));
        std::vector<RsCell> sub;
        for (int i = 0; i < nb; ++i)
          if (hflag[(size_t)i]) sub.push_back(hc[(size_t)i]);
        if (!sub.empty()) {
          HIPCHK(hipMemcpy(dsub.p, sub.data(), sizeof(RsCell) * sub.size(), hipMemcpyHostToDevice));
          e = launch_rs_stream(dsub.as<RsCell>(), (int)sub.size(), rcc, nullptr);
        }
      } else {
        e = launch_rs_stream(dcells.as<RsCell>(), nb, rcc, nullptr);
      }
      if (e) return hip_fail((hipError_t)e, "rstream stream launch");
      if (mix_lds) {   // gen_mix_gaussian: sample.int's rejection is unbounded; check the flag
        HIPCHK(hipMemcpy(hst.data(), dst.p, sizeof(RsState) * (size_t)nb, hipMemcpyDeviceToHost));
        for (int i = 0; i < nb; ++i)
          if (hst[(size_t)i].pad[1])
            return fail(DCOR_ENOMEM, "rstream: cell %d's sample.int ran past its word buffer", i0 + i);
      }
      e = launch_rs_materialise(dcells.as<RsCell>(), nb, rcc, nullptr, mix_lds);
      if (e) return hip_fail((hipError_t)e, "rstream materialise launch");
      for (int i = 0; i < nb; ++i)
        if (int st = rs_estimate(cells[i0 + i], hc[(size_t)i], rcc,
                                 dout.as<dcor_rep_out>() + (size_t)i * B + done)) return st;
    }
    for (int i = 0; i < nb; ++i) {
      dcor_rep_out* o = dout.as<dcor_rep_out>() + (size_t)i * B;
      if (int st = dcor_accumulate_launch(o, B, cells[i0 + i].rho, acc.as<dcor_accum>() + 2 * i,
                                          nullptr)) return st;
    }
    HIPCHK(hipMemcpy(h_acc + 2 * i0, acc.p, sizeof(dcor_accum) * 2 * (size_t)nb, hipMemcpyDeviceToHost));
    if (h_detail)
      HIPCHK(hipMemcpy(h_detail + (size_t)i0 * B, dout.p, sizeof(dcor_rep_out) * (size_t)B * (size_t)nb,
                       hipMemcpyDeviceToHost));
    i0 += nb;
  }
  return DCOR_OK;
}

int dcor_rstream_draws(const dcor_cell* cell, int64_t reps, const dcor_rs_draws* h) {
  if (!cell || !h || reps < 1 || reps > 65535) return fail(DCOR_EINVAL, "bad rstream_draws arguments");
  if (int st = need_device()) return st;
  RsPlan p;
  if (int st = rs_plan(*cell, p)) return st;
  const int32_t rc = (int32_t)reps;
  DevBuf buf, dst, dcell;
  HIPCHK(buf.alloc(rs_cell_bytes(p, rc)));
  HIPCHK(dst.alloc(sizeof(RsState)));
  HIPCHK(dcell.alloc(sizeof(RsCell)));
  RsState hs;
  rs_seed((int32_t)cell->seed, hs);
  char* base = buf.as<char>();
  rs_carve(p, rc, base);
  p.c.st = dst.as<RsState>();
  HIPCHK(hipMemcpy(dst.p, &hs, sizeof(hs), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dcell.p, &p.c, sizeof(RsCell), hipMemcpyHostToDevice));
  int e = launch_rs_stream(dcell.as<RsCell>(), 1, rc, nullptr);
  if (!e) e = launch_rs_materialise(dcell.as<RsCell>(), 1, rc, nullptr,
                                    p.c.shuffle ? rs_mix_lds_bytes(p.c.n) : 0);
  if (e) return hip_fail((hipError_t)e, "rstream launch");
  const RsCell& c = p.c;
  const size_t R = (size_t)reps, n = (size_t)c.n, k = (size_t)c.k, ns = (size_t)c.nsim;
  auto get = [&](void* dst_h, const void* src_d, size_t bytes) -> int {
    if (dst_h && src_d) HIPCHK(hipMemcpy(dst_h, src_d, bytes, hipMemcpyDeviceToHost));
    return DCOR_OK;
  };
  int st = 0;
  st |= get(h->X, c.X, R * n * 8);
  st |= get(h->Y, c.Y, R * n * 8);
  st |= get(h->lap_ni_sc, c.lap_nsc, R * 32);
  st |= get(h->lap_int_sc, c.lap_isc, R * 32);
  st |= get(h->lap_ni_x, c.lap_x, R * k * 8);
  st |= get(h->lap_ni_y, c.lap_y, R * k * 8);
  st |= get(h->flips, c.flips, R * ((n + 31) / 32) * 4);
  st |= get(h->lap_local, c.lap_local, R * n * 8);
  st |= get(h->lap_scalar, c.lap_scalar, R * 8);
  st |= get(h->mix_z, c.mix_z, R * ns * 8);
  st |= get(h->mix_l, c.mix_l, R * ns * 8);
  return st ? DCOR_EHIP : DCOR_OK;
}

int dcor_rstream_mt_jump(int32_t seed, int64_t J, uint32_t* h_out) {
  if (!h_out || J < 0) return fail(DCOR_EINVAL, "bad mt_jump arguments");
  if (mt_charpoly_degree() != 19937) return fail(DCOR_EINVAL, "MT19937 characteristic polynomial not found");
  return mt_jump_window(seed, J, h_out);
}

int dcor_rstream_words(int32_t seed, int64_t count, uint32_t* h_out) {
  if (!h_out || count < 1 || count > ((int64_t)1 << 30)) return fail(DCOR_EINVAL, "bad rstream_words arguments");
  if (int st = need_device()) return st;
  RsCell c;
  std::memset(&c, 0, sizeof(c));
  c.pre = count;
  DevBuf words, idx, dst, dcell;
  HIPCHK(words.alloc(sizeof(uint32_t) * (size_t)(count + 2 * 624 + 64)));
  HIPCHK(idx.alloc(16));
  HIPCHK(dst.alloc(sizeof(RsState)));
  HIPCHK(dcell.alloc(sizeof(RsCell)));
  RsState hs;
  rs_seed(seed, hs);
  c.st = dst.as<RsState>(); c.words = words.as<uint32_t>();
  c.words_cap = count + 2 * 624 + 64;
  c.rep_off = idx.as<int64_t>(); c.exp_end = idx.as<int64_t>() + 1;
  HIPCHK(hipMemcpy(dst.p, &hs, sizeof(hs), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dcell.p, &c, sizeof(RsCell), hipMemcpyHostToDevice));
  const int e = launch_rs_stream(dcell.as<RsCell>(), 1, 1, nullptr);
  if (e) return hip_fail((hipError_t)e, "rstream words launch");
  HIPCHK(hipMemcpy(h_out, words.p, sizeof(uint32_t) * (size_t)count, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

}  // extern "C"

extern "C" {

int dcor_rstream_hrs_draws(int64_t n, int64_t k, int64_t m, int64_t nsim, int64_t runs,
                           const int32_t* h_ni_seeds, const int32_t* h_int_seeds, int32_t* d_perm,
                           double* d_lap_x, double* d_lap_y, double* d_lap_local,
                           double* d_lap_central, double* d_mix_z, double* d_mix_l, void* stream) {
  if (n < 2 || n > RS_HRS_NMAX || k < 1 || m < 1 || k * m > n || nsim < 1 || runs < 0 ||
      runs > 0x7fffffff)
    return fail(DCOR_EINVAL, "rstream_hrs_draws: need 2 <= n <= %d, k*m <= n, nsim >= 1",
                RS_HRS_NMAX);
  if (h_ni_seeds && (!d_perm || !d_lap_x || !d_lap_y))
    return fail(DCOR_EINVAL, "rstream_hrs_draws: NI outputs missing");
  if (h_int_seeds && (!d_lap_local || !d_lap_central || !d_mix_z || !d_mix_l))
    return fail(DCOR_EINVAL, "rstream_hrs_draws: INT outputs missing");
  if (runs == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  if (h_ni_seeds) {
    DevBuf ds;
    if (int st = upload(ds, h_ni_seeds, (size_t)runs)) return st;
    const int e = launch_rs_hrs_ni(ds.as<int32_t>(), runs, n, k * m, k, d_perm, d_lap_x, d_lap_y,
                                   stream);
    if (e) return hip_fail((hipError_t)e, "rstream hrs NI launch");
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  }
  if (h_int_seeds) {
    const int64_t pre = n + 1 + 2 * nsim, rep_max = pre + 18 * nsim;
    const size_t per_run = al256(((size_t)rep_max + 2 * 624 + 64) * 4) + 2 * al256(8) +
                           al256((size_t)nsim * 8) + sizeof(RsState) + sizeof(RsCell);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(runs, (int64_t)(rs_budget() / per_run)));
    std::vector<RsState> hst((size_t)chunk);
    std::vector<RsCell> hc((size_t)chunk);
    for (int64_t r0 = 0; r0 < runs; r0 += chunk) {
      const int64_t nr = std::min<int64_t>(chunk, runs - r0);
      const size_t words_b = al256(((size_t)rep_max + 2 * 624 + 64) * 4);
      const size_t off_st = (size_t)nr * (words_b + 2 * al256(8) + al256((size_t)nsim * 8));
      const size_t off_cells = off_st + al256(sizeof(RsState) * (size_t)nr);
      void* arena = nullptr;
      if (int st = rs_arena_get(off_cells + al256(sizeof(RsCell) * (size_t)nr), &arena))
        return st;
      char* base = (char*)arena;
      RsState* dst = (RsState*)((char*)arena + off_st);
      for (int64_t i = 0; i < nr; ++i) {
        RsCell& c = hc[(size_t)i];
        std::memset(&c, 0, sizeof(c));
        c.n = n; c.k = 0; c.nsim = nsim; c.family = RS_FAMILY_HRS_INT; c.has_mix = 1;
        c.pre = pre;
        c.words = (uint32_t*)base; base += words_b;
        c.words_cap = rep_max + 2 * 624 + 64;
        c.rep_off = (int64_t*)base; base += al256(8);
        c.exp_end = (int64_t*)base; base += al256(8);
        c.expv = (double*)base; base += al256((size_t)nsim * 8);
        c.lap_local = d_lap_local + (size_t)(r0 + i) * (size_t)n;
        c.lap_scalar = d_lap_central + (r0 + i);
        c.mix_z = d_mix_z + (size_t)(r0 + i) * (size_t)nsim;
        c.mix_l = d_mix_l + (size_t)(r0 + i) * (size_t)nsim;
        c.st = dst + i;
        rs_seed(h_int_seeds[r0 + i], hst[(size_t)i]);
      }
      HIPCHK(hipMemcpy(dst, hst.data(), sizeof(RsState) * (size_t)nr, hipMemcpyHostToDevice));
      RsCell* dcells = (RsCell*)((char*)arena + off_cells);
      HIPCHK(hipMemcpy(dcells, hc.data(), sizeof(RsCell) * (size_t)nr, hipMemcpyHostToDevice));
      int e = launch_rs_stream(dcells, (int)nr, 1, stream);
      if (!e) e = launch_rs_materialise(dcells, (int)nr, 1, stream);
      if (e) return hip_fail((hipError_t)e, "rstream hrs INT launch");
      HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    }
  }
  return DCOR_OK;
}

}  // extern "C"

// ============================================== R-surface helpers (R/dcor*.R) ===
extern "C" {

int dcor_int_subg_sd_uc(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                        double eta1, double eta2, int hrs, double lam_s, double lam_o,
                        double lam_r, double delta, const double* lap_local, double* sd_uc) {
  if (!X || !Y || !lap_local || !sd_uc) return fail(DCOR_EINVAL, "int_subg_sd_uc: null argument");
  if (int st = need_device()) return st;
  dcor_premat_subg d;
  std::memset(&d, 0, sizeof(d));
  d.n = n; d.reps = 1; d.eps1 = eps1; d.eps2 = eps2; d.eta1 = eta1; d.eta2 = eta2; d.alpha = 0.05;
  d.hrs = hrs; d.lam_x = d.lam_y = NAN; d.lam_s = lam_s; d.lam_o = lam_o; d.lam_r = lam_r;
  d.delta = delta; d.nsim = 1;
  PrematSubgConst p;
  if (int st = premat_subg_const(&d, p)) return st;
  DevBuf bX, bY, bl, bo;
  if (int st = upload(bX, X, (size_t)n)) return st;
  if (int st = upload(bY, Y, (size_t)n)) return st;
  if (int st = upload(bl, lap_local, (size_t)n)) return st;
  HIPCHK(bo.alloc(sizeof(double)));
  p.X = bX.as<double>(); p.Y = bY.as<double>(); p.lap_local = bl.as<double>();
  const int rc = launch_uc_sd(p, bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "uc_sd launch");
  HIPCHK(hipMemcpy(sd_uc, bo.p, sizeof(double), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_dp_mean(const double* x, int64_t n, double lo, double hi, double eps, double lap,
                 double* out) {
  if (!x || !out || n < 1) return fail(DCOR_EINVAL, "dp_mean: bad argument");
  if (int st = need_device()) return st;
  const double s_mu = (hi - lo) / ((double)n * eps);  // real-data-sims.R:69
  const double lap2[2] = {lap, 0.0};
  DevBuf bx, bl, bo;
  if (int st = upload(bx, x, (size_t)n)) return st;
  if (int st = upload(bl, lap2, 2)) return st;
  HIPCHK(bo.alloc(sizeof(double) * 2));
  const int rc = launch_dp_sd(bx.as<double>(), n, lo, hi, s_mu, 0.0, bl.as<double>(),
                              bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "dp_mean launch");
  HIPCHK(hipMemcpy(out, bo.p, sizeof(double), hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_standardize_dp(const double* x, int64_t n, double lo, double hi, double mean, double sd,
                        double eps, double* out) {
  if ((n > 0 && (!x || !out)) || n < 0) return fail(DCOR_EINVAL, "standardize_dp: bad argument");
  if (n == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  const double den = r_max(sd, eps);  // max(priv$sd, eps), real-data-sims.R:89
  DevBuf bx, bo;
  if (int st = upload(bx, x, (size_t)n)) return st;
  HIPCHK(bo.alloc(sizeof(double) * (size_t)n));
  const int rc = launch_standardize_dp(bx.as<double>(), n, lo, hi, mean, den, bo.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "standardize_dp launch");
  HIPCHK(hipMemcpy(out, bo.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_gen_bernoulli(const double* u, const double* v, int64_t n, double rho, double* X,
                       double* Y) {
  if (n < 0 || (n > 0 && (!u || !v || !X || !Y))) return fail(DCOR_EINVAL, "gen_bernoulli: bad argument");
  if (!(std::fabs(rho) <= 1)) return fail(DCOR_EINVAL, "gen_bernoulli: abs(rho) <= 1 is not TRUE (vert-cor.R:79)");
  if (n == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  const double p11 = 0.25 + rho / 4, p10 = 0.25 - rho / 4, p01 = p10;  // vert-cor.R:80-82
  DevBuf bu, bv, bX, bY;
  if (int st = upload(bu, u, (size_t)n)) return st;
  if (int st = upload(bv, v, (size_t)n)) return st;
  HIPCHK(bX.alloc(sizeof(double) * (size_t)n));
  HIPCHK(bY.alloc(sizeof(double) * (size_t)n));
  const int rc = launch_gen_bernoulli(bu.as<double>(), bv.as<double>(), n, p01 / 0.5, p11 / 0.5,
                                      bX.as<double>(), bY.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "gen_bernoulli launch");
  HIPCHK(hipMemcpy(X, bX.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Y, bY.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_gen_bounded_factor(const double* U, const double* E1, const double* E2, int64_t n,
                            double* X, double* Y) {
  if (n < 0 || (n > 0 && (!U || !E1 || !E2 || !X || !Y)))
    return fail(DCOR_EINVAL, "gen_bounded_factor: bad argument");
  if (n == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  DevBuf bU, b1, b2, bX, bY;
  if (int st = upload(bU, U, (size_t)n)) return st;
  if (int st = upload(b1, E1, (size_t)n)) return st;
  if (int st = upload(b2, E2, (size_t)n)) return st;
  HIPCHK(bX.alloc(sizeof(double) * (size_t)n));
  HIPCHK(bY.alloc(sizeof(double) * (size_t)n));
  const int rc = launch_gen_bounded_factor(bU.as<double>(), b1.as<double>(), b2.as<double>(), n,
                                           bX.as<double>(), bY.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "gen_bounded_factor launch");
  HIPCHK(hipMemcpy(X, bX.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Y, bY.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

static int mvn_run(const double* z0, int64_t n0, const double* z1, int64_t n1, const int32_t* perm,
                   const MvnConst& m, double* X, double* Y) {
  const int64_t n = n0 + n1;
  if (n == 0) return DCOR_OK;
  if (int st = need_device()) return st;
  DevBuf b0, b1, bp, bX, bY;
  if (int st = upload(b0, z0, (size_t)(2 * n0))) return st;
  if (int st = upload(b1, z1, (size_t)(2 * n1))) return st;
  if (perm) { if (int st = upload(bp, perm, (size_t)n)) return st; }
  HIPCHK(bX.alloc(sizeof(double) * (size_t)n));
  HIPCHK(bY.alloc(sizeof(double) * (size_t)n));
  const int rc = launch_mvrnorm_apply(b0.as<double>(), n0, b1.as<double>(), n1,
                                      perm ? bp.as<int32_t>() : nullptr, m, bX.as<double>(),
                                      bY.as<double>(), nullptr);
  if (rc) return hip_fail((hipError_t)rc, "mvrnorm launch");
  HIPCHK(hipMemcpy(X, bX.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(Y, bY.p, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost));
  return DCOR_OK;
}

int dcor_mvrnorm(const double* z, int64_t n, const double mu[2], const double sigma[2],
                 double rho, double* X, double* Y) {
  if (n < 0 || !mu || !sigma || (n > 0 && (!z || !X || !Y))) return fail(DCOR_EINVAL, "mvrnorm: bad argument");
  if (!mvrnorm_pd(sigma, rho)) return fail(DCOR_EINVAL, "mvrnorm: 'Sigma' is not positive definite");
  MvnConst m;
  std::memset(&m, 0, sizeof(m));
  rs_mvrnorm_factor(sigma, rho, m.A0);
  m.mu0[0] = mu[0]; m.mu0[1] = mu[1];
  return mvn_run(z, n, nullptr, 0, nullptr, m, X, Y);
}

int dcor_mix_gaussian(const double* z0, int64_t n0, const double* z1, int64_t n1,
                      const int32_t* perm, double rho, const double mu0[2], const double sigma0[2],
                      const double mu1[2], const double sigma1[2], double* X, double* Y) {
  if (n0 < 0 || n1 < 0 || !mu0 || !sigma0 || !mu1 || !sigma1 ||
      (n0 + n1 > 0 && (!perm || !X || !Y || (n0 && !z0) || (n1 && !z1))))
    return fail(DCOR_EINVAL, "gen_mix_gaussian: bad argument");
  for (int64_t i = 0; i < n0 + n1; ++i)
    if (perm[i] < 0 || perm[i] >= n0 + n1) return fail(DCOR_EINVAL, "gen_mix_gaussian: perm out of range");
  if (!mvrnorm_pd(sigma0, rho) || !mvrnorm_pd(sigma1, rho))
    return fail(DCOR_EINVAL, "gen_mix_gaussian: mvrnorm 'Sigma' is not positive definite");
  MvnConst m;
  rs_mvrnorm_factor(sigma0, rho, m.A0);
  rs_mvrnorm_factor(sigma1, rho, m.A1);
  m.mu0[0] = mu0[0]; m.mu0[1] = mu0[1]; m.mu1[0] = mu1[0]; m.mu1[1] = mu1[1];
  return mvn_run(z0, n0, z1, n1, perm, m, X, Y);
}

}  // extern "C"
