// dcor_kernels.hip -- gfx950 kernels of the DP-correlation Monte-Carlo hot path.
//
// One 256-thread workgroup (4 wave64) owns one replicate.  Fused kernels generate
// their samples with Philox (nothing materialised in HBM), pre-materialised kernels
// stream caller-provided samples and noise.  fp64 throughout (R `double`); batch
// sign counts and flip sums are exact integers.  See DESIGN.md for the roofline.
#include <hip/hip_runtime.h>

#include "dcor_device.h"
#include "dcor_engine.h"

namespace dcor {

// --------------------------------------------------------------- DGP helpers
struct DgpGen {
  DgpConst g;
  uint32_t rep, k0, k1;
  uint32_t cidx;   // cached Philox block index (Bernoulli: two samples per block)
  U4 cw;

  __device__ __forceinline__ void init(const DgpConst& gc, uint32_t r, uint32_t a, uint32_t b) {
    g = gc; rep = r; k0 = a; k1 = b; cidx = 0xffffffffu;
  }
  // sample i -> (x, y).  lapw: if non-null receives the DGP_B block's (w2,w3)
  // unit Laplace (sub-G local noise).
  __device__ __forceinline__ void gen(uint32_t i, double& x, double& y, double* lap) {
    if (g.dgp == DCOR_DGP_GAUSSIAN) {
      const U4 w = draw(i, rep, DCOR_SITE_DGP_A, k0, k1);
      double z1, z2;
      normal_pair(w, &z1, &z2);
      x = g.mu0 + (g.a00 * z1 + g.a01 * z2);
      y = g.mu1 + (g.a10 * z1 + g.a11 * z2);
      if (lap) {
        const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
        *lap = unit_laplace(u53(v.w2, v.w3));
      }
    } else if (g.dgp == DCOR_DGP_BERNOULLI) {
      const uint32_t bi = i >> 1;
      if (bi != cidx) { cw = draw(bi, rep, DCOR_SITE_DGP_A, k0, k1); cidx = bi; }
      const uint32_t wa = (i & 1) ? cw.w2 : cw.w0;
      const uint32_t wb = (i & 1) ? cw.w3 : cw.w1;
      const double u = (double)wa * 0x1p-32, v = (double)wb * 0x1p-32;
      x = (u < 0.5) ? 1.0 : 0.0;
      y = (x == 0.0) ? (v < g.thr0 ? 1.0 : 0.0) : (v < g.thr1 ? 1.0 : 0.0);
      if (lap) {
        const U4 v2 = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
        *lap = unit_laplace(u53(v2.w2, v2.w3));
      }
    } else {
      const U4 w = draw(i, rep, DCOR_SITE_DGP_A, k0, k1);
      const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
      const double U = -g.cU + g.cU2 * u53(w.w0, w.w1);
      x = U + (-g.cE + g.cE2 * u53(w.w2, w.w3));
      y = U + (-g.cE + g.cE2 * u53(v.w0, v.w1));
      if (lap) *lap = unit_laplace(u53(v.w2, v.w3));
    }
  }
};

// sign((a - mu)/sd) exactly as R computes it (sd > 0): the quotient has the sign of
// the numerator unless it underflows, which needs |a - mu| < sd * 2^-1000.
__device__ __forceinline__ int sgn_std(double a, double mu, double sd, bool& bad) {
  const double d = a - mu;
  if (fabs(d) >= sd * 0x1p-1000) return (d > 0) - (d < 0);
  const double q = d / sd;
  bad |= (q != q);
  return (q > 0) - (q < 0);
}
__device__ __forceinline__ int sgn_raw(double a, bool& bad) {
  bad |= (a != a);
  return (a > 0) - (a < 0);
}

struct FlipGen {  // sign-family INT flips, 4 per Philox block (SITE_FLIP)
  uint32_t cidx;
  U4 cw;
  __device__ __forceinline__ int get(uint32_t i, uint32_t rep, uint32_t k0, uint32_t k1,
                                     double p) {
    const uint32_t bi = i >> 2;
    if (bi != cidx) { cw = draw(bi, rep, DCOR_SITE_FLIP, k0, k1); cidx = bi; }
    const uint32_t q = i & 3;
    const uint32_t w = q == 0 ? cw.w0 : (q == 1 ? cw.w1 : (q == 2 ? cw.w2 : cw.w3));
    return ((double)w * 0x1p-32 < p) ? 1 : -1;  // 2*S - 1
  }
};

// mixquant inside the workgroup: keys = z + c*l from Philox, then order statistic.
__device__ __forceinline__ double mixquant_fused(const MixConst& mx, double c, uint32_t rep,
                                                 uint32_t k0, uint32_t k1, double* keys,
                                                 int* nan_cnt) {
  if (threadIdx.x == 0) *nan_cnt = 0;
  __syncthreads();
  int nn = 0;
  for (int b = threadIdx.x; 2 * b < mx.nsim; b += DCOR_BLOCK) {
    const U4 wz = draw((uint32_t)b, rep, DCOR_SITE_MIX_Z, k0, k1);
    const U4 wl = draw((uint32_t)b, rep, DCOR_SITE_MIX_L, k0, k1);
    double z0, z1;
    normal_pair(wz, &z0, &z1);
    const double l0 = unit_laplace(u53(wl.w0, wl.w1));
    const double l1 = unit_laplace(u53(wl.w2, wl.w3));
    double v0 = z0 + c * l0;
    if (v0 != v0) { v0 = __longlong_as_double(0x7ff0000000000000LL); ++nn; }
    keys[2 * b] = v0;
    if (2 * b + 1 < mx.nsim) {
      double v1 = z1 + c * l1;
      if (v1 != v1) { v1 = __longlong_as_double(0x7ff0000000000000LL); ++nn; }
      keys[2 * b + 1] = v1;
    }
  }
  if (nn) atomicAdd(nan_cnt, nn);
  __syncthreads();
  return lds_select(keys, mx.nsim, mx.P, mx.pos, nan_cnt);
}

__device__ __forceinline__ double mixquant_loaded(const MixConst& mx, double c, const double* z,
                                                  const double* l, double* keys, int* nan_cnt) {
  if (threadIdx.x == 0) *nan_cnt = 0;
  __syncthreads();
  int nn = 0;
  for (int i = threadIdx.x; i < mx.nsim; i += DCOR_BLOCK) {
    double v = z[i] + c * l[i];
    if (v != v) { v = __longlong_as_double(0x7ff0000000000000LL); ++nn; }
    keys[i] = v;
  }
  if (nn) atomicAdd(nan_cnt, nn);
  __syncthreads();
  return lds_select(keys, mx.nsim, mx.P, mx.pos, nan_cnt);
}

#define MIX_MAX 2048

// ------------------------------------------------- sign-family epilogues
struct SignStd { double muNx, sdNx, muNy, sdNy, muIx, sdIx, muIy, sdIy; };

__device__ __forceinline__ void priv_std_from_sums(const SignConst& c, const double v[4],
                                                   const double lap[8], SignStd& s) {
  // vert-cor.R:335-344 with mean(xc) = sum/n (R: LD mean, agrees to rounding)
  const double mx = v[0] / c.nd, m2x = v[1] / c.nd, my = v[2] / c.nd, m2y = v[3] / c.nd;
  s.muNx = mx + c.s_mu_x * lap[0];
  s.sdNx = sqrt(rmax((m2x + c.s_m2_x * lap[1]) - s.muNx * s.muNx, 1e-12));
  s.muNy = my + c.s_mu_y * lap[2];
  s.sdNy = sqrt(rmax((m2y + c.s_m2_y * lap[3]) - s.muNy * s.muNy, 1e-12));
  s.muIx = mx + c.s_mu_x * lap[4];
  s.sdIx = sqrt(rmax((m2x + c.s_m2_x * lap[5]) - s.muIx * s.muIx, 1e-12));
  s.muIy = my + c.s_mu_y * lap[6];
  s.sdIy = sqrt(rmax((m2y + c.s_m2_y * lap[7]) - s.muIy * s.muIy, 1e-12));
}

__device__ __forceinline__ void ni_sign_result(const SignConst& c, DD sT, DD sT2, bool bad,
                                               double* o) {
  // vert-cor.R:233-254
  const double sumT = sT.hi + sT.lo;
  const double eta = c.inv_k * sumT;
  const double S = sqrt(dd_var(sT, sT2, c.kd));
  o[0] = sin(M_PI * eta / 2.0);
  o[1] = sin(M_PI / 2.0 * rmax(eta - c.crit * S / c.sqrt_k, -1.0));
  o[2] = sin(M_PI / 2.0 * rmin(eta + c.crit * S / c.sqrt_k, 1.0));
  if (bad) o[0] = o[1] = o[2] = dnan();
}

// vert-cor.R:186-194, 281-313.  Returns (rho, eta, se_eta) and the mixquant c*.
__device__ __forceinline__ void int_sign_point(const SignConst& c, long long core, double lapz,
                                               double& rho, double& eta, double& se,
                                               double& cstar) {
  const double Z = c.scale_Z * lapz;
  const double eta0 = c.coefZ * (double)core + Z;
  rho = sin(M_PI * eta0 / 2.0);
  eta = 1.0 - acos(rho) * 2.0 / M_PI;
  const double h = 1.0 - acos(rho) * 2.0 / M_PI;
  const double s2 = 1.0 - c.q2 * (h * h);
  se = 1.0 / sqrt(c.nd) * sqrt(s2) * c.ratio;
  cstar = 2.0 / (sqrt(c.nd * s2) * c.eps_r);
}

// ===================================================== fused sign family ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_fused(SignConst c, dcor_rep_out* out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  __shared__ double lap[10];
  __shared__ double keys[MIX_MAX];
  __shared__ int nan_cnt;
  const uint32_t rep = (uint32_t)(c.rep_begin + blockIdx.x);
  const int tid = threadIdx.x;
  if (tid < 5) {
    const U4 w = draw((uint32_t)tid, rep, DCOR_SITE_SCALAR, c.k0, c.k1);
    lap[2 * tid] = unit_laplace(u53(w.w0, w.w1));
    lap[2 * tid + 1] = unit_laplace(u53(w.w2, w.w3));
  }
  DgpGen gen;
  gen.init(c.g, rep, c.k0, c.k1);
  // ---- pass 1: DP mean / second moment sums of the clipped samples (vert-cor.R:328-340)
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  if (c.normalise) {
    for (int64_t i = tid; i < c.n; i += DCOR_BLOCK) {
      double x, y;
      gen.gen((uint32_t)i, x, y, nullptr);
      const double xc = rclip(x, c.L), yc = rclip(y, c.L);
      v[0] += xc; v[1] += xc * xc; v[2] += yc; v[3] += yc * yc;
    }
  }
  block_sum<4>(v, red);
  SignStd s;
  {
    double l8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) l8[q] = lap[q];
    priv_std_from_sums(c, v, l8, s);
  }
  // ---- pass 2: regenerate, signs vs the four private centres, batch counts, flips
  FlipGen fl;
  fl.cidx = 0xffffffffu;
  bool bad = false;
  DD sT{0.0, 0.0}, sT2{0.0, 0.0};
  long long core = 0;
  gen.cidx = 0xffffffffu;
  for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
    int cx = 0, cy = 0;
    const int64_t i0 = j * c.m;
    for (int r = 0; r < c.m; ++r) {
      const uint32_t i = (uint32_t)(i0 + r);
      double x, y;
      gen.gen(i, x, y, nullptr);
      int nx, ny, ix, iy;
      if (c.normalise) {
        const double xc = rclip(x, c.L), yc = rclip(y, c.L);
        nx = sgn_std(xc, s.muNx, s.sdNx, bad);
        ny = sgn_std(yc, s.muNy, s.sdNy, bad);
        ix = sgn_std(xc, s.muIx, s.sdIx, bad);
        iy = sgn_std(yc, s.muIy, s.sdIy, bad);
      } else {
        nx = ix = sgn_raw(x, bad);
        ny = iy = sgn_raw(y, bad);
      }
      cx += nx; cy += ny;
      core += fl.get(i, rep, c.k0, c.k1, c.pflip) * ix * iy;
    }
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);
    const double xt = (double)cx / c.md + c.bx * unit_laplace(u53(w.w0, w.w1));
    const double yt = (double)cy / c.md + c.by * unit_laplace(u53(w.w2, w.w3));
    const double T = c.md * xt * yt;
    dd_acc(sT, T);
    dd_acc(sT2, T * T);
  }
  for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) {  // tail: INT only
    double x, y;
    gen.gen((uint32_t)i, x, y, nullptr);
    int ix, iy;
    if (c.normalise) {
      ix = sgn_std(rclip(x, c.L), s.muIx, s.sdIx, bad);
      iy = sgn_std(rclip(y, c.L), s.muIy, s.sdIy, bad);
    } else {
      ix = sgn_raw(x, bad);
      iy = sgn_raw(y, bad);
    }
    core += fl.get((uint32_t)i, rep, c.k0, c.k1, c.pflip) * ix * iy;
  }
  DD d2[2] = {sT, sT2};
  block_sum_dd<2>(d2, red);
  core = block_sum_i(core, redi);
  const long long nbad = block_sum_i(bad ? 1 : 0, redi);
  double o[6];
  ni_sign_result(c, d2[0], d2[1], nbad != 0, o);
  double rho, eta, se, cstar;
  int_sign_point(c, core, lap[8], rho, eta, se, cstar);
  double w;
  if (c.mode_normal)
    w = mixquant_fused(c.mix, cstar, rep, c.k0, c.k1, keys, &nan_cnt) * se;
  else
    w = c.w_laplace;
  o[3] = rho;
  o[4] = sin(M_PI / 2.0 * rmax(eta - w, -1.0));
  o[5] = sin(M_PI / 2.0 * rmin(eta + w, 1.0));
  if (nbad) o[3] = o[4] = o[5] = dnan();
  if (tid == 0) {
    dcor_rep_out r{o[0], o[1], o[2], o[3], o[4], o[5]};
    out[blockIdx.x] = r;
  }
}

// ===================================================== fused sub-G family ===
__device__ __forceinline__ void ni_subg_result(const SubgConst& c, DD sP, DD sT, DD sT2,
                                               double* o) {
  // ver-cor-subG.R:51-59
  const double rho = c.m_over_k * (sP.hi + sP.lo);
  const double se = sqrt(dd_var(sT, sT2, c.kd)) / c.sqrt_k;
  o[0] = rho;
  o[1] = rmax(rho - c.crit * se, -1.0);
  o[2] = rmin(rho + c.crit * se, 1.0);
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_subg_fused(SubgConst c, dcor_rep_out* out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ double lapz;
  __shared__ double keys[MIX_MAX];
  __shared__ int nan_cnt;
  const uint32_t rep = (uint32_t)(c.rep_begin + blockIdx.x);
  const int tid = threadIdx.x;
  if (tid == 0) {
    const U4 w = draw(4u, rep, DCOR_SITE_SCALAR, c.k0, c.k1);
    lapz = unit_laplace(u53(w.w0, w.w1));
  }
  DgpGen gen;
  gen.init(c.g, rep, c.k0, c.k1);
  DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
  for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
    double sx = 0.0, sy = 0.0;
    const int64_t i0 = j * c.m;
    for (int r = 0; r < c.m; ++r) {
      double x, y, l;
      gen.gen((uint32_t)(i0 + r), x, y, &l);
      sx += rclip(x, c.l1);
      sy += rclip(y, c.l2);
      const double S = c.sender_is_X ? x : y, O = c.sender_is_X ? y : x;
      const double Uc = rclip((rclip(S, c.ls) + c.bs * l) * O, c.lr);
      dd_acc(sU, Uc);
      dd_acc(sU2, Uc * Uc);
    }
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);
    const double xt = sx / c.md + c.bx * unit_laplace(u53(w.w0, w.w1));
    const double yt = sy / c.md + c.by * unit_laplace(u53(w.w2, w.w3));
    dd_acc(sP, xt * yt);
    const double T = c.md * xt * yt;
    dd_acc(sT, T);
    dd_acc(sT2, T * T);
  }
  for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) {
    double x, y, l;
    gen.gen((uint32_t)i, x, y, &l);
    const double S = c.sender_is_X ? x : y, O = c.sender_is_X ? y : x;
    const double Uc = rclip((rclip(S, c.ls) + c.bs * l) * O, c.lr);
    dd_acc(sU, Uc);
    dd_acc(sU2, Uc * Uc);
  }
  DD d5[5] = {sP, sT, sT2, sU, sU2};
  block_sum_dd<5>(d5, red);
  double o[6];
  ni_subg_result(c, d5[0], d5[1], d5[2], o);
  // ver-cor-subG.R:91-103
  const DD mU = dd_div_d(d5[3], c.nd);
  const double rho = (mU.hi + mU.lo) + c.s_central * lapz;
  const double sd = sqrt(dd_var(d5[3], d5[4], c.nd));
  const double se_norm = sqrt(sd * sd + c.sn2x2);
  const double cstar = 2.0 / (c.sqrt_n * sd * c.eps_r);
  const double q = mixquant_fused(c.mix, cstar, rep, c.k0, c.k1, keys, &nan_cnt);
  const double width = q * se_norm / c.sqrt_n;
  o[3] = rho;
  o[4] = rmax(rho - width, -1.0);
  o[5] = rmin(rho + width, 1.0);
  if (tid == 0) {
    dcor_rep_out r{o[0], o[1], o[2], o[3], o[4], o[5]};
    out[blockIdx.x] = r;
  }
}

// ================================================== pre-materialised sign ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_sign(PrematSignConst p, dcor_rep_out* out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  __shared__ double keys[MIX_MAX];
  __shared__ int nan_cnt;
  const SignConst& c = p.s;
  const int64_t rep = blockIdx.x;
  const int tid = threadIdx.x;
  const double* X = p.X + rep * p.xy_stride;
  const double* Y = p.Y + rep * p.xy_stride;
  const double* lni = p.lap_ni_sc + rep * 4;
  const double* lin = p.lap_int_sc + rep * 4;
  const double* lx = p.lap_ni_x + rep * c.k;
  const double* ly = p.lap_ni_y + rep * c.k;
  const uint32_t* fw = p.flips + rep * p.flip_words;
  DD v[4] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
  if (c.normalise) {
    for (int64_t i = tid; i < c.n; i += DCOR_BLOCK) {
      const double xc = rclip(X[i], c.L), yc = rclip(Y[i], c.L);
      dd_acc(v[0], xc); dd_acc(v[1], xc * xc); dd_acc(v[2], yc); dd_acc(v[3], yc * yc);
    }
  }
  block_sum_dd<4>(v, red);
  SignStd s;
  {
    // means from the double-double sums (R: long-double mean), then vert-cor.R:335-344
    double mean[4], l8[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const DD m = dd_div_d(v[q], c.nd);
      mean[q] = m.hi + m.lo;
      l8[q] = lni[q];
      l8[4 + q] = lin[q];
    }
    s.muNx = mean[0] + c.s_mu_x * l8[0];
    s.sdNx = sqrt(rmax((mean[1] + c.s_m2_x * l8[1]) - s.muNx * s.muNx, 1e-12));
    s.muNy = mean[2] + c.s_mu_y * l8[2];
    s.sdNy = sqrt(rmax((mean[3] + c.s_m2_y * l8[3]) - s.muNy * s.muNy, 1e-12));
    s.muIx = mean[0] + c.s_mu_x * l8[4];
    s.sdIx = sqrt(rmax((mean[1] + c.s_m2_x * l8[5]) - s.muIx * s.muIx, 1e-12));
    s.muIy = mean[2] + c.s_mu_y * l8[6];
    s.sdIy = sqrt(rmax((mean[3] + c.s_m2_y * l8[7]) - s.muIy * s.muIy, 1e-12));
  }
  bool bad = false;
  DD sT{0, 0}, sT2{0, 0};
  long long core = 0;
  for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
    int cx = 0, cy = 0;
    const int64_t i0 = j * c.m;
    for (int r = 0; r < c.m; ++r) {
      const int64_t i = i0 + r;
      const double x = X[i], y = Y[i];
      int nx, ny, ix, iy;
      if (c.normalise) {
        const double xc = rclip(x, c.L), yc = rclip(y, c.L);
        nx = sgn_std(xc, s.muNx, s.sdNx, bad);
        ny = sgn_std(yc, s.muNy, s.sdNy, bad);
        ix = sgn_std(xc, s.muIx, s.sdIx, bad);
        iy = sgn_std(yc, s.muIy, s.sdIy, bad);
      } else {
        nx = ix = sgn_raw(x, bad);
        ny = iy = sgn_raw(y, bad);
      }
      cx += nx; cy += ny;
      const int f = ((fw[i >> 5] >> (i & 31)) & 1u) ? 1 : -1;
      core += f * ix * iy;
    }
    const double xt = (double)cx / c.md + c.bx * lx[j];
    const double yt = (double)cy / c.md + c.by * ly[j];
    const double T = c.md * xt * yt;
    dd_acc(sT, T);
    dd_acc(sT2, T * T);
  }
  for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) {
    const double x = X[i], y = Y[i];
    int ix, iy;
    if (c.normalise) {
      ix = sgn_std(rclip(x, c.L), s.muIx, s.sdIx, bad);
      iy = sgn_std(rclip(y, c.L), s.muIy, s.sdIy, bad);
    } else {
      ix = sgn_raw(x, bad);
      iy = sgn_raw(y, bad);
    }
    const int f = ((fw[i >> 5] >> (i & 31)) & 1u) ? 1 : -1;
    core += f * ix * iy;
  }
  DD d2[2] = {sT, sT2};
  block_sum_dd<2>(d2, red);
  core = block_sum_i(core, redi);
  const long long nbad = block_sum_i(bad ? 1 : 0, redi);
  double o[6];
  ni_sign_result(c, d2[0], d2[1], nbad != 0, o);
  double rho, eta, se, cstar;
  int_sign_point(c, core, p.lap_z[rep], rho, eta, se, cstar);
  double w;
  if (c.mode_normal)
    w = mixquant_loaded(c.mix, cstar, p.mix_z + rep * c.mix.nsim, p.mix_l + rep * c.mix.nsim,
                        keys, &nan_cnt) * se;
  else
    w = c.w_laplace;
  o[3] = rho;
  o[4] = sin(M_PI / 2.0 * rmax(eta - w, -1.0));
  o[5] = sin(M_PI / 2.0 * rmin(eta + w, 1.0));
  if (nbad) o[3] = o[4] = o[5] = dnan();
  if (tid == 0) {
    dcor_rep_out r{o[0], o[1], o[2], o[3], o[4], o[5]};
    out[rep] = r;
  }
}

// ================================================== pre-materialised sub-G ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_subg(PrematSubgConst p, dcor_rep_out* out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ double keys[MIX_MAX];
  __shared__ int nan_cnt;
  const SubgConst& c = p.s;
  const int64_t rep = blockIdx.x;
  const int tid = threadIdx.x;
  const double* X = p.X + rep * p.xy_stride;
  const double* Y = p.Y + rep * p.xy_stride;
  const double* S = c.sender_is_X ? X : Y;
  const double* O = c.sender_is_X ? Y : X;
  const double* lx = p.lap_ni_x + rep * c.k;
  const double* ly = p.lap_ni_y + rep * c.k;
  const double* ll = p.lap_local + rep * c.n;
  DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
  auto int_term = [&](int64_t i) {
    const double ov = p.hrs ? rclip(O[i], p.lo_) : O[i];
    const double Uc = rclip((rclip(S[i], c.ls) + c.bs * ll[i]) * ov, c.lr);
    dd_acc(sU, Uc);
    dd_acc(sU2, Uc * Uc);
  };
  auto batch_term = [&](int64_t j, DD bx, DD by) {
    const DD xb = dd_div_d(bx, c.md), yb = dd_div_d(by, c.md);
    const double xt = (xb.hi + xb.lo) + c.bx * lx[j];
    const double yt = (yb.hi + yb.lo) + c.by * ly[j];
    dd_acc(sP, xt * yt);
    const double T = c.md * xt * yt;
    dd_acc(sT, T);
    dd_acc(sT2, T * T);
  };
  if (p.perm == nullptr) {
    // contiguous batches: each element read once by its batch owner (NI + INT)
    for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
      DD bx{0, 0}, by{0, 0};
      const int64_t i0 = j * c.m;
      for (int r = 0; r < c.m; ++r) {
        const int64_t i = i0 + r;
        dd_acc(bx, rclip(X[i], c.l1));
        dd_acc(by, rclip(Y[i], c.l2));
        int_term(i);
      }
      batch_term(j, bx, by);
    }
    for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) int_term(i);
  } else {
    // HRS: random batches idx = sample.int(n, k*m) (real-data-sims.R:131)
    const int32_t* pm = p.perm + rep * (c.k * c.m);
    for (int64_t i = tid; i < c.n; i += DCOR_BLOCK) int_term(i);
    for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
      DD bx{0, 0}, by{0, 0};
      for (int r = 0; r < c.m; ++r) {
        const int64_t i = pm[j * c.m + r];
        dd_acc(bx, rclip(X[i], c.l1));
        dd_acc(by, rclip(Y[i], c.l2));
      }
      batch_term(j, bx, by);
    }
  }
  DD d5[5] = {sP, sT, sT2, sU, sU2};
  block_sum_dd<5>(d5, red);
  double o[6];
  ni_subg_result(c, d5[0], d5[1], d5[2], o);
  const DD mU = dd_div_d(d5[3], c.nd);
  const double rho = (mU.hi + mU.lo) + c.s_central * p.lap_central[rep];
  const double sd = sqrt(dd_var(d5[3], d5[4], c.nd));
  double width;
  if (!p.hrs) {
    const double se_norm = sqrt(sd * sd + c.sn2x2);
    const double cstar = 2.0 / (c.sqrt_n * sd * c.eps_r);
    const double q = mixquant_loaded(c.mix, cstar, p.mix_z + rep * c.mix.nsim,
                                     p.mix_l + rep * c.mix.nsim, keys, &nan_cnt);
    width = q * se_norm / c.sqrt_n;
  } else if (sd == 0.0) {
    width = p.crit_sqrt2_s;
  } else {
    const double cstar = (2.0 * c.lr) / (c.sqrt_n * sd * c.eps_r);
    const double q = mixquant_loaded(c.mix, cstar, p.mix_z + rep * c.mix.nsim,
                                     p.mix_l + rep * c.mix.nsim, keys, &nan_cnt);
    width = q * (sd / c.sqrt_n);
  }
  o[3] = rho;
  o[4] = rmax(rho - width, -1.0);
  o[5] = rmin(rho + width, 1.0);
  if (tid == 0) {
    dcor_rep_out r{o[0], o[1], o[2], o[3], o[4], o[5]};
    out[rep] = r;
  }
}

// ======================================================== accumulation ===
// Deterministic per-method summary of `count` records (one workgroup).
__global__ __launch_bounds__(DCOR_BLOCK) void k_accumulate(const dcor_rep_out* rec, int64_t count,
                                                           double rho, dcor_accum* acc) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  for (int meth = 0; meth < 2; ++meth) {
    DD s[6] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}};
    long long cnt[4] = {0, 0, 0, 0};  // cover, cover_na, na_est, na_ci
    for (int64_t b = threadIdx.x; b < count; b += DCOR_BLOCK) {
      const double* r = &rec[b].ni_hat + 3 * meth;
      const double est = r[0], lo = r[1], hi = r[2];
      const bool nae = (est != est), nal = (lo != lo), nah = (hi != hi);
      if (nae) ++cnt[2]; else {
        dd_acc(s[0], est);
        dd_acc(s[1], est * est);
        const double e = est - rho;
        dd_acc(s[2], e * e);
      }
      if (nal || nah) ++cnt[3]; else {
        dd_acc(s[3], hi - lo);
        dd_acc(s[4], lo);
        dd_acc(s[5], hi);
      }
      // R: rho >= lo && rho <= hi with NA three-valued logic
      const int a = nal ? 2 : (rho >= lo ? 1 : 0);
      const int bq = nah ? 2 : (rho <= hi ? 1 : 0);
      int cv;
      if (a == 0) cv = 0; else if (a == 1) cv = bq; else cv = (bq == 0) ? 0 : 2;
      if (cv == 1) ++cnt[0]; else if (cv == 2) ++cnt[1];
    }
    block_sum_dd<6>(s, red);
    long long tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) tot[q] = block_sum_i(cnt[q], redi);
    if (threadIdx.x == 0) {
      dcor_accum a;
      a.n = count; a.n_cover = tot[0]; a.n_cover_na = tot[1]; a.n_na_est = tot[2]; a.n_na_ci = tot[3];
      a.reserved[0] = a.reserved[1] = a.reserved[2] = 0;
      a.est[0] = s[0].hi; a.est[1] = s[0].lo; a.est2[0] = s[1].hi; a.est2[1] = s[1].lo;
      a.se2[0] = s[2].hi; a.se2[1] = s[2].lo; a.len[0] = s[3].hi; a.len[1] = s[3].lo;
      a.lo[0] = s[4].hi; a.lo[1] = s[4].lo; a.hi[0] = s[5].hi; a.hi[1] = s[5].lo;
      acc[meth] = a;
    }
  }
}

// ================================================== single-call helpers ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_mixquant(const double* z, const double* l,
                                                         MixConst mx, double c, double* out) {
  __shared__ double keys[MIX_MAX];
  __shared__ int nan_cnt;
  const double q = mixquant_loaded(mx, c, z, l, keys, &nan_cnt);
  if (threadIdx.x == 0) *out = q;
}

// priv_standardize (vert-cor.R:322-348) over one vector (one workgroup).
__global__ __launch_bounds__(DCOR_BLOCK) void k_priv_standardize(const double* v, int64_t n,
                                                                 double L, double s_mu,
                                                                 double s_m2, const double* lap2,
                                                                 double* out) {
  __shared__ double red[16 * DCOR_WAVES];
  DD a[2] = {{0, 0}, {0, 0}};
  for (int64_t i = threadIdx.x; i < n; i += DCOR_BLOCK) {
    const double xc = rclip(v[i], L);
    dd_acc(a[0], xc);
    dd_acc(a[1], xc * xc);
  }
  block_sum_dd<2>(a, red);
  const double nd = (double)n;
  const DD m1 = dd_div_d(a[0], nd), m2 = dd_div_d(a[1], nd);
  const double mu = (m1.hi + m1.lo) + s_mu * lap2[0];
  const double m2p = (m2.hi + m2.lo) + s_m2 * lap2[1];
  const double sd = sqrt(rmax(m2p - mu * mu, 1e-12));
  for (int64_t i = threadIdx.x; i < n; i += DCOR_BLOCK) out[i] = (rclip(v[i], L) - mu) / sd;
}

// dp_sd (real-data-sims.R:73-84): out = {mean, sd}.
__global__ __launch_bounds__(DCOR_BLOCK) void k_dp_sd(const double* x, int64_t n, double lo,
                                                      double hi, double s_mu, double s_m2,
                                                      const double* lap2, double* out) {
  __shared__ double red[16 * DCOR_WAVES];
  DD a[2] = {{0, 0}, {0, 0}};
  for (int64_t i = threadIdx.x; i < n; i += DCOR_BLOCK) {
    const double xc = rclip_lohi(x[i], lo, hi);
    dd_acc(a[0], xc);
    dd_acc(a[1], xc * xc);
  }
  block_sum_dd<2>(a, red);
  const double nd = (double)n;
  const DD m1 = dd_div_d(a[0], nd), m2 = dd_div_d(a[1], nd);
  const double mu = (m1.hi + m1.lo) + s_mu * lap2[0];
  const double m2p = (m2.hi + m2.lo) + s_m2 * lap2[1];
  if (threadIdx.x == 0) {
    out[0] = mu;
    out[1] = sqrt(rmax(m2p - mu * mu, 0.0));
  }
}

// ============================================================== draws ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_draws(int kind, uint32_t k0, uint32_t k1,
                                                      uint32_t site, int64_t rep_begin,
                                                      int64_t count, double* out) {
  const int64_t r = blockIdx.y;
  const uint32_t rep = (uint32_t)(rep_begin + r);
  const int64_t npair = (count + 1) / 2;
  for (int64_t b = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x; b < npair;
       b += (int64_t)gridDim.x * DCOR_BLOCK) {
    const U4 w = draw((uint32_t)b, rep, site, k0, k1);
    double a, c;
    if (kind == 1) {
      normal_pair(w, &a, &c);
    } else if (kind == 0) {
      a = unit_laplace(u53(w.w0, w.w1));
      c = unit_laplace(u53(w.w2, w.w3));
    } else {
      a = u53(w.w0, w.w1);
      c = u53(w.w2, w.w3);
    }
    double* o = out + r * count;
    o[2 * b] = a;
    if (2 * b + 1 < count) o[2 * b + 1] = c;
  }
}

// ============================================================ launchers ===
static inline int last_err() { return (int)hipGetLastError(); }

int launch_sign_fused(const SignConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  hipLaunchKernelGGL(k_sign_fused, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}
int launch_subg_fused(const SubgConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  hipLaunchKernelGGL(k_subg_fused, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}
int launch_premat_sign(const PrematSignConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  hipLaunchKernelGGL(k_premat_sign, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}
int launch_premat_subg(const PrematSubgConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  hipLaunchKernelGGL(k_premat_subg, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}
int launch_accumulate(const dcor_rep_out* d_out, int64_t count, double rho, dcor_accum* acc,
                      void* stream) {
  hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, d_out,
                     count, rho, acc);
  return last_err();
}
int launch_mixquant(const double* z, const double* l, int32_t nsim, double c, int32_t pos,
                    double* out, void* stream) {
  MixConst mx;
  mx.nsim = nsim; mx.pos = pos; mx.P = 1;
  while (mx.P < nsim) mx.P <<= 1;
  mx.pad = 0;
  hipLaunchKernelGGL(k_mixquant, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, z, l, mx,
                     c, out);
  return last_err();
}
int launch_priv_standardize(const double* v, int64_t n, double L, double s_mu, double s_m2,
                            const double* lap2, double* out, void* stream) {
  hipLaunchKernelGGL(k_priv_standardize, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, v,
                     n, L, s_mu, s_m2, lap2, out);
  return last_err();
}
int launch_draws(int kind, uint32_t k0, uint32_t k1, uint32_t site, int64_t rep_begin,
                 int64_t reps, int64_t count, double* out, void* stream) {
  if (reps <= 0 || count <= 0) return 0;
  const int64_t npair = (count + 1) / 2;
  int64_t gx = (npair + DCOR_BLOCK - 1) / DCOR_BLOCK;
  if (gx > 4096) gx = 4096;
  hipLaunchKernelGGL(k_draws, dim3((unsigned)gx, (unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, kind, k0, k1, site, rep_begin, count, out);
  return last_err();
}
int launch_dp_sd(const double* x, int64_t n, double lo, double hi, double s_mu, double s_m2,
                 const double* lap2, double* out2, void* stream) {
  hipLaunchKernelGGL(k_dp_sd, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, x, n, lo, hi,
                     s_mu, s_m2, lap2, out2);
  return last_err();
}

}  // namespace dcor
