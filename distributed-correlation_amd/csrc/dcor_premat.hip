// dcor_premat.hip -- pre-materialised (explicit-input, HBM-streaming) kernels, the
// accumulation kernel, single-call helpers (mixquant, priv_standardize, dp_sd) and the
// on-device draw generator.  One 256-thread workgroup per replicate.
#include <hip/hip_runtime.h>

#include "dcor_common.h"

namespace dcor {


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
  bool bad_ni = false, bad_int = false;  // NaN seen by NI (first k*m) / INT (all n)
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
        nx = sgn_std(xc, s.muNx, s.sdNx, bad_ni);
        ny = sgn_std(yc, s.muNy, s.sdNy, bad_ni);
        ix = sgn_std(xc, s.muIx, s.sdIx, bad_int);
        iy = sgn_std(yc, s.muIy, s.sdIy, bad_int);
      } else {
        nx = ix = sgn_raw(x, bad_ni);
        ny = iy = sgn_raw(y, bad_ni);
        bad_int |= bad_ni;
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
      ix = sgn_std(rclip(x, c.L), s.muIx, s.sdIx, bad_int);
      iy = sgn_std(rclip(y, c.L), s.muIy, s.sdIy, bad_int);
    } else {
      ix = sgn_raw(x, bad_int);
      iy = sgn_raw(y, bad_int);
    }
    const int f = ((fw[i >> 5] >> (i & 31)) & 1u) ? 1 : -1;
    core += f * ix * iy;
  }
  DD d2[2] = {sT, sT2};
  block_sum_dd<2>(d2, red);
  core = block_sum_i(core, redi);
  const long long nbad = block_sum_i((bad_ni ? 1LL : 0LL) + (bad_int ? (1LL << 20) : 0LL), redi);
  const bool any_ni = (nbad & 0xFFFFF) != 0, any_int = (nbad >> 20) != 0;
  double o[6];
  ni_sign_result(c, d2[0], d2[1], any_ni, o);
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
  if (any_int) o[3] = o[4] = o[5] = dnan();
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
