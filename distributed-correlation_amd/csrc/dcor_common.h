// dcor_common.h -- device helpers shared by the fused and pre-materialised kernels:
// R-exact sign of a standardised value, mixquant order statistic from loaded draws, and
// the NI / INT epilogues of both estimator families (cited R lines inline).
#pragma once
#include "dcor_device.h"
#include "dcor_engine.h"

namespace dcor {

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

// mixquant over keys already in registers: zv[s], lv[s] = z[i], l[i] for i = tid + s*DCOR_BLOCK
// (a caller can issue these loads before c is known).
__device__ __forceinline__ double mixquant_regs(const MixConst& mx, double c,
                                                const double (&zv)[SEL_VPT],
                                                const double (&lv)[SEL_VPT], SelScratch* sc) {
  if (threadIdx.x == 0) sc->nan_cnt = 0;
  __syncthreads();
  double val[SEL_VPT];
  int nn = 0;
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s) {
    const int i = threadIdx.x + s * DCOR_BLOCK;
    val[s] = dnan();
    if (i < mx.nsim) {
      val[s] = zv[s] + c * lv[s];
      nn += (val[s] != val[s]);
    }
  }
  if (nn) atomicAdd(&sc->nan_cnt, nn);
  __syncthreads();
  return value_select(val, mx.pos, mx.nsim - sc->nan_cnt, sc);
}

__device__ __forceinline__ void mixquant_prefetch(const MixConst& mx, const double* z,
                                                  const double* l, double (&zv)[SEL_VPT],
                                                  double (&lv)[SEL_VPT]) {
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s) {
    const int i = threadIdx.x + s * DCOR_BLOCK;
    zv[s] = i < mx.nsim ? z[i] : 0.0;
    lv[s] = i < mx.nsim ? l[i] : 0.0;
  }
}

__device__ __forceinline__ double mixquant_loaded(const MixConst& mx, double c, const double* z,
                                                  const double* l, SelScratch* sc) {
  if (threadIdx.x == 0) sc->nan_cnt = 0;
  __syncthreads();
  double val[SEL_VPT];
  int nn = 0;
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s) {
    const int i = threadIdx.x + s * DCOR_BLOCK;
    val[s] = dnan();
    if (i < mx.nsim) {
      val[s] = z[i] + c * l[i];
      nn += (val[s] != val[s]);
    }
  }
  if (nn) atomicAdd(&sc->nan_cnt, nn);
  __syncthreads();
  return value_select(val, mx.pos, mx.nsim - sc->nan_cnt, sc);
}

#define MIX_MAX 2048

// ------------------------------------------------- sign-family epilogues
struct SignStd { double muNx, sdNx, muNy, sdNy, muIx, sdIx, muIy, sdIy; };

// vert-cor.R:335-344 from mean(xc), mean(xc^2), mean(yc), mean(yc^2): NI thresholds with
// draws lap[0..3], INT thresholds (fresh noise, :271-272) with lap[4..7].
__device__ __forceinline__ void priv_std_from_means(const SignConst& c, double mx, double m2x,
                                                    double my, double m2y, const double lap[8],
                                                    SignStd& s) {
  s.muNx = mx + c.s_mu_x * lap[0];
  s.sdNx = sqrt(rmax((m2x + c.s_m2_x * lap[1]) - s.muNx * s.muNx, 1e-12));
  s.muNy = my + c.s_mu_y * lap[2];
  s.sdNy = sqrt(rmax((m2y + c.s_m2_y * lap[3]) - s.muNy * s.muNy, 1e-12));
  s.muIx = mx + c.s_mu_x * lap[4];
  s.sdIx = sqrt(rmax((m2x + c.s_m2_x * lap[5]) - s.muIx * s.muIx, 1e-12));
  s.muIy = my + c.s_mu_y * lap[6];
  s.sdIy = sqrt(rmax((m2y + c.s_m2_y * lap[7]) - s.muIy * s.muIy, 1e-12));
}

__device__ __forceinline__ void priv_std_from_sums(const SignConst& c, const double v[4],
                                                   const double lap[8], SignStd& s) {
  // mean(xc) = sum/n (R: LD mean, agrees to rounding)
  priv_std_from_means(c, v[0] / c.nd, v[1] / c.nd, v[2] / c.nd, v[3] / c.nd, lap, s);
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

__device__ __forceinline__ void ni_subg_result(const SubgConst& c, DD sP, DD sT, DD sT2,
                                               double* o) {
  // ver-cor-subG.R:51-59
  const double rho = c.m_over_k * (sP.hi + sP.lo);
  const double se = sqrt(dd_var(sT, sT2, c.kd)) / c.sqrt_k;
  o[0] = rho;
  o[1] = rmax(rho - c.crit * se, -1.0);
  o[2] = rmin(rho + c.crit * se, 1.0);
}


}  // namespace dcor
