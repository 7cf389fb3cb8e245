/*
 * dcor_r.c -- R `.Call` shim over include/dcor.h: the binding of the reference's R surface
 * (R/dcor.R, R/dcor_subG.R, R/dcor_hrs.R).  Built by R CMD SHLIB against libdcor.so:
 *
 *   R CMD SHLIB -o dcor_r.so dcor_r.c -I../../include -L../dcor -ldcor -Wl,-rpath,$(realpath ../dcor)
 *
 * R is absent from the build image; tests/test_r_shim.py compiles this file
 * against a stub of the R C API (tests/rstub/) and calls its entry points through ctypes.
 * Contract: inputs are borrowed REAL()/INTEGER() views; outputs are allocated here with
 * allocVector / allocMatrix; nothing C-owned is live when Rf_error longjmps (scratch comes from
 * R_alloc, which R frees on the jump).
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <string.h>

#include "dcor.h"

static void dcor_stop(int st) {
  char msg[512];
  dcor_last_error(msg, sizeof msg);
  Rf_error("dcor: %s (status %d)", msg, st);
}

static double num(SEXP x) { return Rf_asReal(x); }
static const double* dptr_or_null(SEXP x) { return Rf_isNull(x) ? NULL : REAL(x); }

static SEXP triple(const double o[3]) {
  SEXP r = PROTECT(allocVector(REALSXP, 3));
  memcpy(REAL(r), o, 3 * sizeof(double));
  UNPROTECT(1);
  return r;
}

SEXP dcor_R_lambda_n(SEXP n, SEXP eta) { return ScalarReal(dcor_lambda_n(num(n), num(eta))); }

SEXP dcor_R_lambda_INT_n(SEXP n, SEXP eta_s, SEXP eta_r, SEXP eps_s) {
  SEXP r = PROTECT(allocVector(REALSXP, 2));
  dcor_lambda_int_n(num(n), num(eta_s), num(eta_r), num(eps_s), REAL(r));
  UNPROTECT(1);
  return r;
}

SEXP dcor_R_lambda_from_priv(SEXP lo, SEXP hi, SEXP mean, SEXP sd, SEXP eps_sd) {
  return ScalarReal(dcor_lambda_from_priv(num(lo), num(hi), num(mean), num(sd), num(eps_sd)));
}

SEXP dcor_R_lambda_receiver_from_noise(SEXP ls, SEXP lo, SEXP es, SEXP delta) {
  return ScalarReal(dcor_lambda_receiver_from_noise(num(ls), num(lo), num(es), num(delta)));
}

SEXP dcor_R_mixquant(SEXP z, SEXP l, SEXP c, SEXP p) {
  double o;
  const int st = dcor_mixquant(REAL(z), REAL(l), XLENGTH(z), num(c), num(p), &o);
  if (st) dcor_stop(st);
  return ScalarReal(o);
}

SEXP dcor_R_priv_standardize(SEXP v, SEXP eps, SEXP L, SEXP lap) {
  SEXP r = PROTECT(allocVector(REALSXP, XLENGTH(v)));
  const int st = dcor_priv_standardize(REAL(v), XLENGTH(v), num(eps), num(L), REAL(lap), REAL(r));
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_dp_sd(SEXP x, SEXP lo, SEXP hi, SEXP e1, SEXP e2, SEXP lap) {
  double o[2];
  const int st = dcor_dp_sd(REAL(x), XLENGTH(x), num(lo), num(hi), num(e1), num(e2), REAL(lap), o);
  if (st) dcor_stop(st);
  SEXP r = PROTECT(allocVector(REALSXP, 2));
  REAL(r)[0] = o[0];
  REAL(r)[1] = o[1];
  UNPROTECT(1);
  return r;
}

SEXP dcor_R_dp_mean(SEXP x, SEXP lo, SEXP hi, SEXP eps, SEXP lap) {
  double o;
  const int st = dcor_dp_mean(REAL(x), XLENGTH(x), num(lo), num(hi), num(eps), num(lap), &o);
  if (st) dcor_stop(st);
  return ScalarReal(o);
}

SEXP dcor_R_standardize_dp(SEXP x, SEXP lo, SEXP hi, SEXP mean, SEXP sd, SEXP eps) {
  SEXP r = PROTECT(allocVector(REALSXP, XLENGTH(x)));
  const int st = dcor_standardize_dp(REAL(x), XLENGTH(x), num(lo), num(hi), num(mean), num(sd),
                                     num(eps), REAL(r));
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_ci_NI_signbatch(SEXP X, SEXP Y, SEXP e1, SEXP e2, SEXP alpha, SEXP normalise,
                            SEXP lap_sc, SEXP lap_x, SEXP lap_y) {
  double o[3];
  const int st = dcor_ci_ni_signbatch(REAL(X), REAL(Y), XLENGTH(X), num(e1), num(e2), num(alpha),
                                      Rf_asLogical(normalise), dptr_or_null(lap_sc), REAL(lap_x),
                                      REAL(lap_y), o);
  if (st) dcor_stop(st);
  return triple(o);
}

SEXP dcor_R_ci_INT_signflip(SEXP X, SEXP Y, SEXP e1, SEXP e2, SEXP alpha, SEXP mode,
                            SEXP normalise, SEXP lap_sc, SEXP flips, SEXP lap_z, SEXP mz, SEXP ml) {
  const R_xlen_t n = XLENGTH(X);
  unsigned char* fl = (unsigned char*)R_alloc(n, 1); /* R-managed: freed on longjmp */
  for (R_xlen_t i = 0; i < n; ++i) fl[i] = (unsigned char)(INTEGER(flips)[i] != 0);
  double o[3];
  const int st = dcor_ci_int_signflip(REAL(X), REAL(Y), n, num(e1), num(e2), num(alpha),
                                      Rf_asInteger(mode), Rf_asLogical(normalise),
                                      dptr_or_null(lap_sc), fl, num(lap_z), REAL(mz), REAL(ml),
                                      XLENGTH(mz), o);
  if (st) dcor_stop(st);
  return triple(o);
}

SEXP dcor_R_correlation_NI_subG(SEXP X, SEXP Y, SEXP e1, SEXP e2, SEXP eta1, SEXP eta2,
                                SEXP alpha, SEXP hrs, SEXP lam_x, SEXP lam_y, SEXP perm,
                                SEXP lap_x, SEXP lap_y) {
  double o[3];
  const int st = dcor_correlation_ni_subg(
      REAL(X), REAL(Y), XLENGTH(X), num(e1), num(e2), num(eta1), num(eta2), num(alpha),
      Rf_asLogical(hrs), num(lam_x), num(lam_y), Rf_isNull(perm) ? NULL : INTEGER(perm),
      REAL(lap_x), REAL(lap_y), o);
  if (st) dcor_stop(st);
  return triple(o);
}

SEXP dcor_R_ci_INT_subG(SEXP X, SEXP Y, SEXP e1, SEXP e2, SEXP eta1, SEXP eta2, SEXP alpha,
                        SEXP hrs, SEXP lam_s, SEXP lam_o, SEXP lam_r, SEXP delta, SEXP lap_local,
                        SEXP lap_central, SEXP mz, SEXP ml) {
  double o[3];
  const int st = dcor_ci_int_subg(REAL(X), REAL(Y), XLENGTH(X), num(e1), num(e2), num(eta1),
                                  num(eta2), num(alpha), Rf_asLogical(hrs), num(lam_s),
                                  num(lam_o), num(lam_r), num(delta), REAL(lap_local),
                                  num(lap_central), REAL(mz), REAL(ml), XLENGTH(mz), o);
  if (st) dcor_stop(st);
  return triple(o);
}

/* HRS ci_INT_subG's sd(Uc) (lam = lambda_sender, lambda_other, lambda_receiver, delta_clip). */
SEXP dcor_R_int_subg_sd_uc(SEXP X, SEXP Y, SEXP e1, SEXP e2, SEXP eta1, SEXP eta2, SEXP lam,
                           SEXP lap_local) {
  if (XLENGTH(lam) != 4) Rf_error("dcor: lam must hold 4 numbers");
  const double* l = REAL(lam);
  double sd;
  const int st = dcor_int_subg_sd_uc(REAL(X), REAL(Y), XLENGTH(X), num(e1), num(e2), num(eta1),
                                     num(eta2), 1, l[0], l[1], l[2], l[3], REAL(lap_local), &sd);
  if (st) dcor_stop(st);
  return ScalarReal(sd);
}

/* n x 2 matrix (columns X, Y) for the DGP wrappers. */
static SEXP xy_matrix(R_xlen_t n) { return allocMatrix(REALSXP, (int)n, 2); }

SEXP dcor_R_gen_bernoulli(SEXP u, SEXP v, SEXP rho) {
  const R_xlen_t n = XLENGTH(u);
  SEXP r = PROTECT(xy_matrix(n));
  const int st = dcor_gen_bernoulli(REAL(u), REAL(v), n, num(rho), REAL(r), REAL(r) + n);
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_gen_bounded_factor(SEXP U, SEXP E1, SEXP E2) {
  const R_xlen_t n = XLENGTH(U);
  SEXP r = PROTECT(xy_matrix(n));
  const int st = dcor_gen_bounded_factor(REAL(U), REAL(E1), REAL(E2), n, REAL(r), REAL(r) + n);
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_mvrnorm(SEXP z, SEXP n_, SEXP mu, SEXP sigma, SEXP rho) {
  const R_xlen_t n = (R_xlen_t)num(n_);
  if (XLENGTH(z) != 2 * n || XLENGTH(mu) != 2 || XLENGTH(sigma) != 2)
    Rf_error("dcor: mvrnorm needs 2n normals, mu[2], sigma[2]");
  SEXP r = PROTECT(xy_matrix(n));
  const int st = dcor_mvrnorm(REAL(z), n, REAL(mu), REAL(sigma), num(rho), REAL(r), REAL(r) + n);
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_mix_gaussian(SEXP z0, SEXP n0_, SEXP z1, SEXP n1_, SEXP perm, SEXP rho, SEXP mu0,
                         SEXP sigma0, SEXP mu1, SEXP sigma1) {
  const R_xlen_t n0 = (R_xlen_t)num(n0_), n1 = (R_xlen_t)num(n1_);
  if (XLENGTH(z0) != 2 * n0 || XLENGTH(z1) != 2 * n1 || XLENGTH(perm) != n0 + n1)
    Rf_error("dcor: gen_mix_gaussian needs 2 n0 + 2 n1 normals and a permutation of n");
  SEXP r = PROTECT(xy_matrix(n0 + n1));
  const int st = dcor_mix_gaussian(REAL(z0), n0, REAL(z1), n1, INTEGER(perm), num(rho), REAL(mu0),
                                   REAL(sigma0), REAL(mu1), REAL(sigma1), REAL(r),
                                   REAL(r) + (n0 + n1));
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

/* One grid: cells given as parallel vectors (one element per cell).  rng_r: R's own streams
 * (dcor_rstream_grid_run, one device) instead of the Philox engine, which shards every cell's
 * replicates over `devices` (0-based HIP ids; empty: every visible GPU). */
SEXP dcor_R_grid_run(SEXP family, SEXP dgp, SEXP n, SEXP rho, SEXP eps1, SEXP eps2, SEXP alpha,
                     SEXP mu1, SEXP mu2, SEXP s1, SEXP s2, SEXP normalise, SEXP mode, SEXP seed,
                     SEXP B, SEXP want_detail, SEXP mix, SEXP rng_r, SEXP nsim, SEXP devices) {
  /* mix: gen_mix_gaussian's mu0[2], sigma0[2], mu1[2], sigma1[2], pi_mix (ver-cor-subG.R:116-118) */
  if (XLENGTH(mix) != 9) Rf_error("dcor_grid: mix must hold 9 numbers");
  const double* mx = REAL(mix);
  const int nc = LENGTH(n);
  const long long b = (long long)Rf_asReal(B);
  dcor_cell* cells = (dcor_cell*)R_alloc(nc, sizeof(dcor_cell));
  for (int i = 0; i < nc; ++i) {
    memset(&cells[i], 0, sizeof(dcor_cell));
    cells[i].family = INTEGER(family)[i];
    cells[i].dgp = INTEGER(dgp)[i];
    cells[i].n = (int64_t)REAL(n)[i];
    cells[i].rho = REAL(rho)[i];
    cells[i].eps1 = REAL(eps1)[i];
    cells[i].eps2 = REAL(eps2)[i];
    cells[i].alpha = REAL(alpha)[i];
    cells[i].mu[0] = REAL(mu1)[i]; cells[i].mu[1] = REAL(mu2)[i];
    cells[i].sigma[0] = REAL(s1)[i]; cells[i].sigma[1] = REAL(s2)[i];
    cells[i].eta1 = cells[i].eta2 = 1.0;
    cells[i].normalise = LOGICAL(normalise)[i];
    cells[i].ci_mode = INTEGER(mode)[i];
    cells[i].nsim = (int64_t)REAL(nsim)[i];
    cells[i].seed = (uint64_t)REAL(seed)[i];
    cells[i].mix_mu0[0] = mx[0]; cells[i].mix_mu0[1] = mx[1];
    cells[i].mix_sigma0[0] = mx[2]; cells[i].mix_sigma0[1] = mx[3];
    cells[i].mix_mu1[0] = mx[4]; cells[i].mix_mu1[1] = mx[5];
    cells[i].mix_sigma1[0] = mx[6]; cells[i].mix_sigma1[1] = mx[7];
    cells[i].mix_pi = mx[8];
  }
  SEXP acc = PROTECT(allocVector(RAWSXP, (R_xlen_t)nc * 2 * sizeof(dcor_accum)));
  SEXP det = PROTECT(Rf_asLogical(want_detail) ? allocVector(REALSXP, (R_xlen_t)nc * b * 6)
                                               : allocVector(REALSXP, 0));
  dcor_rep_out* dp = XLENGTH(det) ? (dcor_rep_out*)REAL(det) : NULL;
  const int st = Rf_asLogical(rng_r)
      ? dcor_rstream_grid_run(cells, nc, b, (dcor_accum*)RAW(acc), dp)
      : dcor_grid_run_multi(cells, nc, b, LENGTH(devices) ? INTEGER(devices) : NULL,
                            LENGTH(devices), (dcor_accum*)RAW(acc), dp);
  if (st) { UNPROTECT(2); dcor_stop(st); }
  /* summaries: [cell][method][mse, bias, var, coverage, ci_length] */
  SEXP sm = PROTECT(allocVector(REALSXP, (R_xlen_t)nc * 2 * 5));
  for (int i = 0; i < nc; ++i)
    for (int m = 0; m < 2; ++m)
      dcor_accum_finalize((dcor_accum*)RAW(acc) + 2 * i + m, cells[i].rho,
                          (dcor_summary*)(REAL(sm) + (2 * i + m) * 5));
  SEXP out = PROTECT(allocVector(VECSXP, 2));
  SET_VECTOR_ELT(out, 0, sm);
  SET_VECTOR_ELT(out, 1, det);
  UNPROTECT(4);
  return out;
}

static const R_CallMethodDef calls[] = {
    {"dcor_R_lambda_n", (DL_FUNC)&dcor_R_lambda_n, 2},
    {"dcor_R_lambda_INT_n", (DL_FUNC)&dcor_R_lambda_INT_n, 4},
    {"dcor_R_lambda_from_priv", (DL_FUNC)&dcor_R_lambda_from_priv, 5},
    {"dcor_R_lambda_receiver_from_noise", (DL_FUNC)&dcor_R_lambda_receiver_from_noise, 4},
    {"dcor_R_mixquant", (DL_FUNC)&dcor_R_mixquant, 4},
    {"dcor_R_priv_standardize", (DL_FUNC)&dcor_R_priv_standardize, 4},
    {"dcor_R_dp_sd", (DL_FUNC)&dcor_R_dp_sd, 6},
    {"dcor_R_dp_mean", (DL_FUNC)&dcor_R_dp_mean, 5},
    {"dcor_R_standardize_dp", (DL_FUNC)&dcor_R_standardize_dp, 6},
    {"dcor_R_ci_NI_signbatch", (DL_FUNC)&dcor_R_ci_NI_signbatch, 9},
    {"dcor_R_ci_INT_signflip", (DL_FUNC)&dcor_R_ci_INT_signflip, 12},
    {"dcor_R_correlation_NI_subG", (DL_FUNC)&dcor_R_correlation_NI_subG, 13},
    {"dcor_R_ci_INT_subG", (DL_FUNC)&dcor_R_ci_INT_subG, 16},
    {"dcor_R_int_subg_sd_uc", (DL_FUNC)&dcor_R_int_subg_sd_uc, 8},
    {"dcor_R_gen_bernoulli", (DL_FUNC)&dcor_R_gen_bernoulli, 3},
    {"dcor_R_gen_bounded_factor", (DL_FUNC)&dcor_R_gen_bounded_factor, 3},
    {"dcor_R_mvrnorm", (DL_FUNC)&dcor_R_mvrnorm, 5},
    {"dcor_R_mix_gaussian", (DL_FUNC)&dcor_R_mix_gaussian, 10},
    {"dcor_R_grid_run", (DL_FUNC)&dcor_R_grid_run, 20},
    {NULL, NULL, 0}};

void R_init_dcor_r(DllInfo* dll) {
  R_registerRoutines(dll, NULL, calls, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
