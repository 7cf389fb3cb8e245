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
#include <math.h>
#include <string.h>

#include "dcor.h"

static void dcor_stop(int st) {
  char msg[512];
  dcor_last_error(msg, sizeof msg);
  Rf_error("dcor: %s (status %d)", msg, st);
}

static double num(SEXP x) { return Rf_asReal(x); }
static const double* dptr_or_null(SEXP x) { return Rf_isNull(x) ? NULL : REAL(x); }

/* Argument checks the R wrappers always satisfy, for direct .Call use: the C side reads exactly
 * these lengths. */
static void need_len(SEXP x, R_xlen_t n, const char* what) {
  if (XLENGTH(x) != n) Rf_error("dcor: %s must have length %lld (got %lld)", what, (long long)n,
                                (long long)XLENGTH(x));
}
static void need_same_xy(SEXP X, SEXP Y) {
  if (XLENGTH(X) != XLENGTH(Y)) Rf_error("dcor: X and Y must have the same length");
}
/* The NI batch count the entry reads k Laplace draws for (vert-cor.R:207-208; ver-cor-subG.R:36-38;
 * real-data-sims.R:126-130). */
static R_xlen_t ni_k(R_xlen_t n, double e1, double e2, int subg, int hrs) {
  double m = ceil(8.0 / (e1 * e2));
  if (subg && m > (double)n) m = (double)n;
  double k = m > 0 ? floor((double)n / m) : 0;
  if (hrs && k < 2) k = 2;
  return (R_xlen_t)k;
}

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
  need_len(l, XLENGTH(z), "l");
  double o;
  const int st = dcor_mixquant(REAL(z), REAL(l), XLENGTH(z), num(c), num(p), &o);
  if (st) dcor_stop(st);
  return ScalarReal(o);
}

SEXP dcor_R_priv_standardize(SEXP v, SEXP eps, SEXP L, SEXP lap) {
  need_len(lap, 2, "lap");
  SEXP r = PROTECT(allocVector(REALSXP, XLENGTH(v)));
  const int st = dcor_priv_standardize(REAL(v), XLENGTH(v), num(eps), num(L), REAL(lap), REAL(r));
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_dp_sd(SEXP x, SEXP lo, SEXP hi, SEXP e1, SEXP e2, SEXP lap) {
  need_len(lap, 2, "lap");
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
  need_same_xy(X, Y);
  if (!Rf_isNull(lap_sc)) need_len(lap_sc, 4, "lap_sc");
  const R_xlen_t k = ni_k(XLENGTH(X), num(e1), num(e2), 0, 0);
  need_len(lap_x, k, "lap_x");
  need_len(lap_y, k, "lap_y");
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
  need_same_xy(X, Y);
  need_len(flips, n, "flips");
  if (!Rf_isNull(lap_sc)) need_len(lap_sc, 4, "lap_sc");
  need_len(ml, XLENGTH(mz), "mix_l");
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
  need_same_xy(X, Y);
  const int hrs_ = Rf_asLogical(hrs);
  const R_xlen_t k = ni_k(XLENGTH(X), num(e1), num(e2), 1, hrs_);
  need_len(lap_x, k, "lap_x");
  need_len(lap_y, k, "lap_y");
  if (!Rf_isNull(perm) && hrs_) {
    const R_xlen_t m = k == 2 && ni_k(XLENGTH(X), num(e1), num(e2), 1, 0) < 2
                           ? XLENGTH(X) / 2 : (R_xlen_t)fmin(ceil(8.0 / (num(e1) * num(e2))), (double)XLENGTH(X));
    need_len(perm, k * m, "perm");
  }
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
  need_same_xy(X, Y);
  need_len(lap_local, XLENGTH(X), "lap_local");
  need_len(ml, XLENGTH(mz), "mix_l");
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
  need_same_xy(X, Y);
  need_len(lap_local, XLENGTH(X), "lap_local");
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
  if (XLENGTH(v) != n) Rf_error("dcor: gen_bernoulli needs u and v of the same length");
  SEXP r = PROTECT(xy_matrix(n));
  const int st = dcor_gen_bernoulli(REAL(u), REAL(v), n, num(rho), REAL(r), REAL(r) + n);
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

SEXP dcor_R_gen_bounded_factor(SEXP U, SEXP E1, SEXP E2) {
  const R_xlen_t n = XLENGTH(U);
  if (XLENGTH(E1) != n || XLENGTH(E2) != n)
    Rf_error("dcor: gen_bounded_factor needs U, E1 and E2 of the same length");
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
  if (XLENGTH(mu0) != 2 || XLENGTH(sigma0) != 2 || XLENGTH(mu1) != 2 || XLENGTH(sigma1) != 2)
    Rf_error("dcor: gen_mix_gaussian needs mu0, sigma0, mu1, sigma1 of length 2");
  SEXP r = PROTECT(xy_matrix(n0 + n1));
  const int st = dcor_mix_gaussian(REAL(z0), n0, REAL(z1), n1, INTEGER(perm), num(rho), REAL(mu0),
                                   REAL(sigma0), REAL(mu1), REAL(sigma1), REAL(r),
                                   REAL(r) + (n0 + n1));
  UNPROTECT(1);
  if (st) dcor_stop(st);
  return r;
}

/* ---- the grid scripts' output tables (vert-cor.R:556-597; ver-cor-subG.R:301-333) ---------- */
/* run_sim_one's detail columns: vert-cor.R:367-385 (sign family) and ver-cor-subG.R:170-172 +
 * 201-206 (sub-G); then the setting columns the merge loops append. */
static const char* const DETAIL_SIGN[17] = {
    "repl", "ni_hat", "int_hat", "ni_se2", "int_se2", "ni_low", "ni_up", "int_low", "int_up",
    "ni_cover", "int_cover", "ni_ci_len", "int_ci_len", "n", "rho_true", "eps1", "eps2"};
static const char* const DETAIL_SUBG[17] = {
    "repl", "ni_hat", "ni_low", "ni_up", "int_hat", "int_low", "int_up", "ni_se2", "int_se2",
    "ni_cover", "int_cover", "ni_ci_len", "int_ci_len", "n", "rho_true", "eps1", "eps2"};
static const char* const SUMM_COLS[9] = {"n", "rho_true", "eps1", "eps2", "mse", "bias",
                                         "coverage", "ci_len", "method"};

static void set_frame_attrs(SEXP df, const char* const* names, int ncol, R_xlen_t nrow) {
  SEXP nm = PROTECT(allocVector(STRSXP, ncol));
  for (int j = 0; j < ncol; ++j) SET_STRING_ELT(nm, j, mkChar(names[j]));
  setAttrib(df, R_NamesSymbol, nm);
  SEXP rn = PROTECT(allocVector(INTSXP, 2));   /* compact row names c(NA, -nrow) */
  INTEGER(rn)[0] = NA_INTEGER;
  INTEGER(rn)[1] = -(int)nrow;
  setAttrib(df, R_RowNamesSymbol, rn);
  setAttrib(df, R_ClassSymbol, mkString("data.frame"));
  UNPROTECT(2);
}

/* R's `rho >= lo && rho <= up` (vert-cor.R:405,416) / `rho >= lo & rho <= up` (ver-cor-subG.R:
 * 203-204): FALSE if either comparison is FALSE, NA if neither is and one is NA, else TRUE. */
static int r_cover(double rho, double lo, double up) {
  const int a = ISNAN(lo) ? NA_INTEGER : (rho >= lo), b = ISNAN(up) ? NA_INTEGER : (rho <= up);
  if (a == 0 || b == 0) return 0;
  if (a == NA_INTEGER || b == NA_INTEGER) return NA_INTEGER;
  return 1;
}

/* detail_all = rbindlist of the cells' run_sim_one detail frames with n, rho_true, eps1, eps2
 * appended (vert-cor.R:556-568; ver-cor-subG.R:303-314).  The column order and the cover type
 * follow the family of the first cell: integer 0/1/NA for the sign family, whose frame starts the
 * columns as NA_integer_ (vert-cor.R:381-382), logical for sub-G (ver-cor-subG.R:203-204). */
static SEXP detail_all_frame(const dcor_cell* cells, int nc, long long B, const double* rec) {
  const int sign = cells[0].family == DCOR_FAMILY_SIGN;
  const char* const* names = sign ? DETAIL_SIGN : DETAIL_SUBG;
  const R_xlen_t nrow = (R_xlen_t)nc * B;
  SEXP df = PROTECT(allocVector(VECSXP, 17));
  SEXP col[17];
  for (int j = 0; j < 17; ++j) {
    const char* nm = names[j];
    const int type = strcmp(nm, "repl") == 0 ? INTSXP
                     : (strcmp(nm, "ni_cover") == 0 || strcmp(nm, "int_cover") == 0)
                         ? (sign ? INTSXP : LGLSXP) : REALSXP;
    col[j] = allocVector(type, nrow);
    SET_VECTOR_ELT(df, j, col[j]);
  }
  for (int i = 0; i < nc; ++i) {
    const double rho = cells[i].rho;
    for (long long b = 0; b < B; ++b) {
      const R_xlen_t r = (R_xlen_t)i * B + b;
      const double* o = rec + 6 * r;   /* ni_hat, ni_low, ni_up, int_hat, int_low, int_up */
      for (int j = 0; j < 17; ++j) {
        const char* nm = names[j];
        double v = 0;
        int iv = 0, is_int = 0;
        if (!strcmp(nm, "repl")) { iv = (int)(b + 1); is_int = 1; }
        else if (!strcmp(nm, "ni_hat")) v = o[0];
        else if (!strcmp(nm, "ni_low")) v = o[1];
        else if (!strcmp(nm, "ni_up")) v = o[2];
        else if (!strcmp(nm, "int_hat")) v = o[3];
        else if (!strcmp(nm, "int_low")) v = o[4];
        else if (!strcmp(nm, "int_up")) v = o[5];
        else if (!strcmp(nm, "ni_se2")) v = (o[0] - rho) * (o[0] - rho);      /* (hat - rho)^2 */
        else if (!strcmp(nm, "int_se2")) v = (o[3] - rho) * (o[3] - rho);
        else if (!strcmp(nm, "ni_cover")) { iv = r_cover(rho, o[1], o[2]); is_int = 1; }
        else if (!strcmp(nm, "int_cover")) { iv = r_cover(rho, o[4], o[5]); is_int = 1; }
        else if (!strcmp(nm, "ni_ci_len")) v = o[2] - o[1];                     /* diff(ci) */
        else if (!strcmp(nm, "int_ci_len")) v = o[5] - o[4];
        else if (!strcmp(nm, "n")) v = (double)cells[i].n;
        else if (!strcmp(nm, "rho_true")) v = rho;
        else if (!strcmp(nm, "eps1")) v = cells[i].eps1;
        else v = cells[i].eps2;
        if (is_int) ((int*)(TYPEOF(col[j]) == INTSXP ? (void*)INTEGER(col[j]) : (void*)LOGICAL(col[j])))[r] = iv;
        else REAL(col[j])[r] = v;
      }
    }
  }
  set_frame_attrs(df, names, 17, nrow);
  UNPROTECT(1);
  return df;
}

/* summ_all = rbindlist(summ_NI, summ_INT) (vert-cor.R:573-597; ver-cor-subG.R:319-333): per
 * (n, rho_true, eps1, eps2) group of detail_all (data.table's `by`, groups in first-appearance
 * order) mse, bias = mean(hat) - mean(rho_true), coverage, ci_len, then `method`.  From the device
 * accumulators: cells sharing a key are pooled by merging their accumulators in cell order, and
 * dcor_accum_finalize takes the means (NA if any member is NA, as mean() without na.rm). */
static SEXP summ_all_frame(const dcor_cell* cells, int nc, const dcor_accum* acc) {
  int* grp = (int*)R_alloc(nc, sizeof(int));
  int* first = (int*)R_alloc(nc, sizeof(int));
  int ng = 0;
  for (int i = 0; i < nc; ++i) {
    int g = -1;
    for (int q = 0; q < ng && g < 0; ++q) {
      const dcor_cell* c = &cells[first[q]];
      if ((double)c->n == (double)cells[i].n && c->rho == cells[i].rho && c->eps1 == cells[i].eps1 &&
          c->eps2 == cells[i].eps2)
        g = q;
    }
    if (g < 0) { g = ng++; first[g] = i; }
    grp[i] = g;
  }
  dcor_accum* pooled = (dcor_accum*)R_alloc((size_t)ng * 2, sizeof(dcor_accum));
  memset(pooled, 0, (size_t)ng * 2 * sizeof(dcor_accum));
  for (int i = 0; i < nc; ++i)
    for (int m = 0; m < 2; ++m) dcor_accum_merge(&pooled[2 * grp[i] + m], &acc[2 * i + m]);
  const R_xlen_t nrow = 2 * (R_xlen_t)ng;
  SEXP df = PROTECT(allocVector(VECSXP, 9));
  for (int j = 0; j < 8; ++j) SET_VECTOR_ELT(df, j, allocVector(REALSXP, nrow));
  SEXP meth = allocVector(STRSXP, nrow);
  SET_VECTOR_ELT(df, 8, meth);
  for (int m = 0; m < 2; ++m)             /* summ_NI rows first, then summ_INT */
    for (int g = 0; g < ng; ++g) {
      const dcor_cell* c = &cells[first[g]];
      dcor_summary sm;
      dcor_accum_finalize(&pooled[2 * g + m], c->rho, &sm);
      const R_xlen_t r = (R_xlen_t)m * ng + g;
      const double v[8] = {(double)c->n, c->rho, c->eps1, c->eps2, sm.mse, sm.bias, sm.coverage,
                           sm.ci_length};
      for (int j = 0; j < 8; ++j) REAL(VECTOR_ELT(df, j))[r] = v[j];
      SET_STRING_ELT(meth, r, mkChar(m == 0 ? "NI" : "INT"));
    }
  set_frame_attrs(df, SUMM_COLS, 9, nrow);
  UNPROTECT(1);
  return df;
}

/* One grid: cells given as parallel vectors (one element per cell).  rng_r: R's own streams
 * (dcor_rstream_grid_run, one device) instead of the Philox engine, which shards every cell's
 * replicates over `devices` (0-based HIP ids; empty: every visible GPU).  Returns
 * list(summary [cell][method][mse, bias, var, coverage, ci_length], detail records (nc B x 6, or
 * empty), detail_all (data.frame, or NULL without detail), summ_all (data.frame)). */
SEXP dcor_R_grid_run(SEXP family, SEXP dgp, SEXP n, SEXP rho, SEXP eps1, SEXP eps2, SEXP alpha,
                     SEXP mu1, SEXP mu2, SEXP s1, SEXP s2, SEXP normalise, SEXP mode, SEXP seed,
                     SEXP B, SEXP want_detail, SEXP mix, SEXP rng_r, SEXP nsim, SEXP devices) {
  /* mix: gen_mix_gaussian's mu0[2], sigma0[2], mu1[2], sigma1[2], pi_mix (ver-cor-subG.R:116-118) */
  if (XLENGTH(mix) != 9) Rf_error("dcor_grid: mix must hold 9 numbers");
  const double* mx = REAL(mix);
  const int nc = LENGTH(n);
  {
    SEXP per_cell[] = {family, dgp, rho, eps1, eps2, alpha, mu1, mu2, s1, s2, normalise, mode, seed, nsim};
    for (size_t q = 0; q < sizeof per_cell / sizeof per_cell[0]; ++q)
      if (LENGTH(per_cell[q]) != nc) Rf_error("dcor_grid: every per-cell argument needs %d values", nc);
  }
  const double bd = Rf_asReal(B);
  if (!(bd >= 1) || bd != floor(bd)) Rf_error("dcor_grid: B must be a positive whole number");
  const long long b = (long long)bd;
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
  const int detail = Rf_asLogical(want_detail) == 1;
  SEXP acc = PROTECT(allocVector(RAWSXP, (R_xlen_t)nc * 2 * sizeof(dcor_accum)));
  SEXP det = PROTECT(detail ? allocVector(REALSXP, (R_xlen_t)nc * b * 6) : allocVector(REALSXP, 0));
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
  SEXP out = PROTECT(allocVector(VECSXP, 4));
  SET_VECTOR_ELT(out, 0, sm);
  SET_VECTOR_ELT(out, 1, det);
  if (detail && nc > 0) SET_VECTOR_ELT(out, 2, detail_all_frame(cells, nc, b, REAL(det)));
  if (nc > 0) SET_VECTOR_ELT(out, 3, summ_all_frame(cells, nc, (const dcor_accum*)RAW(acc)));
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
