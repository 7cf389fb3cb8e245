/*
 * dcor_rstream.c -- CPU restatement of R's own random streams as the reference's replicate
 * loop consumes them (the "R-stream" mode).
 *
 * TEST INFRASTRUCTURE ONLY, like dcor_oracle.c: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * What is restated.  R's generators are not in /root/reference; this follows R's C sources
 * (R >= 3.6 defaults: RNGkind "Mersenne-Twister", "Inversion", "Rejection"):
 *   set.seed(s)      RNG_Init: seed = 69069 seed + 1 fifty times, then 625 more words;
 *                    word 0 is MT's position (set to 624), words 1..624 the state.
 *   unif_rand()      MT19937 genrand: tempered word * 2.3283064365386963e-10, then fixup
 *                    into (0, 1).
 *   norm_rand()      INVERSION: u = (int)(2^27 u1) + u2, qnorm5(u / 2^27) (AS241).
 *   exp_rand()       Ahrens & Dieter (1972), algorithm SA, with R's q[] table.
 *   rbinom(1, p)     the inverse-cdf branch (n p < 30) of R's rbinom.
 *   runif(a, b)      a + (b - a) u; a == b returns a without drawing.
 *   extraDistr::rlaplace(n, mu, sigma)  mu - sigma sign(u) log(1 - 2|u|), u = runif(-.5, .5)
 *                    (vert-cor.R:106,188).
 *   MASS::mvrnorm    eigen(Sigma, symmetric = TRUE) -> LAPACK dsyevr; for a 2x2 matrix
 *                    dsytrd is the identity and dstemr takes its n = 2 branch (dlaev2), R
 *                    reverses to decreasing order; X = mu + (V %*% diag(sqrt(ev))) %*% t(Z)
 *                    with reference-BLAS dgemm accumulation order (vert-cor.R:389-394).
 * Draw order per replicate: SURVEY.md Appendix A (vert-cor.R:392-417; ver-cor-subG.R:174-197).
 *
 * PARITY STATUS.  R is absent from this image.  The generators are pinned by values R
 * prints for set.seed(1/42/123) followed by runif/rnorm/rexp (tests/golden/r_known_values.json,
 * 7-8 significant digits), and qnorm5 against scipy's ndtri; the eigen() branch is pinned by
 * the vectors R prints for two 2x2 matrices.  Everything else is "parity unpinned".
 *
 * log().  R calls the platform libm.  Here, and bit-identically on the GPU, log is an
 * accurate double-double evaluation (rs_log: relative error below 2^-69 before the final
 * rounding), i.e. correctly rounded except with probability ~2^-16 per call; glibc's log
 * (<= 0.52 ulp) agrees with it on almost every input (tests/test_rstream.py measures it).
 * Draws that need no log (uniforms, Bernoulli, exp_rand, 85 % of normals) are exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dcor.h"
#include "dcor_oracle.h"
#define DCOR_TABLE_ATTR
#include "../distributed-correlation_amd/csrc/dcor_tables.h"

/* --------------------------------------------------------------- MT19937 */
#define MT_N 624
#define MT_M 397

void orc_rs_set_seed(orc_rs_state* st, int32_t seed) {
  uint32_t s = (uint32_t)seed;
  for (int j = 0; j < 50; ++j) s = 69069u * s + 1u;           /* initial scrambling */
  uint32_t words[MT_N + 1];
  for (int j = 0; j < MT_N + 1; ++j) { s = 69069u * s + 1u; words[j] = s; }
  for (int j = 0; j < MT_N; ++j) st->mt[j] = words[j + 1];
  st->mti = MT_N;                                              /* FixupSeeds(initial) */
}

uint32_t orc_rs_word(orc_rs_state* st) {
  static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
  uint32_t* mt = st->mt;
  uint32_t y;
  if (st->mti >= MT_N) {
    int kk;
    for (kk = 0; kk < MT_N - MT_M; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < MT_N - 1; kk++) {
      y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
      mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt[MT_N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    st->mti = 0;
  }
  y = mt[st->mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double orc_rs_word_unif(uint32_t w) {
  const double i2_32m1 = 2.328306437080797e-10; /* 1/(2^32 - 1) */
  const double x = (double)w * 2.3283064365386963e-10;
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

double orc_rs_unif(orc_rs_state* st) { return orc_rs_word_unif(orc_rs_word(st)); }

/* ------------------------------------------------------- accurate log ---- */
static inline void two_sum(double a, double b, double* s, double* e) {
  const double t = a + b, bb = t - a;
  *s = t;
  *e = (a - (t - bb)) + (b - bb);
}

double orc_rs_log(double x) {
  /* x positive, normal, finite (all R-stream arguments are).  x = 2^k z with z in
   * [0.6875, 1.375); r = z/c - 1 = z*invc - 1 is exact as rh + e; log1p(r) with r^2/2 in
   * double-double and the r^3.. tail in double; log c as a double-double from the table. */
  uint64_t ix;
  memcpy(&ix, &x, 8);
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127u);
  const int64_t k = (int64_t)tmp >> 52;
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  double z;
  memcpy(&z, &iz, 8);
  const double invc = dcor_log_tab[i][0], lch = dcor_log_tab[i][1], lcl = dcor_log_tab_lo[i];
  const double p = z * invc;
  const double pe = fma(z, invc, -p);
  double r1, r2;
  two_sum(p - 1.0, pe, &r1, &r2);               /* r = r1 + r2 exactly */
  const double s2 = r1 * r1;
  const double s2e = fma(r1, r1, -s2);
  const double h = -0.5 * s2;                    /* exact */
  const double hl = -0.5 * (s2e + 2.0 * r1 * r2);
  double t = DCOR_RS_LOG1P_C10;
  t = fma(t, r1, DCOR_RS_LOG1P_C9);
  t = fma(t, r1, DCOR_RS_LOG1P_C8);
  t = fma(t, r1, DCOR_RS_LOG1P_C7);
  t = fma(t, r1, DCOR_RS_LOG1P_C6);
  t = fma(t, r1, DCOR_RS_LOG1P_C5);
  t = fma(t, r1, DCOR_RS_LOG1P_C4);
  t = fma(t, r1, DCOR_RS_LOG1P_C3);
  const double tail = (r1 * s2) * t;
  double a1, a2;
  two_sum(r1, h, &a1, &a2);                      /* log1p(r) = a1 + (a2 + ...) */
  const double kd = (double)k;
  double s, se, s3, se3;
  two_sum(kd * DCOR_LN2_HI, lch, &s, &se);       /* k ln2_hi is exact */
  two_sum(s, a1, &s3, &se3);
  const double lo = se + se3 + (a2 + hl + r2 + tail) + (kd * DCOR_LN2_LO + lcl);
  return s3 + lo;
}

/* ------------------------------------------------------ qnorm5 (AS241) --- */
double orc_rs_qnorm5(double p) {
  /* R's qnorm(p, 0, 1, lower.tail = TRUE, log.p = FALSE) for p in (0, 1) */
  const double q = p - 0.5;
  double r, val;
  if (fabs(q) <= .425) {
    r = .180625 - q * q;
    val = q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r +
                    67265.770927008700853) * r + 45921.953931549871457) * r +
                  13731.693765509461125) * r + 1971.5909503065514427) * r +
                133.14166789178437745) * r + 3.387132872796366608) /
          (((((((r * 5226.495278852545925 + 28729.085735721942674) * r +
                39307.89580009271061) * r + 21213.794301586595867) * r +
              5394.1960214247511077) * r + 687.1870074920579083) * r +
            42.313330701600911252) * r + 1.);
    return val;
  }
  r = (q > 0) ? (0.5 - p + 0.5) : p;            /* R_DT_CIv(p) : p */
  r = sqrt(-orc_rs_log(r));
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
  if (q < 0.0) val = -val;
  return val;
}

/* ----------------------------------------------------------- variates ---- */
double orc_rs_norm_words(uint32_t w1, uint32_t w2) {
  const double BIG = 134217728.0; /* 2^27 */
  double u = orc_rs_word_unif(w1);
  u = (int)(BIG * u) + orc_rs_word_unif(w2);
  return orc_rs_qnorm5(u / BIG);
}

double orc_rs_norm(orc_rs_state* st) {
  const uint32_t w1 = orc_rs_word(st);
  const uint32_t w2 = orc_rs_word(st);
  return orc_rs_norm_words(w1, w2);
}

/* q[k-1] = sum_{j=1..k} ln2^j / j!  (R's exp_rand table, sexp.c) */
const double orc_rs_exp_q[16] = {
    0.6931471805599453, 0.9333736875190459, 0.9888777961838675, 0.9984959252914960040,
    0.9998292811061389, 0.9999833164100727, 0.9999985691438767, 0.9999998906925558,
    0.9999999924734159, 0.9999999995283275, 0.9999999999728814, 0.9999999999985598,
    0.9999999999999289, 0.9999999999999968, 0.9999999999999999, 1.0000000000000000};

double orc_rs_exp(orc_rs_state* st) {
  const double* q = orc_rs_exp_q;
  double a = 0.;
  double u = orc_rs_unif(st);
  while (u <= 0. || u >= 1.) u = orc_rs_unif(st);
  for (;;) {
    u += u;
    if (u > 1.) break;
    a += q[0];
  }
  u -= 1.;
  if (u <= q[0]) return a + u;
  int i = 0;
  double ustar = orc_rs_unif(st), umin = ustar;
  do {
    ustar = orc_rs_unif(st);
    if (umin > ustar) umin = ustar;
    i++;
  } while (u > q[i]);
  return a + umin * q[0];
}

double orc_rs_rbinom1(orc_rs_state* st, double pp) {
  /* rbinom(1, pp): size 1 < 30/p always takes the inverse-cdf branch */
  if (pp == 0.) return 0.;
  if (pp == 1.) return 1.;
  const int n = 1;
  const double p = fmin(pp, 1. - pp);
  const double q = 1. - p;
  const double r = p / q;
  const double g = r * (n + 1);
  const double qn = q; /* R_pow_int(q, 1) */
  int ix;
  for (;;) {
    ix = 0;
    double f = qn;
    double u = orc_rs_unif(st);
    for (;;) {
      if (u < f) goto finis;
      if (ix > 110) break;
      u -= f;
      ix++;
      f *= (g / ix - r);
    }
  }
finis:
  if (pp > 0.5) ix = n - ix;
  return (double)ix;
}

double orc_rs_runif(orc_rs_state* st, double a, double b) {
  if (!isfinite(a) || !isfinite(b) || b < a) return NAN;
  if (a == b) return a;
  double u;
  do { u = orc_rs_unif(st); } while (u <= 0 || u >= 1);
  return a + (b - a) * u;
}

double orc_rs_laplace_unit_word(uint32_t w) {
  /* extraDistr::rlaplace(1, 0, 1): 0 - 1*sign(u)*log(1 - 2|u|), u = runif(-.5, .5).  The
   * engine scales unit draws by sigma: sigma*(-sign(u) log(..)) == 0 - sigma*sign(u)*log(..)
   * bit for bit. */
  const double u = -0.5 + (0.5 - -0.5) * orc_rs_word_unif(w);
  if (u == 0.0) return 0.0;
  const double l = orc_rs_log(1.0 - 2.0 * fabs(u));
  return (u > 0) ? -l : l;
}

/* ------------------------------------------------------ MASS::mvrnorm ---- */
static void dlaev2(double a, double b, double c, double* rt1, double* rt2, double* cs1,
                   double* sn1) {
  double sm = a + c, df = a - c, adf = fabs(df), tb = b + b, ab = fabs(tb);
  double acmx, acmn, rt, cs, ct, tn;
  int sgn1, sgn2;
  if (fabs(a) > fabs(c)) { acmx = a; acmn = c; } else { acmx = c; acmn = a; }
  if (adf > ab) {
    const double t = ab / adf;
    rt = adf * sqrt(1.0 + t * t);
  } else if (adf < ab) {
    const double t = adf / ab;
    rt = ab * sqrt(1.0 + t * t);
  } else {
    rt = ab * sqrt(2.0);
  }
  if (sm < 0.0) {
    *rt1 = 0.5 * (sm - rt);
    sgn1 = -1;
    *rt2 = (acmx / *rt1) * acmn - (b / *rt1) * b;
  } else if (sm > 0.0) {
    *rt1 = 0.5 * (sm + rt);
    sgn1 = 1;
    *rt2 = (acmx / *rt1) * acmn - (b / *rt1) * b;
  } else {
    *rt1 = 0.5 * rt;
    *rt2 = -0.5 * rt;
    sgn1 = 1;
  }
  if (df >= 0.0) { cs = df + rt; sgn2 = 1; } else { cs = df - rt; sgn2 = -1; }
  const double acs = fabs(cs);
  if (acs > ab) {
    ct = -tb / cs;
    *sn1 = 1.0 / sqrt(1.0 + ct * ct);
    *cs1 = ct * *sn1;
  } else {
    if (ab == 0.0) {
      *cs1 = 1.0;
      *sn1 = 0.0;
    } else {
      tn = -cs / tb;
      *cs1 = 1.0 / sqrt(1.0 + tn * tn);
      *sn1 = tn * *cs1;
    }
  }
  if (sgn1 == sgn2) {
    tn = *cs1;
    *cs1 = -*sn1;
    *sn1 = tn;
  }
}

void orc_rs_eigen2(double a, double b, double c, double values[2], double vectors[4]) {
  /* eigen(matrix(c(a, b, b, c), 2), symmetric = TRUE): values decreasing, vectors
   * column-major {V11, V21, V12, V22} */
  double r1, r2, cs, sn;
  dlaev2(a, b, c, &r1, &r2, &cs, &sn);
  int swap = 0;
  if (r1 < r2) { const double t = r1; r1 = r2; r2 = t; swap = 1; }
  /* dstemr: W(1) = R2 with Z(:,1), W(2) = R1 with Z(:,2); R reverses the order */
  const double z1a = swap ? cs : -sn, z1b = swap ? sn : cs;
  const double z2a = swap ? -sn : cs, z2b = swap ? cs : sn;
  values[0] = r1; values[1] = r2;
  vectors[0] = z2a; vectors[1] = z2b;
  vectors[2] = z1a; vectors[3] = z1b;
}

void orc_rs_mvrnorm_factor(const double sigma[2], double rho, double A[4]) {
  /* Sigma as vert-cor.R:389-390 / ver-cor-subG.R:119-122; A = V %*% diag(sqrt(pmax(ev, 0)))
   * row-major {A11, A12, A21, A22} with dgemm's accumulation (C = 0; C += D(l,j) V(i,l)). */
  const double s11 = sigma[0] * sigma[0], s12 = sigma[0] * sigma[1] * rho,
               s22 = sigma[1] * sigma[1];
  double ev[2], V[4];
  orc_rs_eigen2(s11, s12, s22, ev, V);
  const double d0 = sqrt(fmax(ev[0], 0.0)), d1 = sqrt(fmax(ev[1], 0.0));
  const double V11 = V[0], V21 = V[1], V12 = V[2], V22 = V[3];
  A[0] = (0.0 + d0 * V11) + 0.0 * V12;
  A[1] = (0.0 + 0.0 * V11) + d1 * V12;
  A[2] = (0.0 + d0 * V21) + 0.0 * V22;
  A[3] = (0.0 + 0.0 * V21) + d1 * V22;
}

/* ----------------------------------------------- replicate draw driver --- */
static void rs_laplace_n(orc_rs_state* st, int64_t n, double* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = orc_rs_laplace_unit_word(orc_rs_word(st));
}

static void rs_mixquant_draws(orc_rs_state* st, int64_t nsim, double* z, double* l) {
  /* rnorm(nsim) + c*rexp(nsim)*(2*rbinom(nsim,1,0.5)-1)  (vert-cor.R:47): l = +-rexp */
  for (int64_t j = 0; j < nsim; ++j) z[j] = orc_rs_norm(st);
  for (int64_t j = 0; j < nsim; ++j) l[j] = orc_rs_exp(st);
  for (int64_t j = 0; j < nsim; ++j) l[j] = l[j] * (2 * orc_rs_rbinom1(st, 0.5) - 1);
}

int orc_rs_geometry(const void* cellp, int64_t* k_out, int* mix_out) {
  const dcor_cell* c = (const dcor_cell*)cellp;
  const int64_t n = c->n;
  double m = ceil(8.0 / (c->eps1 * c->eps2));
  if (c->family == DCOR_FAMILY_SUBG && m > (double)n) m = (double)n;
  const double kd = floor((double)n / m);
  if (!(kd >= 1)) return DCOR_EKLT1;
  *k_out = (int64_t)kd;
  if (c->family == DCOR_FAMILY_SUBG) {
    *mix_out = 1;
  } else {
    const double eps_r = (c->eps1 >= c->eps2) ? c->eps2 : c->eps1;
    int mode = c->ci_mode;
    if (mode == DCOR_MODE_AUTO) mode = (sqrt((double)n) * eps_r > 0.5) ? DCOR_MODE_NORMAL : DCOR_MODE_LAPLACE;
    *mix_out = (mode == DCOR_MODE_NORMAL);
  }
  return DCOR_OK;
}

int orc_rs_draw_rep(orc_rs_state* st, const void* cellp, orc_rs_draws* d) {
  const dcor_cell* c = (const dcor_cell*)cellp;
  const int64_t n = c->n, nsim = c->nsim;
  int64_t k;
  int mix;
  int s = orc_rs_geometry(cellp, &k, &mix);
  if (s) return s;
  /* 1. DGP */
  if (c->dgp == DCOR_DGP_GAUSSIAN) {
    double A[4];
    orc_rs_mvrnorm_factor(c->sigma, c->rho, A);
    double* z = (double*)malloc(sizeof(double) * (size_t)(2 * n));
    for (int64_t i = 0; i < 2 * n; ++i) z[i] = orc_rs_norm(st);   /* matrix(rnorm(2n), n) */
    for (int64_t i = 0; i < n; ++i) {
      d->X[i] = c->mu[0] + ((0.0 + z[i] * A[0]) + z[n + i] * A[1]);
      d->Y[i] = c->mu[1] + ((0.0 + z[i] * A[2]) + z[n + i] * A[3]);
    }
    free(z);
  } else if (c->dgp == DCOR_DGP_BERNOULLI) {
    double* u = (double*)malloc(sizeof(double) * (size_t)(2 * n));
    for (int64_t i = 0; i < 2 * n; ++i) u[i] = orc_rs_runif(st, 0.0, 1.0);
    orc_gen_bernoulli(u, u + n, n, c->rho, d->X, d->Y);
    free(u);
  } else if (c->dgp == DCOR_DGP_BOUNDED_FACTOR) {
    const double cU = sqrt(3 * c->rho), cE = sqrt(3 * (1 - c->rho));
    double* U = (double*)malloc(sizeof(double) * (size_t)n);
    for (int64_t i = 0; i < n; ++i) U[i] = orc_rs_runif(st, -cU, cU);
    for (int64_t i = 0; i < n; ++i) d->X[i] = U[i] + orc_rs_runif(st, -cE, cE);
    for (int64_t i = 0; i < n; ++i) d->Y[i] = U[i] + orc_rs_runif(st, -cE, cE);
    free(U);
  } else if (c->dgp == DCOR_DGP_MIX_GAUSSIAN) {
    /* gen_mix_gaussian (ver-cor-subG.R:113-136): labels <- rbinom(n, 1, pi_mix);
     * rbind(mvrnorm(n0, mu0, S0), mvrnorm(n1, mu1, S1))[sample.int(n), ], clipped to [-1, 1] */
    uint8_t* lab = (uint8_t*)malloc((size_t)n);
    int64_t n0 = 0;
    for (int64_t i = 0; i < n; ++i) {
      lab[i] = (uint8_t)orc_rs_rbinom1(st, c->mix_pi);
      n0 += (lab[i] == 0);
    }
    const int64_t n1 = n - n0;
    double A0[4], A1[4];
    orc_rs_mvrnorm_factor(c->mix_sigma0, c->rho, A0);
    orc_rs_mvrnorm_factor(c->mix_sigma1, c->rho, A1);
    double* z = (double*)malloc(sizeof(double) * (size_t)(2 * n + 1));
    for (int64_t i = 0; i < 2 * n; ++i) z[i] = orc_rs_norm(st);  /* 2 n0 then 2 n1 normals */
    double* rx = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    double* ry = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    for (int64_t r = 0; r < n0; ++r) {
      rx[r] = c->mix_mu0[0] + ((0.0 + z[r] * A0[0]) + z[n0 + r] * A0[1]);
      ry[r] = c->mix_mu0[1] + ((0.0 + z[r] * A0[2]) + z[n0 + r] * A0[3]);
    }
    const double* z1 = z + 2 * n0;
    for (int64_t r = 0; r < n1; ++r) {
      rx[n0 + r] = c->mix_mu1[0] + ((0.0 + z1[r] * A1[0]) + z1[n1 + r] * A1[1]);
      ry[n0 + r] = c->mix_mu1[1] + ((0.0 + z1[r] * A1[2]) + z1[n1 + r] * A1[3]);
    }
    int32_t* perm = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    orc_rs_sample_int(st, n, n, perm);
    for (int64_t i = 0; i < n; ++i) {     /* pmax(pmin(out, 1), -1) */
      double x = rx[perm[i]], y = ry[perm[i]];
      x = (x > 1.0) ? 1.0 : x; x = (x < -1.0) ? -1.0 : x;
      y = (y > 1.0) ? 1.0 : y; y = (y < -1.0) ? -1.0 : y;
      d->X[i] = x; d->Y[i] = y;
    }
    free(lab); free(z); free(rx); free(ry); free(perm);
  } else {
    return DCOR_EINVAL;
  }
  d->has_mix = mix;
  d->k = k;
  if (c->family == DCOR_FAMILY_SIGN) {
    /* 2. ci_NI_signbatch: priv_standardize X then Y (2 draws each), then rLap(k) x2 */
    if (c->normalise) rs_laplace_n(st, 4, d->lap_sc);
    rs_laplace_n(st, k, d->lap_ni_x);
    rs_laplace_n(st, k, d->lap_ni_y);
    /* 3. ci_INT_signflip: fresh standardisation, rbinom(n, 1, p), Z, then mixquant */
    if (c->normalise) rs_laplace_n(st, 4, d->lap_sc + 4);
    const int sender_is_X = (c->eps1 >= c->eps2);
    const double eps_s = sender_is_X ? c->eps1 : c->eps2;
    const double p = exp(eps_s) / (exp(eps_s) + 1);
    for (int64_t i = 0; i < n; ++i) d->flips[i] = (uint8_t)orc_rs_rbinom1(st, p);
    d->lap_scalar = orc_rs_laplace_unit_word(orc_rs_word(st));
  } else {
    /* 2. correlation_NI_subG: rLap(k) x2; 3. ci_INT_subG: rLap(n), rLap(1), mixquant */
    rs_laplace_n(st, k, d->lap_ni_x);
    rs_laplace_n(st, k, d->lap_ni_y);
    rs_laplace_n(st, n, d->lap_local);
    d->lap_scalar = orc_rs_laplace_unit_word(orc_rs_word(st));
  }
  if (mix) rs_mixquant_draws(st, nsim, d->mix_z, d->mix_l);
  return DCOR_OK;
}

int orc_rs_sim(const void* cellp, int64_t B, double* out) {
  /* run_sim_one's loop with R's streams: set.seed(seed), then B replicates in order
   * (vert-cor.R:364,392-419; ver-cor-subG.R:169,174-198).  out: B x 6. */
  const dcor_cell* c = (const dcor_cell*)cellp;
  const int64_t n = c->n, nsim = c->nsim;
  if (n < 1 || !(c->eps1 > 0) || !(c->eps2 > 0) || c->seed > 0x7fffffffull) return DCOR_EINVAL;
  if (orc_cell_check(c)) return DCOR_EINVAL;
  int64_t k;
  int mix;
  int s = orc_rs_geometry(cellp, &k, &mix);
  if (s) return s;
  orc_rs_state st;
  orc_rs_set_seed(&st, (int32_t)c->seed);
  orc_rs_draws d;
  memset(&d, 0, sizeof(d));
  d.X = (double*)malloc(sizeof(double) * (size_t)n);
  d.Y = (double*)malloc(sizeof(double) * (size_t)n);
  d.lap_ni_x = (double*)malloc(sizeof(double) * (size_t)k);
  d.lap_ni_y = (double*)malloc(sizeof(double) * (size_t)k);
  d.flips = (uint8_t*)malloc((size_t)n);
  d.lap_local = (double*)malloc(sizeof(double) * (size_t)n);
  d.mix_z = (double*)malloc(sizeof(double) * (size_t)(nsim + 1));
  d.mix_l = (double*)malloc(sizeof(double) * (size_t)(nsim + 1));
  for (int64_t b = 0; b < B && s == DCOR_OK; ++b) {
    s = orc_rs_draw_rep(&st, cellp, &d);
    if (s) break;
    double* o = out + 6 * b;
    if (c->family == DCOR_FAMILY_SIGN) {
      s = orc_ci_ni_signbatch(d.X, d.Y, n, c->eps1, c->eps2, c->alpha, c->normalise, d.lap_sc,
                              d.lap_ni_x, d.lap_ni_y, o);
      int md;
      if (!s)
        s = orc_ci_int_signflip(d.X, d.Y, n, c->eps1, c->eps2, c->alpha, c->ci_mode,
                                c->normalise, d.lap_sc + 4, d.flips, d.lap_scalar, d.mix_z,
                                d.mix_l, nsim, o + 3, &md);
    } else {
      s = orc_ni_subg(d.X, d.Y, n, c->eps1, c->eps2, c->eta1, c->eta2, c->alpha, 0, NAN, NAN,
                      NULL, d.lap_ni_x, d.lap_ni_y, o, NULL);
      if (!s)
        s = orc_int_subg(d.X, d.Y, n, c->eps1, c->eps2, c->eta1, c->eta2, c->alpha, 0, NAN, NAN,
                         NAN, NAN, d.lap_local, d.lap_scalar, d.mix_z, d.mix_l, nsim, o + 3,
                         NULL);
    }
  }
  free(d.X); free(d.Y); free(d.lap_ni_x); free(d.lap_ni_y); free(d.flips); free(d.lap_local);
  free(d.mix_z); free(d.mix_l);
  return s;
}

/* ------------------------------------------- HRS runs (real-data-sims.R) --- */
/* R_unif_index(dn) (R >= 3.6, sample.kind "Rejection"): rbits(ceil(log2(dn))) until < dn;
 * rbits takes floor(unif_rand() * 65536) per 16 bits. */
static double rs_unif_index(orc_rs_state* st, double dn) {
  if (dn <= 0) return 0.0;
  const int bits = (int)ceil(log2(dn));
  double dv;
  do {
    int64_t v = 0;
    for (int nn = 0; nn <= bits; nn += 16) {
      const int v1 = (int)floor(orc_rs_unif(st) * 65536);
      v = 65536 * v + v1;
    }
    dv = (double)(v & (((int64_t)1 << bits) - 1));
  } while (dn <= dv);
  return dv;
}

void orc_rs_sample_int(orc_rs_state* st, int64_t n, int64_t k, int32_t* out) {
  /* sample.int(n, k) without replacement (do_sample, uniform): 0-based */
  int32_t* x = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  for (int64_t i = 0; i < n; i++) x[i] = (int32_t)i;
  int64_t nn = n;
  for (int64_t i = 0; i < k; i++) {
    const int64_t j = (int64_t)rs_unif_index(st, (double)nn);
    out[i] = x[j];
    x[j] = x[--nn];
  }
  free(x);
}

void orc_rs_hrs_ni_draws(int32_t seed, int64_t n, int64_t k, int64_t m, int32_t* perm,
                         double* lap_x, double* lap_y) {
  /* run_NI_once (real-data-sims.R:357-373): set.seed, then correlation_NI_subG's draws:
   * idx <- sample.int(n, k*m) (:131), rLap(k) X, rLap(k) Y (:136-137; rLap :58-61) */
  orc_rs_state st;
  orc_rs_set_seed(&st, seed);
  orc_rs_sample_int(&st, n, k * m, perm);
  rs_laplace_n(&st, k, lap_x);
  rs_laplace_n(&st, k, lap_y);
}

void orc_rs_hrs_int_draws(int32_t seed, int64_t n, int64_t nsim, double* lap_local,
                          double* lap_central, double* mix_z, double* mix_l) {
  /* run_INT_once (real-data-sims.R:375-402): set.seed, then ci_INT_subG's draws: rLap(n)
   * (:224/:228), rLap(1) (:232), mixquant(nsim = 2000) (:161-164, :240-241) */
  orc_rs_state st;
  orc_rs_set_seed(&st, seed);
  rs_laplace_n(&st, n, lap_local);
  *lap_central = orc_rs_laplace_unit_word(orc_rs_word(&st));
  rs_mixquant_draws(&st, nsim, mix_z, mix_l);
}
