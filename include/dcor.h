/*
 * dcor.h -- C-ABI of the MI355X (gfx950) engine for the Monte-Carlo hot path of
 * abhinavc3/distributed-correlation (DP correlation across two servers, NI + INT).
 *
 * Drop-in boundary.  The reference's surface is a set of R closures
 * (vert-cor.R, ver-cor-subG.R, real-data-sims.R); its R wrappers call these
 * entry points through `.Call`.  Plain C types only: no torch,
 * no C++ across the ABI.  Every compute entry point runs on the GPU; there is no
 * CPU fallback (a missing device is an error, DCOR_ENODEV / DCOR_EHIP).
 *
 * Conventions
 *  - Status: every entry returns int (DCOR_OK = 0).  The message of the last
 *    failure on the calling thread is read with dcor_last_error().
 *  - Ownership: inputs are borrowed for the duration of the call; outputs go to
 *    caller-allocated buffers.  `*_launch` entries take DEVICE pointers and a
 *    hipStream_t (as void*) and are asynchronous; all other entries take HOST
 *    pointers and are synchronous.
 *  - Noise: explicit-input entries take UNIT-scale draws (Laplace(0,1), flip bits,
 *    mixquant normals/Laplace); the entry scales them exactly as the R code scales
 *    its own draws (scale * unit is bit-identical to extraDistr::rlaplace's
 *    mu - sigma*sign(u)*log(1-2|u|) at mu = 0).
 *  - NA: a statistic R would return as NA (e.g. sd of k = 1 batch products) is
 *    returned as NaN.
 */
#ifndef DCOR_H
#define DCOR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCOR_OK 0
#define DCOR_EINVAL 1  /* bad n / eps / lengths: the reference's stopifnot()          */
#define DCOR_EKLT1 2   /* fewer than one full batch (vert-cor.R:127,209; subG.R:38)    */
#define DCOR_EHIP 3    /* HIP runtime error                                            */
#define DCOR_ENOMEM 4
#define DCOR_ENODEV 5  /* no gfx950 device visible                                     */
#define DCOR_EFORK 6   /* called in a process forked (mclapply) after its parent had used the
                          engine: HIP does not survive fork(); run the grid from the parent
                          with one dcor_grid_run call instead            */

enum { DCOR_FAMILY_SIGN = 0, DCOR_FAMILY_SUBG = 1 };
enum { DCOR_DGP_GAUSSIAN = 0, DCOR_DGP_BERNOULLI = 1, DCOR_DGP_BOUNDED_FACTOR = 2,
       DCOR_DGP_MIX_GAUSSIAN = 3 /* gen_mix_gaussian, ver-cor-subG.R:113-133 */ };
enum { DCOR_MODE_AUTO = 0, DCOR_MODE_NORMAL = 1, DCOR_MODE_LAPLACE = 2 };

/* One (distribution, rho, eps, n) grid cell.  Replaces one row of
 * expand.grid(n, rho, eps_idx) plus run_sim_one's arguments
 * (vert-cor.R:356-362,507-511,542-552; ver-cor-subG.R:159-167,265-288). */
typedef struct dcor_cell {
  int32_t family;    /* DCOR_FAMILY_SIGN: ci_NI_signbatch + ci_INT_signflip          */
                     /* DCOR_FAMILY_SUBG: correlation_NI_subG + ci_INT_subG          */
  int32_t dgp;       /* DCOR_DGP_*                                                    */
  int64_t n;         /* samples per replicate                                         */
  double rho, eps1, eps2, alpha;
  double mu[2], sigma[2]; /* Gaussian DGP (MASS::mvrnorm), vert-cor.R:389-394          */
  double eta1, eta2;      /* sub-G calibration, ver-cor-subG.R:26                      */
  int32_t normalise;      /* sign family priv_standardize switch, vert-cor.R:211       */
  int32_t ci_mode;        /* DCOR_MODE_*, vert-cor.R:294-296                           */
  int64_t nsim;           /* mixquant draws (1000; 2000 in real-data-sims.R:161)       */
  uint64_t seed;          /* per-cell seed (R: 1e6 + i, vert-cor.R:552): Philox key    */
  /* DCOR_DGP_MIX_GAUSSIAN (ver-cor-subG.R:113-116; R defaults mu0 (0,0), sigma0 (1,1),
   * mu1 (3,3), sigma1 (2,.5), pi_mix .5): label ~ Bern(pi_mix), (X, Y) ~ mvrnorm of that
   * component with correlation rho, then pmax(pmin(., 1), -1). */
  double mix_mu0[2], mix_sigma0[2], mix_mu1[2], mix_sigma1[2];
  double mix_pi;
} dcor_cell;

/* Per-replicate result: the six numbers of one row of run_sim_one's `detail`
 * (vert-cor.R:401-417); se2 / cover / ci_len derive from these and rho. */
typedef struct dcor_rep_out {
  double ni_hat, ni_lo, ni_hi;
  double int_hat, int_lo, int_hi;
} dcor_rep_out;

/* Per-(cell, method) summary accumulator, mergeable across replicate ranges and
 * GPUs (sums are double-double {hi, lo}).  Finalised by dcor_accum_finalize into
 * run_sim_one's summary row (vert-cor.R:422-430; ver-cor-subG.R:208-210). */
typedef struct dcor_accum {
  int64_t n;          /* replicates accumulated                                      */
  int64_t n_cover;    /* cover TRUE  (rho >= lo && rho <= hi, R three-valued logic)  */
  int64_t n_cover_na; /* cover NA                                                    */
  int64_t n_na_est;   /* estimate NA                                                 */
  int64_t n_na_ci;    /* lo or hi NA                                                 */
  int64_t reserved[3];
  double est[2], est2[2], se2[2], len[2], lo[2], hi[2];
} dcor_accum;

/* mse, bias, var, coverage, ci_length: the summary columns. */
typedef struct dcor_summary {
  double mse, bias, var, coverage, ci_length;
} dcor_summary;

/* ------------------------------------------------------------------------ */
const char* dcor_version(void);
/* sha256 (hex) of the engine sources this library was built from (csrc/ + include/dcor.h), stamped
 * by the build (__graft_entry__.build_engine), which rebuilds whenever it differs from the tree's. */
const char* dcor_source_hash(void);
int dcor_last_error(char* buf, size_t len);
/* Number of visible HIP devices (0 on a host without GPU; never fails). */
int dcor_device_count(void);
/* Release the library-owned scratch: per (host thread, device) the one-pass sign kernel's
 * chunk x n x 4 B slab of per-sample codes, the grid tables and the auxiliary stream, and stop
 * dcor_grid_run_multi's persistent device workers.  Each host thread has its own, so threads never
 * share scratch; launches of ONE thread on different streams of one device must be ordered by the
 * caller.  Call when no work is in flight.  In a process forked after its parent used the engine
 * it makes no HIP call and returns DCOR_EFORK. */
int dcor_shutdown(void);
/* Implementation switches for A/B runs and tests (no reference counterpart).  The library reads
 * no environment variable: a replicate's bits are a function of (cell, seed, replicate) alone
 * (vert-cor.R:364's per-cell set.seed contract), and the defaults of every switch are a function of
 * the cell geometry.  `name` is one of the switches DESIGN.md lists ("DCOR_TILED",
 * "DCOR_CODE_WINDOW", ...); value NULL restores its default; name NULL restores every default.
 * Returns DCOR_EINVAL for an unknown name.  Process-wide; set it when no work is in flight.
 * dcor_get_variant copies the current value (empty when unset) into buf and returns 1 if set, 0 if
 * not, -1 for an unknown name. */
int dcor_set_variant(const char* name, const char* value);
int dcor_get_variant(const char* name, char* buf, size_t len);
/* Device and pinned-host allocations the library has made so far (its scratch arenas, staging
 * buffers, panels and the host-pointer entries' transfer buffers): a repeated call of the same
 * shape on warm contexts adds none. */
int64_t dcor_alloc_count(void);
/* Device bytes held by the library's scratch arenas over every live context. */
int64_t dcor_device_bytes(void);
/* How dcor_sim_launch splits rep_count replicates of `cell` into launches: *nchunks chunks of at
 * most *chunk replicates (the one-pass sign path's slab chunks; 1 x rep_count for every other kernel
 * family).  Planning only: no device work.  bench.py times its live pass ceilings at this chunk. */
int dcor_sim_chunking(const dcor_cell* cell, int64_t rep_count, int64_t* chunk, int64_t* nchunks);
/* Measurement only (bench.py's roofline, not part of the reference surface): one pass of the
 * one-pass sign path (the workgroup kernels dcor_sim_launch runs for cells with n > 16384 and
 * normalise = TRUE; a smaller cell runs passes 1-3 in them too, with the same per-replicate records
 * and tie batches as its wave kernels -- its results may differ from theirs in the low bits, since
 * the workgroup and wave reductions add the compensated sums in different orders) over replicates rep_begin .. rep_begin + reps - 1 as ONE chunk,
 * on `stream`, in the calling thread's scratch arena.  which: 1 pass 1 (writes the slab and the
 * clipped sums; for the Gaussian DGP it also regenerates its slow samples), 2 pass 2 (reads the slab
 * and sums), 3 the epilogue (reads pass 2's partials); 11 the pass-1 ceiling and 12 the pass-2
 * ceiling (Gaussian DGP, m = 8): the same loops with their memory side removed, at the real passes'
 * waves per SIMD -- their time is the instruction stream's own issue-bound time on this GPU; 13 the
 * pass-1 ceiling at its own (higher) occupancy; 14 / 15 the pass-1 ceiling plus only its slab stores
 * / plus only its slow-sample list and regenerations (what each costs).  Run 1, 2, 3 in that order
 * on the same cell and reps (12 after 1).  No result is returned; time them with events. */
int dcor_diag_sign_pass(const dcor_cell* cell, int64_t rep_begin, int64_t reps, int which, void* stream);
/* Measurement only: passes 1 and 2 (as dcor_diag_sign_pass 1, 2, on the null stream) and, per
 * replicate, the number of NI batches whose record codes tied a private centre's code and took the
 * exact regeneration fix-up (the rare path of the one-pass sign kernels) into h_ties[reps]. */
int dcor_diag_sign_ties(const dcor_cell* cell, int64_t rep_begin, int64_t reps, int64_t* h_ties);

/* ---- calibration scalars (host closed forms) ----------------------------- */
/* lambda_n, ver-cor-subG.R:1 (= real-data-sims.R:109). */
double dcor_lambda_n(double n, double eta);
/* lambda_INT_n, ver-cor-subG.R:3-7 (= real-data-sims.R:154-158). out = {lambda_s, lambda_r}. */
void dcor_lambda_int_n(double n, double eta_s, double eta_r, double eps_s, double out[2]);
/* lambda_receiver_from_noise, real-data-sims.R:170-174. */
double dcor_lambda_receiver_from_noise(double lam_s, double lam_o, double eps_s, double delta);
/* lambda_from_priv(lo, hi, priv, eps_sd), real-data-sims.R:103-106 (priv = {mean, sd}). */
double dcor_lambda_from_priv(double lo, double hi, double mean, double sd, double eps_sd);
/* qnorm(p) (R's qnorm, used as qnorm(1 - alpha/2)). */
double dcor_qnorm(double p);

/* ---- fused Monte-Carlo engine (the hot path) ----------------------------- */
/* Replicates [rep_begin, rep_begin + rep_count) of one cell, one workgroup per
 * replicate: Philox DGP -> clip -> reduce -> Laplace -> NI + INT estimate + CI.
 * Replaces run_sim_one's loop body (vert-cor.R:392-419; ver-cor-subG.R:174-198).
 * d_out: rep_count device records.  Per-replicate results depend only on
 * (seed, rep), never on the range split, so any sharding over GPUs is exact.
 * Asynchronous with stream semantics for d_out: every kernel that writes d_out runs after the
 * work enqueued on `stream` before the call, and work enqueued on `stream` after the call runs
 * after all of this call's kernels.  Kernels that only touch library scratch (the one-pass sign
 * path's passes 1 and 2, on two library streams) may start earlier, beside the previous call's
 * tail. */
int dcor_sim_launch(const dcor_cell* cell, int64_t rep_begin, int64_t rep_count,
                    dcor_rep_out* d_out, void* stream);
/* Deterministic per-method accumulation of `count` records into d_acc[0] (NI)
 * and d_acc[1] (INT) (overwrites).  Replaces the summarise() closures
 * (vert-cor.R:422-437; ver-cor-subG.R:201-217). */
int dcor_accumulate_launch(const dcor_rep_out* d_out, int64_t count, double rho,
                           dcor_accum* d_acc, void* stream);
/* Host helpers over accumulators. */
void dcor_accum_merge(dcor_accum* dst, const dcor_accum* src);
void dcor_accum_finalize(const dcor_accum* acc, double rho, dcor_summary* out);
/* Whole grid on the current device, synchronous, host buffers (dcor_grid_run_multi with the
 * current device).  h_acc: 2*ncells accumulators (NI, INT per cell); h_detail: NULL or ncells*B
 * records, cell-major. */
int dcor_grid_run(const dcor_cell* cells, int ncells, int64_t B, dcor_accum* h_acc,
                  dcor_rep_out* h_detail);

/* The batched grid on the CURRENT device, asynchronous on `stream`: replicates
 * [rep_begin[i], rep_begin[i] + rep_count[i]) of every cell i.  The replicates of all cells of one
 * kernel family run in the same launches (one workgroup or wave per replicate, each cell's
 * constants from a device table), so a grid of small cells -- the reference grids' B = 250 --
 * fills the GPU like one large cell.  d_out: sum(rep_count) records, cell-major (cell i's first at
 * sum_{j<i} rep_count[j]); d_acc: 2*ncells accumulators (NI, INT per cell) of those records,
 * byte-identical to dcor_accumulate_launch on each cell's records.  Per-replicate results equal
 * dcor_sim_launch's.  The scratch and tables are the calling thread's (one set per thread and
 * device); ncells <= 65535. */
int dcor_grid_launch(const dcor_cell* cells, int ncells, const int64_t* rep_begin,
                     const int64_t* rep_count, dcor_rep_out* d_out, dcor_accum* d_acc,
                     void* stream);
/* The grid over several GPUs of one node, synchronous, host buffers: every cell's B replicates are
 * split into contiguous ranges, shard g = [g B / G, (g+1) B / G) on device_ids[g] from its own host
 * thread (a device may appear more than once; with more than one shard the threads are persistent
 * workers, one per (device, listing), whose scratch survives across calls until dcor_shutdown);
 * accumulators are merged in device-list order, so the summary is deterministic for a given list,
 * and per-replicate records do not depend on it.  Device memory is bounded whatever B is: the
 * replicates run through a record buffer of DCOR_GRID_REC_MB (default 256) MiB in passes of whole
 * accumulate blocks, so the accumulators equal dcor_accumulate_launch over each cell's records.
 * device_ids = NULL / ndev = 0: every visible device.  Replaces mclapply over cells
 * (vert-cor.R:534-553; ver-cor-subG.R:294-295). */
int dcor_grid_run_multi(const dcor_cell* cells, int ncells, int64_t B, const int* device_ids,
                        int ndev, dcor_accum* h_acc, dcor_rep_out* h_detail);

/* ---- R-stream mode ------------------------------------- */
/* The same grid as dcor_grid_run, but every replicate consumes R's OWN random stream: cell
 * i starts from set.seed(cells[i].seed) (R's Mersenne-Twister / Inversion defaults) and
 * draws in run_sim_one's call order (vert-cor.R:364,392-419; ver-cor-subG.R:169,174-198;
 * SURVEY.md Appendix A): mvrnorm / gen_bernoulli / gen_bounded_factor, priv_standardize and
 * batch Laplace (extraDistr::rlaplace), rbinom flips, mixquant's rnorm / rexp / rbinom.
 * Replicate b of a cell therefore equals the reference's replicate b for that seed, up to
 * libm rounding of log.  seed must fit set.seed's 32-bit integer; every DGP
 * (gen_mix_gaussian: n <= 65536).  Synchronous, host buffers, like dcor_grid_run. */
int dcor_rstream_grid_run(const dcor_cell* cells, int ncells, int64_t B, dcor_accum* h_acc,
                          dcor_rep_out* h_detail);
/* The explicit inputs R-stream replicates 0 .. reps-1 of one cell consume (HOST buffers,
 * rep-major; a NULL pointer skips that array): the parity hook of the R-stream mode. */
typedef struct dcor_rs_draws {
  double *X, *Y;                  /* [reps][n]                                        */
  double *lap_ni_sc, *lap_int_sc; /* [reps][4] unit Laplace (sign family, normalise)   */
  double *lap_ni_x, *lap_ni_y;    /* [reps][k]                                        */
  uint32_t* flips;                /* [reps][ceil(n/32)] rbinom(n, 1, p) bits (sign)    */
  double* lap_local;              /* [reps][n] (sub-G)                                */
  double* lap_scalar;             /* [reps] Z (sign) / central Laplace (sub-G)        */
  double *mix_z, *mix_l;          /* [reps][nsim] rnorm, rexp*(2*rbinom-1)             */
} dcor_rs_draws;
int dcor_rstream_draws(const dcor_cell* cell, int64_t reps, const dcor_rs_draws* h);
/* The first `count` tempered Mersenne-Twister words after set.seed(seed), from the GPU
 * generator (unif_rand() = fixup(word * 2^-32)). */
int dcor_rstream_words(int32_t seed, int64_t count, uint32_t* h_out);
/* Jump-ahead of R's Mersenne-Twister stream (host computation, no device): the 624 raw state words
 * J words past the first generated block of set.seed(seed) -- raw words 624 + J .. 624 + J + 623 of
 * the stream (raw word 624 + k = the k-th word MT generates; tempering makes the k-th unif_rand).
 * By x^J mod phi (phi: MT19937's characteristic polynomial, Berlekamp-Massey); the device does
 * the same per segment when one long stream is generated by many workgroups. */
int dcor_rstream_mt_jump(int32_t seed, int64_t J, uint32_t* h_out);
/* The HRS runs' noise on R's streams (real-data-sims.R:355-404), in the explicit-input layout
 * of dcor_premat_subg (hrs = 1), DEVICE outputs, synchronous on `stream`:
 *  run r, NI: set.seed(h_ni_seeds[r]); sample.int(n, k*m) -> d_perm[r][k*m] (0-based), then
 *    rLap(k) twice -> d_lap_x[r][k], d_lap_y[r][k] (unit scale);
 *  run r, INT: set.seed(h_int_seeds[r]); rLap(n) -> d_lap_local[r][n], rLap(1) ->
 *    d_lap_central[r], mixquant(nsim) -> d_mix_z[r][nsim], d_mix_l[r][nsim].
 * The reference seeds run `rep` at eps index idx with 10 + 37 rep + 1000 idx (NI) and
 * 20 + 41 rep + 1000 idx (INT).  A NULL seed array skips that half.  2 <= n <= 65536. */
int dcor_rstream_hrs_draws(int64_t n, int64_t k, int64_t m, int64_t nsim, int64_t runs,
                           const int32_t* h_ni_seeds, const int32_t* h_int_seeds, int32_t* d_perm,
                           double* d_lap_x, double* d_lap_y, double* d_lap_local,
                           double* d_lap_central, double* d_mix_z, double* d_mix_l, void* stream);

/* ---- pre-materialised (explicit-input) batch mode: HBM streaming --------- */
/* Sign family, R replicates.  Per-replicate arrays are laid out rep-major with
 * the given strides (a stride of 0 shares one array across replicates). */
typedef struct dcor_premat_sign {
  int64_t n, reps;
  double eps1, eps2, alpha;
  int32_t normalise, ci_mode;
  int64_t nsim;
  const double* X;          /* [reps][xy_stride] (xy_stride 0: shared)            */
  const double* Y;
  int64_t xy_stride;
  const double* lap_ni_sc;  /* [reps][4]  mu_X, m2_X, mu_Y, m2_Y (vert-cor.R:214-215) */
  const double* lap_ni_x;   /* [reps][k]  (vert-cor.R:230)                        */
  const double* lap_ni_y;   /* [reps][k]  (vert-cor.R:231)                        */
  const double* lap_int_sc; /* [reps][4]  fresh standardisation (vert-cor.R:271-272) */
  const uint32_t* flips;    /* [reps][ceil(n/32)] bit i of word i/32 = S_i (vert-cor.R:175) */
  const double* lap_z;      /* [reps]     Z (vert-cor.R:188)                      */
  const double* mix_z;      /* [reps][nsim] rnorm(nsim)  (vert-cor.R:47)          */
  const double* mix_l;      /* [reps][nsim] rexp*(2*rbinom-1)                     */
} dcor_premat_sign;

/* Sub-Gaussian family (simulation variant, hrs = 0, ver-cor-subG.R:25-108) or the
 * HRS variant (hrs = 1, real-data-sims.R:115-147,176-252).  Every array must be aligned to
 * its element size (8 B; perm 4 B), else DCOR_EINVAL. */
typedef struct dcor_premat_subg {
  int64_t n, reps;
  double eps1, eps2, eta1, eta2, alpha;
  int32_t hrs, reserved;
  double lam_x, lam_y;                 /* NI overrides (NaN: lambda_n)             */
  double lam_s, lam_o, lam_r, delta;   /* INT overrides (NaN: defaults)            */
  int64_t nsim;
  const double* X;
  const double* Y;
  int64_t xy_stride;
  const int32_t* perm;      /* hrs: [reps][k*m] 0-based sample.int(n,k*m)-1; else NULL */
  const double* lap_ni_x;   /* [reps][k]                                          */
  const double* lap_ni_y;   /* [reps][k]                                          */
  const double* lap_local;  /* [reps][n]  rLap(n, 2*lambda_s/eps_s)               */
  const double* lap_central;/* [reps]                                             */
  const double* mix_z;      /* [reps][nsim]                                       */
  const double* mix_l;      /* [reps][nsim]                                       */
} dcor_premat_subg;

/* Whether a shared panel (DEVICE pointers) is dictionary-codable: *ok = 1 iff n <= 65536 and
 * both columns hold at most 256 distinct doubles and no NaN.  dcor_premat_subg_launch with a
 * shared panel (xy_stride 0) and random batches (perm) then runs the LDS-resident coded kernel;
 * otherwise the L2-gather kernel.  Synchronous; results never depend on the path. */
int dcor_panel_dict_probe(const double* d_X, const double* d_Y, int64_t n, int* ok);

/* A shared (X, Y) panel prepared once for many pre-materialised sub-G launches: the HRS panel
 * of real-data-sims.R, reused by every replicate of the eps sweep (real-data-sims.R:345-404).
 * Create encodes the panel on `stream` and waits for it (dictionary codes when codable, see
 * the probe above);
 * the device arrays d_X, d_Y must stay valid and unchanged until destroy. */
typedef struct dcor_panel dcor_panel;
int dcor_panel_create(const double* d_X, const double* d_Y, int64_t n, void* stream,
                      dcor_panel** out);
/* *coded = 1 if the panel is dictionary-coded (create synchronises once to learn it). */
int dcor_panel_coded(const dcor_panel* panel, int* coded);
int dcor_panel_destroy(dcor_panel* panel);
/* dcor_premat_subg_launch over a prepared panel: d->X, d->Y must be the panel's arrays,
 * d->xy_stride 0, d->n the panel's n.  Skips the per-launch encoding. */
int dcor_premat_subg_panel_launch(const dcor_premat_subg* d, const dcor_panel* panel,
                                  dcor_rep_out* d_out, void* stream);

/* HRS replicates rep_begin .. rep_begin + d->reps - 1 with the noise drawn inside the kernel
 * (real-data-sims.R:115-147 NI, 176-252 INT; the replicate loop of 345-448): the Philox
 * streams the HRS driver otherwise materialises in HBM -- dcor_perm_launch(seed_ni,
 * DCOR_SITE_PERM), dcor_draws_launch(Laplace, seed_ni, 11 / 12) for the NI batches,
 * (Laplace, seed_int, 13) local and (Laplace, seed_int, 14, count 1) central INT noise,
 * (normal, seed_int, 15) and (Laplace, seed_int, 16) for mixquant.  Results equal
 * dcor_premat_subg_panel_launch on those arrays to within the compensated sums' rounding.
 * d->hrs must be 1; d's noise pointers are ignored.  Any panel: a dictionary-coded one runs
 * from LDS codes; an uncoded one (continuous values) with n <= 65536 gathers its clipped
 * samples from L2 (same results bit for bit as the coded kernel on a codable panel); larger
 * uncoded panels materialise the same streams per chunk and run the pre-materialised kernels. */
int dcor_hrs_fused_launch(const dcor_premat_subg* d, const dcor_panel* panel, uint64_t seed_ni,
                          uint64_t seed_int, int64_t rep_begin, dcor_rep_out* d_out, void* stream);

/* Segments of the HRS eps sweep (real-data-sims.R:345-448: for each eps, R NI runs under
 * set.seed(10 + 37 rep + 1000 idx) and R INT runs under set.seed(20 + 41 rep + 1000 idx),
 * :402-437) on one prepared panel, pre-materialised: for every segment, replicates rep_begin ..
 * rep_begin + reps - 1 at eps1 = eps2 = eps with Philox keys seed_ni / seed_int, their noise
 * drawn into a stream-ordered buffer (the dcor_perm_launch / dcor_draws_launch sites listed for
 * dcor_hrs_fused_launch) and run by dcor_premat_subg_panel_launch, records to d_out[out_row ..].
 * Each record equals the same replicate of dcor_premat_subg_panel_launch on those draws bit for
 * bit (the host loop of dcor.hrs.hrs_replicates, run natively; one host call per sweep instead
 * of eight launches from the host per eps).  base supplies n, X, Y (the panel's), alpha, nsim,
 * hrs = 1, lam_x / lam_y (NI) and lam_s / lam_o (INT) and delta > 0; per segment eta = 1 and
 * lam_r = dcor_lambda_receiver_from_noise(lam_s, lam_o, eps, delta).  Every segment is
 * checked before anything is enqueued. */
typedef struct dcor_hrs_segment {
  double eps;
  uint64_t seed_ni, seed_int;
  int64_t rep_begin, reps, out_row;
} dcor_hrs_segment;
int dcor_hrs_sweep_launch(const dcor_premat_subg* base, const dcor_panel* panel,
                          const dcor_hrs_segment* segs, int64_t nseg, dcor_rep_out* d_out,
                          void* stream);

int dcor_premat_sign_launch(const dcor_premat_sign* d, dcor_rep_out* d_out, void* stream);
int dcor_premat_subg_launch(const dcor_premat_subg* d, dcor_rep_out* d_out, void* stream);

/* Batch geometry (m, k) the estimators use; family selects the guard
 * (sub-G: m>n => m=n; HRS: k<2 => k=2, m=floor(n/2)).  Returns DCOR_EKLT1 if k<1. */
int dcor_batch_geometry(int64_t n, double eps1, double eps2, int family, int hrs,
                        int64_t km[2]);

/* ---- single-call host-pointer forms: the R `.Call` targets --------------- */
/* ci_NI_signbatch (vert-cor.R:204-255). out = {rho_hat, lo, hi}. */
int dcor_ci_ni_signbatch(const double* X, const double* Y, int64_t n, double eps1,
                         double eps2, double alpha, int normalise, const double lap_sc[4],
                         const double* lap_x, const double* lap_y, double out[3]);
/* ci_INT_signflip (vert-cor.R:260-317); flips one byte (0/1) per sample. */
int dcor_ci_int_signflip(const double* X, const double* Y, int64_t n, double eps1,
                         double eps2, double alpha, int mode, int normalise,
                         const double lap_sc[4], const uint8_t* flips, double lap_z,
                         const double* mix_z, const double* mix_l, int64_t nsim,
                         double out[3]);
/* correlation_NI_subG (ver-cor-subG.R:25-62; hrs: real-data-sims.R:115-147). */
int dcor_correlation_ni_subg(const double* X, const double* Y, int64_t n, double eps1,
                             double eps2, double eta1, double eta2, double alpha, int hrs,
                             double lam_x, double lam_y, const int32_t* perm,
                             const double* lap_x, const double* lap_y, double out[3]);
/* ci_INT_subG (ver-cor-subG.R:67-108; hrs: real-data-sims.R:176-252). */
int dcor_ci_int_subg(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                     double eta1, double eta2, double alpha, int hrs, double lam_s,
                     double lam_o, double lam_r, double delta, const double* lap_local,
                     double lap_central, const double* mix_z, const double* mix_l,
                     int64_t nsim, double out[3]);
/* mixquant (ver-cor-subG.R:8-13): sort(z + c*l)[ceiling(p*nsim)]. */
int dcor_mixquant(const double* z, const double* l, int64_t nsim, double c, double p,
                  double* out);
/* priv_standardize (vert-cor.R:322-348): the DP mean / second-moment helper. */
int dcor_priv_standardize(const double* v, int64_t n, double eps_norm, double L_raw,
                          const double lap[2], double* out);
/* dp_sd (real-data-sims.R:73-84): out = {mean, sd}; lap = {mean, m2} unit draws. */
int dcor_dp_sd(const double* x, int64_t n, double lo, double hi, double eps1, double eps2,
               const double lap[2], double out[2]);

/* ---- R-surface helpers: the arithmetic half of R wrappers that draw with R's RNG ----------
 * The R wrappers (R/dcor*.R) make the reference's own RNG calls in the reference's order, so
 * .Random.seed advances exactly as it does under the reference, and hand the draws to these
 * entries, which evaluate the rest on the GPU in R's operation order.  Host pointers,
 * synchronous. */
/* sd(Uc) of ci_INT_subG's clipped products for given X, Y and unit local noise
 * (ver-cor-subG.R:87-99; hrs: real-data-sims.R:221-236): the HRS wrapper needs it to take the
 * sd(Uc) == 0 branch (real-data-sims.R:237-238), which draws no mixquant values, before drawing
 * anything.  Same lambda rules as dcor_ci_int_subg. */
int dcor_int_subg_sd_uc(const double* X, const double* Y, int64_t n, double eps1, double eps2,
                        double eta1, double eta2, int hrs, double lam_s, double lam_o,
                        double lam_r, double delta, const double* lap_local, double* sd_uc);
/* dp_mean (real-data-sims.R:64-70) of n non-NA values: mean(pmin(pmax(x, lo), hi)) +
 * (hi - lo)/(n eps) * lap, lap a unit Laplace draw. */
int dcor_dp_mean(const double* x, int64_t n, double lo, double hi, double eps, double lap,
                 double* out);
/* standardize_dp (real-data-sims.R:87-90): (pmin(pmax(x, lo), hi) - mean) / max(sd, eps). */
int dcor_standardize_dp(const double* x, int64_t n, double lo, double hi, double mean, double sd,
                        double eps, double* out);
/* gen_bernoulli (vert-cor.R:78-98) from u = runif(n), v = runif(n); |rho| <= 1. */
int dcor_gen_bernoulli(const double* u, const double* v, int64_t n, double rho, double* X,
                       double* Y);
/* gen_bounded_factor (ver-cor-subG.R:141-154): cbind(U + E1, U + E2) from its three runif draws. */
int dcor_gen_bounded_factor(const double* U, const double* E1, const double* E2, int64_t n,
                            double* X, double* Y);
/* MASS::mvrnorm(n, mu, Sigma) with Sigma = [[s1^2, s1 s2 rho], [s1 s2 rho, s2^2]]
 * (vert-cor.R:389-394) from z = rnorm(2n): LAPACK's eigenvectors (dsyevr / dlaev2) and dgemm's
 * summation order, so X, Y equal R's.  DCOR_EINVAL if Sigma is not positive definite. */
int dcor_mvrnorm(const double* z, int64_t n, const double mu[2], const double sigma[2],
                 double rho, double* X, double* Y);
/* gen_mix_gaussian (ver-cor-subG.R:115-136) from its draws: n0 labels 0 (rbinom), z0 = rnorm(2 n0),
 * z1 = rnorm(2 n1), perm = sample.int(n) - 1 (0-based); rows clipped to [-1, 1]. */
int dcor_mix_gaussian(const double* z0, int64_t n0, const double* z1, int64_t n1,
                      const int32_t* perm, double rho, const double mu0[2], const double sigma0[2],
                      const double mu1[2], const double sigma1[2], double* X, double* Y);

/* On-device unit draws from the engine's Philox streams (pre-materialised inputs
 * generated in HBM, e.g. the HRS noise of BASELINE config C5).  kind: 0 unit Laplace,
 * 1 standard normal (Box-Muller pairs), 2 uniform (0,1).  Element e of replicate r uses
 * block (e/2, r, site) and words (0,1) / (2,3) for e even / odd.  d_out: [reps][count];
 * count < 2^31, rep_begin + reps <= 2^32, reps <= 65535. */
int dcor_draws_launch(int kind, uint64_t seed, int site, int64_t rep_begin, int64_t reps,
                      int64_t count, double* d_out, void* stream);

/* The cell's DGP samples from the fused engine's draw contract (the sites below): d_X, d_Y
 * [reps][n] for replicates rep_begin .. rep_begin + reps - 1 -- the (X, Y) every fused kernel
 * generates for those replicates (gen_bernoulli, mvrnorm, gen_bounded_factor, gen_mix_gaussian
 * of vert-cor.R:78-98,389-394 / ver-cor-subG.R:113-154). */
int dcor_dgp_launch(const dcor_cell* cell, int64_t rep_begin, int64_t reps, double* d_X,
                    double* d_Y, void* stream);

/* On-device keyed random batches for the HRS NI estimator: d_out[r][t] = P_r(t), t < count,
 * where P_r is a pseudo-random permutation of [0, n) (4-round Feistel, cycle-walked, keyed by
 * Philox block (0, rep_begin + r, site, 0)) -- the role of sample.int(n, k*m) 0-based
 * (real-data-sims.R:131).  d_out: [reps][count] int32. */
int dcor_perm_launch(uint64_t seed, int site, int64_t rep_begin, int64_t reps, int64_t n,
                     int64_t count, int32_t* d_out, void* stream);

/* Draw-site contract of the fused engine (DESIGN.md "RNG"): Philox4x32-10 with
 * key = (seed lo32, seed hi32), counter = (index, rep, site, 0) unless noted.
 * Gaussian DGP sample i: block (i, rep, DGP_A) = (w0, w1, w2, w3); z1 = ziggurat(w0, w2 & 0xffff),
 * z2 = ziggurat(w1, w2 >> 16), INT flip = (w3 < ceil(p 2^32)).  A ziggurat draw that misses the
 * fast test continues on blocks (i, rep, ZIG, 2a + which) (attempt a >= 1 draws its layer and
 * magnitude there; every attempt's wedge uniform is words 2,3) and, in the base layer, on tail
 * blocks (i, rep, ZIG_TAIL, 2t + which); which = 0 for z1, 1 for z2. */
enum {
  DCOR_SITE_DGP_A = 1,   /* 1 Gaussian sample + its flip / 2 Bernoulli samples / U,E1 */
  DCOR_SITE_DGP_B = 2,   /* bounded-factor E2 (w0,w1) ; sub-G local Laplace (w2,w3) */
  DCOR_SITE_FLIP = 3,    /* sign-family INT flips, 4 samples per block (bounded factor, mixture) */
  DCOR_SITE_NI_LAP = 4,  /* batch j: Laplace X (w0,w1), Y (w2,w3)                  */
  DCOR_SITE_SCALAR = 5,  /* blocks 0..4: NI mu/m2 X, NI mu/m2 Y, INT mu/m2 X, INT mu/m2 Y, Z */
  DCOR_SITE_MIX_Z = 6,   /* mixquant normals, 2 per block                         */
  DCOR_SITE_MIX_L = 7,   /* mixquant unit Laplace, 2 per block                    */
  DCOR_SITE_PERM = 8,    /* HRS random-batch permutation keys (dcor_perm_launch)  */
  DCOR_SITE_ZIG = 9,     /* Gaussian DGP ziggurat retries (counter word 3 = 2 attempt + which) */
  DCOR_SITE_ZIG_TAIL = 10 /* Gaussian DGP ziggurat tail (counter word 3 = 2 step + which) */
};

#ifdef __cplusplus
}
#endif
#endif /* DCOR_H */
