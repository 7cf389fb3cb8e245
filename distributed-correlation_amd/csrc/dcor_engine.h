// dcor_engine.h -- launch-time constant blocks shared by the host C-ABI and the kernels.
//
// Every data-independent scalar of the R estimators (lambda, m, k, Laplace scales,
// qnorm, exp(eps_s) ratios, mixquant order-statistic index ...) is evaluated ONCE on
// the host with the R operation order (see dcor_capi.cpp) and handed to the kernel by
// value, so the per-replicate kernel only does the data-dependent arithmetic.
#pragma once
#include <stdint.h>

#include "../../include/dcor.h"

namespace dcor {

// The current value of an implementation switch set by dcor_set_variant (dcor_capi.cpp), or
// nullptr when it is at its default.  Never the environment: see include/dcor.h.
const char* variant(const char* name);

struct DgpConst {
  int32_t dgp;
  int32_t nan_dgp;                      // gen_bounded_factor with rho outside [0, 1]: sqrt(3 rho)
                                        // or sqrt(3 (1 - rho)) is NaN, runif(n, NaN, NaN) gives
                                        // NaN, so every estimate of the replicate is NaN
  double mu0, mu1, a00, a01, a10, a11;  // Gaussian: X = mu + A z  (MASS::mvrnorm)
  double thr0, thr1;                    // Bernoulli: p01/0.5, p11/0.5
  uint64_t T0, T1;                      // ceil(thr*2^32): u32*2^-32 < thr  <=>  u32 < T
  uint32_t T0_24, T1_24;                // Bernoulli Y: 24-bit v < ceil(thr*2^24)
  double cU, cU2, cE, cE2;              // bounded factor: -c + (c - -c) * u
  double xmu[2][2], xa[2][4];           // mixture: per-component mu and mvrnorm factor
  uint32_t T24, pad2;                   // mixture label: u24 < T24 = ceil(pi_mix * 2^24)
};

struct MixConst {
  int32_t nsim, pos, P, pad;  // R: sort(x)[ceiling(p*nsim)] -> 0-based pos; P = pow2 >= nsim
};

// Sign family: ci_NI_signbatch + ci_INT_signflip (vert-cor.R:204-317).
struct SignConst {
  int64_t n, k;
  int64_t rep_begin;
  uint32_t k0, k1;          // Philox key (seed lo, hi)
  int32_t m, normalise, sender_is_X, mode_normal;
  DgpConst g;
  MixConst mix;
  double nd, md, kd;
  double L;                                   // sqrt(2*log(n))
  double s_mu_x, s_m2_x, s_mu_y, s_m2_y;      // priv_standardize Laplace scales
  double bx, by;                              // 2/(m*eps1), 2/(m*eps2)
  double inv_k, crit, sqrt_k;
  double pflip;                               // exp(eps_s)/(exp(eps_s)+1)
  uint64_t flipT;                             // ceil(pflip*2^32): flip <=> u32 < flipT
  uint32_t flipT24;                           // ceil(pflip*2^24): Bernoulli DGP spare-bit flips
  int32_t md_pow2;                            // m is a power of two: count / m == count * inv_md
  double inv_md;
  double scale_Z, coefZ, q2, ratio, inv_sqrt_n, eps_r, w_laplace;
  double cbase_x, cinv_x, cbase_y, cinv_y;    // monotone code maps of clip(x), clip(y)
  float cinv_xf, cnb_xf, cinv_yf, cnb_yf;     // the same maps in fp32 / 65535: t = fma(v, inv, -base*inv)
  int32_t pieces;                             // pass 2 by 8-record pieces: m / 8 for m % 8 == 0,
                                              // 16 <= m <= 8 SIGN_PIECES_MAX; else 0
  int32_t pad_pc;
};
// Pass 2's piece path (m % 8 == 0, 16 <= m <= 8 SIGN_PIECES_MAX): a wave's 64 lanes read 64
// consecutive 8-record pieces (2 KB, coalesced), and each batch's P = m / 8 piece counts meet in
// the wave's LDS buffer of 64 P words (dynamic shared memory: DCOR_WAVES x 64 x P_max x 4 B).
#define SIGN_PIECES_MAX 31
inline int32_t sign_pieces(int64_t m) { return (m % 8 == 0 && m >= 16 && m <= 8 * SIGN_PIECES_MAX) ? (int32_t)(m / 8) : 0; }
inline size_t sign_piece_lds(int32_t pmax) { return (size_t)4 * 64 * (size_t)pmax * sizeof(uint32_t); }

// Sub-G family: correlation_NI_subG + ci_INT_subG (ver-cor-subG.R:25-108).
struct SubgConst {
  int64_t n, k;
  int64_t rep_begin;
  uint32_t k0, k1;
  int32_t m, sender_is_X;
  DgpConst g;
  MixConst mix;
  double nd, md, kd;
  double l1, l2;                    // lambda_n(n, eta1/2)
  double bx, by;                    // 2*l1/(m*eps1), 2*l2/(m*eps2)
  double m_over_k, crit, sqrt_k;
  double ls, lr, bs;                // lambda_s, lambda_r, 2*lambda_s/eps_s
  double s_central, sn2x2;          // 2*lr/(n*eps_r), 2*(s_central^2)
  double sqrt_n, eps_r;
  int32_t md_pow2, pad4;            // m is a power of two: sum / m == sum * inv_md
  double inv_md;
};

// Pre-materialised sign family.
struct PrematSignConst {
  SignConst s;          // scalars (dgp/key unused)
  const double* X; const double* Y; int64_t xy_stride;
  const double* lap_ni_sc; const double* lap_ni_x; const double* lap_ni_y;
  const double* lap_int_sc; const uint32_t* flips; int64_t flip_words;
  const double* lap_z; const double* mix_z; const double* mix_l;
};

// Pre-materialised sub-G (simulation or HRS variant).
struct PrematSubgConst {
  SubgConst s;
  int32_t hrs, dict_built;  // dict_built: 1 coded panel built (dcor_panel), 2 built and known coded
  double lo_;                        // HRS: lambda_other (clip of the non-sender)
  double crit_sqrt2_s;               // HRS: qnorm*sqrt(2)*(2*lr/(n*eps_r))  (sd==0 branch)
  const double* X; const double* Y; int64_t xy_stride;
  const int32_t* perm;
  const double* lap_ni_x; const double* lap_ni_y; const double* lap_local;
  const double* lap_central; const double* mix_z; const double* mix_l;
  // HRS with a shared panel (xy_stride 0): clipped panel packed once per launch,
  // xyc[i] = (clip(X_i, l1), clip(Y_i, l2)) for the NI gathers, soc[i] = (clip(S_i, ls),
  // clip(O_i, lo)) for the INT stream.  nullptr: read X / Y directly.
  const double2* xyc; const double2* soc;
  // Shared panel, random batches, n <= DCOR_DICT_NMAX: dictionary-coded panel built on device
  // per launch (k_panel_dict).  dict_ok is set by the device: 1 -> the coded kernel runs,
  // 0 (more than 256 distinct values in a column, a NaN or an infinity) -> the L2-gather kernel runs.
  uint16_t* dict_codes; double* dict_vals; int* dict_ok;
  // Coded-panel kernel only: each replicate's sums are split over `slices` work items (0 or 1:
  // one), whose partials part[rep * slices + t] the epilogue merges in slice order.
  int32_t slices, pad_;
};
#define DCOR_DICT_NMAX 65536
// Slices per replicate in the prepared coded-panel kernel (partials: 80 B each).  1: measured
// best -- 2 slices even out a persistent grid's last round but cost 25 % in per-item start-up
// and reduction (r01 A/B: 590-605 us vs 735-760 us per 8192 replicates).
#define DCOR_DICT_SLICES 1
size_t premat_dict_lds_bytes(int64_t n);
// codes: n u16 (16-B padded), dict: 512 doubles, ok: 1 int (device).
int launch_panel_dict(const double* X, const double* Y, int64_t n, uint16_t* codes, double* dict,
                      int* ok, void* stream);

// Kernel launchers (dcor_kernels.hip).  Return hipError_t as int.
int launch_sign_fused(const SignConst& c, int64_t reps, dcor_rep_out* out, void* stream);
// One-pass sign algorithm: pass-1 / pass-2 kernels over replicate chunks of `chunk`;
// scratch = chunk * n * 4 B of codes; sums = chunk * 4 doubles followed by chunk
// SignPartial records (48 B).
// Bernoulli sign family (bit planes): scratch = chunk * 3 * 4*ceil(n/256) u64, part = chunk
// SignPartial records (48 B each).
struct SignPartial;
int launch_sign_bern(SignConst c, int64_t reps, int64_t chunk, uint64_t* scratch,
                     SignPartial* part, dcor_rep_out* out, void* stream);
// One-pass sign engine buffers: two slabs (chunk * n * 4 B) and two sums/partials areas
// (chunk * 80 B), an auxiliary stream and two events (fork / join) for the two-stream
// chunk pipeline; aux == nullptr runs every chunk on the caller's stream.
// lib[0], lib[1]: the library streams the chunks alternate on (null: everything on the caller's
// stream).  cross: the previous call ran on the same streams and scratch layout, so passes 1 and 2
// start without waiting for the caller's stream (they touch library memory only); every kernel that
// writes `out` waits for ev_entry, the caller's stream at this call.
struct CodesBufs {
  uint32_t* slab[2];
  double* sums[2];
  void* lib[2];
  void* ev_entry;
  void* ev_end[2];
  bool cross;
};
int launch_sign_fused_codes(const SignConst& c, int64_t reps, int64_t chunk, const CodesBufs& bf,
                            dcor_rep_out* out, void* stream);
// One pass of the one-pass sign path as a single chunk (dcor_diag_sign_pass).
int launch_sign_diag(const SignConst& c, int64_t reps, int which, uint32_t* slab, double* sums,
                     void* part, dcor_rep_out* out, void* stream);
int launch_subg_fused(const SubgConst& c, int64_t reps, dcor_rep_out* out, void* stream);
int launch_dgp(const DgpConst& g, uint32_t k0, uint32_t k1, int64_t rep_begin, int64_t reps,
               int64_t n, double* X, double* Y, void* stream);

// ---- batched grid launches (dcor_grid_launch): many cells' replicates per launch ----------
// One work item = one replicate: the cell's constants come from a device table, so a launch
// covers any mix of cells of one kernel family and DGP (no per-cell launches, no per-cell
// occupancy cliff at the reference grids' B = 250).
struct GridItem {
  uint32_t cell;      // index into the launch's constant table
  uint32_t rep;       // replicate index: the Philox counter
  uint64_t scratch;   // first element of the replicate's scratch (codes: u32 records; Bernoulli
                      // planes: u64 words)
  uint64_t out;       // index of its output record
};
// A run of consecutive replicates of one cell inside one chunk launch; the launch's work items
// are expanded from these on the device (launch_grid_expand), so the host plans O(cells + chunks)
// records instead of one per replicate.
struct GridPiece {
  uint32_t cell;        // index into the launch's constant table
  uint32_t rep0;        // replicate of the first item
  uint64_t item0;       // first item index (within the chunk launch)
  uint64_t count;       // items
  uint64_t out0;        // output record of the first item
  uint64_t scr0;        // scratch element of the first item
  uint64_t scr_stride;  // scratch elements per item
};
int launch_grid_expand(const GridPiece* pieces, int64_t npieces, GridItem* items, void* stream);
enum GridKind { GK_SIGN_CODES = 0, GK_SIGN_REGEN = 1, GK_SIGN_BERN_W = 2, GK_SIGN_BERN = 3, GK_SUBG = 4,
                GK_SIGN_CODES_W = 5, GK_SUBG_W = 6 };
// sub-G cells up to this n run one wave per replicate (GK_SUBG_W), in the grid and dcor_sim_launch
#define SUBG_W_NMAX 16384
// one-pass sign cells up to this n run the wave-per-replicate kernels (GK_SIGN_CODES_W), in the
// grid and in dcor_sim_launch alike, so a replicate's bits do not depend on the entry point
#define SIGN_W_NMAX 16384
// per-item scratch of the kinds that use it
#define GRID_BERN_W_NMAX 16384
// doubles per replicate handed from the one-pass sign kernel's pass 1 to pass 2
#define SIGN_SUMS 8
// The one-pass sign path's per-replicate scratch ("item", in u32 words): n u16 records, two per
// word, padded to 64 words (256 B).
__host__ __device__ inline uint64_t sign_rec_words(int64_t n) { return ((uint64_t)(n + 1) / 2 + 63) & ~(uint64_t)63; }
__host__ __device__ inline uint64_t sign_item_words(int64_t n, int /*dgp*/) { return sign_rec_words(n); }
// bytes of a SignPartial (pass 2 -> epilogue; dcor_fused.hip)
#define SIGN_PARTIAL_BYTES 48
// Pass 1 + pass 2 over `nitems` items (scratch: the items' code slabs; sums: SIGN_SUMS doubles per
// item; part: per-item SignPartial), then the wave epilogue writing out[item.out].
// pmax: the largest SignConst.pieces of the launch's cells (its pass-2 LDS, sign_piece_lds).
int launch_grid_sign_codes(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                           uint32_t* scratch, double* sums, SignPartial* part, int vpl32, int pmax,
                           dcor_rep_out* out, void* stream);
// Small cells: wave pass 1 + wave pass 2 / epilogue (sums: SIGN_SUMS doubles per item, no partials).
int launch_grid_sign_codes_w(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                             uint32_t* scratch, double* sums, int vpl32, int pmax, dcor_rep_out* out,
                             void* stream);
int launch_grid_sign_regen(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                           dcor_rep_out* out, void* stream);
int launch_grid_sign_bern(bool wave, const SignConst* cells, const GridItem* items, int64_t nitems,
                          uint64_t* scratch, SignPartial* part, int vpl32, dcor_rep_out* out,
                          void* stream);
int launch_grid_subg_w(int dgp, const SubgConst* cells, const GridItem* items, int64_t nitems, int vpl32,
                       dcor_rep_out* out, void* stream);
int launch_grid_subg(int dgp, const SubgConst* cells, const GridItem* items, int64_t nitems,
                     dcor_rep_out* out, void* stream);
// Accumulators of grid cells, computed in passes over bounded record buffers.  Cell c's records
// are partitioned as launch_accumulate partitions them (accumulate_blocks(count) blocks of
// accumulate_per(count)); a pass holds whole blocks.  Entry: blocks [blo, bhi) of one cell whose
// records start (at block blo) at rec[base]; poff: the cell's first partial in `part` (cells with
// more than one block).  The block partials and their merge are byte-identical to
// launch_accumulate on the cell's records alone.
struct AccEntry {
  int64_t base, blo, bhi, count, poff;
  double rho;
  int32_t cell, pad;
};
struct AccCell {   // a multi-block cell for the final merge
  int64_t count, poff;
  int32_t cell, pad;
};
int accumulate_blocks(int64_t count);
int64_t accumulate_per(int64_t count);
int launch_accumulate_pass(const dcor_rep_out* rec, const AccEntry* ent, int nent, int max_span,
                           dcor_accum* part, dcor_accum* acc, void* stream);
int launch_accumulate_merge_cells(const AccCell* cells, int ncells, const dcor_accum* part,
                                  dcor_accum* acc, void* stream);
int launch_premat_sign(const PrematSignConst& c, int64_t reps, dcor_rep_out* out, void* stream);
// part: reps * 80 B scratch (stream -> epilogue partial sums).
// epi_stream / ev: if non-null the epilogue runs on epi_stream after an event recorded on
// `stream` behind the streaming kernels (chunk pipelining).
// HRS replicates [rep_begin, rep_begin + reps) with in-kernel Philox noise over a coded panel
// (c.dict_codes / c.dict_vals set), or over an uncoded one (c.xyc / c.soc: 2 x n double2 of
// scratch the launch packs; n <= DCOR_DICT_NMAX); part: reps * 80 B.
int launch_hrs_fused(const PrematSubgConst& c, uint64_t seed_ni, uint64_t seed_int,
                     int64_t rep_begin, int64_t reps, void* part, dcor_rep_out* out, void* stream);
// int_stream / ev_fork / ev_join: an auxiliary stream and two events for the tiled path's INT kernel
// (DCOR_TILED_INT=2); without them that mode runs the INT sums inside the tiled kernel.
int launch_premat_subg(const PrematSubgConst& c, int64_t reps, void* part, dcor_rep_out* out,
                       void* stream, void* epi_stream = nullptr, void* ev = nullptr,
                       void* int_stream = nullptr, void* ev_fork = nullptr, void* ev_join = nullptr);
int launch_accumulate(const dcor_rep_out* d_out, int64_t count, double rho, dcor_accum* acc,
                      void* stream);
int launch_mixquant(const double* z, const double* l, int32_t nsim, double c, int32_t pos,
                    double* out, void* stream);
int launch_priv_standardize(const double* v, int64_t n, double L, double s_mu, double s_m2,
                            const double* lap2, double* out, void* stream);
int launch_draws(int kind, uint32_t k0, uint32_t k1, uint32_t site, int64_t rep_begin,
                 int64_t reps, int64_t count, double* out, void* stream);
int launch_perm(uint32_t k0, uint32_t k1, uint32_t site, int64_t rep_begin, int64_t reps,
                int64_t n, int64_t count, int32_t* out, void* stream);
// Every Philox noise array of `reps` HRS replicates in one launch: element for element the
// launch_perm (seed_ni, DCOR_SITE_PERM) and launch_draws (Laplace seed_ni 11 / 12, Laplace
// seed_int 13 / 14, normal 15, Laplace 16) outputs, rows [reps][count] as theirs.
struct HrsNoise {
  uint64_t seed_ni, seed_int;
  int64_t rep_begin, n, k, km, nsim;
  int32_t* perm;
  double *lap_x, *lap_y, *lap_local, *lap_central, *mix_z, *mix_l;
};
int launch_hrs_noise(const HrsNoise& j, int64_t reps, void* stream);
int launch_dp_sd(const double* x, int64_t n, double lo, double hi, double s_mu, double s_m2,
                 const double* lap2, double* out2, void* stream);
// R-surface transforms (dcor_premat.hip): the arithmetic half of the R wrappers' DGPs and DP
// helpers, whose random draws the wrappers take with R's own RNG.
struct MvnConst {          // MASS::mvrnorm factors A = V diag(sqrt(ev)) (row-major 2x2) and means
  double A0[4], mu0[2];    // component 0 (the only one for a plain mvrnorm)
  double A1[4], mu1[2];    // component 1 (gen_mix_gaussian)
};
int launch_uc_sd(const PrematSubgConst& p, double* out, void* stream);
int launch_standardize_dp(const double* x, int64_t n, double lo, double hi, double mean, double den,
                          double* out, void* stream);
int launch_gen_bernoulli(const double* u, const double* v, int64_t n, double t0, double t1,
                         double* X, double* Y, void* stream);
int launch_gen_bounded_factor(const double* U, const double* E1, const double* E2, int64_t n,
                              double* X, double* Y, void* stream);
int launch_mvrnorm_apply(const double* z0, int64_t n0, const double* z1, int64_t n1,
                         const int32_t* perm, const MvnConst& m, double* X, double* Y, void* stream);

// R-stream mode (dcor_rstream.hip): R's Mersenne-Twister state as set.seed leaves it.
struct RsState {
  uint32_t mt[624];
  int32_t mti;
  int32_t pad[3];
};
// One grid cell of an R-stream batch: the replicate's word layout,
// the host-evaluated transform constants, and the cell's device buffers for a chunk of rc
// replicates (carved from one allocation by the host).
struct RsCell {
  int64_t n, k, nsim;
  int64_t dgp_words;   // words of the DGP segment
  int64_t pre;         // words of a replicate before its exp_rand segment (or all of them)
  int32_t family, dgp, normalise, has_mix;
  int32_t flip_on, flip_inv, flip_const, u_draw, e_draw, pad;
  double flip_q;       // rbinom(1, pp): ix = (u >= flip_q)
  double A[4], mu[2];  // mvrnorm: X = mu + ((0 + z1 A0) + z2 A1), Y likewise with A2, A3
  double bern_t0, bern_t1;
  double cU, cE, u_const, e_const;
  RsState* st;
  uint32_t* words;     // rc * rep_max + 624 tempered words
  int64_t* rep_off;    // [rc] first word of each replicate
  int64_t* exp_end;    // [rc] first word after each replicate's exp_rand segment
  double* expv;        // [rc][nsim] rexp values
  double *X, *Y;       // [rc][n]
  double *lap_nsc, *lap_isc;   // [rc][4] standardisation draws (sign, normalise)
  double *lap_x, *lap_y;       // [rc][k]
  uint32_t* flips;             // [rc][ceil(n/32)]
  double* lap_local;           // [rc][n] (sub-G)
  double* lap_scalar;          // [rc] Z (sign) / central (sub-G)
  double *mix_z, *mix_l;       // [rc][nsim]
  // gen_mix_gaussian (ver-cor-subG.R:113-136): `pre_a` words of labels + normals, then
  // sample.int(n) (variable, `shuffle` = 1), then the rest of `pre`
  int64_t pre_a;
  int32_t shuffle, lab_on, lab_inv, lab_const;
  double lab_q;                // rbinom(1, pi_mix): ix = (u >= lab_q)
  double mA0[4], mA1[4], mmu0[2], mmu1[2];
  int64_t* shuf_end;           // [rc] first word after each replicate's sample.int
  int32_t* shuf;               // [rc][n] the shuffled row order (0-based)
  int64_t words_cap;           // capacity of `words`; the walker stops (RsState.pad[1] = 1)
                               // rather than overrun it
  // The jump path (launch_rsj): the chunk's stream generated segment-parallel from MT19937
  // jump-ahead windows, the walk replaced by pointer doubling over consumption positions
  // 0 .. jN (jN: the chunk's word budget; position jN stands for "past the budget").
  uint32_t* raw;               // [RSJ_L] raw words of the chunk's first segment (state block first)
  uint8_t* tlift;              // T_k(P) - P, the words 2^k exp_rand draws from P take (levels
                               // k < RSJ_T16 uint16, then uint32; level k at RSJ_TBYTES(k, jN + 1))
  int32_t* glift;              // [jlg][jN + 1]: G_k(P) = the start 2^k replicates on from P
  int32_t* jflag;              // set when the chunk ran past jN (the host re-runs it by k_rs_stream)
  int64_t jN, jpost;           // word budget; fixed words after the exp_rand segment (rbinom)
  int32_t jlt, jlg;            // levels of T and of G
};
// Raw words per jump segment (a multiple of 624, >= 624 + 19937 + 624 so segment 0 holds the
// base window every jump combines), and 64-bit words per jump polynomial.
#define RSJ_L (624 * 48)
#define RSJ_PW 312
// T levels below RSJ_T16 fit 16 bits (a draw takes <= 17 words: 17 * 2^11 < 65536)
#define RSJ_T16 12
#define RSJ_TBYTES(k, S) \
  ((k) <= RSJ_T16 ? 2 * (int64_t)(S) * (k) : 2 * (int64_t)(S) * RSJ_T16 + 4 * (int64_t)(S) * ((k) - RSJ_T16))
// Runs the jump path over d_cells[0..ncells): generation (segment 0 sequential, the rest from
// the nseg - 1 jump polynomials), the walk by pointer doubling, the exp_rand values and the
// .Random.seed after the chunk.  The polynomials as set-bit lists: polynomial s at
// d_pidx[d_poff[s] .. d_poff[s + 1]), two 16-bit bit indices per word, each list padded to a
// multiple of 8 indices with RSJ_PAD.  max_pos: the largest jN + 1; max_lt /
// max_lg: the largest jlt / jlg; max_exp: the largest rc * nsim.
#define RSJ_PAD (19936 + 624)
int launch_rsj(RsCell* d_cells, int ncells, int32_t rc, const uint32_t* d_poff, const uint32_t* d_pidx, int nseg,
               int64_t max_pos, int max_lt, int max_lg, int64_t max_exp, void* stream);
// RsCell.family for the HRS INT runs: rLap(n), rLap(1), mixquant (real-data-sims.R:375-402)
#define RS_FAMILY_HRS_INT 2
int launch_rs_stream(RsCell* d_cells, int ncells, int32_t rc, void* stream);
// The HRS NI runs: sample.int(n, k*m) and rLap(k) twice after set.seed(seeds[r]); n <= RS_HRS_NMAX.
#define RS_HRS_NMAX 65536
size_t rs_hrs_ni_lds_bytes(int64_t n);
int launch_rs_hrs_ni(const int32_t* d_seeds, int64_t runs, int64_t n, int64_t km, int64_t k,
                     int32_t* perm, double* lx, double* ly, void* stream);
// lds: dynamic LDS for gen_mix_gaussian cells (rs_mix_lds_bytes(max n)), else 0
int launch_rs_materialise(const RsCell* d_cells, int ncells, int32_t rc, void* stream,
                          size_t lds = 0);
size_t rs_mix_lds_bytes(int64_t n);
#define RS_MIX_NMAX 65536

}  // namespace dcor
