// dcor_premat.hip -- pre-materialised (explicit-input, HBM-streaming) kernels, the
// accumulation kernel, single-call helpers (mixquant, priv_standardize, dp_sd) and the
// on-device draw generator.  One 256-thread workgroup per replicate.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "dcor_common.h"

namespace dcor {


// ================================================== pre-materialised sign ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_sign(PrematSignConst p, dcor_rep_out* out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  __shared__ SelScratch sel;
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
                        &sel) * se;
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
// Streaming kernel (one workgroup per replicate): NI batch means + INT clipped products,
// compensated partial sums -> SubgPartial.  The mixquant / CI epilogue is a second kernel,
// so the streaming kernel carries no sort scratch and keeps many loads in flight (each
// thread issues UNR iterations' loads before using them).
struct SubgPartial { double s[10]; };  // sP, sT, sT2, sU, sU2 as (hi, lo)

#define SUBG_UNR 4

// Pack the shared HRS panel once per launch (the clips of the per-sample paths, so the values
// are identical) for the uncoded persistent kernels (k_premat_subg_dict<.., true>,
// k_hrs_fused_l2): one 16-B gather per NI sample instead of two 8-B ones, no per-rep clips.
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_xy_pack(PrematSubgConst p,
                                                               double2* __restrict__ xyc,
                                                               double2* __restrict__ soc) {
  const SubgConst& c = p.s;
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i >= c.n) return;
  const double x = p.X[i], y = p.Y[i];
  const double sv = c.sender_is_X ? x : y, ov = c.sender_is_X ? y : x;
  xyc[i] = make_double2(rclip(x, c.l1), rclip(y, c.l2));
  soc[i] = make_double2(rclip(sv, c.ls), rclip(ov, p.lo_));
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_subg_stream(PrematSubgConst p,
                                                                   const int* __restrict__ dict_ok,
                                                                   SubgPartial* __restrict__ part) {
  __shared__ double red[16 * DCOR_WAVES];
  if (dict_ok != nullptr && *dict_ok) return;  // the dictionary-coded kernel owns this launch
  const SubgConst& c = p.s;
  const int64_t rep = blockIdx.x;
  const int tid = threadIdx.x;
  const double* __restrict__ X = p.X + rep * p.xy_stride;
  const double* __restrict__ Y = p.Y + rep * p.xy_stride;
  const double* __restrict__ S = c.sender_is_X ? X : Y;
  const double* __restrict__ O = c.sender_is_X ? Y : X;
  const double* __restrict__ lx = p.lap_ni_x + rep * c.k;
  const double* __restrict__ ly = p.lap_ni_y + rep * c.k;
  const double* __restrict__ ll = p.lap_local + rep * c.n;
  DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
  auto int_term = [&](double sv, double ov0, double l) {   // ver-cor-subG.R:88-90; rds:222-232
    const double ov = p.hrs ? rclip(ov0, p.lo_) : ov0;
    const double Uc = rclip((rclip(sv, c.ls) + c.bs * l) * ov, c.lr);
    ks_acc(sU, Uc);
    ks_acc(sU2, Uc * Uc);
  };
  auto batch_term = [&](double lxj, double lyj, DD bx, DD by) {  // ver-cor-subG.R:44-55
    const DD xb = dd_div_d(bx, c.md), yb = dd_div_d(by, c.md);
    const double xt = (xb.hi + xb.lo) + c.bx * lxj;
    const double yt = (yb.hi + yb.lo) + c.by * lyj;
    ks_acc(sP, xt * yt);
    const double T = c.md * xt * yt;
    ks_acc(sT, T);
    ks_acc(sT2, T * T);
  };
  if (p.perm == nullptr) {
    // contiguous batches: each element read once by its batch owner (NI + INT)
    for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
      DD bx{0, 0}, by{0, 0};
      const int64_t i0 = j * c.m;
      for (int r = 0; r < c.m; ++r) {
        const int64_t i = i0 + r;
        const double xv = X[i], yv = Y[i];
        dd_acc(bx, rclip(xv, c.l1));
        dd_acc(by, rclip(yv, c.l2));
        int_term(c.sender_is_X ? xv : yv, c.sender_is_X ? yv : xv, ll[i]);
      }
      batch_term(lx[j], ly[j], bx, by);
    }
    for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) int_term(S[i], O[i], ll[i]);
  } else {
    // HRS: random batches idx = sample.int(n, k*m) (real-data-sims.R:131).
    // INT over all n: UNR coalesced loads in flight per thread.
    const int64_t step = (int64_t)DCOR_BLOCK * SUBG_UNR;
    int64_t i = tid;
    for (; i + (SUBG_UNR - 1) * DCOR_BLOCK < c.n; i += step) {
      double l[SUBG_UNR], sv[SUBG_UNR], ov[SUBG_UNR];
#pragma unroll
      for (int u = 0; u < SUBG_UNR; ++u) {
        l[u] = ll[i + u * DCOR_BLOCK];
        sv[u] = S[i + u * DCOR_BLOCK];
        ov[u] = O[i + u * DCOR_BLOCK];
      }
#pragma unroll
      for (int u = 0; u < SUBG_UNR; ++u) int_term(sv[u], ov[u], l[u]);
    }
    for (; i < c.n; i += DCOR_BLOCK) int_term(S[i], O[i], ll[i]);
    // NI over batches: perm rows gathered from the (cache-resident) panel.
    const int32_t* __restrict__ pm = p.perm + rep * (c.k * c.m);
    if (c.m == 2) {
      int64_t j = tid;
      for (; j + (SUBG_UNR - 1) * DCOR_BLOCK < c.k; j += step) {
        int32_t i0[SUBG_UNR], i1[SUBG_UNR];
        double ax[SUBG_UNR], ay[SUBG_UNR];
#pragma unroll
        for (int u = 0; u < SUBG_UNR; ++u) {
          const int64_t jj = j + u * DCOR_BLOCK;
          const int2 pr = *reinterpret_cast<const int2*>(pm + 2 * jj);
          i0[u] = pr.x; i1[u] = pr.y;
          ax[u] = lx[jj]; ay[u] = ly[jj];
        }
#pragma unroll
        for (int u = 0; u < SUBG_UNR; ++u) {
          const DD bx = two_sum(rclip(X[i0[u]], c.l1), rclip(X[i1[u]], c.l1));
          const DD by = two_sum(rclip(Y[i0[u]], c.l2), rclip(Y[i1[u]], c.l2));
          batch_term(ax[u], ay[u], bx, by);
        }
      }
      for (; j < c.k; j += DCOR_BLOCK) {
        const DD bx = two_sum(rclip(X[pm[2 * j]], c.l1), rclip(X[pm[2 * j + 1]], c.l1));
        const DD by = two_sum(rclip(Y[pm[2 * j]], c.l2), rclip(Y[pm[2 * j + 1]], c.l2));
        batch_term(lx[j], ly[j], bx, by);
      }
    } else {
      for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
        DD bx{0, 0}, by{0, 0};
        for (int r = 0; r < c.m; ++r) {
          const int64_t ii = pm[j * c.m + r];
          dd_acc(bx, rclip(X[ii], c.l1));
          dd_acc(by, rclip(Y[ii], c.l2));
        }
        batch_term(lx[j], ly[j], bx, by);
      }
    }
  }
  DD d5[5] = {sP, sT, sT2, sU, sU2};
  block_sum_dd<5>(d5, red);
  if (tid == 0) {
    SubgPartial q;
#pragma unroll
    for (int v = 0; v < 5; ++v) { q.s[2 * v] = d5[v].hi; q.s[2 * v + 1] = d5[v].lo; }
    part[rep] = q;
  }
}


// NI result, INT estimate, mixquant, INT CI of replicate `rep` from its five sums
// (ver-cor-subG.R:51-59, 91-103; real-data-sims.R:233-243), in two halves around the mixquant:
// premat_subg_pre gives the NI triple, the INT point estimate, sd and c* (and whether the CI takes
// a mixquant at all: the HRS sd == 0 branch does not); premat_subg_post the CI from quant(c*).
struct SubgPre {
  double o[3];
  double rho, sd, cstar;
  bool quant;
};
__device__ __forceinline__ SubgPre premat_subg_pre(const PrematSubgConst& p, const DD (&d5)[5],
                                                   double lapc) {
  const SubgConst& c = p.s;
  SubgPre r;
  ni_subg_result(c, d5[0], d5[1], d5[2], r.o);
  const DD mU = dd_div_d(d5[3], c.nd);
  r.rho = (mU.hi + mU.lo) + c.s_central * lapc;
  r.sd = sqrt(dd_var(d5[3], d5[4], c.nd));
  r.quant = !p.hrs || r.sd != 0.0;
  r.cstar = !p.hrs ? 2.0 / (c.sqrt_n * r.sd * c.eps_r) : (2.0 * c.lr) / (c.sqrt_n * r.sd * c.eps_r);
  return r;
}
__device__ __forceinline__ dcor_rep_out premat_subg_post(const PrematSubgConst& p, const SubgPre& r,
                                                         double qq) {
  const SubgConst& c = p.s;
  double width;
  if (!p.hrs) {
    const double se_norm = sqrt(r.sd * r.sd + c.sn2x2);
    width = qq * se_norm / c.sqrt_n;
  } else if (r.sd == 0.0) {
    width = p.crit_sqrt2_s;
  } else {
    width = qq * (r.sd / c.sqrt_n);
  }
  return dcor_rep_out{r.o[0], r.o[1], r.o[2], r.rho, rmax(r.rho - width, -1.0), rmin(r.rho + width, 1.0)};
}

// quant(c*) is the mixquant (workgroup- or wave-level, called uniformly); `writer` is the one
// thread that stores the record.
template <class Quant>
__device__ __forceinline__ void premat_subg_finish_q(const PrematSubgConst& p, int64_t rep,
                                                     const DD (&d5)[5], Quant&& quant, bool writer,
                                                     dcor_rep_out* out, double lapc) {
  const SubgPre r = premat_subg_pre(p, d5, lapc);
  const double qq = r.quant ? quant(r.cstar) : 0.0;
  const dcor_rep_out o = premat_subg_post(p, r, qq);
  if (writer) out[rep] = o;
}

__device__ __forceinline__ void premat_subg_finish(const PrematSubgConst& p, int64_t rep,
                                                   const DD (&d5)[5], SelScratch* sel,
                                                   dcor_rep_out* out) {
  const MixConst& mx = p.s.mix;
  premat_subg_finish_q(p, rep, d5, [&](double cs) {
    return mixquant_loaded(mx, cs, p.mix_z + rep * mx.nsim, p.mix_l + rep * mx.nsim, sel);
  }, threadIdx.x == 0, out, p.lap_central[rep]);
}

// The five sums of replicate `rep`: its p.slices partials merged in slice order.
__device__ __forceinline__ void load_partials(const PrematSubgConst& p,
                                              const SubgPartial* __restrict__ part, int64_t rep,
                                              DD (&d5)[5]) {
  const int S = p.slices > 1 ? p.slices : 1;
  const SubgPartial q = part[rep * S];
#pragma unroll
  for (int v = 0; v < 5; ++v) d5[v] = two_sum(q.s[2 * v], q.s[2 * v + 1]);
  for (int t = 1; t < S; ++t) {
    const SubgPartial r = part[rep * S + t];
#pragma unroll
    for (int v = 0; v < 5; ++v) d5[v] = dd_add(d5[v], DD{r.s[2 * v], r.s[2 * v + 1]});
  }
}

// Wave-per-replicate epilogue (four replicates per workgroup, no workgroup barriers): the
// mixquant keys z + c l are loaded VPL per lane and selected with wave_select.
template <int VPL>
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_subg_epilogue_w(PrematSubgConst p, int64_t reps,
                                                                       const SubgPartial* __restrict__ part,
                                                                       dcor_rep_out* out) {
  __shared__ WaveSel wsel[DCOR_WAVES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t rep = (int64_t)blockIdx.x * DCOR_WAVES + wv;
  if (rep >= reps) return;  // whole waves only
  DD d5[5];
  load_partials(p, part, rep, d5);
  const MixConst& mx = p.s.mix;
  const double* z = p.mix_z + rep * mx.nsim;
  const double* l = p.mix_l + rep * mx.nsim;
  premat_subg_finish_q(p, rep, d5, [&](double cs) {
    double val[VPL];
#pragma unroll
    for (int s = 0; s < VPL; ++s) {
      const int i = lane + 64 * s;
      val[s] = i < mx.nsim ? z[i] + cs * l[i] : dnan();  // NaN keys are dropped (R's sort)
    }
    return wave_select<VPL>(val, mx.pos, &wsel[wv]);
  }, lane == 0, out, p.lap_central[rep]);
}

// Epilogue of the streaming kernels that hand their sums over through SubgPartial.
// The scalar half (sums, NI triple, sd, c*) runs in wave 0 only and c* reaches the other waves
// through LDS: the four waves computed it redundantly before, a quarter of the kernel's fp64 work.
__global__ __launch_bounds__(DCOR_BLOCK) void k_premat_subg_epilogue(PrematSubgConst p,
                                                                     const SubgPartial* __restrict__ part,
                                                                     dcor_rep_out* out) {
  __shared__ SelScratch sel;
  __shared__ double bc[2];  // c*, and 1.0 when the CI takes a mixquant
  const int64_t rep = blockIdx.x;
  const MixConst& mx = p.s.mix;
  double zv[SEL_VPT], lv[SEL_VPT];  // the mixquant draws do not depend on c*: load them first
  mixquant_prefetch(mx, p.mix_z + rep * mx.nsim, p.mix_l + rep * mx.nsim, zv, lv);
  SubgPre r{};
  if (threadIdx.x < 64) {
    DD d5[5];
    load_partials(p, part, rep, d5);
    r = premat_subg_pre(p, d5, p.lap_central[rep]);
    if (threadIdx.x == 0) { bc[0] = r.cstar; bc[1] = r.quant ? 1.0 : 0.0; }
  }
  __syncthreads();
  const double qq = bc[1] != 0.0 ? mixquant_regs(mx, bc[0], zv, lv, &sel) : 0.0;
  if (threadIdx.x == 0) out[rep] = premat_subg_post(p, r, qq);
}

// ------------------------------------------- dictionary-coded shared panel (HRS) ---
// Survey panels take few distinct values (HRS wave 2: 46 clipped ages, 201 clipped BMIs), so
// the shared panel is stored as one byte-pair code per sample plus two value dictionaries:
// 2 B per sample instead of 16 B, small enough to sit in LDS.  Every random NI batch gather
// and every INT panel read then hits LDS, and only the per-replicate noise / permutation
// streams touch HBM.  The values are the panel's own doubles, so results are unchanged.
// k_panel_dict builds the dictionaries with an LDS hash table (one workgroup); if a column
// has more than 256 distinct values (or a NaN or an infinity), it clears *ok and the L2-gather
// kernel runs: the coded kernels rely on a finite dictionary.
#define DICT_SLOTS 1024
#define DICT_MAX 256
#define DICT_THREADS 1024
__device__ __forceinline__ uint32_t dict_hash(unsigned long long key) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 54);  // 10 bits
}

__global__ __launch_bounds__(DICT_THREADS) void k_panel_dict(const double* __restrict__ X,
                                                           const double* __restrict__ Y, int64_t n,
                                                           uint16_t* __restrict__ codes,
                                                           double* __restrict__ dict, int* ok) {
  __shared__ unsigned long long tab[2][DICT_SLOTS];
  __shared__ int16_t sid[2][DICT_SLOTS];
  __shared__ int cnt[2], bad, wtot[2][DICT_THREADS / 64];
  const unsigned long long EMPTY = ~0ull;  // a NaN pattern: NaN inputs are rejected anyway
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int s = tid; s < DICT_SLOTS; s += DICT_THREADS) { tab[0][s] = EMPTY; tab[1][s] = EMPTY; }
  if (tid == 0) { cnt[0] = cnt[1] = 0; bad = 0; }
  __syncthreads();
  for (int64_t i0 = tid; i0 < n; i0 += 4 * DICT_THREADS) {
    double xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * DICT_THREADS;
      xv[u] = i < n ? X[i] : 0.0;
      yv[u] = i < n ? Y[i] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cpt = q & 1, u = q >> 1;
      if (i0 + u * DICT_THREADS >= n) break;
      if (*(volatile int*)&bad) break;
      const double v = cpt == 0 ? xv[u] : yv[u];
      if (!(fabs(v) <= 1.7976931348623157e308)) { bad = 1; break; }   // NaN or +-Inf
      const unsigned long long key = (unsigned long long)__double_as_longlong(v);
      uint32_t h = dict_hash(key);
      // Plain reads find a present key without an atomic (most samples repeat a value); the
      // CAS only runs on an empty slot.  The table is at most 1/4 full (256 of 1024).
      for (int probe = 0; probe < DICT_SLOTS; ++probe) {
        unsigned long long cur = *(volatile unsigned long long*)&tab[cpt][h];
        if (cur == EMPTY) {
          cur = atomicCAS(&tab[cpt][h], EMPTY, key);
          if (cur == EMPTY) {
            if (atomicAdd(&cnt[cpt], 1) >= DICT_MAX) bad = 1;
            break;
          }
        }
        if (cur == key) break;
        if (*(volatile int*)&bad) break;
        h = (h + 1) & (DICT_SLOTS - 1);
      }
    }
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) *ok = 0;
    return;
  }
  // dense ids in slot order: wave ballot ranks + a scan over the 16 wave totals
  for (int cpt = 0; cpt < 2; ++cpt) {
    const bool occ = tab[cpt][tid] != EMPTY;
    const unsigned long long b = __ballot(occ);
    const int below = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[cpt][wv] = __popcll(b);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += wtot[cpt][w];
    if (occ) {
      sid[cpt][tid] = (int16_t)(base + below);
      dict[cpt * DICT_MAX + base + below] = __longlong_as_double((long long)tab[cpt][tid]);
    }
  }
  if (tid < DICT_MAX) {  // unused entries are defined (never referenced by a code)
    if (tid >= cnt[0]) dict[tid] = 0.0;
    if (tid >= cnt[1]) dict[DICT_MAX + tid] = 0.0;
  }
  __syncthreads();
  for (int64_t i0 = tid; i0 < n; i0 += 4 * DICT_THREADS) {
    double xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * DICT_THREADS;
      xv[u] = i < n ? X[i] : 0.0;
      yv[u] = i < n ? Y[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * DICT_THREADS;
      if (i >= n) break;
      uint32_t id[2];
#pragma unroll
      for (int cpt = 0; cpt < 2; ++cpt) {
        const unsigned long long key = (unsigned long long)__double_as_longlong(cpt == 0 ? xv[u] : yv[u]);
        uint32_t h = dict_hash(key);
        while (tab[cpt][h] != key) h = (h + 1) & (DICT_SLOTS - 1);  // present by construction
        id[cpt] = (uint32_t)sid[cpt][h];
      }
      codes[i] = (uint16_t)(id[0] | (id[1] << 8));
    }
  }
  if (tid == 0) *ok = 1;
}

// Streaming kernel over the dictionary-coded panel: persistent workgroups of DICT_NT threads
// (the coded panel is loaded into LDS once per workgroup; 47 KB of LDS at n = 19,433 leaves
// three workgroups = 24 waves per CU to keep HBM loads in flight), work items grid-strided.
// A work item is one slice of one replicate: slice t of S takes the t-th share of the INT
// sample pairs and of the NI batch pairs, and writes its five compensated sums to
// part[rep * S + t]; the epilogue merges the S partials in slice order.  Slicing evens out the
// last round of a persistent grid (replicate counts rarely divide by the workgroup count).  The noise /
// permutation streams are read once, 16 B per lane, non-temporal.  Dynamic LDS layout: four
// clipped dictionaries dX, dY (NI clips), dS, dO (INT sender / other clips), the reduction
// scratch, then the n codes.
#define DICT_NT 512
#define DICT_NW (DICT_NT / 64)
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef int iv4 __attribute__((ext_vector_type(4)));
typedef int iv2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int64_t share(int64_t total, int t, int S) { return total * t / S; }

// L2 = true: the same kernel for a panel that has no dictionary -- the clipped panel packed in
// HBM (xyc, soc; 32 B per sample, L2-resident at survey sizes), each INT sample pair read as two
// coalesced double2, each NI sample gathered from L2.  Only the reduction scratch is in LDS.
template <int DUNR, int WPE, bool L2>  // 16-B loads in flight per thread; waves per SIMD
__global__ __launch_bounds__(DICT_NT, WPE) void k_premat_subg_dict(PrematSubgConst p,
                                                             const uint16_t* __restrict__ codes_g,
                                                             const double* __restrict__ dict_g,
                                                             const int* __restrict__ dict_ok,
                                                             int64_t reps,
                                                             SubgPartial* __restrict__ part) {
  extern __shared__ double dsm[];
  // the coded kernel owns a launch whose device probe found a dictionary, else the L2 kernel
  if (L2 ? (dict_ok != nullptr && *dict_ok != 0) : (*dict_ok == 0)) return;
  const SubgConst& c = p.s;
  const int tid = threadIdx.x;
  const int S = p.slices > 1 ? p.slices : 1;
  double* dX = dsm;
  double* dY = dsm + DICT_MAX;
  double* dS = dsm + 2 * DICT_MAX;
  double* dO = dsm + 3 * DICT_MAX;
  double* red = L2 ? dsm : dsm + 4 * DICT_MAX;
  uint16_t* cod = reinterpret_cast<uint16_t*>(dsm + 4 * DICT_MAX + 20 * DICT_NW);
  const double2* __restrict__ xyp = p.xyc;
  const double2* __restrict__ sop = p.soc;
  if constexpr (!L2) {
    if (tid < DICT_MAX) {
      const double x = dict_g[tid], y = dict_g[DICT_MAX + tid];
      dX[tid] = rclip(x, c.l1);                                   // real-data-sims.R:126-127
      dY[tid] = rclip(y, c.l2);
      const double sv = c.sender_is_X ? x : y, ov = c.sender_is_X ? y : x;
      dS[tid] = rclip(sv, c.ls);                                  // real-data-sims.R:222-227
      dO[tid] = p.hrs ? rclip(ov, p.lo_) : ov;
    }
    const int64_t nv = (c.n * 2 + 15) / 16;                      // 16-B words of codes
    const uint4* src = reinterpret_cast<const uint4*>(codes_g);
    uint4* dst = reinterpret_cast<uint4*>(cod);
    for (int64_t w = tid; w < nv; w += DICT_NT) dst[w] = src[w];
    __syncthreads();
  }
  // the clipped values of sample i: NI (x, y) and INT (sender, other)
  auto ni_xy = [&](int64_t i) -> double2 {
    if constexpr (L2) {
      return xyp[i];
    } else {
      const uint32_t a = cod[i];
      return make_double2(dX[a & 255u], dY[a >> 8]);
    }
  };
  const int64_t items = reps * S;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int64_t rep = it / S;
    const int t = (int)(it - rep * S);
    const double* __restrict__ lx = p.lap_ni_x + rep * c.k;
    const double* __restrict__ ly = p.lap_ni_y + rep * c.k;
    const double* __restrict__ ll = p.lap_local + rep * c.n;
    const int32_t* __restrict__ pm = p.perm + rep * (c.k * c.m);
    DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
    auto uval = [&](int64_t i, double l) {  // ver-cor-subG.R:88-90; real-data-sims.R:222-232
      double sv, ov;
      if constexpr (L2) {
        const double2 v = sop[i];
        sv = v.x; ov = v.y;
      } else {
        const uint32_t cd = cod[i];
        sv = dS[cd & 255u]; ov = dO[cd >> 8];
      }
      // coded panel: every dictionary value is finite (k_panel_dict), so is the noise, so the
      // product is never NaN and R's NaN-preserving clip reduces to min + max
      if constexpr (L2) return rclip((sv + c.bs * l) * ov, c.lr);
      else return rclip_fin((sv + c.bs * l) * ov, c.lr);
    };
    auto uterm = [&](int64_t i, double l) {
      const double Uc = uval(i, l);
      ks_acc(sU, Uc);
      ks_acc(sU2, Uc * Uc);
    };
    // an INT sample pair's two terms (a batch pair's) added plainly, the pair sum compensated:
    // half the TwoSum chains of per-term sums
    auto uterm2 = [&](int64_t i, double l0, double l1) {
      const double U0 = uval(i, l0), U1 = uval(i + 1, l1);
      ks_acc(sU, U0 + U1);
      ks_acc(sU2, U0 * U0 + U1 * U1);
    };
    // INT stream: sample pairs (2q, 2q + 1) whatever the row's alignment, so a replicate's sums
    // never depend on where its row sits in the launch (odd n: every other row starts 8 B off a
    // 16-B boundary and reads its pairs as two 8-B loads).  Slice S-1 takes the odd tail sample.
    {
      const bool al16 = (reinterpret_cast<uintptr_t>(ll) & 15) == 0;
      const int64_t np = c.n >> 1;
      const int64_t q0 = share(np, t, S), q1 = share(np, t + 1, S);
      const dv2* l2 = reinterpret_cast<const dv2*>(ll);
      auto ldp = [&](int64_t qq) -> dv2 {
        if (al16) return __builtin_nontemporal_load(l2 + qq);
        dv2 v;
        v.x = __builtin_nontemporal_load(ll + 2 * qq);
        v.y = __builtin_nontemporal_load(ll + 2 * qq + 1);
        return v;
      };
      int64_t q = q0 + tid;
      for (; q + (DUNR - 1) * DICT_NT < q1; q += DUNR * DICT_NT) {
        dv2 v[DUNR];
#pragma unroll
        for (int u = 0; u < DUNR; ++u) v[u] = ldp(q + u * DICT_NT);
#pragma unroll
        for (int u = 0; u < DUNR; ++u) uterm2(2 * (q + u * DICT_NT), v[u].x, v[u].y);
      }
      for (; q < q1; q += DICT_NT) {
        const dv2 v = ldp(q);
        uterm2(2 * q, v.x, v.y);
      }
      if (tid == DICT_NT - 1 && t == S - 1 && (c.n & 1)) uterm(c.n - 1, ll[c.n - 1]);
    }
    // workgroup sums: wave sums into a scratch half alternating per item (a wave can run at
    // most one barrier ahead), then lane v < 5 folds sum v over the waves in wave order.  The
    // INT sums are wave-reduced here, so they are not live across the NI loop.
    double* rb = red + (((it - blockIdx.x) / gridDim.x) & 1) * (10 * DICT_NW);
    auto wave_put = [&](int v, DD a) {
      a = wave_sum_dd(a);
      if ((tid & 63) == 0) {
        rb[(2 * v) * DICT_NW + (tid >> 6)] = a.hi;
        rb[(2 * v + 1) * DICT_NW + (tid >> 6)] = a.lo;
      }
    };
    wave_put(3, sU);
    wave_put(4, sU2);
    if (c.m == 2) {  // real-data-sims.R:131-137 with the exact two-value batch mean
      auto pair = [&](int a0, int b0, double lxj, double lyj) {
        const double2 a = ni_xy(a0), b = ni_xy(b0);
        const double xt = (a.x + b.x) * 0.5 + c.bx * lxj;
        const double yt = (a.y + b.y) * 0.5 + c.by * lyj;
        ks_acc(sP, xt * yt);
        const double T = c.md * xt * yt;
        ks_acc(sT, T);
        ks_acc(sT2, T * T);
      };
      // batches j, j + 1 (indices iv4, noise x2 / y2): the pair's terms added plainly
      auto pair2 = [&](iv4 pr, dv2 lx2, dv2 ly2) {
        const double2 a0 = ni_xy(pr.x), b0 = ni_xy(pr.y), a1 = ni_xy(pr.z), b1 = ni_xy(pr.w);
        const double xt0 = (a0.x + b0.x) * 0.5 + c.bx * lx2.x, yt0 = (a0.y + b0.y) * 0.5 + c.by * ly2.x;
        const double xt1 = (a1.x + b1.x) * 0.5 + c.bx * lx2.y, yt1 = (a1.y + b1.y) * 0.5 + c.by * ly2.y;
        const double T0 = c.md * xt0 * yt0, T1 = c.md * xt1 * yt1;
        ks_acc(sP, xt0 * yt0 + xt1 * yt1);
        ks_acc(sT, T0 + T1);
        ks_acc(sT2, T0 * T0 + T1 * T1);
      };
      // two batches (2q, 2q + 1) per lane whatever the rows' alignment (odd k: every other row
      // is 8 B off a 16-B boundary and reads int2 / double pairs instead of int4 / double2)
      const bool al = ((reinterpret_cast<uintptr_t>(pm) | reinterpret_cast<uintptr_t>(lx) |
                        reinterpret_cast<uintptr_t>(ly)) & 15) == 0;
      const int64_t np = c.k >> 1;
      const int64_t q0 = share(np, t, S), q1 = share(np, t + 1, S);
      const iv4* p4 = reinterpret_cast<const iv4*>(pm);
      const dv2* x2 = reinterpret_cast<const dv2*>(lx);
      const dv2* y2 = reinterpret_cast<const dv2*>(ly);
      auto ldb = [&](int64_t qq, iv4& pr, dv2& ax, dv2& ay) {
        if (al) {
          pr = __builtin_nontemporal_load(p4 + qq);
          ax = __builtin_nontemporal_load(x2 + qq);
          ay = __builtin_nontemporal_load(y2 + qq);
        } else {
          const iv2* p2 = reinterpret_cast<const iv2*>(pm);  // rows of 2k int32: 8-B aligned
          const iv2 a = __builtin_nontemporal_load(p2 + 2 * qq), b = __builtin_nontemporal_load(p2 + 2 * qq + 1);
          pr.x = a.x; pr.y = a.y; pr.z = b.x; pr.w = b.y;
          ax.x = __builtin_nontemporal_load(lx + 2 * qq);
          ax.y = __builtin_nontemporal_load(lx + 2 * qq + 1);
          ay.x = __builtin_nontemporal_load(ly + 2 * qq);
          ay.y = __builtin_nontemporal_load(ly + 2 * qq + 1);
        }
      };
      int64_t q = q0 + tid;
      for (; q + (DUNR / 2 - 1) * DICT_NT < q1; q += (DUNR / 2) * DICT_NT) {
        iv4 pr[DUNR / 2];
        dv2 ax[DUNR / 2], ay[DUNR / 2];
#pragma unroll
        for (int u = 0; u < DUNR / 2; ++u) ldb(q + u * DICT_NT, pr[u], ax[u], ay[u]);
#pragma unroll
        for (int u = 0; u < DUNR / 2; ++u) pair2(pr[u], ax[u], ay[u]);
      }
      for (; q < q1; q += DICT_NT) {
        iv4 pr;
        dv2 ax, ay;
        ldb(q, pr, ax, ay);
        pair2(pr, ax, ay);
      }
      if (tid == DICT_NT - 1 && t == S - 1 && (c.k & 1))
        pair(pm[2 * (c.k - 1)], pm[2 * (c.k - 1) + 1], lx[c.k - 1], ly[c.k - 1]);
    } else {
      for (int64_t j = share(c.k, t, S) + tid; j < share(c.k, t + 1, S); j += DICT_NT) {
        DD bx{0, 0}, by{0, 0};
        for (int r = 0; r < c.m; ++r) {
          const double2 a = ni_xy(pm[j * c.m + r]);
          dd_acc(bx, a.x);
          dd_acc(by, a.y);
        }
        const DD xb = dd_div_d(bx, c.md), yb = dd_div_d(by, c.md);
        const double xt = (xb.hi + xb.lo) + c.bx * lx[j];
        const double yt = (yb.hi + yb.lo) + c.by * ly[j];
        ks_acc(sP, xt * yt);
        const double T = c.md * xt * yt;
        ks_acc(sT, T);
        ks_acc(sT2, T * T);
      }
    }
    wave_put(0, sP);
    wave_put(1, sT);
    wave_put(2, sT2);
    __syncthreads();
    if (tid < 5) {
      const DD a = fold_waves_dd<DICT_NW>(rb + (2 * tid) * DICT_NW, rb + (2 * tid + 1) * DICT_NW);
      part[it].s[2 * tid] = a.hi;
      part[it].s[2 * tid + 1] = a.lo;
    }
  }
}

// Uncoded shared panel, m = 2, k even, n < 65536: the L2-gather kernel's replicate with the
// NI gathers served from LDS tiles instead of L2 (real-data-sims.R:115-147, 176-252).  Per
// replicate the workgroup sweeps the panel in tiles of consecutive samples (tile_pairs INT
// sample pairs each); filling a tile reads the packed clipped panel (k_premat_xy_pack: xyc, soc)
// from L2, coalesced, and the INT noise from HBM, adds the INT terms of its pairs, and stores
// the NI clips (clip(X, l1), clip(Y, l2)) to LDS.  Every thread holds the sample indices of its
// NQ batch pairs in registers (u16) and, per tile, adds the LDS entry of each index that falls in
// the tile to its batch sums: an index outside the tile reads a -0.0 sentinel, and -0.0 + a = a,
// a + -0.0 = a, so each batch sum ends as fl(a + b) = fl(b + a) whatever the tiles' order.  A
// random 16-B L2 gather per NI sample (19,432 per C5 replicate) becomes a share of a coalesced
// tile fill plus an LDS read.  Batch pairs beyond NQ * NT per thread take further rounds of
// tiles (NI only).  Threads own INT pairs and NI batch pairs q = tid (mod NT), ascending, as in
// the L2 kernel; PG adds the two terms of an INT pair (of a batch pair) plainly and compensates
// the pair sums, as the L2 kernel does, so with NT = 512 and NA = 1 the sums are its bit for bit.
// Measured (C5-continuous, 8192 replicates, round 4, with the epilogue): 1.05 ms with the INT
// stream in the first round's fills; timing ablations (wrong results, round 4) took 0.68 ms without
// it, 0.91 without the gathers, 0.93 without the NI noise.  The INT stream therefore runs in a kernel of its
// own by default (k_premat_subg_int; tiled_kernel() below).  A round issues all its batch-index
// loads, and later all its noise loads, before it waits for any: one HBM round trip each per
// round (a per-pair branch around each load had made them five).
// NT threads per workgroup; NQ batch pairs per thread per round; FU fill pairs per loop trip; GB
// batch pairs gathered per scheduling group; NA accumulator sets; WPE waves per SIMD.
// INTK = false: the INT sums are left to k_premat_subg_int (s[6..9] of each partial); the kernel
// then streams no INT bytes, writes s[0..5] only and needs 106 VGPRs instead of 128.
// Measured and dropped (round 5, C5-continuous, one box): the NI noise of the first 1-5 batch pairs
// loaded before the tile sweeps instead of after them -- 1.08e7-1.10e7 replicates/s with 0, 1 or 2
// pairs (it had looked like +9 % while the loads still branched on alignment at run time), 4 and 5
// pairs spill.
// AL: the caller's perm / lap_ni_x / lap_ni_y are 16-B aligned (every row is then, k being even):
// 16-B loads; otherwise element loads of the same values.  The launcher picks the instantiation, so
// the arithmetic -- and every replicate's bits -- does not depend on the buffers' alignment, and the
// aligned kernel carries no run-time branch around its loads (measured, round 5: the branch took
// the tiled kernel from 496 to 551 us per 8192 C5-continuous replicates).
// NI-only kernels (INTK = false) fill a tile by LDS-direct loads (global_load_lds_dwordx4, 1 KB per
// wave-instruction, no VGPR staging), every wave's share issued at once and waited for once, instead
// of the register-staged copy loop the INT-sum form needs (round 6: the same time, 2 fewer VGPRs).
// ENQ: the NI noise of the first ENQ batch pairs is loaded when the round's last tile has been filled,
// before its gathers, so those loads' HBM latency runs under the gathers (the rest after them); the
// loads move, the arithmetic does not.  C5-continuous (round 6, two boxes): ENQ 3 1.29e7-1.30e7
// replicates/s against 1.26e7-1.27e7 for ENQ 0 (4 VGPRs spill at the 128 cap); ENQ 2 1.28e7-1.29e7;
// ENQ 4 and 5 spill 12 and 25 VGPRs, 1.21e7-1.23e7 and 1.01e7; ENQ 3 with the NI sums created after
// the sweeps (no spill) 1.28e7.
template <int NT, int NQ, int FU, int GB, int NA, int WPE, bool PG = false, bool INTK = true, bool AL = true,
          int ENQ = 0>
__global__ __launch_bounds__(NT, WPE) void k_premat_subg_tiled(PrematSubgConst p,
                                                              const int* __restrict__ dict_ok,
                                                              int64_t reps, int64_t tile_pairs_,
                                                              SubgPartial* __restrict__ part) {
  constexpr int NW = NT / 64;
  extern __shared__ double dsm[];
  if (dict_ok != nullptr && *dict_ok != 0) return;  // the coded kernel owns this launch
  const SubgConst& c = p.s;
  const uint32_t tid = threadIdx.x;
  double* red = dsm;
  double2* tile = reinterpret_cast<double2*>(dsm + 20 * NW);
  const double2* __restrict__ xy = p.xyc;  // clip(X, l1), clip(Y, l2): the NI values
  const double2* __restrict__ so = p.soc;  // clip(S, ls), clip(O, lo): the INT values
  // every index fits 32 bits (n < 65536): VGPR offsets from uniform bases
  const uint32_t n = (uint32_t)c.n;
  const uint32_t nbp = (uint32_t)(c.k >> 1);  // batch pairs (k even)
  const uint32_t tile_pairs = (uint32_t)tile_pairs_;
  // the panel tile in LDS (its index; the panel is every replicate's) and the sweep direction
  uint32_t held = 0xFFFFFFFFu, dir = 0u;
  for (int64_t it = blockIdx.x; it < reps; it += gridDim.x) {
    const int64_t rep = it;
    const double* __restrict__ ll = p.lap_local + rep * c.n;
    // batch pair q's four indices and two noise pairs (AL above)
    const int* __restrict__ pr_row = p.perm + rep * (c.k * 2);
    const double* __restrict__ x_row = p.lap_ni_x + rep * c.k;
    const double* __restrict__ y_row = p.lap_ni_y + rep * c.k;
    auto ld_pr = [&](uint32_t q) -> iv4 {
      if constexpr (AL) return __builtin_nontemporal_load(reinterpret_cast<const iv4*>(pr_row) + q);
      iv4 v;
      v.x = __builtin_nontemporal_load(pr_row + 4 * q);
      v.y = __builtin_nontemporal_load(pr_row + 4 * q + 1);
      v.z = __builtin_nontemporal_load(pr_row + 4 * q + 2);
      v.w = __builtin_nontemporal_load(pr_row + 4 * q + 3);
      return v;
    };
    auto ld_nz = [&](const double* __restrict__ row, uint32_t q) -> dv2 {
      if constexpr (AL) return __builtin_nontemporal_load(reinterpret_cast<const dv2*>(row) + q);
      dv2 v;
      v.x = __builtin_nontemporal_load(row + 2 * q);
      v.y = __builtin_nontemporal_load(row + 2 * q + 1);
      return v;
    };
    // two independent accumulator sets (the first / second sample of an INT pair, the first /
    // second batch of a batch pair): twice the fp64 dependency chains in flight per thread at
    // two waves per SIMD; the sets are merged with dd_add before the wave reduction
    DD sP[NA] = {}, sT[NA] = {}, sT2[NA] = {}, sU[NA] = {}, sU2[NA] = {};
    auto merged = [](const DD (&a)[NA]) { return NA == 1 ? a[0] : dd_add(a[0], a[NA - 1]); };
    auto uterm = [&](double2 v, double l, int w) {  // ver-cor-subG.R:88-90; rds:222-232
      const double Uc = rclip((v.x + c.bs * l) * v.y, c.lr);
      ks_acc(sU[w % NA], Uc);
      ks_acc(sU2[w % NA], Uc * Uc);
    };
    // PG: an INT pair's two terms added plainly, the pair sum compensated
    auto uterm2 = [&](double2 v0, double l0, double2 v1, double l1) {
      const double U0 = rclip((v0.x + c.bs * l0) * v0.y, c.lr);
      const double U1 = rclip((v1.x + c.bs * l1) * v1.y, c.lr);
      ks_acc(sU[0], U0 + U1);
      ks_acc(sU2[0], U0 * U0 + U1 * U1);
    };
    // INT sample pairs (2q, 2q + 1) whatever the row's alignment, as in the L2 kernel (a row 8 B off
    // a 16-B boundary reads its pairs as two 8-B loads); the odd tail sample joins the last tile.
    const bool al16 = (reinterpret_cast<uintptr_t>(ll) & 15) == 0;
    const uint32_t h = 0u;
    const uint32_t np = n >> 1;
    const dv2* __restrict__ l2 = reinterpret_cast<const dv2*>(ll);
    auto ldp = [&](uint32_t qq) -> dv2 {
      if (al16) return __builtin_nontemporal_load(l2 + qq);
      dv2 v;
      v.x = __builtin_nontemporal_load(ll + 2 * qq);
      v.y = __builtin_nontemporal_load(ll + 2 * qq + 1);
      return v;
    };
    const uint32_t ntiles = np > 0 ? (np + tile_pairs - 1) / tile_pairs : 1u;
    double* rb = red + (((it - blockIdx.x) / gridDim.x) & 1) * (10 * NW);
    auto wave_put = [&](int v, DD a) {
      a = wave_sum_dd(a);
      if ((tid & 63) == 0) {
        rb[(2 * v) * NW + (tid >> 6)] = a.hi;
        rb[(2 * v + 1) * NW + (tid >> 6)] = a.lo;
      }
    };
    // rounds of NQ * NT batch pairs; the INT terms ride along the first round's fills
    for (uint32_t qb = 0; qb == 0 || qb < nbp; qb += (uint32_t)NQ * NT) {
      const bool first = INTK && qb == 0;
      uint32_t sa[NQ], sb[NQ];  // (a | b << 16) of the pair's two batches
      double ax[NQ][2], ay[NQ][2];
      // every load of the round first (a pair past the last re-reads the last), then the packing:
      // one HBM round trip per round instead of one per batch pair
      iv4 pr[NQ];
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const uint32_t q = qb + tid + (uint32_t)u * NT;
        pr[u] = ld_pr(q < nbp ? q : nbp - 1);
      }
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const uint32_t q = qb + tid + (uint32_t)u * NT;
        sa[u] = sb[u] = 0xFFFFFFFFu;  // 65535 is never a sample index (n < 65536)
        if (q < nbp) {
          sa[u] = (uint32_t)pr[u].x | ((uint32_t)pr[u].y << 16);
          sb[u] = (uint32_t)pr[u].z | ((uint32_t)pr[u].w << 16);
        }
        ax[u][0] = ax[u][1] = ay[u][0] = ay[u][1] = -0.0;
      }
      // NI noise of this round's batch pairs (past the last pair: the last pair's), every load issued
      // before any is used: one round trip per round
      dv2 nx[NQ], ny[NQ];
      auto load_noise = [&](int u) {
        const uint32_t q = qb + tid + (uint32_t)u * NT, qc = q < nbp ? q : nbp - 1;
        nx[u] = ld_nz(x_row, qc);
        ny[u] = ld_nz(y_row, qc);
      };
      for (uint32_t ti = 0; ti < ntiles; ++ti) {
        // NI-only kernel: every other round sweeps the tiles in reverse, so it starts on the tile
        // the previous round (of this replicate or the last) ended on, still in LDS
        const uint32_t tp = (!INTK && dir) ? ntiles - 1 - ti : ti;
        const uint32_t pa = tp * tile_pairs;
        const uint32_t pb = pa + tile_pairs < np ? pa + tile_pairs : np;
        const uint32_t lo = tp == 0 ? 0u : h + 2 * pa;
        const uint32_t hi = tp == ntiles - 1 ? n : h + 2 * pb;
        const uint32_t tn = hi - lo;
        if (INTK || tp != held) {
          __syncthreads();  // the previous tile's readers are done
          if constexpr (!INTK) {
            // xy[lo, hi) -> tile[0, tn): chunk cc of 64 entries by wave cc mod NW, lane-linear
            const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
            for (uint32_t cc = wv; cc * 64u < tn; cc += (uint32_t)NW) {
              const uint32_t t = cc * 64u + lane;
              if (t < tn)
                __builtin_amdgcn_global_load_lds((const void*)(xy + lo + t),
                                                 (__attribute__((address_space(3))) void*)(tile + cc * 64u), 16, 0, 0);
            }
            if (tid == 0) tile[tn] = make_double2(-0.0, -0.0);  // the out-of-tile sentinel
            __builtin_amdgcn_s_waitcnt(0x0F70);                 // vmcnt(0): this wave's copies landed
            __syncthreads();
            held = tp;
          }
        }
        if (INTK) {   // (the barrier above has run)
          // fill: this thread's INT pairs q = tid (mod NT) in [pa, pb), FU per loop trip
          uint32_t q = pa + ((tid + NT - pa % NT) % NT);
          for (; q + (FU - 1) * NT < pb; q += FU * NT) {
            double2 a0[FU], a1[FU], s0[FU], s1[FU];
            dv2 lv[FU];
#pragma unroll
            for (int u = 0; u < FU; ++u) {
              const uint32_t i = h + 2 * (q + u * NT);
              a0[u] = xy[i]; a1[u] = xy[i + 1];
              if (first) {
                s0[u] = so[i]; s1[u] = so[i + 1];
                lv[u] = ldp(q + u * NT);
              }
            }
#pragma unroll
            for (int u = 0; u < FU; ++u) {
              const uint32_t i = h + 2 * (q + u * NT);
              tile[i - lo] = a0[u];
              tile[i + 1 - lo] = a1[u];
              if (first) {
                if (PG) {
                  uterm2(s0[u], lv[u].x, s1[u], lv[u].y);
                } else {
                  uterm(s0[u], lv[u].x, 0);
                  uterm(s1[u], lv[u].y, 1);
                }
              }
            }
          }
          for (; q < pb; q += NT) {
            const uint32_t i = h + 2 * q;
            tile[i - lo] = xy[i];
            tile[i + 1 - lo] = xy[i + 1];
            if (first) {
              const dv2 l = ldp(q);
              if (PG) {
                uterm2(so[i], l.x, so[i + 1], l.y);
              } else {
                uterm(so[i], l.x, 0);
                uterm(so[i + 1], l.y, 1);
              }
            }
          }
          if (tp == ntiles - 1 && h + 2 * np < n && tid == NT - 1) tile[n - 1 - lo] = xy[n - 1];
          if (tid == 0) tile[tn] = make_double2(-0.0, -0.0);  // the out-of-tile sentinel
          __syncthreads();
          held = tp;
        }
        if (ENQ > 0 && ti + 1 == ntiles) {
#pragma unroll
          for (int u = 0; u < ENQ; ++u) load_noise(u);
        }
        // gather: every index of this thread's batch pairs against the tile
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          const uint32_t i0 = sa[u] & 0xFFFFu, i1 = sa[u] >> 16, i2 = sb[u] & 0xFFFFu, i3 = sb[u] >> 16;
          const double2 t0 = tile[min(i0 - lo, tn)], t1 = tile[min(i1 - lo, tn)];
          const double2 t2 = tile[min(i2 - lo, tn)], t3 = tile[min(i3 - lo, tn)];
          ax[u][0] = (ax[u][0] + t0.x) + t1.x;
          ay[u][0] = (ay[u][0] + t0.y) + t1.y;
          ax[u][1] = (ax[u][1] + t2.x) + t3.x;
          ay[u][1] = (ay[u][1] + t2.y) + t3.y;
          // GB pairs' LDS reads in flight at a time: the scheduler would otherwise hoist all 4 NQ
          // reads (16 VGPRs each) above the adds
          if ((u + 1) % GB == 0) __builtin_amdgcn_sched_barrier(0);
        }
      }
      dir ^= 1u;
      if (first) {
        if (tid == NT - 1 && h + 2 * np < n) uterm(so[n - 1], ll[n - 1], 1);
        wave_put(3, merged(sU));
        wave_put(4, merged(sU2));
      }
      // NI terms of this round's batch pairs, ascending q (real-data-sims.R:131-137)
#pragma unroll
      for (int u = ENQ; u < NQ; ++u) load_noise(u);
#pragma unroll
      for (int u = 0; u < NQ; ++u) {
        const uint32_t q = qb + tid + (uint32_t)u * NT;
        if (q < nbp) {
          const dv2 lx = nx[u], ly = ny[u];
          if (PG) {  // the pair's two batch terms added plainly, the pair sums compensated
            const double xt0 = ax[u][0] * 0.5 + c.bx * lx[0], yt0 = ay[u][0] * 0.5 + c.by * ly[0];
            const double xt1 = ax[u][1] * 0.5 + c.bx * lx[1], yt1 = ay[u][1] * 0.5 + c.by * ly[1];
            const double T0 = c.md * xt0 * yt0, T1 = c.md * xt1 * yt1;
            ks_acc(sP[0], xt0 * yt0 + xt1 * yt1);
            ks_acc(sT[0], T0 + T1);
            ks_acc(sT2[0], T0 * T0 + T1 * T1);
          } else {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const double xt = ax[u][b] * 0.5 + c.bx * lx[b];
              const double yt = ay[u][b] * 0.5 + c.by * ly[b];
              ks_acc(sP[b % NA], xt * yt);
              const double T = c.md * xt * yt;
              ks_acc(sT[b % NA], T);
              ks_acc(sT2[b % NA], T * T);
            }
          }
        }
      }
    }
    wave_put(0, merged(sP));
    wave_put(1, merged(sT));
    wave_put(2, merged(sT2));
    __syncthreads();
    if (tid < (INTK ? 5u : 3u)) {
      const DD a = fold_waves_dd<NW>(rb + (2 * tid) * NW, rb + (2 * tid + 1) * NW);
      part[it].s[2 * tid] = a.hi;
      part[it].s[2 * tid + 1] = a.lo;
    }
  }
}

// The INT sums of the tiled kernel's replicates in a kernel of their own (real-data-sims.R:
// 176-252; ver-cor-subG.R:88-90): the packed clipped (S, O) panel and each replicate's local noise
// streamed once, R replicates per workgroup sharing every panel load, with no tile phases or
// barriers between the loads.  The work split and summation order are the tiled kernel's (INT
// pairs q = t (mod 512) ascending in logical thread t, the odd tail sample last in thread 511,
// wave sums folded over the 8 logical waves in order): 256 threads stand for the 512 logical
// threads t and t + 256, so the sums are the tiled and L2 kernels' bit for bit.  Writes s[6..9]
// of each replicate's partial; k_premat_subg_tiled<.., INTK = false> writes s[0..5].
// The INT kernel's replicates per workgroup (R), pair slots loaded per step and minimum waves per
// SIMD: 4, 1, 4 (100 VGPRs, 2048 workgroups at 8192 replicates) measured 0.54 of 8 TB/s for
// C5-continuous (round 4) against 0.53-0.54 for 2, 2, 1 and 2, 1, 1, 0.52 for 2, 1, 8 (spills) and
// 0.47 for 2, 2, 6 (spills).
#define DCOR_INT_WPE 4
template <int R>
__global__ __launch_bounds__(256, DCOR_INT_WPE) void k_premat_subg_int(PrematSubgConst p, int64_t reps,
                                                         SubgPartial* __restrict__ part) {
  constexpr int LNW = 8;                 // logical waves (512 logical threads)
  __shared__ double red[R][4][LNW];      // [replicate][sU.hi, sU.lo, sU2.hi, sU2.lo][logical wave]
  const SubgConst& c = p.s;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = (uint32_t)c.n, np = n >> 1;
  const double2* __restrict__ so = p.soc;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const double* ll[R];
  bool al[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t rep = r0 + r < reps ? r0 + r : reps - 1;  // a short last group recomputes, never writes
    ll[r] = p.lap_local + rep * c.n;
    al[r] = (reinterpret_cast<uintptr_t>(ll[r]) & 15) == 0;
  }
  auto ldp = [&](int r, uint32_t q) -> dv2 {
    if (al[r]) return __builtin_nontemporal_load(reinterpret_cast<const dv2*>(ll[r]) + q);
    dv2 v;
    v.x = __builtin_nontemporal_load(ll[r] + 2 * q);
    v.y = __builtin_nontemporal_load(ll[r] + 2 * q + 1);
    return v;
  };
  DD sU[R][2] = {}, sU2[R][2] = {};      // [replicate][logical thread tid, tid + 256]
  // Pair p belongs to logical thread p mod 512, so the pairs q = tid (mod 512) go to set 0 and
  // q = tid + 256 (mod 512) to set 1, each set in ascending order, as in the 512-thread kernels.
  // One loop per set, one pair slot per trip (its loads first, then its terms; the set a
  // compile-time index).  Measured (round 5, per 8192 C5-continuous replicates, one box): 245 us, as
  // round 4's loop (which summed both sets into one); both slots of a 512-pair trip in one loop body
  // took 269 us (the second slot's loads waited behind the first's terms and its branch), or 354 us
  // with both slots' loads issued first.
  auto sweep = [&](uint32_t q0, auto set_tag) {
    constexpr int SET = decltype(set_tag)::value;
    for (uint32_t q = q0; q < np; q += 512) {
      const double2 v0 = so[2 * q], v1 = so[2 * q + 1];
      dv2 l[R];
#pragma unroll
      for (int r = 0; r < R; ++r) l[r] = ldp(r, q);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double U0 = rclip((v0.x + c.bs * l[r].x) * v0.y, c.lr);
        const double U1 = rclip((v1.x + c.bs * l[r].y) * v1.y, c.lr);
        ks_acc(sU[r][SET], U0 + U1);
        ks_acc(sU2[r][SET], U0 * U0 + U1 * U1);
      }
    }
  };
  sweep(tid, std::integral_constant<int, 0>());
  sweep(tid + 256, std::integral_constant<int, 1>());
  if (tid == 255 && 2 * np < n) {        // logical thread 511: the odd tail sample
    const double2 v = so[n - 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double Uc = rclip((v.x + c.bs * ll[r][n - 1]) * v.y, c.lr);
      ks_acc(sU[r][1], Uc);
      ks_acc(sU2[r][1], Uc * Uc);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int set = 0; set < 2; ++set) {
      const DD a = wave_sum_dd(sU[r][set]), a2 = wave_sum_dd(sU2[r][set]);
      if ((tid & 63) == 0) {
        const int w = set * 4 + (int)(tid >> 6);
        red[r][0][w] = a.hi; red[r][1][w] = a.lo;
        red[r][2][w] = a2.hi; red[r][3][w] = a2.lo;
      }
    }
  __syncthreads();
  if (tid < 2 * R) {
    const int r = (int)tid >> 1, v = (int)tid & 1;
    const DD a = fold_waves_dd<LNW>(red[r][2 * v], red[r][2 * v + 1]);
    if (r0 + r < reps) {
      part[r0 + r].s[6 + 2 * v] = a.hi;
      part[r0 + r].s[7 + 2 * v] = a.lo;
    }
  }
}

// ======================================================== accumulation ===
// Deterministic per-method summary of `count` records (one workgroup).
// Stage 1: block b folds records [b*per, min((b+1)*per, count)) of both methods into a
// partial accumulator pair part[2b], part[2b+1].  Stage 2 merges the partials in block
// order (deterministic for a given count).
__device__ __forceinline__ void acc_record(double est, double lo, double hi, double rho, DD* s,
                                           long long* cnt) {
  const bool nae = (est != est), nal = (lo != lo), nah = (hi != hi);
  if (nae) ++cnt[2]; else {
    ks_acc(s[0], est);
    ks_acc(s[1], est * est);
    const double e = est - rho;
    ks_acc(s[2], e * e);
  }
  if (nal || nah) ++cnt[3]; else {
    ks_acc(s[3], hi - lo);
    ks_acc(s[4], lo);
    ks_acc(s[5], hi);
  }
  // R: rho >= lo && rho <= hi with NA three-valued logic
  const int a = nal ? 2 : (rho >= lo ? 1 : 0);
  const int bq = nah ? 2 : (rho <= hi ? 1 : 0);
  int cv;
  if (a == 0) cv = 0; else if (a == 1) cv = bq; else cv = (bq == 0) ? 0 : 2;
  if (cv == 1) ++cnt[0]; else if (cv == 2) ++cnt[1];
}

__device__ __forceinline__ void acc_write(dcor_accum* dst, int64_t n, const DD* s, const long long* t) {
  dcor_accum a;
  a.n = n; a.n_cover = t[0]; a.n_cover_na = t[1]; a.n_na_est = t[2]; a.n_na_ci = t[3];
  a.reserved[0] = a.reserved[1] = a.reserved[2] = 0;
  a.est[0] = s[0].hi; a.est[1] = s[0].lo; a.est2[0] = s[1].hi; a.est2[1] = s[1].lo;
  a.se2[0] = s[2].hi; a.se2[1] = s[2].lo; a.len[0] = s[3].hi; a.len[1] = s[3].lo;
  a.lo[0] = s[4].hi; a.lo[1] = s[4].lo; a.hi[0] = s[5].hi; a.hi[1] = s[5].lo;
  *dst = a;
}

// One accumulate block: records [b0, b1) of one cell (both methods) into dst[0], dst[1].  Every
// accumulate kernel runs this body, so a block's partial is the same bits whichever kernel, launch
// or pass computed it.
__device__ __forceinline__ void acc_block_body(const dcor_rep_out* rec, int64_t b0, int64_t b1,
                                               double rho, dcor_accum* dst, double* red,
                                               long long* redi) {
  for (int meth = 0; meth < 2; ++meth) {
    DD s[6] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}};
    long long cnt[4] = {0, 0, 0, 0};  // cover, cover_na, na_est, na_ci
    for (int64_t b = b0 + threadIdx.x; b < b1; b += DCOR_BLOCK) {
      const double* r = &rec[b].ni_hat + 3 * meth;
      acc_record(r[0], r[1], r[2], rho, s, cnt);
    }
    block_sum_dd<6>(s, red);
    long long tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) tot[q] = block_sum_i(cnt[q], redi);
    if (threadIdx.x == 0) acc_write(dst + meth, b1 > b0 ? b1 - b0 : 0, s, tot);
  }
}

// Merge nb block partials (part[2 b + meth]) in block order into acc[0], acc[1].
__device__ __forceinline__ void acc_merge_body(const dcor_accum* part, int64_t nb, int64_t count,
                                               dcor_accum* acc, double* red, long long* redi) {
  for (int meth = 0; meth < 2; ++meth) {
    DD s[6] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}};
    long long cnt[4] = {0, 0, 0, 0};
    for (int64_t b = threadIdx.x; b < nb; b += DCOR_BLOCK) {
      const dcor_accum& a = part[2 * b + meth];
      s[0] = dd_add(s[0], DD{a.est[0], a.est[1]});
      s[1] = dd_add(s[1], DD{a.est2[0], a.est2[1]});
      s[2] = dd_add(s[2], DD{a.se2[0], a.se2[1]});
      s[3] = dd_add(s[3], DD{a.len[0], a.len[1]});
      s[4] = dd_add(s[4], DD{a.lo[0], a.lo[1]});
      s[5] = dd_add(s[5], DD{a.hi[0], a.hi[1]});
      cnt[0] += a.n_cover; cnt[1] += a.n_cover_na; cnt[2] += a.n_na_est; cnt[3] += a.n_na_ci;
    }
    block_sum_dd<6>(s, red);
    long long tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) tot[q] = block_sum_i(cnt[q], redi);
    if (threadIdx.x == 0) acc_write(acc + meth, count, s, tot);
  }
}

// launch_accumulate's partition of `count` records: ~2048 per block, at most 512 blocks.
__host__ __device__ __forceinline__ int64_t acc_nblocks(int64_t count) {
  int64_t nb = (count + 2047) / 2048;
  if (nb < 1) nb = 1;
  if (nb > 512) nb = 512;
  return nb;
}
__host__ __device__ __forceinline__ int64_t acc_per(int64_t count, int64_t nb) {
  return (count + nb - 1) / nb > 0 ? (count + nb - 1) / nb : 1;
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_accumulate(const dcor_rep_out* rec, int64_t count,
                                                           int64_t per, double rho,
                                                           dcor_accum* part) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  const int64_t b0 = (int64_t)blockIdx.x * per;
  const int64_t b1 = (b0 + per < count) ? b0 + per : count;
  acc_block_body(rec, b0, b1, rho, part + 2 * blockIdx.x, red, redi);
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_accumulate_merge(const dcor_accum* part, int nb,
                                                                 int64_t count, dcor_accum* acc) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  acc_merge_body(part, nb, count, acc, red, redi);
}

// Pass form for the batched grid: entry j of a pass names blocks [blo, bhi) of one cell's
// partition (acc_nblocks of the cell's count), whose records sit in this pass's buffer at
// rec + base (record r of the cell -- cell-relative -- at rec[base + r - blo per]).  Block (t, j)
// runs block blo + t exactly as k_accumulate would on the cell alone; a one-block cell writes its
// accumulators directly, the others their partial at part[2 (poff + b)].
__global__ __launch_bounds__(DCOR_BLOCK) void k_accumulate_pass(const dcor_rep_out* rec,
                                                                const AccEntry* __restrict__ ent,
                                                                dcor_accum* part, dcor_accum* acc) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  const AccEntry e = ent[blockIdx.y];
  const int64_t b = e.blo + (int64_t)blockIdx.x;
  if (b >= e.bhi) return;
  const int64_t nb = acc_nblocks(e.count), per = acc_per(e.count, nb);
  const int64_t r0 = b * per;
  const int64_t r1 = (r0 + per < e.count) ? r0 + per : e.count;
  dcor_accum* dst = nb == 1 ? acc + 2 * (int64_t)e.cell : part + 2 * (e.poff + b);
  // the same records, thread assignment and order as k_accumulate's block b on the cell alone
  acc_block_body(rec + e.base + (r0 - e.blo * per), 0, r1 - r0, e.rho, dst, red, redi);
}

// Merge of every multi-block cell's partials after the last pass (cells[] lists them).
__global__ __launch_bounds__(DCOR_BLOCK) void k_accumulate_merge_cells(const AccCell* __restrict__ cells,
                                                                       const dcor_accum* part,
                                                                       dcor_accum* acc) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  const AccCell c = cells[blockIdx.x];
  acc_merge_body(part + 2 * c.poff, acc_nblocks(c.count), c.count, acc + 2 * (int64_t)c.cell, red, redi);
}

// ================================================== single-call helpers ===
__global__ __launch_bounds__(DCOR_BLOCK) void k_mixquant(const double* z, const double* l,
                                                         MixConst mx, double c, double* out) {
  __shared__ SelScratch sel;
  const double q = mixquant_loaded(mx, c, z, l, &sel);
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

// ================================================ R-surface transforms ===
// The elementwise halves of the R wrappers' DGP and DP helpers: the wrapper draws with R's own
// RNG calls (so .Random.seed advances exactly as in the reference) and the GPU does the
// arithmetic, in R's operation order.

// sd(Uc) of ci_INT_subG's clipped products (ver-cor-subG.R:88-99; real-data-sims.R:221-236),
// one workgroup: the HRS wrapper's test of the sd(Uc) == 0 branch (real-data-sims.R:237).
__global__ __launch_bounds__(DCOR_BLOCK) void k_uc_sd(PrematSubgConst p, double* out) {
  __shared__ double red[16 * DCOR_WAVES];
  const SubgConst& c = p.s;
  const double* S = c.sender_is_X ? p.X : p.Y;
  const double* O = c.sender_is_X ? p.Y : p.X;
  DD a[2] = {{0, 0}, {0, 0}};
  for (int64_t i = threadIdx.x; i < c.n; i += DCOR_BLOCK) {
    const double ov = p.hrs ? rclip(O[i], p.lo_) : O[i];
    const double Uc = rclip((rclip(S[i], c.ls) + c.bs * p.lap_local[i]) * ov, c.lr);
    ks_acc(a[0], Uc);
    ks_acc(a[1], Uc * Uc);
  }
  block_sum_dd<2>(a, red);
  if (threadIdx.x == 0) out[0] = sqrt(dd_var(a[0], a[1], c.nd));
}

// standardize_dp (real-data-sims.R:87-90): (pmin(pmax(x, lo), hi) - mean) / max(sd, eps).
__global__ __launch_bounds__(DCOR_BLOCK) void k_standardize_dp(const double* x, int64_t n, double lo,
                                                               double hi, double mean, double den,
                                                               double* out) {
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i < n) out[i] = (rclip_lohi(x[i], lo, hi) - mean) / den;
}

// gen_bernoulli from its uniforms u, v (vert-cor.R:85-97).
__global__ __launch_bounds__(DCOR_BLOCK) void k_gen_bernoulli(const double* u, const double* v,
                                                              int64_t n, double t0, double t1,
                                                              double* X, double* Y) {
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i >= n) return;
  const double x = (u[i] < 0.5) ? 1.0 : 0.0;                           // :88
  X[i] = x;
  Y[i] = (x == 0.0) ? (v[i] < t0 ? 1.0 : 0.0) : (v[i] < t1 ? 1.0 : 0.0);  // :92-96
}

// cbind(U + E1, U + E2) of gen_bounded_factor (ver-cor-subG.R:153).
__global__ __launch_bounds__(DCOR_BLOCK) void k_gen_bounded_factor(const double* U, const double* E1,
                                                                   const double* E2, int64_t n,
                                                                   double* X, double* Y) {
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i >= n) return;
  X[i] = U[i] + E1[i];
  Y[i] = U[i] + E2[i];
}

// MASS::mvrnorm's transform of Z = matrix(rnorm(2n), n) (column 1 = z[0..n), column 2 =
// z[n..2n)): mu + (V diag(sqrt(ev))) %*% t(Z) in dgemm's order, transposed back.  With `perm`
// (gen_mix_gaussian, ver-cor-subG.R:127-135): rows of rbind(mvrnorm(n0), mvrnorm(n1)) taken in
// sample.int(n) order and clipped to [-1, 1]; z1 holds component 1's 2 n1 normals.
__global__ __launch_bounds__(DCOR_BLOCK) void k_mvrnorm_apply(const double* z0, int64_t n0,
                                                              const double* z1, int64_t n1,
                                                              const int32_t* perm, MvnConst m,
                                                              double* X, double* Y) {
  const int64_t n = n0 + n1;
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i >= n) return;
  const int64_t src = perm ? (int64_t)perm[i] : i;
  double xv, yv;
  if (src < n0) {
    const double a = z0[src], b = z0[n0 + src];
    xv = m.mu0[0] + ((0.0 + a * m.A0[0]) + b * m.A0[1]);
    yv = m.mu0[1] + ((0.0 + a * m.A0[2]) + b * m.A0[3]);
  } else {
    const int64_t t = src - n0;
    const double a = z1[t], b = z1[n1 + t];
    xv = m.mu1[0] + ((0.0 + a * m.A1[0]) + b * m.A1[1]);
    yv = m.mu1[1] + ((0.0 + a * m.A1[2]) + b * m.A1[3]);
  }
  if (perm) {   // pmax(pmin(out, 1), -1)
    xv = rclip_lohi(xv, -1.0, 1.0);
    yv = rclip_lohi(yv, -1.0, 1.0);
  }
  X[i] = xv;
  Y[i] = yv;
}

// ============================================================== draws ===
// Pairs b = b0, b0 + bstride, ... of one replicate row: element 2b and 2b + 1 from Philox block
// (b, rep, site).  The row's values do not depend on how the pairs are dealt to lanes.
// 32-bit pair indices: count < 2^31 (the launchers' rows), so the loop and its store offsets need
// no 64-bit arithmetic.
__device__ __forceinline__ void draws_span(int kind, uint32_t k0, uint32_t k1, uint32_t site,
                                           uint32_t rep, int64_t count, double* __restrict__ o,
                                           int64_t b0_, int64_t bstride_) {
  const uint32_t npair = (uint32_t)((count + 1) / 2), bstride = (uint32_t)bstride_;
  const uint32_t cnt = (uint32_t)count;
  for (uint32_t b = (uint32_t)b0_; b < npair; b += bstride) {
    const U4 w = draw(b, rep, site, k0, k1);
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
    o[2u * b] = a;
    if (2u * b + 1u < cnt) o[2u * b + 1u] = c;
  }
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_draws(int kind, uint32_t k0, uint32_t k1,
                                                      uint32_t site, int64_t rep_begin,
                                                      int64_t count, double* out) {
  const int64_t r = blockIdx.y;
  draws_span(kind, k0, k1, site, (uint32_t)(rep_begin + r), count, out + r * count,
             (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x, (int64_t)gridDim.x * DCOR_BLOCK);
}

// ========================================================== permutation ===
// Keyed pseudo-random permutation of [0, n): a 4-round unbalanced Feistel network on exactly
// bits = ceil(log2 n) bits (high part c = bits - a, low part a = bits / 2; the part widths
// alternate each round and return after four), cycle-walked into [0, n) -- at least half the
// domain is accepted, so a wave rarely walks long.  Round functions use only full-rate 24-bit
// multiplies.  out[r][t] = P_r(t), t < count, is a random ordered subset of size `count`: the
// role of sample.int(n, k*m) (real-data-sims.R:131) for the HRS random batches.  Round keys:
// Philox block (0, rep, site, 0).  Restated in oracle/ (orc_perm) for bit-exact tests.
__device__ __forceinline__ uint32_t feistel_f(uint32_t r, uint32_t k, uint32_t mask) {
  uint32_t t = __umul24((r ^ k) & 0xFFFFFFu, 0x9E3779u);
  t ^= t >> 15;
  t = __umul24(t & 0xFFFFFFu, 0x85EBCBu);
  t ^= t >> 13;
  return t & mask;
}

// One pass of the four rounds on (c + a)-bit x.
__device__ __forceinline__ uint32_t feistel_pass(uint32_t x, int a, int c, const U4& kk) {
  const uint32_t ma = (1u << a) - 1u, mc = (1u << c) - 1u;
  uint32_t H = x >> a, L = x & ma;              // (c bits, a bits)
  uint32_t t;
  t = H ^ feistel_f(L, kk.w0, mc); H = L; L = t;  // (a, c)
  t = H ^ feistel_f(L, kk.w1, ma); H = L; L = t;  // (c, a)
  t = H ^ feistel_f(L, kk.w2, mc); H = L; L = t;  // (a, c)
  t = H ^ feistel_f(L, kk.w3, ma); H = L; L = t;  // (c, a)
  return (H << a) | L;
}

// P_r(t) = the first of pass(t), pass(pass(t)), ... inside [0, n).  Each lane owns the strided
// sequence t, t + stride, ... and applies one pass per loop trip, moving to its next t as soon
// as the current one lands: lanes stay busy while their walks differ in length (a loop per t
// would run every lane of a wave to the longest of its 64 walks, ~3.4x the mean for n just
// above a power of two).  The launcher gives every lane about 16 values of t.
__device__ __forceinline__ void perm_span(uint32_t k0, uint32_t k1, uint32_t site, uint32_t rep,
                                          uint32_t n, int a, int c, int64_t count,
                                          int32_t* __restrict__ o, uint32_t t, uint32_t stride) {
  const U4 kk = draw(0u, rep, site, k0, k1);
  const uint32_t cnt = (uint32_t)count;  // count <= n < 2^31
  uint32_t x = t;
  while (t < cnt) {
    x = feistel_pass(x, a, c, kk);
    if (x < n) {
      o[t] = (int32_t)x;
      t += stride;
      x = t;
    }
  }
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_perm(uint32_t k0, uint32_t k1, uint32_t site,
                                                     int64_t rep_begin, uint32_t n, int a, int c,
                                                     int64_t count, int32_t* out) {
  const int64_t r = blockIdx.y;
  perm_span(k0, k1, site, (uint32_t)(rep_begin + r), n, a, c, count, out + r * count,
            blockIdx.x * DCOR_BLOCK + threadIdx.x, gridDim.x * DCOR_BLOCK);
}

// All seven noise arrays of an HRS launch (HrsNoise) in one grid: blockIdx.y is the replicate,
// blockIdx.x ranges [g[i], g[i+1]) are the permutation row (i = 0) and the six draw rows, each
// dealt exactly as its own launch would deal it (perm_span / draws_span), so every element equals
// the separate launches' bit for bit.  One launch instead of seven: the HRS sweep's small
// per-eps launches are launch-latency bound.
struct HrsNoiseArgs {
  HrsNoise j;
  uint32_t g[8];
  int pa, pc;
};
__global__ __launch_bounds__(DCOR_BLOCK) void k_hrs_noise(HrsNoiseArgs q) {
  const int64_t r = blockIdx.y;
  const uint32_t rep = (uint32_t)(q.j.rep_begin + r);
  const uint32_t bx = blockIdx.x, tid = threadIdx.x;
  const uint32_t n0 = (uint32_t)q.j.seed_ni, n1 = (uint32_t)(q.j.seed_ni >> 32);
  const uint32_t i0 = (uint32_t)q.j.seed_int, i1 = (uint32_t)(q.j.seed_int >> 32);
  int part = 0;
#pragma unroll
  for (int i = 1; i < 7; ++i) part += bx >= q.g[i] ? 1 : 0;
  const uint32_t lo = q.g[part], span = q.g[part + 1] - lo;
  const int64_t b0 = (int64_t)(bx - lo) * DCOR_BLOCK + tid, bs = (int64_t)span * DCOR_BLOCK;
  const int64_t k = q.j.k, n = q.j.n, ns = q.j.nsim;
  switch (part) {
    case 0: perm_span(n0, n1, DCOR_SITE_PERM, rep, (uint32_t)n, q.pa, q.pc, q.j.km,
                      q.j.perm + r * q.j.km, (uint32_t)b0, (uint32_t)bs); break;
    case 1: draws_span(0, n0, n1, 11u, rep, k, q.j.lap_x + r * k, b0, bs); break;
    case 2: draws_span(0, n0, n1, 12u, rep, k, q.j.lap_y + r * k, b0, bs); break;
    case 3: draws_span(0, i0, i1, 13u, rep, n, q.j.lap_local + r * n, b0, bs); break;
    case 4: draws_span(0, i0, i1, 14u, rep, 1, q.j.lap_central + r, b0, bs); break;
    case 5: draws_span(1, i0, i1, 15u, rep, ns, q.j.mix_z + r * ns, b0, bs); break;
    default: draws_span(0, i0, i1, 16u, rep, ns, q.j.mix_l + r * ns, b0, bs); break;
  }
}

// ========================================================= fused HRS ===
// The HRS replicate of k_premat_subg_dict with its noise drawn in the kernel instead of read
// from HBM: the same Philox streams the HRS driver materialises (dcor_perm_launch with
// seed_ni, DCOR_SITE_PERM; dcor_draws_launch Laplace seed_ni sites 11 / 12 for the NI
// batches, seed_int sites 13 / 14 for the INT local / central noise, normal site 15 and
// Laplace site 16 for mixquant), so every replicate equals the pre-materialised pipeline's
// bit for bit.  real-data-sims.R:115-147 (NI) and 176-252 (INT) per replicate.
struct HrsKeys {
  uint32_t ni0, ni1, in0, in1;  // Philox keys (seed_ni, seed_int)
  uint32_t rep_begin;
  int pa, pc;                   // Feistel split of ceil(log2 n) bits (launch_perm)
};
#define HRS_SITE_NI_X 11u
#define HRS_SITE_NI_Y 12u
#define HRS_SITE_LOCAL 13u
#define HRS_SITE_CENTRAL 14u
#define HRS_SITE_MIX_Z 15u
#define HRS_SITE_MIX_L 16u

template <int WPE>
__global__ __launch_bounds__(DICT_NT, WPE) void k_hrs_fused(PrematSubgConst p, HrsKeys hk,
                                                           const uint16_t* __restrict__ codes_g,
                                                           const double* __restrict__ dict_g,
                                                           int64_t reps,
                                                           SubgPartial* __restrict__ part,
                                                           uint16_t* __restrict__ scr,
                                                           int64_t scr_stride) {
  extern __shared__ double dsm[];
  const SubgConst& c = p.s;
  const int tid = threadIdx.x;
  double* dX = dsm;
  double* dY = dsm + DICT_MAX;
  double* dS = dsm + 2 * DICT_MAX;
  double* dO = dsm + 3 * DICT_MAX;
  double* red = dsm + 4 * DICT_MAX;
  uint16_t* cod = reinterpret_cast<uint16_t*>(dsm + 4 * DICT_MAX + 20 * DICT_NW);
  if (tid < DICT_MAX) {
    const double x = dict_g[tid], y = dict_g[DICT_MAX + tid];
    dX[tid] = rclip(x, c.l1);
    dY[tid] = rclip(y, c.l2);
    const double sv = c.sender_is_X ? x : y, ov = c.sender_is_X ? y : x;
    dS[tid] = rclip(sv, c.ls);
    dO[tid] = rclip(ov, p.lo_);
  }
  {
    const int64_t nv = (c.n * 2 + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(codes_g);
    uint4* dst = reinterpret_cast<uint4*>(cod);
    for (int64_t w = tid; w < nv; w += DICT_NT) dst[w] = src[w];
  }
  __syncthreads();
  const uint32_t n = (uint32_t)c.n;
  for (int64_t it = blockIdx.x; it < reps; it += gridDim.x) {
    const uint32_t rep = hk.rep_begin + (uint32_t)it;
    DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
    auto uval = [&](uint32_t cd, double l) {  // real-data-sims.R:222-232
      // finite dictionary (k_panel_dict) and noise: the product is never NaN
      return rclip_fin((dS[cd & 255u] + c.bs * l) * dO[cd >> 8], c.lr);
    };
    auto uterm = [&](double Uc) {
      ks_acc(sU, Uc);
      ks_acc(sU2, Uc * Uc);
    };
    // a pair of INT terms (of NI batches) is added plainly and the pair sum compensated: half
    // the TwoSum chains of per-term sums
    auto uterm2 = [&](double U0, double U1) {
      ks_acc(sU, U0 + U1);
      ks_acc(sU2, U0 * U0 + U1 * U1);
    };
    // Phase A: the panel codes at the permuted batch slots, gs[t] = code[P(t)], t < k m, into
    // this workgroup's scratch row (L2-resident, reused by every replicate of the workgroup).
    // Each lane walks its strided run of t and moves to the next t as soon as a walk lands,
    // so lanes stay busy while walk lengths differ.  Phase B reads the row after a barrier.
    const U4 kk = draw(0u, rep, DCOR_SITE_PERM, hk.ni0, hk.ni1);
    uint16_t* __restrict__ gs = scr + (int64_t)blockIdx.x * scr_stride;
    {
      const uint32_t km = (uint32_t)(c.k * c.m);
      uint32_t t = (uint32_t)tid, x = t;
      while (t < km) {
        x = feistel_pass(x, hk.pa, hk.pc, kk);
        if (x < n) {
          gs[t] = cod[x];
          t += DICT_NT;
          x = t;
        }
      }
    }
    {  // INT local noise: block b -> samples 2b, 2b+1
      const int64_t nb = c.n >> 1;
      for (int64_t b = tid; b < nb; b += DICT_NT) {
        const U4 w = draw((uint32_t)b, rep, HRS_SITE_LOCAL, hk.in0, hk.in1);
        uterm2(uval(cod[2 * b], unit_laplace(u53(w.w0, w.w1))),
               uval(cod[2 * b + 1], unit_laplace(u53(w.w2, w.w3))));
      }
      if ((c.n & 1) && tid == DICT_NT - 1) {
        const U4 w = draw((uint32_t)nb, rep, HRS_SITE_LOCAL, hk.in0, hk.in1);
        uterm(uval(cod[c.n - 1], unit_laplace(u53(w.w0, w.w1))));
      }
    }
    double* rb = red + (((it - blockIdx.x) / gridDim.x) & 1) * (10 * DICT_NW);
    auto wave_put = [&](int v, DD a) {
      a = wave_sum_dd(a);
      if ((tid & 63) == 0) {
        rb[(2 * v) * DICT_NW + (tid >> 6)] = a.hi;
        rb[(2 * v + 1) * DICT_NW + (tid >> 6)] = a.lo;
      }
    };
    wave_put(3, sU);
    wave_put(4, sU2);
    __syncthreads();  // phase A's scratch row is complete
    auto nterm = [&](double xt, double yt) {  // real-data-sims.R:133-137
      ks_acc(sP, xt * yt);
      const double T = c.md * xt * yt;
      ks_acc(sT, T);
      ks_acc(sT2, T * T);
    };
    auto nterm2 = [&](double xt0, double yt0, double xt1, double yt1) {
      const double T0 = c.md * xt0 * yt0, T1 = c.md * xt1 * yt1;
      ks_acc(sP, xt0 * yt0 + xt1 * yt1);
      ks_acc(sT, T0 + T1);
      ks_acc(sT2, T0 * T0 + T1 * T1);
    };
    if (c.m == 2) {  // batches 2q, 2q+1 share one Philox block of X noise and one of Y noise
      const uint32_t* __restrict__ g2 = reinterpret_cast<const uint32_t*>(gs);  // batch j's codes
      auto xt_of = [&](uint32_t ab, double lxj) {
        return (dX[(ab & 0xFFFFu) & 255u] + dX[(ab >> 16) & 255u]) * 0.5 + c.bx * lxj;
      };
      auto yt_of = [&](uint32_t ab, double lyj) {
        return (dY[(ab & 0xFFFFu) >> 8] + dY[(ab >> 16) >> 8]) * 0.5 + c.by * lyj;
      };
      for (int64_t q = tid; 2 * q < c.k; q += DICT_NT) {
        const U4 wx = draw((uint32_t)q, rep, HRS_SITE_NI_X, hk.ni0, hk.ni1);
        const U4 wy = draw((uint32_t)q, rep, HRS_SITE_NI_Y, hk.ni0, hk.ni1);
        const uint32_t ab0 = g2[2 * q];
        const double xt0 = xt_of(ab0, unit_laplace(u53(wx.w0, wx.w1)));
        const double yt0 = yt_of(ab0, unit_laplace(u53(wy.w0, wy.w1)));
        if (2 * q + 1 < c.k) {
          const uint32_t ab1 = g2[2 * q + 1];
          nterm2(xt0, yt0, xt_of(ab1, unit_laplace(u53(wx.w2, wx.w3))),
                 yt_of(ab1, unit_laplace(u53(wy.w2, wy.w3))));
        } else {
          nterm(xt0, yt0);
        }
      }
    } else {
      for (int64_t j = tid; j < c.k; j += DICT_NT) {
        const U4 wx = draw((uint32_t)(j >> 1), rep, HRS_SITE_NI_X, hk.ni0, hk.ni1);
        const U4 wy = draw((uint32_t)(j >> 1), rep, HRS_SITE_NI_Y, hk.ni0, hk.ni1);
        const double lxj = unit_laplace((j & 1) ? u53(wx.w2, wx.w3) : u53(wx.w0, wx.w1));
        const double lyj = unit_laplace((j & 1) ? u53(wy.w2, wy.w3) : u53(wy.w0, wy.w1));
        DD bx{0, 0}, by{0, 0};
        for (int r = 0; r < c.m; ++r) {
          const uint32_t a = gs[j * c.m + r];
          dd_acc(bx, dX[a & 255u]);
          dd_acc(by, dY[a >> 8]);
        }
        const DD xb = dd_div_d(bx, c.md), yb = dd_div_d(by, c.md);
        nterm((xb.hi + xb.lo) + c.bx * lxj, (yb.hi + yb.lo) + c.by * lyj);
      }
    }
    wave_put(0, sP);
    wave_put(1, sT);
    wave_put(2, sT2);
    __syncthreads();
    if (tid < 5) {
      const DD a = fold_waves_dd<DICT_NW>(rb + (2 * tid) * DICT_NW, rb + (2 * tid + 1) * DICT_NW);
      part[it].s[2 * tid] = a.hi;
      part[it].s[2 * tid + 1] = a.lo;
    }
  }
}

// k_hrs_fused for a panel that is not dictionary-codable (continuous values): the same
// replicate, work split and summation order, with the clipped panel packed once per launch in
// HBM (xyc = NI clips, soc = INT sender / other clips, k_premat_xy_pack; 32 B per sample, L2-
// resident at survey sizes) instead of LDS codes.  LDS holds this replicate's permuted batch
// indices (u16, n <= 65536), written by phase A's Feistel walks; phase B gathers the two
// samples of each batch from L2.  The clipped values are the coded kernel's dictionary entries,
// so on a codable panel both kernels return the same bits.
template <int WPE>
__global__ __launch_bounds__(DICT_NT, WPE) void k_hrs_fused_l2(PrematSubgConst p, HrsKeys hk,
                                                              int64_t reps,
                                                              SubgPartial* __restrict__ part) {
  extern __shared__ double dsm[];
  const SubgConst& c = p.s;
  const int tid = threadIdx.x;
  double* red = dsm;
  uint16_t* gs = reinterpret_cast<uint16_t*>(dsm + 20 * DICT_NW);
  const double2* __restrict__ xy = p.xyc;
  const double2* __restrict__ so = p.soc;
  const uint32_t n = (uint32_t)c.n;
  for (int64_t it = blockIdx.x; it < reps; it += gridDim.x) {
    const uint32_t rep = hk.rep_begin + (uint32_t)it;
    DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
    auto uval = [&](double2 v, double l) {  // real-data-sims.R:222-232
      return rclip((v.x + c.bs * l) * v.y, c.lr);
    };
    auto uterm = [&](double Uc) {
      ks_acc(sU, Uc);
      ks_acc(sU2, Uc * Uc);
    };
    auto uterm2 = [&](double U0, double U1) {  // as k_hrs_fused: pair sums compensated
      ks_acc(sU, U0 + U1);
      ks_acc(sU2, U0 * U0 + U1 * U1);
    };
    // Phase A: gs[t] = P(t), t < k m (sample.int(n, k*m) - 1, real-data-sims.R:131); the
    // previous item's readers are past the barrier that ends its reduction.
    const U4 kk = draw(0u, rep, DCOR_SITE_PERM, hk.ni0, hk.ni1);
    {
      const uint32_t km = (uint32_t)(c.k * c.m);
      uint32_t t = (uint32_t)tid, x = t;
      while (t < km) {
        x = feistel_pass(x, hk.pa, hk.pc, kk);
        if (x < n) {
          gs[t] = (uint16_t)x;
          t += DICT_NT;
          x = t;
        }
      }
    }
    {  // INT local noise: block b -> samples 2b, 2b+1
      const int64_t nb = c.n >> 1;
      for (int64_t b = tid; b < nb; b += DICT_NT) {
        const U4 w = draw((uint32_t)b, rep, HRS_SITE_LOCAL, hk.in0, hk.in1);
        const double2 v0 = so[2 * b], v1 = so[2 * b + 1];
        uterm2(uval(v0, unit_laplace(u53(w.w0, w.w1))), uval(v1, unit_laplace(u53(w.w2, w.w3))));
      }
      if ((c.n & 1) && tid == DICT_NT - 1) {
        const U4 w = draw((uint32_t)nb, rep, HRS_SITE_LOCAL, hk.in0, hk.in1);
        uterm(uval(so[c.n - 1], unit_laplace(u53(w.w0, w.w1))));
      }
    }
    double* rb = red + (((it - blockIdx.x) / gridDim.x) & 1) * (10 * DICT_NW);
    auto wave_put = [&](int v, DD a) {
      a = wave_sum_dd(a);
      if ((tid & 63) == 0) {
        rb[(2 * v) * DICT_NW + (tid >> 6)] = a.hi;
        rb[(2 * v + 1) * DICT_NW + (tid >> 6)] = a.lo;
      }
    };
    wave_put(3, sU);
    wave_put(4, sU2);
    __syncthreads();  // phase A's index row is complete
    auto nterm = [&](double xt, double yt) {  // real-data-sims.R:133-137
      ks_acc(sP, xt * yt);
      const double T = c.md * xt * yt;
      ks_acc(sT, T);
      ks_acc(sT2, T * T);
    };
    auto nterm2 = [&](double xt0, double yt0, double xt1, double yt1) {
      const double T0 = c.md * xt0 * yt0, T1 = c.md * xt1 * yt1;
      ks_acc(sP, xt0 * yt0 + xt1 * yt1);
      ks_acc(sT, T0 + T1);
      ks_acc(sT2, T0 * T0 + T1 * T1);
    };
    if (c.m == 2) {
      const uint32_t* __restrict__ g2 = reinterpret_cast<const uint32_t*>(gs);
      for (int64_t q = tid; 2 * q < c.k; q += DICT_NT) {
        const uint32_t ab0 = g2[2 * q];
        const uint32_t ab1 = 2 * q + 1 < c.k ? g2[2 * q + 1] : 0u;
        const U4 wx = draw((uint32_t)q, rep, HRS_SITE_NI_X, hk.ni0, hk.ni1);
        const U4 wy = draw((uint32_t)q, rep, HRS_SITE_NI_Y, hk.ni0, hk.ni1);
        const double2 a0 = xy[ab0 & 0xFFFFu], b0 = xy[ab0 >> 16];
        const double xt0 = (a0.x + b0.x) * 0.5 + c.bx * unit_laplace(u53(wx.w0, wx.w1));
        const double yt0 = (a0.y + b0.y) * 0.5 + c.by * unit_laplace(u53(wy.w0, wy.w1));
        if (2 * q + 1 < c.k) {
          const double2 a1 = xy[ab1 & 0xFFFFu], b1 = xy[ab1 >> 16];
          nterm2(xt0, yt0, (a1.x + b1.x) * 0.5 + c.bx * unit_laplace(u53(wx.w2, wx.w3)),
                 (a1.y + b1.y) * 0.5 + c.by * unit_laplace(u53(wy.w2, wy.w3)));
        } else {
          nterm(xt0, yt0);
        }
      }
    } else {
      for (int64_t j = tid; j < c.k; j += DICT_NT) {
        const U4 wx = draw((uint32_t)(j >> 1), rep, HRS_SITE_NI_X, hk.ni0, hk.ni1);
        const U4 wy = draw((uint32_t)(j >> 1), rep, HRS_SITE_NI_Y, hk.ni0, hk.ni1);
        const double lxj = unit_laplace((j & 1) ? u53(wx.w2, wx.w3) : u53(wx.w0, wx.w1));
        const double lyj = unit_laplace((j & 1) ? u53(wy.w2, wy.w3) : u53(wy.w0, wy.w1));
        DD bx{0, 0}, by{0, 0};
        for (int r = 0; r < c.m; ++r) {
          const double2 v = xy[gs[j * c.m + r]];
          dd_acc(bx, v.x);
          dd_acc(by, v.y);
        }
        const DD xb = dd_div_d(bx, c.md), yb = dd_div_d(by, c.md);
        nterm((xb.hi + xb.lo) + c.bx * lxj, (yb.hi + yb.lo) + c.by * lyj);
      }
    }
    wave_put(0, sP);
    wave_put(1, sT);
    wave_put(2, sT2);
    __syncthreads();
    if (tid < 5) {
      const DD a = fold_waves_dd<DICT_NW>(rb + (2 * tid) * DICT_NW, rb + (2 * tid + 1) * DICT_NW);
      part[it].s[2 * tid] = a.hi;
      part[it].s[2 * tid + 1] = a.lo;
    }
  }
}

// Epilogue of k_hrs_fused: central Laplace and mixquant draws generated here.  Thread t holds
// the pairs of Philox blocks t + 256 s (order is irrelevant to an order statistic).
__global__ __launch_bounds__(DCOR_BLOCK) void k_hrs_fused_epilogue(PrematSubgConst p, HrsKeys hk,
                                                                   const SubgPartial* __restrict__ part,
                                                                   dcor_rep_out* out) {
  __shared__ SelScratch sel;
  const int64_t r = blockIdx.x;
  const uint32_t rep = hk.rep_begin + (uint32_t)r;
  const MixConst& mx = p.s.mix;
  double zv[SEL_VPT], lv[SEL_VPT];
  bool have[SEL_VPT];
#pragma unroll
  for (int s = 0; s < SEL_VPT / 2; ++s) {
    const int b = threadIdx.x + s * DCOR_BLOCK;
    have[2 * s] = 2 * b < mx.nsim;
    have[2 * s + 1] = 2 * b + 1 < mx.nsim;
    zv[2 * s] = zv[2 * s + 1] = lv[2 * s] = lv[2 * s + 1] = 0.0;
    if (have[2 * s]) {
      const U4 wz = draw((uint32_t)b, rep, HRS_SITE_MIX_Z, hk.in0, hk.in1);
      const U4 wl = draw((uint32_t)b, rep, HRS_SITE_MIX_L, hk.in0, hk.in1);
      normal_pair(wz, &zv[2 * s], &zv[2 * s + 1]);
      lv[2 * s] = unit_laplace(u53(wl.w0, wl.w1));
      lv[2 * s + 1] = unit_laplace(u53(wl.w2, wl.w3));
    }
  }
  // the scalar half in wave 0 only (as k_premat_subg_epilogue); c* reaches the others through LDS
  __shared__ double bc[2];
  SubgPre pre{};
  if (threadIdx.x < 64) {
    const U4 wc = draw(0u, rep, HRS_SITE_CENTRAL, hk.in0, hk.in1);
    DD d5[5];
    load_partials(p, part, r, d5);
    pre = premat_subg_pre(p, d5, unit_laplace(u53(wc.w0, wc.w1)));
    if (threadIdx.x == 0) { bc[0] = pre.cstar; bc[1] = pre.quant ? 1.0 : 0.0; sel.nan_cnt = 0; }
  }
  __syncthreads();
  double qq = 0.0;
  if (bc[1] != 0.0) {
    const double cs = bc[0];
    double val[SEL_VPT];
    int nn = 0;
#pragma unroll
    for (int s = 0; s < SEL_VPT; ++s) {
      val[s] = dnan();
      if (have[s]) {
        val[s] = zv[s] + cs * lv[s];
        nn += (val[s] != val[s]);
      }
    }
    if (nn) atomicAdd(&sel.nan_cnt, nn);
    __syncthreads();
    qq = value_select(val, mx.pos, mx.nsim - sel.nan_cnt, &sel);
  }
  if (threadIdx.x == 0) out[r] = premat_subg_post(p, pre, qq);
}

int launch_hrs_fused(const PrematSubgConst& c, uint64_t seed_ni, uint64_t seed_int,
                     int64_t rep_begin, int64_t reps, void* part, dcor_rep_out* out,
                     void* stream) {
  if (reps <= 0) return 0;
  HrsKeys hk;
  hk.ni0 = (uint32_t)seed_ni; hk.ni1 = (uint32_t)(seed_ni >> 32);
  hk.in0 = (uint32_t)seed_int; hk.in1 = (uint32_t)(seed_int >> 32);
  hk.rep_begin = (uint32_t)rep_begin;
  int bits = 1;
  while ((1ll << bits) < c.s.n) ++bits;
  hk.pa = bits / 2; hk.pc = bits - hk.pa;
  const int wsel = [] {
    const char* e = dcor::variant("DCOR_HRS_WPE");
    return (e && std::atoi(e) == 4) ? 4 : 6;
  }();
  const bool l2 = c.xyc != nullptr;  // uncoded panel: packed clips in HBM, indices in LDS
  const size_t lds = l2 ? (size_t)(20 * DICT_NW) * sizeof(double) +
                              (size_t)((c.s.k * c.s.m * 2 + 15) / 16) * 16
                        : premat_dict_lds_bytes(c.s.n);
  if (l2)
    hipLaunchKernelGGL(k_premat_xy_pack, dim3((unsigned)((c.s.n + DCOR_BLOCK - 1) / DCOR_BLOCK)),
                       dim3(DCOR_BLOCK), 0, (hipStream_t)stream, c, (double2*)c.xyc,
                       (double2*)c.soc);
  typedef void (*FusedK)(PrematSubgConst, HrsKeys, const uint16_t*, const double*, int64_t,
                         SubgPartial*, uint16_t*, int64_t);
  typedef void (*FusedL2K)(PrematSubgConst, HrsKeys, int64_t, SubgPartial*);
  const FusedK kern = wsel == 4 ? k_hrs_fused<4> : k_hrs_fused<6>;
  const FusedL2K kern_l2 = wsel == 4 ? k_hrs_fused_l2<4> : k_hrs_fused_l2<6>;
  const void* kf = l2 ? (const void*)kern_l2 : (const void*)kern;
  // per call: the attribute is per device, and one process may drive several GPUs
  if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) != hipSuccess)
    return (int)hipGetLastError();
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (int)hipGetLastError();
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return (int)hipGetLastError();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, DICT_NT, lds) != hipSuccess)
    return (int)hipGetLastError();
  const int64_t slots = (int64_t)cus * (per_cu < 1 ? 1 : per_cu);
  const int64_t grid = reps < slots ? reps : slots;
  if (l2) {
    hipLaunchKernelGGL(kern_l2, dim3((unsigned)grid), dim3(DICT_NT), lds, (hipStream_t)stream, c,
                       hk, reps, (SubgPartial*)part);
    hipLaunchKernelGGL(k_hrs_fused_epilogue, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                       (hipStream_t)stream, c, hk, (const SubgPartial*)part, out);
    return (int)hipGetLastError();
  }
  const int64_t stride = (c.s.k * c.s.m + 63) & ~(int64_t)63;  // u16 codes per scratch row
  void* scr = nullptr;
  if (hipMallocAsync(&scr, (size_t)(grid * stride * 2), (hipStream_t)stream) != hipSuccess)
    return (int)hipGetLastError();
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(DICT_NT), lds,
                     (hipStream_t)stream, c, hk, c.dict_codes, c.dict_vals, reps,
                     (SubgPartial*)part, (uint16_t*)scr, stride);
  (void)hipFreeAsync(scr, (hipStream_t)stream);
  hipLaunchKernelGGL(k_hrs_fused_epilogue, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, hk, (const SubgPartial*)part, out);
  return (int)hipGetLastError();
}

// ============================================================ launchers ===
static inline int last_err() { return (int)hipGetLastError(); }

int launch_premat_sign(const PrematSignConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  hipLaunchKernelGGL(k_premat_sign, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}
int launch_panel_dict(const double* X, const double* Y, int64_t n, uint16_t* codes, double* dict,
                      int* ok, void* stream) {
  hipLaunchKernelGGL(k_panel_dict, dim3(1), dim3(DICT_THREADS), 0, (hipStream_t)stream, X, Y, n,
                     codes, dict, ok);
  return last_err();
}

size_t premat_dict_lds_bytes(int64_t n) {
  return (size_t)(4 * DICT_MAX + 20 * DICT_NW) * sizeof(double) + (size_t)((n * 2 + 15) / 16) * 16;
}

typedef void (*DictKernel)(PrematSubgConst, const uint16_t*, const double*, const int*, int64_t,
                           SubgPartial*);
// Coded-panel kernel variant: (16-B loads in flight per thread, waves per SIMD).  The kernel
// reads at ~5.8 TB/s in every variant (r01 A/B: 590-605 us per 8192 replicates); the default
// keeps two 512-thread workgroups per CU.  DCOR_DICT_VARIANT=1..3 selects the others for A/B.
static DictKernel dict_kernel() {
  static const DictKernel ks[4] = {k_premat_subg_dict<4, 4, false>, k_premat_subg_dict<4, 6, false>,
                                   k_premat_subg_dict<8, 4, false>, k_premat_subg_dict<6, 6, false>};
  const int v = [] {
    const char* e = dcor::variant("DCOR_DICT_VARIANT");
    const int x = e ? std::atoi(e) : 0;
    return (x >= 0 && x < 4) ? x : 0;
  }();
  return ks[v];
}

// Uncoded shared-panel kernel variant (16-B loads in flight per thread, waves per SIMD);
// DCOR_L2_VARIANT=1..3 selects the others for A/B.
static DictKernel l2_kernel() {
  static const DictKernel ks[4] = {k_premat_subg_dict<4, 8, true>, k_premat_subg_dict<4, 4, true>,
                                   k_premat_subg_dict<8, 8, true>, k_premat_subg_dict<8, 4, true>};
  const int v = [] {
    const char* e = dcor::variant("DCOR_L2_VARIANT");
    const int x = e ? std::atoi(e) : 0;
    return (x >= 0 && x < 4) ? x : 0;
  }();
  return ks[v];
}

// Tiled uncoded-panel kernel variants (threads, batch pairs per thread per round, fill unroll,
// gather group, accumulator sets, waves per SIMD, pair-grouped sums, INT sums in the kernel) and
// the LDS each workgroup may give its tile.  C5-continuous, 8192 replicates per launch (call incl.
// the epilogue; round 4, one box):
//   in-kernel INT sums, two 512-thread workgroups per CU, four 80-KB tiles   1.05 ms (0.39 of 8 TB/s)
//   INT sums in k_premat_subg_int (serial), same tiled kernel               0.87 ms (0.47)
//   INT sums in k_premat_subg_int, one 1024-thread workgroup per CU with
//     two 156-KB tiles and one round of batch pairs (default)               0.82 ms (0.50)
// Without the INT stream the tiled kernel needs 116 VGPRs instead of 128 (and no spills), and its
// tile fills read the L2-resident panel only.  The 512-thread variant's sums are the L2-gather
// kernel's bit for bit in every INT mode; the 1024-thread variant splits the batch pairs over
// 1024 threads, so its NI sums differ from those in the low bits.  Measured and dropped: one
// 512-thread workgroup per CU with ten batch pairs per thread (one round; 200 VGPRs, 0.38-0.40),
// L2 warm-up loads of the noise phase during the last tile (0.39), barriers that wait for LDS
// traffic only (no change), a wider fill unroll (no change), the INT kernel on the auxiliary
// stream beside the tiled kernel (DCOR_TILED_INT=2: the two share the CUs' issue and memory
// pipelines, 0.47).  DCOR_TILED_VARIANT=0 selects the 512-thread variant; DCOR_TILED=0 the
// L2-gather kernel.
struct TiledKernel {
  void (*k)(PrematSubgConst, const int*, int64_t, int64_t, SubgPartial*);
  int nt;
  size_t lds_budget;
};
// Where the tiled path's INT sums run (DCOR_TILED_INT): 0 inside the tiled kernel's first round of
// tile fills; 1 (default) in k_premat_subg_int before it on the same stream; 2 in
// k_premat_subg_int on the library's auxiliary stream beside it.
static int tiled_int_mode() {
  const int m = [] {
    const char* e = dcor::variant("DCOR_TILED_INT");
    const int x = e ? std::atoi(e) : 1;
    return (x >= 0 && x <= 2) ? x : 1;
  }();
  return m;
}
#ifndef DCOR_INT_R
#define DCOR_INT_R 4
#endif
static TiledKernel tiled_kernel(bool intk, bool al) {
  static const TiledKernel ks[2][2][2] = {
      {{{k_premat_subg_tiled<512, 5, 1, 1, 1, 4, true, true, false>, 512, 80 * 1024},
        {k_premat_subg_tiled<512, 5, 1, 1, 1, 4, true, true, true>, 512, 80 * 1024}},
       {{k_premat_subg_tiled<512, 5, 1, 1, 1, 4, true, false, false>, 512, 80 * 1024},
        {k_premat_subg_tiled<512, 5, 1, 1, 1, 4, true, false, true>, 512, 80 * 1024}}},
      {{{k_premat_subg_tiled<1024, 5, 1, 1, 1, 4, true, true, false>, 1024, 160 * 1024},
        {k_premat_subg_tiled<1024, 5, 1, 1, 1, 4, true, true, true>, 1024, 160 * 1024}},
       {{k_premat_subg_tiled<1024, 5, 1, 1, 1, 4, true, false, false, 3>, 1024, 160 * 1024},
        {k_premat_subg_tiled<1024, 5, 1, 1, 1, 4, true, false, true, 3>, 1024, 160 * 1024}}}};
  const int v = [] {
    const char* e = dcor::variant("DCOR_TILED_VARIANT");
    const int x = e ? std::atoi(e) : 1;
    return (x >= 0 && x < 2) ? x : 1;
  }();
  return ks[v][intk ? 0 : 1][al ? 1 : 0];
}
static bool tiled_enabled() {
  const bool on = [] {
    const char* e = dcor::variant("DCOR_TILED");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// Workgroup slots of the coded-panel kernel (CUs x resident workgroups at this LDS size).
static int premat_dict_slots(int64_t n, int* slots) {
  const size_t lds = premat_dict_lds_bytes(n);
  // per call: the attribute is per device, and one process may drive several GPUs
  if (hipFuncSetAttribute((const void*)dict_kernel(), hipFuncAttributeMaxDynamicSharedMemorySize,
                          150 * 1024) != hipSuccess)
    return last_err();
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return last_err();
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return last_err();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dict_kernel(), DICT_NT, lds) !=
      hipSuccess)
    return last_err();
  *slots = cus * (per_cu < 1 ? 1 : per_cu);
  return 0;
}

int launch_premat_subg(const PrematSubgConst& c0, int64_t reps, void* part, dcor_rep_out* out,
                       void* stream, void* epi_stream, void* ev, void* int_stream, void* ev_fork,
                       void* ev_join) {
  if (reps <= 0) return 0;
  PrematSubgConst c = c0;
  c.slices = 1;
  if (c.dict_codes != nullptr) {
    static_assert(DICT_NT >= DICT_MAX, "dictionary fill assumes one entry per thread");
    if (!c.dict_built)
      hipLaunchKernelGGL(k_panel_dict, dim3(1), dim3(DICT_THREADS), 0, (hipStream_t)stream, c.X,
                         c.Y, c.s.n, c.dict_codes, c.dict_vals, c.dict_ok);
    int slots = 0;
    if (int e = premat_dict_slots(c.s.n, &slots)) return e;
    // a prepared coded panel: no L2-gather kernel shares the partials, so replicates are
    // sliced.  The slice count is fixed (not sized to the launch), so a replicate's sums do
    // not depend on how replicates are split over launches or GPUs.
    if (c.dict_built == 2) c.slices = DCOR_DICT_SLICES;
    const int64_t items = reps * c.slices;
    const int64_t grid = items < (int64_t)slots ? items : (int64_t)slots;
    hipLaunchKernelGGL(dict_kernel(), dim3((unsigned)grid), dim3(DICT_NT),
                       premat_dict_lds_bytes(c.s.n), (hipStream_t)stream, c, c.dict_codes,
                       c.dict_vals, c.dict_ok, reps, (SubgPartial*)part);
  }
  if (c.xyc != nullptr) {
    // shared panel, random batches, no dictionary (or the device probe may find none): the
    // clipped panel packed once, then for m = 2 (k even) and u16 sample indices the tiled kernel,
    // otherwise the persistent kernel gathering it from L2.  The choice depends on the geometry
    // only, never on the caller's buffer alignment (the tiled kernel reads unaligned rows element
    // by element), so a replicate's bits do not either.
    const bool tiled = c.dict_built != 2 && tiled_enabled() && c.s.m == 2 && (c.s.k & 1) == 0 &&
                       c.s.k >= 2 && c.s.n < 65536;
    hipLaunchKernelGGL(k_premat_xy_pack, dim3((unsigned)((c.s.n + DCOR_BLOCK - 1) / DCOR_BLOCK)),
                       dim3(DCOR_BLOCK), 0, (hipStream_t)stream, c, (double2*)c.xyc,
                       (double2*)c.soc);
    if (tiled) {
      // the INT sums in k_premat_subg_int: on the auxiliary stream when the caller gave one
      const int im = tiled_int_mode();
      const bool conc = im == 2 && int_stream != nullptr && ev_fork != nullptr && ev_join != nullptr;
      const bool intk = im == 0 || (im == 2 && !conc);
      // serial: before the tiled kernel; concurrent: submitted after it, so the tiled kernel's
      // persistent workgroups are resident first and the INT workgroups fill what they leave
      auto launch_int = [&](hipStream_t is) {
        hipLaunchKernelGGL(k_premat_subg_int<DCOR_INT_R>, dim3((unsigned)((reps + DCOR_INT_R - 1) / DCOR_INT_R)),
                           dim3(256), 0, is, c, reps, (SubgPartial*)part);
      };
      if (conc && hipEventRecord((hipEvent_t)ev_fork, (hipStream_t)stream) != hipSuccess) return last_err();
      if (!intk && !conc) launch_int((hipStream_t)stream);
      const bool al = ((reinterpret_cast<uintptr_t>(c.perm) | reinterpret_cast<uintptr_t>(c.lap_ni_x) |
                        reinterpret_cast<uintptr_t>(c.lap_ni_y)) & 15) == 0;
      const TiledKernel tk = tiled_kernel(intk, al);
      const int64_t np = c.s.n >> 1;  // INT pairs (at most; h = 1 rows have (n - 1) / 2)
      const size_t red_b = (size_t)(20 * (tk.nt / 64)) * sizeof(double);
      const int64_t tp_max = (int64_t)((tk.lds_budget - red_b) / 16 - 3) / 2;
      const int64_t ntiles = np > 0 ? (np + tp_max - 1) / tp_max : 1;
      const int64_t tile_pairs = np > 0 ? (np + ntiles - 1) / ntiles : 1;
      const size_t lds = red_b + (size_t)(2 * tile_pairs + 3) * 16;
      if (hipFuncSetAttribute((const void*)tk.k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024) != hipSuccess)
        return last_err();
      int dev = 0, cus = 0, per_cu = 0;
      if (hipGetDevice(&dev) != hipSuccess) return last_err();
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return last_err();
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tk.k, tk.nt, lds) != hipSuccess)
        return last_err();
      const int64_t slots = (int64_t)cus * (per_cu < 1 ? 1 : per_cu);
      const int64_t grid = reps < slots ? reps : slots;
      hipLaunchKernelGGL(tk.k, dim3((unsigned)grid), dim3((unsigned)tk.nt), lds, (hipStream_t)stream, c,
                         (const int*)c.dict_ok, reps, tile_pairs, (SubgPartial*)part);
      if (conc) {
        if (hipStreamWaitEvent((hipStream_t)int_stream, (hipEvent_t)ev_fork, 0) != hipSuccess) return last_err();
        launch_int((hipStream_t)int_stream);
        if (hipEventRecord((hipEvent_t)ev_join, (hipStream_t)int_stream) != hipSuccess) return last_err();
        if (hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev_join, 0) != hipSuccess) return last_err();
      }
    } else if (c.dict_built != 2) {
      const DictKernel kl = l2_kernel();
      const size_t lds = (size_t)(20 * DICT_NW) * sizeof(double);
      int dev = 0, cus = 0, per_cu = 0;
      if (hipGetDevice(&dev) != hipSuccess) return last_err();
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return last_err();
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kl, DICT_NT, lds) != hipSuccess)
        return last_err();
      const int64_t slots = (int64_t)cus * (per_cu < 1 ? 1 : per_cu);
      const int64_t grid = reps < slots ? reps : slots;
      hipLaunchKernelGGL(kl, dim3((unsigned)grid), dim3(DICT_NT), lds, (hipStream_t)stream, c,
                         (const uint16_t*)nullptr, (const double*)nullptr, (const int*)c.dict_ok,
                         reps, (SubgPartial*)part);
    }
  } else if (c.dict_built != 2) {  // 2: a prepared panel known to be coded (dcor_panel)
    hipLaunchKernelGGL(k_premat_subg_stream, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                       (hipStream_t)stream, c, (const int*)c.dict_ok, (SubgPartial*)part);
  }
  // workgroup-per-replicate epilogue: measured faster here than the wave-per-replicate form
  // (k_premat_subg_epilogue_w: 2000 loaded keys per wave cost 200+ VGPRs, one wave per SIMD)
  const int wave_epi = [] {
    const char* v = dcor::variant("DCOR_EPILOGUE");
    return v && std::strcmp(v, "wave") == 0;
  }();
  const unsigned gw = (unsigned)((reps + DCOR_WAVES - 1) / DCOR_WAVES);
  if (epi_stream != nullptr) {  // epilogue on a second stream, after this chunk's streaming
    if (hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) != hipSuccess) return last_err();
    if (hipStreamWaitEvent((hipStream_t)epi_stream, (hipEvent_t)ev, 0) != hipSuccess) return last_err();
    stream = epi_stream;
  }
  if (!wave_epi)
    hipLaunchKernelGGL(k_premat_subg_epilogue, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                       (hipStream_t)stream, c, (const SubgPartial*)part, out);
  else if (c.s.mix.nsim <= 1024)
    hipLaunchKernelGGL(k_premat_subg_epilogue_w<16>, dim3(gw), dim3(DCOR_BLOCK), 0,
                       (hipStream_t)stream, c, reps, (const SubgPartial*)part, out);
  else
    hipLaunchKernelGGL(k_premat_subg_epilogue_w<32>, dim3(gw), dim3(DCOR_BLOCK), 0,
                       (hipStream_t)stream, c, reps, (const SubgPartial*)part, out);
  return last_err();
}
int accumulate_blocks(int64_t count) { return (int)acc_nblocks(count); }
int64_t accumulate_per(int64_t count) { return acc_per(count, acc_nblocks(count)); }

int launch_accumulate_pass(const dcor_rep_out* rec, const AccEntry* ent, int nent, int max_span,
                           dcor_accum* part, dcor_accum* acc, void* stream) {
  if (nent <= 0) return 0;
  hipLaunchKernelGGL(k_accumulate_pass, dim3((unsigned)max_span, (unsigned)nent), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, rec, ent, part, acc);
  return last_err();
}

int launch_accumulate_merge_cells(const AccCell* cells, int ncells, const dcor_accum* part,
                                  dcor_accum* acc, void* stream) {
  if (ncells <= 0) return 0;
  hipLaunchKernelGGL(k_accumulate_merge_cells, dim3((unsigned)ncells), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, cells, part, acc);
  return last_err();
}

int launch_accumulate(const dcor_rep_out* d_out, int64_t count, double rho, dcor_accum* acc,
                      void* stream) {
  // ~2048 records per block, at most 512 blocks; 1 block writes acc directly.
  const int64_t nb = acc_nblocks(count), per = acc_per(count, nb);
  if (nb == 1) {
    hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, d_out,
                       count, per, rho, acc);
    return last_err();
  }
  dcor_accum* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, (size_t)nb * 2 * sizeof(dcor_accum), (hipStream_t)stream);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_accumulate, dim3((unsigned)nb), dim3(DCOR_BLOCK), 0, (hipStream_t)stream,
                     d_out, count, per, rho, part);
  hipLaunchKernelGGL(k_accumulate_merge, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, part,
                     (int)nb, count, acc);
  const int rc = last_err();
  (void)hipFreeAsync(part, (hipStream_t)stream);
  return rc;
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
static int64_t draws_gx(int64_t count) {
  const int64_t npair = (count + 1) / 2;
  const int64_t gx = (npair + DCOR_BLOCK - 1) / DCOR_BLOCK;
  return gx > 4096 ? 4096 : gx;
}
// Values of t per lane: ~16 when the launch fills the chip many times over (C5-e2e's 8192
// replicates: 8: 479 us, 32: 491 us, 16: 445-452 us), fewer for small launches (a sweep's 200
// replicates), whose walks are latency bound at a few waves per SIMD.  Results never depend on it.
static int64_t perm_gx(int64_t reps, int64_t count) {
  int64_t v = (count * reps + 4096 * DCOR_BLOCK - 1) / (4096 * DCOR_BLOCK);
  v = v < 2 ? 2 : (v > 16 ? 16 : v);
  const int64_t gx = (count + v * DCOR_BLOCK - 1) / (v * DCOR_BLOCK);
  return gx > 4096 ? 4096 : gx;
}
static void perm_split(int64_t n, int* a, int* c) {
  int bits = 1;
  while ((1ll << bits) < n) ++bits;
  *a = bits / 2;
  *c = bits - *a;
}
int launch_draws(int kind, uint32_t k0, uint32_t k1, uint32_t site, int64_t rep_begin,
                 int64_t reps, int64_t count, double* out, void* stream) {
  if (reps <= 0 || count <= 0) return 0;
  hipLaunchKernelGGL(k_draws, dim3((unsigned)draws_gx(count), (unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, kind, k0, k1, site, rep_begin, count, out);
  return last_err();
}
int launch_perm(uint32_t k0, uint32_t k1, uint32_t site, int64_t rep_begin, int64_t reps,
                int64_t n, int64_t count, int32_t* out, void* stream) {
  if (reps <= 0 || count <= 0) return 0;
  int a, c;
  perm_split(n, &a, &c);
  hipLaunchKernelGGL(k_perm, dim3((unsigned)perm_gx(reps, count), (unsigned)reps), dim3(DCOR_BLOCK),
                     0, (hipStream_t)stream, k0, k1, site, rep_begin, (uint32_t)n, a, c, count, out);
  return last_err();
}
int launch_hrs_noise(const HrsNoise& j, int64_t reps, void* stream) {
  if (reps <= 0) return 0;
  HrsNoiseArgs q;
  q.j = j;
  perm_split(j.n, &q.pa, &q.pc);
  const int64_t gx[7] = {j.km > 0 ? perm_gx(reps, j.km) : 0, draws_gx(j.k), draws_gx(j.k),
                         draws_gx(j.n), draws_gx(1), draws_gx(j.nsim), draws_gx(j.nsim)};
  q.g[0] = 0;
  for (int i = 0; i < 7; ++i) q.g[i + 1] = q.g[i] + (uint32_t)gx[i];
  hipLaunchKernelGGL(k_hrs_noise, dim3(q.g[7], (unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, q);
  return last_err();
}
int launch_dp_sd(const double* x, int64_t n, double lo, double hi, double s_mu, double s_m2,
                 const double* lap2, double* out2, void* stream) {
  hipLaunchKernelGGL(k_dp_sd, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, x, n, lo, hi,
                     s_mu, s_m2, lap2, out2);
  return last_err();
}

static inline dim3 elem_grid(int64_t n) { return dim3((unsigned)((n + DCOR_BLOCK - 1) / DCOR_BLOCK)); }

int launch_uc_sd(const PrematSubgConst& p, double* out, void* stream) {
  hipLaunchKernelGGL(k_uc_sd, dim3(1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, p, out);
  return last_err();
}
int launch_standardize_dp(const double* x, int64_t n, double lo, double hi, double mean, double den,
                          double* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_standardize_dp, elem_grid(n), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, x, n,
                     lo, hi, mean, den, out);
  return last_err();
}
int launch_gen_bernoulli(const double* u, const double* v, int64_t n, double t0, double t1,
                         double* X, double* Y, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_gen_bernoulli, elem_grid(n), dim3(DCOR_BLOCK), 0, (hipStream_t)stream, u, v,
                     n, t0, t1, X, Y);
  return last_err();
}
int launch_gen_bounded_factor(const double* U, const double* E1, const double* E2, int64_t n,
                              double* X, double* Y, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_gen_bounded_factor, elem_grid(n), dim3(DCOR_BLOCK), 0, (hipStream_t)stream,
                     U, E1, E2, n, X, Y);
  return last_err();
}
int launch_mvrnorm_apply(const double* z0, int64_t n0, const double* z1, int64_t n1,
                         const int32_t* perm, const MvnConst& m, double* X, double* Y, void* stream) {
  if (n0 + n1 <= 0) return 0;
  hipLaunchKernelGGL(k_mvrnorm_apply, elem_grid(n0 + n1), dim3(DCOR_BLOCK), 0, (hipStream_t)stream,
                     z0, n0, z1, n1, perm, m, X, Y);
  return last_err();
}

}  // namespace dcor
