// dcor_rstream.hip -- R-stream mode: replicates consume R's OWN random
// streams, so run_sim_one(..., seed) on the GPU returns the reference's per-seed numbers.
//
// R's generator is one sequential Mersenne-Twister stream per set.seed() (vert-cor.R:364;
// ver-cor-subG.R:169), consumed in the call order of SURVEY.md Appendix A.  The engine keeps
// that contract and puts the parallelism where R's stream allows it:
//   k_rs_stream       one 256-thread workgroup per grid cell: MT19937 blocks of 624 words
//                     (the recurrence is parallel: every dependency is >= 227 words back,
//                     so each of a block's three phases is one step of 256 threads), tempered
//                     words streamed to HBM, and the data-dependent consumption --
//                     exp_rand inside mixquant, sample.int's rejection in gen_mix_gaussian --
//                     walked in order, so every replicate's offset in the stream is known.
//                     The MT state is persistent across chunks of replicates
//                     (.Random.seed semantics).
//   k_rs_materialise  one workgroup per (cell, replicate): words -> R's variates (inversion
//                     rnorm with AS241 qnorm, mvrnorm's eigen factor, runif, rbinom,
//                     extraDistr rlaplace, the sample.int row shuffle), written in the
//                     explicit-input layout.
//   then the pre-materialised estimator kernels (dcor_premat.hip) per cell.
//   k_rs_hrs_ni       the HRS NI runs (real-data-sims.R): sample.int(n, k*m) and rLap(k) x2
//                     after each run's own set.seed.
// Every transform uses IEEE basic operations, explicit fma and R's operation order
// (-ffp-contract=off); log is the accurate double-double rs_log (csrc/dcor_tables.h), so the
// GPU matches the CPU restatement oracle/dcor_rstream.c bit for bit.
#include <hip/hip_runtime.h>

#include "dcor_device.h"
#include "dcor_engine.h"

namespace dcor {

// ------------------------------------------------------------ R variates ---
__device__ __forceinline__ double rs_unif(uint32_t w) {
  // MT_genrand's y * 2.3283064365386963e-10, then unif_rand's fixup into (0, 1)
  const double x = (double)w * 2.3283064365386963e-10;
  if (x <= 0.0) return 0.5 * 2.328306437080797e-10;
  return x;  // (1 - x) > 0 for every 32-bit word
}

__device__ __forceinline__ void rs_two_sum(double a, double b, double& s, double& e) {
  const double t = a + b, bb = t - a;
  s = t;
  e = (a - (t - bb)) + (b - bb);
}

__device__ double rs_log(double x) {
  // x positive normal.  log x = k ln2 + log c + log1p(r), r = z*invc - 1 exact as a pair,
  // r^2/2 in double-double, the r^3 .. r^10 tail in double, log c as a double-double.
  const uint64_t ix = (uint64_t)__double_as_longlong(x);
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127u);
  const int64_t k = (int64_t)tmp >> 52;
  const double z = __longlong_as_double((long long)(ix - (tmp & (0xfffull << 52))));
  const double invc = dcor_log_tab[i][0], lch = dcor_log_tab[i][1], lcl = dcor_log_tab_lo[i];
  const double p = z * invc;
  const double pe = fma(z, invc, -p);
  double r1, r2;
  rs_two_sum(p - 1.0, pe, r1, r2);
  const double s2 = r1 * r1;
  const double s2e = fma(r1, r1, -s2);
  const double h = -0.5 * s2;
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
  rs_two_sum(r1, h, a1, a2);
  const double kd = (double)k;
  double s, se, s3, se3;
  rs_two_sum(kd * DCOR_LN2_HI, lch, s, se);
  rs_two_sum(s, a1, s3, se3);
  const double lo = se + se3 + (a2 + hl + r2 + tail) + (kd * DCOR_LN2_LO + lcl);
  return s3 + lo;
}

__device__ double rs_qnorm5(double p) {
  // R's qnorm(p) (qnorm.c, Wichura's AS241) for p in (0, 1), lower tail
  const double q = p - 0.5;
  double r, val;
  if (fabs(q) <= .425) {
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
  r = (q > 0) ? (0.5 - p + 0.5) : p;
  r = sqrt_pos(-rs_log(r));
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

// norm_rand(), INVERSION: u = (int)(2^27 u1) + u2; qnorm5(u / 2^27)
__device__ __forceinline__ double rs_norm(uint32_t w1, uint32_t w2) {
  const double BIG = 134217728.0;
  const double u = (double)(int)(BIG * rs_unif(w1)) + rs_unif(w2);
  return rs_qnorm5(u / BIG);
}

// extraDistr::rlaplace(1, 0, 1) of one word: u = runif(-.5, .5); -sign(u) log(1 - 2|u|)
__device__ __forceinline__ double rs_lap(uint32_t w) {
  const double u = -0.5 + 1.0 * rs_unif(w);
  if (u == 0.0) return 0.0;
  const double l = rs_log(1.0 - 2.0 * fabs(u));
  return (u > 0) ? -l : l;
}

// ------------------------------------------------------------- k_rs_stream ---
#define RS_N 624
#define RS_M 397
#define RS_EXP_MAXW 17   // exp_rand consumes at most 1 + 1 + 15 words

// exp_rand's q[k-1] = sum_{j<=k} ln2^j / j! (R's sexp.c table)
#define RS_Q0 0.6931471805599453
#define RS_Q_TABLE                                                                            \
  {0.6931471805599453, 0.9333736875190459, 0.9888777961838675, 0.9984959252914960040,       \
   0.9998292811061389, 0.9999833164100727, 0.9999985691438767, 0.9999998906925558,         \
   0.9999999924734159, 0.9999999995283275, 0.9999999999728814, 0.9999999999985598,         \
   0.9999999999999289, 0.9999999999999968, 0.9999999999999999, 1.0000000000000000}

// exp_rand (sexp.c) from the draw's first word w: a (the doubling loop's multiple of ln 2) and u,
// and the number of words the draw consumes -- 1 when u <= q[0], else 2 + i for the index i of
// the first q[i] >= u (the do-loop's draws); the value is a + u, or a + q[0] * min of the words
// after the first.
__device__ __forceinline__ int rs_exp_head(uint32_t w, double& a, double& eu) {
  constexpr double q[16] = RS_Q_TABLE;
  a = 0.;
  eu = rs_unif(w);
  for (;;) {
    eu += eu;
    if (eu > 1.) break;
    a += q[0];
  }
  eu -= 1.;
  if (eu <= q[0]) return 1;
  int ie = 1;
#pragma unroll
  for (int t = 1; t < 15; ++t) ie += (eu > q[t]) ? 1 : 0;
  return 2 + ie;
}

__device__ __forceinline__ uint32_t rs_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t rs_untemper(uint32_t y) {
  y ^= y >> 18;
  y ^= (y << 15) & 0xefc60000u;
  uint32_t x = y;
#pragma unroll
  for (int i = 0; i < 4; ++i) x = y ^ ((x << 7) & 0x9d2c5680u);
  y = x;
  x = y ^ (y >> 11);
  x = y ^ (x >> 11);
  return x;
}

#define RS_G __attribute__((address_space(1)))
__device__ __forceinline__ int rs_rl(int v, int s) { return __builtin_amdgcn_readlane(v, s); }
__device__ __forceinline__ int rs_u(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int rs_wrap(int x) { return (x >= 2 * 624) ? x - 2 * 624 : x; }
__device__ __forceinline__ int64_t rs_u64(int64_t v) {
  const int lo = rs_u((int)v), hi = rs_u((int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double rs_rld(double v, int s) {
  const long long b = __double_as_longlong(v);
  const int lo = rs_rl((int)b, s), hi = rs_rl((int)(b >> 32), s);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// One MT19937 block in three phases, each issuing all of its LDS reads before any write:
// kk < 227 reads mt[kk+397] (old); 227 <= kk < 454 reads mt[kk-227] (new, phase 1);
// kk >= 454 reads mt[kk-227] (new, phase 2) and, for kk = 623, mt[0] (new).  One wave.
// NT threads of the workgroup share the phase (NT = 64: one wave).
template <int NT = 64>
__device__ __forceinline__ void rs_mt_phase(uint32_t* mt, int lane, int k0, int k1) {
  constexpr int S = (RS_N - RS_M + NT - 1) / NT;
  uint32_t a[S], b[S], src[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int kk = k0 + lane + NT * i;
    if (kk < k1) {
      a[i] = mt[kk];
      b[i] = mt[kk == RS_N - 1 ? 0 : kk + 1];
      src[i] = mt[kk < RS_N - RS_M ? kk + RS_M : kk - (RS_N - RS_M)];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int kk = k0 + lane + NT * i;
    if (kk < k1) {
      const uint32_t y = (a[i] & 0x80000000u) | (b[i] & 0x7fffffffu);
      mt[kk] = src[i] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
  }
  __syncthreads();
}
template <int NT = 64>
__device__ __forceinline__ void rs_mt_block(uint32_t* mt, int lane) {
  rs_mt_phase<NT>(mt, lane, 0, RS_N - RS_M);
  rs_mt_phase<NT>(mt, lane, RS_N - RS_M, 2 * (RS_N - RS_M));
  rs_mt_phase<NT>(mt, lane, 2 * (RS_N - RS_M), RS_N);
}

// set.seed(seed): RNG_Init's scrambling and 625 words (word 0, the position, is 624)
__device__ __forceinline__ void rs_seed_mt(uint32_t* mt, int32_t seed, int lane) {
  if (lane == 0) {
    uint32_t s = (uint32_t)seed;
    for (int j = 0; j < 50; ++j) s = 69069u * s + 1u;
    s = 69069u * s + 1u;
    for (int j = 0; j < RS_N; ++j) { s = 69069u * s + 1u; mt[j] = s; }
  }
  __syncthreads();
}

// One workgroup per cell.  Its four waves generate each MT block together; every wave runs the
// walk below on the same words (the walk is uniform control flow plus wave-wide window
// classification), so they all call next_block() at the same points, and only wave 0 stores
// the walk's results.  Four waves measured 1.25x (R1) to 1.35x (RG) the one-wave kernel.
// mt[] holds the raw state of the newest block; ring[] the tempered words
// of the last two blocks (slot = absolute word index mod 1248), so exp_rand draws can look
// up to 17 words ahead while the walk stays at most one block behind generation.
// Positions are chunk-relative: P words consumed, Q words produced (and written to HBM).
#define RS_STREAM_NT 256
__global__ __launch_bounds__(RS_STREAM_NT) void k_rs_stream(RsCell* cells, int32_t rc) {
  constexpr int NT = RS_STREAM_NT;
  __shared__ uint32_t mt[RS_N];
  __shared__ uint32_t ring[2 * RS_N];
  // every field in registers: the kernel's stores could alias the descriptor, and a reload
  // from global memory inside the walk costs an L2 round trip per draw
  const RsCell& cg = cells[blockIdx.x];
  const int64_t c_pre = cg.pre, c_nsim = cg.nsim, c_n = cg.n;
  const int c_has_mix = cg.has_mix, c_shuffle = cg.shuffle;
  const int64_t c_pre_a = c_shuffle ? cg.pre_a : cg.pre;  // fixed words before sample.int
  const int64_t c_cap = cg.words_cap;
  int ovf = 0;
  RS_G int64_t* const shuf_end = (RS_G int64_t*)cg.shuf_end;
  // global (not flat) stores: a flat store also counts in lgkmcnt, so every LDS wait behind
  // it would wait for the store to reach memory
  RS_G int64_t* const rep_off = (RS_G int64_t*)cg.rep_off;
  RS_G int64_t* const exp_end = (RS_G int64_t*)cg.exp_end;
  RS_G double* const gexpv = (RS_G double*)cg.expv;
  const int tid = threadIdx.x, lane = tid & 63;
  const bool w0 = tid < 64;  // the wave that stores the walk's results
  RsState* st = cg.st;
  for (int t = tid; t < RS_N; t += NT) mt[t] = st->mt[t];
  // uniform by construction: readfirstlane keeps the walk's counters in scalar registers
  const int mti0 = __builtin_amdgcn_readfirstlane(st->mti);
  int par = __builtin_amdgcn_readfirstlane(st->pad[0]) & 1;  // ring half of mt[]'s block
  const int par0 = par;
  __syncthreads();
  RS_G uint32_t* const out = (RS_G uint32_t*)cg.words;
  int64_t P = 0, Q = 0;
  if (mti0 < RS_N) {                      // the rest of the current block comes first
    for (int t = tid; t < RS_N; t += NT) {
      const uint32_t w = rs_temper(mt[t]);
      ring[par * RS_N + t] = w;
      if (t >= mti0) out[t - mti0] = w;
    }
    Q = RS_N - mti0;
    __syncthreads();
  }
  // ring slot of the consumption point P (absolute word index mod 1248)
  int pslot = (par0 * RS_N + mti0) % (2 * RS_N);
  auto next_block = [&]() {
    rs_mt_block<NT>(mt, tid);
    par ^= 1;
    for (int t = tid; t < RS_N; t += NT) {
      const uint32_t w = rs_temper(mt[t]);
      ring[par * RS_N + t] = w;
      out[Q + t] = w;
    }
    Q += RS_N;
    __syncthreads();
  };
  constexpr double q[16] = RS_Q_TABLE;
  int32_t r = 0;
  // 0: fixed words before sample.int (gen_mix_gaussian) or before exp_rand; 3: sample.int(n);
  // 4: fixed words after it; 1: exp_rand; 2: mixquant's rbinom
  int phase = 0;
  int64_t left = c_pre_a, j = 0, sdn = 0;
  if (tid == 0) rep_off[0] = 0;
  while (r < rc) {
    // the walk is uniform; say so, or the structurizer keeps it in vector registers under
    // exec masks
    P = rs_u64(P); Q = rs_u64(Q); j = rs_u64(j); left = rs_u64(left); sdn = rs_u64(sdn);
    r = rs_u(r); phase = rs_u(phase); par = rs_u(par); pslot = rs_u(pslot);
    if (phase == 3) {
      // sample.int(n): R_unif_index(dn) for dn = n .. 1, rbits(ceil(log2 dn)) until < dn.  Only
      // the consumption matters here (k_rs_materialise replays the swaps); a window of words
      // is classified lane-parallel (v < dn - W accepts, v >= dn rejects whatever came
      // before), anything else goes attempt by attempt.
      if (P == Q) { if (Q + RS_N > c_cap) { ovf = 1; break; } next_block(); continue; }
      const int bits = (sdn <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(sdn - 1));
      const int W = (Q - P < 64) ? (int)(Q - P) : 64;
      const int bits_lo = (sdn - W <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(sdn - W - 1));
      if (bits > 15 || bits != bits_lo || sdn <= 64) {
        const int nw = bits / 16 + 1;
        if (P + nw > Q) { if (Q + RS_N > c_cap) { ovf = 1; break; } next_block(); continue; }
        uint64_t v = 0;
        for (int t = 0; t < nw; ++t) v = 65536ull * v + (ring[rs_wrap(pslot + t)] >> 16);
        v &= (bits >= 63) ? ~0ull : ((1ull << bits) - 1ull);
        P += nw;
        pslot = rs_wrap(pslot + nw);
        if ((int64_t)v < sdn) --sdn;
      } else {
        const uint32_t mask = (1u << bits) - 1u;
        const bool in = lane < W;
        const int64_t v = in ? (int64_t)((ring[rs_wrap(pslot + lane)] >> 16) & mask) : 0;
        const bool sure_acc = in && v < sdn - W, sure_rej = in && v >= sdn;
        if (__ballot(in && !sure_acc && !sure_rej)) {
          for (int l = 0; l < W; ++l)
            if ((int64_t)(uint32_t)rs_rl((int)v, l) < sdn) --sdn;
        } else {
          sdn -= __builtin_popcountll(__ballot(sure_acc));
        }
        P += W;
        pslot = rs_wrap(pslot + W);
      }
      if (sdn == 0) {
        if (tid == 0) shuf_end[r] = P;
        phase = 4;
        left = c_pre - c_pre_a;
      }
      continue;
    }
    if (phase != 1) {
      if (P == Q) { if (Q + RS_N > c_cap) { ovf = 1; break; } next_block(); continue; }
      const int64_t take = (left < Q - P) ? left : Q - P;
      P += take;
      pslot = (int)((pslot + take % (2 * RS_N)) % (2 * RS_N));
      left -= take;
      if (left == 0) {
        if (phase == 0 && c_shuffle) {
          phase = 3; sdn = c_n;
        } else if ((phase == 0 || phase == 4) && c_has_mix) {
          phase = 1; j = 0;
        } else {
          ++r;
          if (r < rc && tid == 0) rep_off[r] = P;
          phase = 0; left = c_pre_a;
        }
      }
      continue;
    }
    if (P + RS_EXP_MAXW > Q) { if (Q + RS_N > c_cap) { ovf = 1; break; } next_block(); continue; }
    // Window of 64 words at P.  Lane l evaluates "an exp_rand draw starting at P + l": R's
    // doubling loop and the draw's length (1, or 2 + the index i where u <= q[i]) depend on
    // that one word only.  The chain of draw starts from P follows by pointer doubling over
    // the lengths; finally every start lane computes and stores its own value.
    const int64_t pos = P + lane;
    double a = 0., eu = 0.;
    int len = 1;
    if (pos < Q) len = rs_exp_head(ring[rs_wrap(pslot + lane)], a, eu);
    // Chain of draw starts from lane 0 by pointer doubling: lane l holds the set M of chain
    // positions reachable from l and the first position J past it; six rounds of
    // M |= M[J], J = J[J] cover the window.
    const int64_t rem = c_nsim - j;
    const int64_t lim = Q - RS_EXP_MAXW - P;   // a draw may start at s <= lim
    uint64_t M = 1ull << lane;
    int J = lane + len;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int src = (J < 64) ? J : 63;
      const uint32_t mlo = (uint32_t)__shfl((int)(uint32_t)M, src);
      const uint32_t mhi = (uint32_t)__shfl((int)(uint32_t)(M >> 32), src);
      const int jj = __shfl(J, src);
      if (J < 64) { M |= ((uint64_t)mhi << 32) | mlo; J = jj; }
    }
    const uint64_t chain = ((uint64_t)(uint32_t)rs_rl((int)(M >> 32), 0) << 32) |
                           (uint32_t)rs_rl((int)(uint32_t)M, 0);
    uint64_t starts = (lim >= 63) ? chain : (chain & ((2ull << lim) - 1ull));
    int64_t cnt = __builtin_popcountll(starts);
    while (cnt > rem) {                        // the segment ends inside this window
      starts &= ~(1ull << (63 - __builtin_clzll(starts)));
      --cnt;
    }
    const int last = 63 - __builtin_clzll(starts);
    const int s = rs_u(last + rs_rl(len, last));
    if (w0 && ((starts >> lane) & 1ull)) {
      double e;
      if (len == 1) {
        e = a + eu;
      } else {                            // umin over the len - 1 following words
        uint32_t wmin = 0xffffffffu;
        for (int t = 1; t < len; ++t) {
          const uint32_t w2 = ring[rs_wrap(pslot + lane + t)];
          wmin = (w2 < wmin) ? w2 : wmin;
        }
        e = a + rs_unif(wmin) * q[0];
      }
      const int idx = __builtin_popcountll(starts & ((1ull << lane) - 1ull));
      gexpv[(int64_t)r * c_nsim + j + idx] = e;
    }
    j += cnt;
    P += s;
    pslot = rs_wrap(pslot + s);
    if (j == c_nsim) {
      if (tid == 0) exp_end[r] = P;
      phase = 2; left = c_nsim;
    }
  }
  if (ovf) {                               // word buffer exhausted (sample.int's rejection
    if (tid == 0) st->pad[1] = 1;         // sampling ran far past its bound): flag, stop
    return;
  }
  // .Random.seed at the consumption point P: in the newest block, just past it, or (after an
  // exp_rand look-ahead) in the previous block, whose raw state is the untempered ring half
  const int64_t o = P + mti0;              // words since the start of the chunk's first block
  const int64_t blk = o / RS_N, newest = (Q + mti0) / RS_N - 1;
  const int off = (int)(o % RS_N);
  if (blk > newest) {                     // P == Q at a block boundary
    for (int t = tid; t < RS_N; t += NT) st->mt[t] = mt[t];
    if (tid == 0) { st->mti = RS_N; st->pad[0] = par; }
  } else if (blk == newest) {
    for (int t = tid; t < RS_N; t += NT) st->mt[t] = mt[t];
    if (tid == 0) { st->mti = off; st->pad[0] = par; }
  } else {
    for (int t = tid; t < RS_N; t += NT) st->mt[t] = rs_untemper(ring[(par ^ 1) * RS_N + t]);
    if (tid == 0) { st->mti = off; st->pad[0] = par ^ 1; }
  }
}

// ------------------------------------------------------------ jump path ---
// k_rs_stream is one workgroup per cell: a single cell (R1: one grid point, B = 1000) runs on
// one CU, generation and walk alike.  The jump path spreads one cell's chunk over the chip:
//   k_rsj_gen0   segment 0 (RSJ_L raw words) sequentially from the state block;
//   k_rsj_jump   segment s >= 1: its first block is sum_{i : g_i = 1} w[624 + i + p] for the jump
//                polynomial g = x^(s RSJ_L - 624) mod phi (dcor_mtjump.cpp) over segment 0's
//                words, then the recurrence; all segments of all cells at once;
//   k_rsj_len    T_0(P) = P + the words an exp_rand draw starting at P consumes;
//   k_rsj_tlift  T_{k+1} = T_k o T_k (16-bit offsets while they fit), k_rsj_glift likewise for G:
//                pointer doubling;
//   k_rsj_g0     G_0(P) = T^nsim(P + pre) + post: the start of the replicate after one at P;
//   k_rsj_chain  P_r = G^r(0) for every r <= rc (binary digits of r), exp_end = T^nsim(P_r + pre);
//   k_rsj_expv   the d-th exp_rand value of replicate r at T^d(P_r + pre);
//   k_rsj_state  .Random.seed at P_rc.
// Positions are clamped at jN, so a chunk whose replicates need more words than the budget
// ends at jN: k_rsj_chain flags it and k_rsj_state leaves the state alone (the host re-runs the
// chunk by k_rs_stream).  Replicates without mixquant (the Laplace CI) have a fixed length: P_r =
// r * pre, no tables.
#define RSJ_NT 256
#define RSJ_JNT 640                         // k_rsj_jump: one lane per window word, 10 waves
#define RSJ_DEG 19937
#define RSJ_BASEW (RSJ_DEG - 1 + RS_N)      // base words one window combines
static_assert(RSJ_PAD == RSJ_BASEW, "the list pad points at the zero words after the base");

__device__ __forceinline__ int64_t rsj_need(int64_t jN, int mti) {  // raw words the chunk may read
  return (mti + jN + 64 + RS_N - 1) / RS_N * RS_N;
}

// T_k(x) - x (levels at t: RSJ_TBYTES)
__device__ __forceinline__ int64_t rsj_tget(const uint8_t* t, int64_t S, int k, int64_t x) {
  const uint8_t* lv = t + RSJ_TBYTES(k, S);
  return (k < RSJ_T16) ? (int64_t)((const uint16_t*)lv)[x] : (int64_t)((const uint32_t*)lv)[x];
}
// x advanced by m exp_rand draws (x and every table entry <= N: T maps N to N)
__device__ __forceinline__ int64_t rsj_adv_t(const uint8_t* t, int64_t S, int64_t x, int64_t m) {
  for (int k = 0; m; ++k, m >>= 1)
    if (m & 1) x += rsj_tget(t, S, k, x);
  return x;
}

__global__ __launch_bounds__(RSJ_NT) void k_rsj_gen0(const RsCell* cells) {
  __shared__ uint32_t mt[RS_N];
  const RsCell& c = cells[blockIdx.x];
  const int tid = threadIdx.x;
  const int mti = c.st->mti;
  for (int t = tid; t < RS_N; t += RSJ_NT) mt[t] = c.st->mt[t];
  __syncthreads();
  const int64_t need = rsj_need(c.jN, mti);
  const int64_t end = need < RSJ_L ? need : RSJ_L;
  RS_G uint32_t* const raw = (RS_G uint32_t*)c.raw;
  RS_G uint32_t* const W = (RS_G uint32_t*)c.words;
  for (int64_t b0 = 0; b0 < end; b0 += RS_N) {
    if (b0) rs_mt_block<RSJ_NT>(mt, tid);
    for (int t = tid; t < RS_N; t += RSJ_NT) {
      const uint32_t v = mt[t];
      raw[b0 + t] = v;
      if (b0 + t >= mti) W[b0 + t - mti] = rs_temper(v);
    }
  }
}

// One workgroup per (segment, cell); lane p < 624 combines window word p over the set-bit list
// of the segment's jump polynomial (host-built, padded to a multiple of 8 with RSJ_PAD, which
// points every lane at a zero word): eight LDS reads in flight per lane, the list in scalar loads.
__global__ __launch_bounds__(RSJ_JNT) void k_rsj_jump(const RsCell* cells, const uint32_t* __restrict__ poff,
                                                      const uint32_t* __restrict__ pidx) {
  extern __shared__ uint32_t rsj_base[];   // raw[624 .. 624 + RSJ_BASEW), then 624 zeros
  __shared__ uint32_t mt[RS_N];
  const RsCell& c = cells[blockIdx.y];
  const int s = blockIdx.x + 1, tid = threadIdx.x;
  const int mti = c.st->mti;
  const int64_t need = rsj_need(c.jN, mti), s0 = (int64_t)s * RSJ_L;
  if (s0 >= need) return;
  const uint32_t* raw = c.raw;
  for (int i = tid; i < RSJ_BASEW + RS_N; i += RSJ_JNT) rsj_base[i] = (i < RSJ_BASEW) ? raw[RS_N + i] : 0u;
  __syncthreads();
  const int p = tid < RS_N ? tid : RS_N - 1;
  const uint32_t* q = rsj_base + p;
  uint32_t acc = 0;
  // pidx: two 16-bit bit indices per word; poff in words
  // (scalar and LDS loads share one wait counter: the next four words are loaded before this
  // step's reads, so waiting for the reads never waits on a fresh scalar load)
  const uint32_t j1 = poff[s];
  uint32_t j = poff[s - 1];
  uint4 nx = make_uint4(0, 0, 0, 0);
  if (j < j1) nx = *(const uint4*)(pidx + j);
  for (; j < j1; j += 4) {
    const uint4 pr = nx;
    if (j + 4 < j1) nx = *(const uint4*)(pidx + j + 4);
    const uint32_t v0 = q[pr.x & 0xffffu], v1 = q[pr.x >> 16], v2 = q[pr.y & 0xffffu], v3 = q[pr.y >> 16];
    const uint32_t v4 = q[pr.z & 0xffffu], v5 = q[pr.z >> 16], v6 = q[pr.w & 0xffffu], v7 = q[pr.w >> 16];
    acc ^= ((v0 ^ v1) ^ (v2 ^ v3)) ^ ((v4 ^ v5) ^ (v6 ^ v7));
  }
  if (tid < RS_N) mt[tid] = acc;
  __syncthreads();
  RS_G uint32_t* const W = (RS_G uint32_t*)c.words;
  const int64_t end = (s0 + RSJ_L < need) ? s0 + RSJ_L : need;
  for (int64_t b0 = s0; b0 < end; b0 += RS_N) {
    if (b0 != s0) rs_mt_block<RSJ_JNT>(mt, tid);
    for (int t = tid; t < RS_N; t += RSJ_JNT) W[b0 + t - mti] = rs_temper(mt[t]);
  }
}

__global__ __launch_bounds__(256) void k_rsj_len(const RsCell* cells) {
  const RsCell& c = cells[blockIdx.y];
  if (!c.has_mix) return;
  const int64_t N = c.jN;
  const uint32_t* W = c.words;
  RS_G uint16_t* const T0 = (RS_G uint16_t*)c.tlift;
  for (int64_t P = (int64_t)blockIdx.x * 256 + threadIdx.x; P <= N; P += (int64_t)gridDim.x * 256) {
    int64_t v = 0;
    if (P < N) {
      double a, eu;
      v = rs_exp_head(W[P], a, eu);
      v = (P + v < N) ? v : N - P;
    }
    T0[P] = (uint16_t)v;
  }
}

// T level k from level k - 1: T_k(P) - P = d(P) + d(P + d(P)), d = T_{k-1} - id
__global__ __launch_bounds__(256) void k_rsj_tlift(const RsCell* cells, int k) {
  const RsCell& c = cells[blockIdx.y];
  if (!c.has_mix || k >= c.jlt) return;
  const int64_t S = c.jN + 1;
  const uint8_t* t = c.tlift;
  uint8_t* const dst = c.tlift + RSJ_TBYTES(k, S);
  for (int64_t P = (int64_t)blockIdx.x * 256 + threadIdx.x; P < S; P += (int64_t)gridDim.x * 256) {
    const int64_t d = rsj_tget(t, S, k - 1, P);
    const int64_t v = d + rsj_tget(t, S, k - 1, P + d);
    if (k < RSJ_T16) ((RS_G uint16_t*)dst)[P] = (uint16_t)v;
    else ((RS_G uint32_t*)dst)[P] = (uint32_t)v;
  }
}

// G level k from level k - 1
__global__ __launch_bounds__(256) void k_rsj_glift(const RsCell* cells, int k) {
  const RsCell& c = cells[blockIdx.y];
  if (!c.has_mix || k >= c.jlg) return;
  const int64_t S = c.jN + 1;
  const int32_t* src = c.glift + (int64_t)(k - 1) * S;
  RS_G int32_t* const dst = (RS_G int32_t*)(c.glift + (int64_t)k * S);
  for (int64_t P = (int64_t)blockIdx.x * 256 + threadIdx.x; P < S; P += (int64_t)gridDim.x * 256)
    dst[P] = src[src[P]];
}

__global__ __launch_bounds__(256) void k_rsj_g0(const RsCell* cells) {
  const RsCell& c = cells[blockIdx.y];
  if (!c.has_mix) return;
  const int64_t N = c.jN, S = N + 1, pre = c.pre, post = c.jpost, nsim = c.nsim;
  const uint8_t* t = c.tlift;
  RS_G int32_t* const G0 = (RS_G int32_t*)c.glift;
  for (int64_t P = (int64_t)blockIdx.x * 256 + threadIdx.x; P < S; P += (int64_t)gridDim.x * 256) {
    int64_t v = N;
    if (P + pre < N) {
      v = rsj_adv_t(t, S, P + pre, nsim) + post;
      v = v < N ? v : N;
    }
    G0[P] = (int32_t)v;
  }
}

__device__ __forceinline__ int64_t rsj_rep_start(const RsCell& c, int64_t r) {
  if (!c.has_mix) return r * c.pre;
  const int64_t S = c.jN + 1;
  int64_t x = 0;
  for (int k = 0; r; ++k, r >>= 1)
    if (r & 1) x = c.glift[(int64_t)k * S + x];
  return x;
}

__global__ __launch_bounds__(256) void k_rsj_chain(const RsCell* cells, int32_t rc) {
  const RsCell c = cells[blockIdx.y];   // by value: the stores below cannot alias it
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r > rc) return;
  const int64_t P = rsj_rep_start(c, r);
  if (r == rc) {
    *c.jflag = (P >= c.jN) ? 1 : 0;
    return;
  }
  c.rep_off[r] = P;
  if (c.has_mix) {
    const int64_t x = P + c.pre;
    c.exp_end[r] = rsj_adv_t(c.tlift, c.jN + 1, x < c.jN ? x : c.jN, c.nsim);
  }
}

__global__ __launch_bounds__(256) void k_rsj_expv(const RsCell* cells, int32_t rc) {
  constexpr double q0 = RS_Q0;
  const RsCell c = cells[blockIdx.y];   // by value: the stores below cannot alias it
  if (!c.has_mix) return;
  const int64_t nsim = c.nsim, N = c.jN, S = N + 1, total = (int64_t)rc * nsim;
  const uint32_t* W = c.words;
  RS_G double* const ev = (RS_G double*)c.expv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / nsim, d = i - r * nsim;
    const int64_t x0 = c.rep_off[r] + c.pre;
    const int64_t x = rsj_adv_t(c.tlift, S, x0 < N ? x0 : N, d);
    double e = 0.0;
    if (x < N) {
      double a, eu;
      const int len = rs_exp_head(W[x], a, eu);
      if (len == 1) {
        e = a + eu;
      } else {
        uint32_t wmin = 0xffffffffu;
        for (int t = 1; t < len; ++t) wmin = (W[x + t] < wmin) ? W[x + t] : wmin;
        e = a + rs_unif(wmin) * q0;
      }
    }
    ev[i] = e;
  }
}

__global__ __launch_bounds__(256) void k_rsj_state(const RsCell* cells, int32_t rc) {
  const RsCell& c = cells[blockIdx.x];
  if (*c.jflag) return;
  RsState* st = c.st;
  const int mti = st->mti;
  const int64_t o = mti + rsj_rep_start(c, rc);
  int64_t blk = o / RS_N;
  int off = (int)(o % RS_N);
  if (off == 0) { --blk; off = RS_N; }   // R's own form: the block consumed, position 624
  __syncthreads();                       // every thread has read st->mti
  for (int t = threadIdx.x; t < RS_N; t += 256)
    st->mt[t] = (blk == 0) ? c.raw[t] : rs_untemper(c.words[blk * RS_N + t - mti]);
  if (threadIdx.x == 0) { st->mti = off; st->pad[0] = 0; st->pad[1] = 0; }
}

int launch_rsj(RsCell* d_cells, int ncells, int32_t rc, const uint32_t* d_poff, const uint32_t* d_pidx, int nseg,
               int64_t max_pos, int max_lt, int max_lg, int64_t max_exp, void* stream) {
  const hipStream_t s = (hipStream_t)stream;
  const unsigned nc = (unsigned)ncells;
  auto blocks = [](int64_t work) {
    const int64_t b = (work + 255) / 256;
    return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
  };
  hipLaunchKernelGGL(k_rsj_gen0, dim3(nc), dim3(RSJ_NT), 0, s, d_cells);
  if (nseg > 1) {
    const size_t lds = (size_t)(RSJ_BASEW + RS_N) * 4;
    // per call: the attribute is per device, and one process may drive several GPUs
    const hipError_t e = hipFuncSetAttribute((const void*)k_rsj_jump,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_rsj_jump, dim3((unsigned)(nseg - 1), nc), dim3(RSJ_JNT), lds, s, d_cells, d_poff, d_pidx);
  }
  const dim3 gp(blocks(max_pos), nc);
  if (max_lt > 0) {
    hipLaunchKernelGGL(k_rsj_len, gp, dim3(256), 0, s, d_cells);
    for (int l = 1; l < max_lt; ++l) hipLaunchKernelGGL(k_rsj_tlift, gp, dim3(256), 0, s, d_cells, l);
    hipLaunchKernelGGL(k_rsj_g0, gp, dim3(256), 0, s, d_cells);
    for (int l = 1; l < max_lg; ++l) hipLaunchKernelGGL(k_rsj_glift, gp, dim3(256), 0, s, d_cells, l);
  }
  hipLaunchKernelGGL(k_rsj_chain, dim3(blocks((int64_t)rc + 1), nc), dim3(256), 0, s, d_cells, rc);
  if (max_exp > 0) hipLaunchKernelGGL(k_rsj_expv, dim3(blocks(max_exp), nc), dim3(256), 0, s, d_cells, rc);
  hipLaunchKernelGGL(k_rsj_state, dim3(nc), dim3(256), 0, s, d_cells, rc);
  return (int)hipGetLastError();
}

// -------------------------------------------------------- k_rs_materialise ---
// sample.int(n) (do_sample's partial Fisher-Yates, R_unif_index rejection) replayed by ONE wave
// from the words at ws: y[i] = the i-th sampled index (0-based).  x[n] (LDS, = identity on
// entry) and mark[(n+31)/32] (LDS, zero on entry) are scratch.  Windows of 64 words are
// classified lane-parallel; the accepted draws' swaps run in parallel unless the bitmap finds
// two equal indices or an index on one of the window's tail slots.  Returns the words used.
__device__ int64_t rs_shuffle_wave(const uint32_t* __restrict__ ws, int64_t n, uint16_t* x,
                                   uint32_t* mark, int32_t* __restrict__ y, int lane) {
  int64_t p = 0, i = 0, dn = n;
  auto swap_one = [&](int64_t v) {
    if (lane == 0) {
      y[i] = (int32_t)x[v];
      x[v] = x[dn - 1];
    }
    ++i;
    --dn;
  };
  while (i < n) {
    i = rs_u64(i); dn = rs_u64(dn); p = rs_u64(p);
    const int bits = (dn <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(dn - 1));
    const int bits_lo = (dn - 64 <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(dn - 65));
    if (bits > 15 || bits != bits_lo || dn <= 64) {
      const uint64_t mask = (bits >= 63) ? ~0ull : ((1ull << bits) - 1ull);
      uint64_t v;
      do {
        v = 0;
        for (int nn = 0; nn <= bits; nn += 16) v = 65536ull * v + (ws[p++] >> 16);
        v &= mask;
      } while ((int64_t)v >= dn);
      swap_one((int64_t)v);
      continue;
    }
    const uint32_t mask = (1u << bits) - 1u;
    const int64_t v = (int64_t)((ws[p + lane] >> 16) & mask);
    const bool sure_acc = v < dn - 64, sure_rej = v >= dn;
    p += 64;
    if (__ballot(!sure_acc && !sure_rej)) {
      for (int l = 0; l < 64; ++l) {
        const int64_t vl = (int64_t)(uint32_t)rs_rl((int)v, l);
        if (vl < dn) swap_one(vl);
      }
      continue;
    }
    const uint64_t A = __ballot(sure_acc);
    const int B = __builtin_popcountll(A);
    const bool acc = sure_acc;
    const int t = __builtin_popcountll(A & ((1ull << lane) - 1ull));
    const int64_t Lt = dn - 1 - t;
    bool clash = false;
    if (acc) clash = (atomicOr(&mark[v >> 5], 1u << (v & 31)) >> (v & 31)) & 1u;
    if (acc && Lt != v) clash |= (mark[Lt >> 5] >> (Lt & 31)) & 1u;
    const bool serial = __ballot(clash) != 0ull;
    if (acc) atomicAnd(&mark[v >> 5], ~(1u << (v & 31)));
    if (!serial) {
      uint16_t a = 0, b = 0;
      if (acc) { a = x[v]; b = x[Lt]; }
      if (acc) { y[i + t] = (int32_t)a; x[v] = b; }
      i += B;
      dn -= B;
    } else {
      for (uint64_t rest = A; rest; rest &= rest - 1ull)
        swap_one((int64_t)(uint32_t)rs_rl((int)v, __builtin_ctzll(rest)));
    }
  }
  return p;
}

size_t rs_mix_lds_bytes(int64_t n) {
  return (size_t)((n + 1) & ~1ll) * 2 + (size_t)((n + 31) / 32) * 4 + 16;
}

__global__ __launch_bounds__(256) void k_rs_materialise(const RsCell* cells, int32_t rc) {
  const RsCell c = cells[blockIdx.x / rc];  // by value: the stores below cannot alias it
  const int64_t r = blockIdx.x % rc;
  const uint32_t* w = c.words + c.rep_off[r];
  const int64_t n = c.n, k = c.k, nsim = c.nsim;
  const int tid = threadIdx.x;
  if (c.family == RS_FAMILY_HRS_INT) {
    // run_INT_once (real-data-sims.R:375-402): rLap(n), rLap(1), mixquant(nsim = 2000)
    double* ll = c.lap_local + r * n;
    for (int64_t i = tid; i < n; i += 256) ll[i] = rs_lap(w[i]);
    if (tid == 0) c.lap_scalar[r] = rs_lap(w[n]);
    const uint32_t* wz = w + n + 1;
    const uint32_t* wb = c.words + c.exp_end[r];
    const double* ev = c.expv + r * nsim;
    for (int64_t jj = tid; jj < nsim; jj += 256) {
      c.mix_z[r * nsim + jj] = rs_norm(wz[2 * jj], wz[2 * jj + 1]);
      c.mix_l[r * nsim + jj] = (rs_unif(wb[jj]) < 0.5) ? -ev[jj] : ev[jj];
    }
    return;
  }
  double* X = c.X + r * n;
  double* Y = c.Y + r * n;
  // 1. DGP
  int64_t o = c.dgp_words;
  if (c.dgp == DCOR_DGP_MIX_GAUSSIAN) {
    // gen_mix_gaussian (ver-cor-subG.R:113-136): labels <- rbinom(n, 1, pi_mix); rows of
    // rbind(mvrnorm(n0, mu0, S0), mvrnorm(n1, mu1, S1)) in sample.int(n) order; clip to [-1, 1]
    extern __shared__ uint32_t rs_msm[];
    __shared__ unsigned long long n0s;
    uint16_t* xs = reinterpret_cast<uint16_t*>(rs_msm);
    uint32_t* mark = rs_msm + ((n + 1) & ~1ll) / 2;
    if (tid == 0) n0s = 0;
    for (int64_t i = tid; i < n; i += 256) xs[i] = (uint16_t)i;
    for (int64_t i = tid; i < (n + 31) / 32; i += 256) mark[i] = 0u;
    __syncthreads();
    unsigned long long z0 = 0;
    for (int64_t i = tid; i < n; i += 256) {
      const uint32_t lab = c.lab_on ? (((rs_unif(w[i]) < c.lab_q) ? 0u : 1u) ^ (uint32_t)c.lab_inv)
                                    : (uint32_t)c.lab_const;
      z0 += (lab == 0);
    }
    atomicAdd(&n0s, z0);
    int32_t* y = c.shuf + r * n;
    const int64_t nlab = c.lab_on ? n : 0;
    __syncthreads();
    if (tid < 64) rs_shuffle_wave(w + nlab + 4 * n, n, xs, mark, y, tid);
    __syncthreads();
    __threadfence_block();
    const int64_t n0 = n0s, n1 = n - n0;
    const uint32_t* wz = w + nlab;      // normals: 2 n0 (component 0) then 2 n1 (component 1)
    for (int64_t i = tid; i < n; i += 256) {
      const int64_t src = y[i];
      double z1, z2, xv, yv;
      if (src < n0) {
        z1 = rs_norm(wz[2 * src], wz[2 * src + 1]);
        z2 = rs_norm(wz[2 * (n0 + src)], wz[2 * (n0 + src) + 1]);
        xv = c.mmu0[0] + ((0.0 + z1 * c.mA0[0]) + z2 * c.mA0[1]);
        yv = c.mmu0[1] + ((0.0 + z1 * c.mA0[2]) + z2 * c.mA0[3]);
      } else {
        const int64_t t = src - n0, b = 2 * n0;
        z1 = rs_norm(wz[2 * (b + t)], wz[2 * (b + t) + 1]);
        z2 = rs_norm(wz[2 * (b + n1 + t)], wz[2 * (b + n1 + t) + 1]);
        xv = c.mmu1[0] + ((0.0 + z1 * c.mA1[0]) + z2 * c.mA1[1]);
        yv = c.mmu1[1] + ((0.0 + z1 * c.mA1[2]) + z2 * c.mA1[3]);
      }
      xv = (xv > 1.0) ? 1.0 : xv; xv = (xv < -1.0) ? -1.0 : xv;   // pmax(pmin(out, 1), -1)
      yv = (yv > 1.0) ? 1.0 : yv; yv = (yv < -1.0) ? -1.0 : yv;
      X[i] = xv;
      Y[i] = yv;
    }
    o = c.shuf_end[r] - c.rep_off[r];
  } else if (c.dgp == DCOR_DGP_GAUSSIAN) {
    // matrix(rnorm(2n), n): column 1 = draws 0..n-1, column 2 = draws n..2n-1;
    // mu + (V diag(sqrt(ev))) %*% t(Z) in dgemm's order
    for (int64_t i = tid; i < n; i += 256) {
      const double z1 = rs_norm(w[2 * i], w[2 * i + 1]);
      const double z2 = rs_norm(w[2 * (n + i)], w[2 * (n + i) + 1]);
      X[i] = c.mu[0] + ((0.0 + z1 * c.A[0]) + z2 * c.A[1]);
      Y[i] = c.mu[1] + ((0.0 + z1 * c.A[2]) + z2 * c.A[3]);
    }
  } else if (c.dgp == DCOR_DGP_BERNOULLI) {
    for (int64_t i = tid; i < n; i += 256) {   // u <- runif(n); v <- runif(n)
      const double u = rs_unif(w[i]), v = rs_unif(w[n + i]);
      const double x = (u < 0.5) ? 1.0 : 0.0;
      X[i] = x;
      Y[i] = (x == 0.0) ? ((v < c.bern_t0) ? 1.0 : 0.0) : ((v < c.bern_t1) ? 1.0 : 0.0);
    }
  } else {  // bounded factor: U, E1, E2 <- runif(n, -c, c); a == b draws nothing
    const int64_t oe1 = c.u_draw ? n : 0, oe2 = oe1 + (c.e_draw ? n : 0);
    for (int64_t i = tid; i < n; i += 256) {
      const double U = c.u_draw ? (-c.cU + (c.cU - -c.cU) * rs_unif(w[i])) : c.u_const;
      const double E1 = c.e_draw ? (-c.cE + (c.cE - -c.cE) * rs_unif(w[oe1 + i])) : c.e_const;
      const double E2 = c.e_draw ? (-c.cE + (c.cE - -c.cE) * rs_unif(w[oe2 + i])) : c.e_const;
      X[i] = U + E1;
      Y[i] = U + E2;
    }
  }
  double* lx = c.lap_x + r * k;
  double* ly = c.lap_y + r * k;
  if (c.family == DCOR_FAMILY_SIGN) {
    // 2. ci_NI_signbatch: standardisation (4), rLap(k) X, rLap(k) Y
    // 3. ci_INT_signflip: standardisation (4), rbinom(n, 1, p), Z
    const int64_t nrm = c.normalise ? 4 : 0;
    if (tid < 4) {
      c.lap_nsc[r * 4 + tid] = c.normalise ? rs_lap(w[o + tid]) : 0.0;
      c.lap_isc[r * 4 + tid] = c.normalise ? rs_lap(w[o + nrm + 2 * k + tid]) : 0.0;
    }
    for (int64_t i = tid; i < k; i += 256) {
      lx[i] = rs_lap(w[o + nrm + i]);
      ly[i] = rs_lap(w[o + nrm + k + i]);
    }
    o += 2 * nrm + 2 * k;
    uint32_t* fw = c.flips + r * ((n + 31) / 32);
    for (int64_t b = tid; b < (n + 31) / 32; b += 256) {
      uint32_t bits = 0;
      for (int t = 0; t < 32; ++t) {
        const int64_t i = b * 32 + t;
        if (i >= n) break;
        // rbinom(1, pp): p = min(pp, 1 - pp), ix = (u >= 1 - p), S = pp > .5 ? 1 - ix : ix
        uint32_t s = c.flip_const;
        if (c.flip_on) s = ((rs_unif(w[o + i]) < c.flip_q) ? 0u : 1u) ^ (uint32_t)c.flip_inv;
        bits |= s << t;
      }
      fw[b] = bits;
    }
    o += c.flip_on ? n : 0;
  } else {
    // 2. correlation_NI_subG: rLap(k) X, rLap(k) Y;  3. ci_INT_subG: rLap(n), rLap(1)
    for (int64_t i = tid; i < k; i += 256) {
      lx[i] = rs_lap(w[o + i]);
      ly[i] = rs_lap(w[o + k + i]);
    }
    o += 2 * k;
    double* ll = c.lap_local + r * n;
    for (int64_t i = tid; i < n; i += 256) ll[i] = rs_lap(w[o + i]);
    o += n;
  }
  if (tid == 0) c.lap_scalar[r] = rs_lap(w[o]);
  o += 1;
  // 4. mixquant: rnorm(nsim), rexp(nsim) (walked by k_rs_stream), rbinom(nsim, 1, .5)
  double* mz = c.mix_z + r * nsim;
  double* ml = c.mix_l + r * nsim;
  if (c.has_mix) {
    const uint32_t* wb = c.words + c.exp_end[r];
    const double* ev = c.expv + r * nsim;
    for (int64_t jj = tid; jj < nsim; jj += 256) {
      mz[jj] = rs_norm(w[o + 2 * jj], w[o + 2 * jj + 1]);
      const double e = ev[jj];
      ml[jj] = (rs_unif(wb[jj]) < 0.5) ? -e : e;   // e * (2 * rbinom(1, .5) - 1)
    }
  } else {
    for (int64_t jj = tid; jj < nsim; jj += 256) { mz[jj] = 0.0; ml[jj] = 0.0; }
  }
}

// ------------------------------------------------------------ k_rs_hrs_ni ---
// run_NI_once (real-data-sims.R:357-373) on R's stream: set.seed(seeds[r]), then
// correlation_NI_subG's draws -- idx <- sample.int(n, k*m) (:131) and rLap(k) twice
// (:136-137).  sample.int without replacement is do_sample's partial Fisher-Yates over
// x[0..n) with R_unif_index's rejection sampling (rbits: 16 bits per word), inherently
// sequential: one wave per run keeps x[] in LDS and walks it in uniform control flow;
// MT blocks are regenerated wave-parallel.  Then the 2k Laplace words, lane-parallel.
__global__ __launch_bounds__(64) void k_rs_hrs_ni(const int32_t* __restrict__ seeds, int64_t n,
                                                  int64_t km, int64_t k, int32_t* __restrict__ perm,
                                                  double* __restrict__ lx, double* __restrict__ ly) {
  extern __shared__ uint32_t rs_sm[];
  uint32_t* mt = rs_sm;
  uint32_t* wb = rs_sm + RS_N;
  uint16_t* x = reinterpret_cast<uint16_t*>(rs_sm + 2 * RS_N);  // n <= 65536: 2 B per index,
                                                                 // so 3 runs share a CU
  const int lane = threadIdx.x;
  const int64_t r = blockIdx.x;
  rs_seed_mt(mt, seeds[r], lane);
  for (int64_t i = lane; i < n; i += 64) x[i] = (uint16_t)i;
  int pos = RS_N;                          // set.seed leaves mti = 624: first use regenerates
  auto refill = [&]() {
    __syncthreads();
    rs_mt_block(mt, lane);
    for (int t = lane; t < RS_N; t += 64) wb[t] = rs_temper(mt[t]);
    __syncthreads();
    pos = 0;
  };
  __syncthreads();
  RS_G int32_t* const pr = (RS_G int32_t*)(perm + r * km);
  // Fast path (one word per attempt, bits <= 15): a window of up to 64 words is evaluated
  // lane-parallel.  With dn the remaining size, v < dn - W accepts and v >= dn rejects
  // whatever the window's earlier draws did; any other v sends the window to the exact
  // in-order path.  The accepted draws' swaps x[j_t] <- x[dn-1-t] then run in parallel
  // unless two j coincide or a j hits one of the window's tail slots (an LDS bitmap
  // detects both); otherwise in order.  Both paths give do_sample's exact sequence.
  uint32_t* mark = reinterpret_cast<uint32_t*>(x + ((n + 1) & ~1ll));
  for (int64_t q = lane; q < (n + 31) / 32; q += 64) mark[q] = 0u;
  __syncthreads();
  int64_t i = 0, dn = n;
  auto take_one = [&](uint64_t v) {        // accept v as the next index (lane 0 swaps)
    if (lane == 0) {
      const int32_t j = (int32_t)v;
      pr[i] = (int32_t)x[j];               // iy[i] = x[j] + 1 (0-based here)
      x[j] = x[dn - 1];
    }
    ++i;
    --dn;
  };
  while (i < km) {
    i = rs_u64(i); dn = rs_u64(dn);
    if (pos == RS_N) refill();
    pos = rs_u(pos);
    const int bits = (dn <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(dn - 1));  // ceil(log2 dn)
    const int W = (RS_N - pos < 64) ? RS_N - pos : 64;
    const int bits_lo = (dn - W <= 1) ? 0 : 64 - __builtin_clzll((unsigned long long)(dn - W - 1));
    if (bits > 15 || bits != bits_lo || dn <= 64) {
      // exact scalar attempt: R_unif_index = rbits(bits) until < dn
      const uint64_t mask = (bits >= 63) ? ~0ull : ((1ull << bits) - 1ull);
      uint64_t v;
      do {
        v = 0;
        for (int nn = 0; nn <= bits; nn += 16) {
          if (pos == RS_N) refill();
          pos = rs_u(pos);
          v = 65536ull * v + (wb[pos] >> 16);  // floor(unif_rand() * 65536)
          ++pos;
        }
        v &= mask;
      } while ((int64_t)v >= dn);
      take_one(v);
      continue;
    }
    const uint32_t mask = (1u << bits) - 1u;
    const bool in = lane < W;
    const int64_t v = in ? (int64_t)((wb[pos + (in ? lane : 0)] >> 16) & mask) : 0;
    const bool sure_acc = in && v < dn - W, sure_rej = in && v >= dn;
    const uint64_t amb = __ballot(in && !sure_acc && !sure_rej);
    if (amb) {                             // exact, in order through the window
      int used = 0;
      for (int l = 0; l < W && i < km; ++l) {
        const int64_t vl = (int64_t)(uint32_t)rs_rl((int)v, l);
        used = l + 1;
        if (vl < dn) take_one((uint64_t)vl);
      }
      pos += used;
      continue;
    }
    uint64_t A = __ballot(sure_acc);
    int used = W;
    const int64_t need = km - i;
    if ((int64_t)__builtin_popcountll(A) > need) {   // the sample ends inside this window
      uint64_t keep = A;
      for (int64_t c = __builtin_popcountll(A); c > need; --c) keep &= ~(1ull << (63 - __builtin_clzll(keep)));
      A = keep;
      used = 64 - __builtin_clzll(A);
    }
    const int B = __builtin_popcountll(A);
    const bool acc = (A >> lane) & 1ull;
    const int t = __builtin_popcountll(A & ((1ull << lane) - 1ull));
    const int64_t Lt = dn - 1 - t;
    bool clash = false;
    if (acc) clash = (atomicOr(&mark[v >> 5], 1u << (v & 31)) >> (v & 31)) & 1u;
    __syncthreads();
    if (acc && Lt != v) clash |= (mark[Lt >> 5] >> (Lt & 31)) & 1u;
    const bool serial = __ballot(clash) != 0ull;
    __syncthreads();
    if (acc) atomicAnd(&mark[v >> 5], ~(1u << (v & 31)));
    if (!serial) {
      uint16_t a = 0, b = 0;
      if (acc) { a = x[v]; b = x[Lt]; }
      __syncthreads();
      if (acc) { pr[i + t] = (int32_t)a; x[v] = b; }
      i += B;
      dn -= B;
    } else {
      for (uint64_t rest = A; rest; rest &= rest - 1ull) {
        const int l = __builtin_ctzll(rest);
        take_one((uint64_t)(uint32_t)rs_rl((int)v, l));
      }
    }
    __syncthreads();
    pos += used;
  }
  // rLap(k) for X, then rLap(k) for Y: the next 2k words
  int64_t t0 = 0;
  const int64_t tot = 2 * k;
  while (t0 < tot) {
    if (pos == RS_N) refill();
    pos = rs_u(pos);
    const int64_t take = ((int64_t)(RS_N - pos) < tot - t0) ? (int64_t)(RS_N - pos) : tot - t0;
    for (int64_t q = lane; q < take; q += 64) {
      const double l = rs_lap(wb[pos + q]);
      const int64_t t = t0 + q;
      if (t < k) lx[r * k + t] = l; else ly[r * k + (t - k)] = l;
    }
    pos += (int)take;
    t0 += take;
  }
}

size_t rs_hrs_ni_lds_bytes(int64_t n) {
  return (size_t)(2 * RS_N) * 4 + (size_t)((n + 1) & ~1ll) * 2 + (size_t)((n + 31) / 32) * 4;
}

int launch_rs_hrs_ni(const int32_t* d_seeds, int64_t runs, int64_t n, int64_t km, int64_t k,
                     int32_t* perm, double* lx, double* ly, void* stream) {
  const size_t lds = rs_hrs_ni_lds_bytes(n);
  // per call: the attribute is per device, and one process may drive several GPUs
  const hipError_t e = hipFuncSetAttribute((const void*)k_rs_hrs_ni,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k_rs_hrs_ni, dim3((unsigned)runs), dim3(64), lds, (hipStream_t)stream, d_seeds,
                     n, km, k, perm, lx, ly);
  return (int)hipGetLastError();
}

int launch_rs_stream(RsCell* d_cells, int ncells, int32_t rc, void* stream) {
  hipLaunchKernelGGL(k_rs_stream, dim3(ncells), dim3(RS_STREAM_NT), 0, (hipStream_t)stream, d_cells, rc);
  return (int)hipGetLastError();
}

int launch_rs_materialise(const RsCell* d_cells, int ncells, int32_t rc, void* stream, size_t lds) {
  if (lds > 64 * 1024) {
    // per call: the attribute is per device, and one process may drive several GPUs
    const hipError_t e = hipFuncSetAttribute((const void*)k_rs_materialise,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k_rs_materialise, dim3((unsigned)(ncells * rc)), dim3(256), lds,
                     (hipStream_t)stream, d_cells, rc);
  return (int)hipGetLastError();
}

}  // namespace dcor
