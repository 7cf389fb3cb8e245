// dcor_device.h -- gfx950 device primitives for the DP-correlation Monte-Carlo engine.
//
//  * Philox4x32-10 counter RNG (key = per-cell seed, counter = (index, rep, site, 0)),
//    the draw-site contract of include/dcor.h.
//  * Uniform / normal / Laplace transforms in fp64 built only from IEEE basic ops and
//    explicit fma(), compiled with -ffp-contract=off, so a draw is a pure function of
//    (seed, rep, site, index) -- identical on any GPU count and reproducible bit for bit
//    by the CPU restatement in oracle/.
//  * Wave64 / workgroup reductions (DPP shuffles + LDS), double-double accumulators.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dcor.h"

#define DCOR_TABLE_ATTR __device__
#include "dcor_tables.h"

#define DCOR_BLOCK 256
#define DCOR_WAVES (DCOR_BLOCK / 64)

namespace dcor {

// ------------------------------------------------------------------ Philox
struct U4 { uint32_t w0, w1, w2, w3; };

// a ^ b ^ k in one gfx950 v_bitop3_b32 (truth table 0x96).  The builtin, not inline asm: the
// compiler does not form bitop3 from a ^ b ^ k by itself, and after an asm statement it pads with
// a hazard s_nop (7.5 per pass-1 sample).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
  return __builtin_amdgcn_bitop3_b32(a, b, k, 0x96);
}

__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
  // 32x32->64 products map to one v_mad_u64_u32 each (hi and lo together); the two
  // xors of each output word are one v_bitop3_b32.
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0), n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

__device__ __forceinline__ U4 draw(uint32_t idx, uint32_t rep, uint32_t site, uint32_t k0,
                                   uint32_t k1) {
  return philox(idx, rep, site, 0u, k0, k1);
}

// (2x+1) * 2^-53 with x the top 52 bits of (a, b): in (0, 1), exact.  Built from bits:
// as_double(1.x) - (1 - 2^-53) is exact (Sterbenz), one v_add_f64.
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  // high word 0x3ff00000 | a >> 12, low word a << 20 | b >> 12: two v_alignbit_b32
  const uint32_t lo = __builtin_amdgcn_alignbit(a, b, 12u);
  const uint32_t hi = __builtin_amdgcn_alignbit(0x3ffu, a, 12u);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo)) - (1.0 - 0x1p-53);
}

// Division-free log for positive normal x (same code as oracle/orc_log): x = 2^k z with
// z in [0.6875, 1.375), r = fma(z, 1/c, -1) against a 256-entry table, log x = k ln2 +
// log c + log1p(r) with a degree-6 polynomial (|r| < 2^-9).  ~12 fp64 ops; <= 2 ulp.
// `tab` is dcor_log8_tab or a copy of it in LDS: a kernel that streams HBM reads its table from LDS,
// because s_waitcnt vmcnt waits in issue order -- a table gather from global memory would wait for
// every stream load issued before it, which defeats the stream's prefetch.
__device__ __forceinline__ double dlog_t(double x, const double2* tab) {
  // The offset's low word is 0, so the reduction lives in the high word (32-bit ops only).
  const uint64_t ix = (uint64_t)__double_as_longlong(x);
  const uint32_t hi = (uint32_t)(ix >> 32), tmp = hi - 0x3fe60000u;
  const int i = (int)((tmp >> 12) & 255u);
  const int k = (int)tmp >> 20;
  const double z = __longlong_as_double(
      (long long)(((uint64_t)(hi - (tmp & 0xfff00000u)) << 32) | (uint32_t)ix));
  const double2 e = tab[i];
  const double invc = e.x, logc = e.y;
  const double r = fma(z, invc, -1.0), kd = (double)k, r2 = r * r;
  double p = fma(r, DCOR_LOG1P_C6, DCOR_LOG1P_C5);
  p = fma(r, p, DCOR_LOG1P_C4);
  p = fma(r, p, DCOR_LOG1P_C3);
  p = fma(r, p, DCOR_LOG1P_C2);
  const double w = fma(kd, DCOR_LN2_HI, logc), lo = fma(kd, DCOR_LN2_LO, r2 * p);
  return w + (r + lo);
}
__device__ __forceinline__ double dlog(double x) {
  return dlog_t(x, reinterpret_cast<const double2*>(dcor_log8_tab));
}
// dcor_log8_tab into LDS (256 double2, 4 KB) by the calling workgroup; the caller synchronises.
__device__ __forceinline__ void log_tab_to_lds(double2* lt, int nthreads) {
  for (int e = threadIdx.x; e < 256; e += nthreads) lt[e] = make_double2(dcor_log8_tab[e][0], dcor_log8_tab[e][1]);
}

// sin(pi t), cos(pi t) for t in [0, 2], given t64 = 64 t (same code as oracle/orc_sincospi):
// j = rint(t64), d = (t64 - j) pi / 64 (|d| <= pi/128), angle addition with the 129-entry
// table of sin / cos(pi j / 64) and degree-7 / 6 polynomials in d.  ~18 fp64 ops.
__device__ __forceinline__ void dsincospi64(double t64, double* sp, double* cp) {
  const double jd = rint(t64), r = t64 - jd;
  const int j = (int)jd;
  const double d = fma(r, DCOR_PI64_HI, r * DCOR_PI64_LO), z = d * d;
  const double sd = fma(d * z, fma(z, fma(z, DCOR_SIN_S7, DCOR_SIN_S5), DCOR_SIN_S3), d);
  const double cm1 = z * fma(z, fma(z, DCOR_COS_C6, DCOR_COS_C4), DCOR_COS_C2);
  const double S = dcor_sincospi_tab[j][0], C = dcor_sincospi_tab[j][1];
  *sp = fma(S, cm1, fma(C, sd, S));
  *cp = fma(C, cm1, fma(-S, sd, C));
}

__device__ __forceinline__ double unit_laplace_t(double u, const double2* tab) {
  const double up = u - 0.5;
  const double g = dlog_t(1.0 - 2.0 * fabs(up), tab);
  return (up > 0) ? -g : g;
}
__device__ __forceinline__ double unit_laplace(double u) {
  return unit_laplace_t(u, reinterpret_cast<const double2*>(dcor_log8_tab));
}

// Correctly rounded sqrt for positive normal x >= 2^-767 (LLVM's own f64 sqrt lowering
// without its tiny-input scaling and 0/inf class fix-ups): rsq + two Goldschmidt steps +
// two fma residual corrections.  Bit-identical to IEEE sqrt on that range (the draws tests
// compare against the CPU's sqrt).  Box-Muller's -2 log(u) >= 2.2e-16 always.
__device__ __forceinline__ double sqrt_pos(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}

// Box-Muller polar pair: radius r = sqrt(-2 log u1) and (cos, sin)(2 pi u2).
__device__ __forceinline__ void normal_polar(const U4& w, double* r, double* s, double* c) {
  const double u1 = u53(w.w0, w.w1);
  const double u2 = u53(w.w2, w.w3);
  *r = sqrt_pos(-2.0 * dlog(u1));
  dsincospi64(u2 * 128.0, s, c);  // t = 2 u2, 64 t exact
}

// The same pair from two 32-bit words (the Gaussian DGP's contract: two samples per Philox
// block): u1 = (a + 1/2) 2^-32 and 64 t = 128 u2 = (b + 1/2) 2^-25, both exact (one v_cvt_f64_u32
// and one fma each).  Radius cut-off sqrt(-2 log 2^-33) = 6.76 (P(R > 6.76) = 1.1e-10).
__device__ __forceinline__ void normal_polar32(uint32_t a, uint32_t b, double* r, double* s,
                                               double* c) {
  const double u1 = fma((double)a, 0x1p-32, 0x1p-33);
  const double t64 = fma((double)b, 0x1p-25, 0x1p-26);
  *r = sqrt_pos(-2.0 * dlog(u1));
  dsincospi64(t64, s, c);
}

// ------------------------------------------------------------- ziggurat
// The Gaussian DGP's normals (Marsaglia & Tsang's ziggurat, 1024 layers, tables in
// dcor_tables.h; same code as oracle/orc_zig).  A draw takes a 32-bit word A and a 16-bit field
// H: j = H >> 5 picks layer L = j >> 1 and sign j & 1, and |u| = (2 x + 1) 2^-38 with the 37 bits
// x = A : H[4:0].  d = 1 + |u| is built from bits (Y = H[4:0] << 27 | 1 << 26 carries the low
// mantissa), so x = fma(d, SX, -SX) = round(|u| SX) with SX = (-1)^s X[L] in one fma; the draw is
// accepted on the fast path when |x| < X[L+1] (the strip lies under the density there): 99.57%
// of draws, so 0.85% of samples (two draws each) take the slow path.
static_assert(DCOR_ZIG_N == 1024, "zig_y*/zig_j* split H as 11 layer-and-sign bits : 5 magnitude bits");
__device__ __forceinline__ double zig_d(uint32_t A, uint32_t Y) {
  const uint32_t hi = __builtin_amdgcn_alignbit(0x3ffu, A, 12u);
  const uint32_t lo = __builtin_amdgcn_alignbit(A, Y, 12u);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint32_t zig_y_lo(uint32_t H16) { return (H16 << 27) | 0x4000000u; }
// z1 takes H = w2 & 0xffff, z2 takes H = w2 >> 16
__device__ __forceinline__ uint32_t zig_y1(uint32_t w2) { return (w2 << 27) | 0x4000000u; }
__device__ __forceinline__ uint32_t zig_y2(uint32_t w2) { return ((w2 << 11) & 0xf8000000u) | 0x4000000u; }
__device__ __forceinline__ uint32_t zig_j1(uint32_t w2) { return (w2 >> 5) & 2047u; }
__device__ __forceinline__ uint32_t zig_j2(uint32_t w2) { return w2 >> 21; }

// The full draw from attempt 0's (A, H): fast test, then the wedge test (L >= 1) against
// f(x) = exp(-x^2/2) compared in logs, or the base layer's tail (L = 0: Marsaglia's x = -log(U1)/r,
// accepted when -2 log(U2) > x^2), and otherwise a new attempt from block (i, rep, ZIG, 2a + which).
// Entry j of the layer table: from the caller's LDS copy `zt` when it has one (pass 1's drain:
// a global load there would wait behind every slab store the wave has in flight), else global.
__device__ __forceinline__ double2 zig_entry(const double2* zt, uint32_t j) {
  return zt ? zt[j] : make_double2(dcor_zig_tab[j][0], dcor_zig_tab[j][1]);
}
__device__ __forceinline__ double zig_slow(uint32_t i, uint32_t which, uint32_t rep, uint32_t k0,
                                        uint32_t k1, uint32_t A, uint32_t H, const double2* zt = nullptr) {
  for (uint32_t a = 0;; ++a) {
    const U4 q = philox(i, rep, DCOR_SITE_ZIG, 2u * a + which, k0, k1);
    if (a > 0) { A = q.w0; H = q.w1 & 0xffffu; }
    const uint32_t j = H >> 5, L = j >> 1;
    const double2 t = zig_entry(zt, j);
    const double x = fma(zig_d(A, zig_y_lo(H)), t.x, -t.x);
    if (fabs(x) < t.y) return x;
    if (L == 0) {
      for (uint32_t t = 0;; ++t) {
        const U4 b = philox(i, rep, DCOR_SITE_ZIG_TAIL, 2u * t + which, k0, k1);
        const double xt = -dlog(u53(b.w0, b.w1)) * DCOR_ZIG_RINV;
        const double yt = -dlog(u53(b.w2, b.w3));
        if (yt + yt > xt * xt) return (j & 1u) ? -(DCOR_ZIG_R + xt) : (DCOR_ZIG_R + xt);
      }
    }
    const double y = fma(u53(q.w2, q.w3), dcor_zig_wedge[L][1], dcor_zig_wedge[L][0]);
    if (dlog(y) < -0.5 * (x * x)) return x;
  }
}

// One draw: the fast path inline, the rest out of line.
__device__ __forceinline__ double zig_draw(uint32_t i, uint32_t which, uint32_t rep, uint32_t k0,
                                           uint32_t k1, uint32_t A, uint32_t H, const double2* zt = nullptr) {
  const uint32_t j = H >> 5;
  const double2 t = zig_entry(zt, j);
  const double x = fma(zig_d(A, zig_y_lo(H)), t.x, -t.x);
  if (fabs(x) < t.y) return x;
  return zig_slow(i, which, rep, k0, k1, A, H, zt);
}

// mu + A z of MASS::mvrnorm (vert-cor.R:389-394) for z = (z1, z2) (same code as oracle/orc_mvn_z).
__device__ __forceinline__ void mvn_z(double z1, double z2, double mu0, double mu1, double a00,
                                      double a01, double a10, double a11, double* x, double* y) {
  *x = fma(a00, z1, fma(a01, z2, mu0));
  *y = fma(a10, z1, fma(a11, z2, mu1));
}

__device__ __forceinline__ void normal_pair(const U4& w, double* z1, double* z2) {
  double r, s, c;
  normal_polar(w, &r, &s, &c);
  *z1 = r * c;
  *z2 = r * s;
}

// mu + A (r c, r s) of MASS::mvrnorm (vert-cor.R:389-394) as one fused form per coordinate:
// fma(r, fma(a01, s, a00 c), mu0) (same code as oracle/orc_mvn_polar).
__device__ __forceinline__ void mvn_polar(double r, double s, double c, double mu0, double mu1,
                                          double a00, double a01, double a10, double a11,
                                          double* x, double* y) {
  *x = fma(r, fma(a01, s, a00 * c), mu0);
  *y = fma(r, fma(a11, s, a10 * c), mu1);
}

// ------------------------------------------------------------- R helpers
__device__ __forceinline__ double rclip(double x, double L) {  // pmax(pmin(x, L), -L)
  // v_min_f64 + v_max_f64 (which return the non-NaN operand), then R's NaN passed through:
  // the same value for every x as the compare-and-select form, in 5 VALU instead of 9
  const double t = fmax(fmin(x, L), -L);
  return (x != x) ? x : t;
}
// Same clip for inputs known not to be NaN (generated samples): one v_min + one v_max.
__device__ __forceinline__ double rclip_fin(double x, double L) { return fmax(fmin(x, L), -L); }
__device__ __forceinline__ double rclip_lohi(double x, double lo, double hi) {  // pmin(pmax(x,lo),hi)
  if (x != x) return x;
  const double t = (x > lo) ? x : lo;
  return (t < hi) ? t : hi;
}
__device__ __forceinline__ double rmax(double a, double b) {
  return (a != a || b != b) ? __longlong_as_double(0x7ff8000000000000LL) : (a > b ? a : b);
}
__device__ __forceinline__ double rmin(double a, double b) {
  return (a != a || b != b) ? __longlong_as_double(0x7ff8000000000000LL) : (a < b ? a : b);
}
__device__ __forceinline__ double dnan() { return __longlong_as_double(0x7ff8000000000000LL); }

// ------------------------------------------------------- double-double
struct DD { double hi, lo; };
__device__ __forceinline__ DD two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  return DD{s, e};
}
__device__ __forceinline__ void dd_acc(DD& acc, double x) {  // acc += x
  const DD t = two_sum(acc.hi, x);
  const double lo = acc.lo + t.lo;
  const DD r = two_sum(t.hi, lo);
  acc = r;
}
// Compensated accumulate (TwoSum into hi, rounding errors summed in lo, no
// renormalisation): 7 flops instead of dd_acc's 13; error ~ n * 2^-106 relative.
__device__ __forceinline__ void ks_acc(DD& acc, double x) {
  const double s = acc.hi + x;
  const double bb = s - acc.hi;
  acc.lo += (acc.hi - (s - bb)) + (x - bb);
  acc.hi = s;
}
__device__ __forceinline__ DD dd_add(DD a, DD b) {
  const DD s = two_sum(a.hi, b.hi);
  const DD t = two_sum(a.lo, b.lo);
  double lo = s.lo + t.hi;
  DD r = two_sum(s.hi, lo);
  lo = r.lo + t.lo;
  return two_sum(r.hi, lo);
}
__device__ __forceinline__ DD two_prod(double a, double b) {
  const double p = a * b;
  return DD{p, fma(a, b, -p)};
}
__device__ __forceinline__ DD dd_mul_d(DD a, double b) {
  DD p = two_prod(a.hi, b);
  p.lo = fma(a.lo, b, p.lo);
  return two_sum(p.hi, p.lo);
}
__device__ __forceinline__ DD dd_mul(DD a, DD b) {
  DD p = two_prod(a.hi, b.hi);
  p.lo = fma(a.hi, b.lo, p.lo);
  p.lo = fma(a.lo, b.hi, p.lo);
  return two_sum(p.hi, p.lo);
}
__device__ __forceinline__ DD dd_div_d(DD a, double b) {
  const double q1 = a.hi / b;
  const DD p = two_prod(q1, b);
  const DD r = dd_add(a, DD{-p.hi, -p.lo});
  const double q2 = r.hi / b;
  return two_sum(q1, q2);
}
__device__ __forceinline__ DD dd_neg(DD a) { return DD{-a.hi, -a.lo}; }

// sample variance (n-1) from double-double sum and sum of squares
__device__ __forceinline__ double dd_var(DD s1, DD s2, double n) {
  if (!(n >= 2)) return dnan();
  const DD mean = dd_div_d(s1, n);
  const DD c = dd_add(s2, dd_neg(dd_mul(s1, mean)));
  const DD v = dd_div_d(c, n - 1.0);
  return v.hi + v.lo;
}

// ------------------------------------------------------------ reductions
// Lane exchanges for the wave all-reduces, without the LDS crossbar (__shfl_xor compiles to
// ds_bpermute_b32 plus index arithmetic): DPP within rows of 16 lanes, the gfx950 permlane swaps
// across rows.  lane_dpp<CTRL>: the value of lane quad_perm / mirror partner; lane_swap<32 | 16>:
// the value pair {own, partner} for partner = lane ^ 32 (permlane32_swap) or lane ^ 16
// (permlane16_swap), in an order that depends on the lane -- callers combine the pair with a
// commutative operation.
template <int CTRL>
__device__ __forceinline__ uint32_t lane_dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t lane_dpp_u64(uint64_t v) {
  return ((uint64_t)lane_dpp_u32<CTRL>((uint32_t)(v >> 32)) << 32) | lane_dpp_u32<CTRL>((uint32_t)v);
}
template <int W>
__device__ __forceinline__ void lane_swap_u32(uint32_t v, uint32_t& a, uint32_t& b) {
  if constexpr (W == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    a = r[0]; b = r[1];
  } else {
    static_assert(W == 16, "permlane16_swap or permlane32_swap");
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    a = r[0]; b = r[1];
  }
}
template <int W>
__device__ __forceinline__ void lane_swap_u64(uint64_t v, uint64_t& a, uint64_t& b) {
  uint32_t al, bl, ah, bh;
  lane_swap_u32<W>((uint32_t)v, al, bl);
  lane_swap_u32<W>((uint32_t)(v >> 32), ah, bh);
  a = ((uint64_t)ah << 32) | al;
  b = ((uint64_t)bh << 32) | bl;
}
// The butterfly of the all-reduces: lanes i^1, i^2 (quad_perm), 7-i within 8 (row_half_mirror),
// 15-i within 16 (row_mirror), rows 0<->1 and 2<->3 (permlane16_swap), halves (permlane32_swap).
// Each step pairs two lanes that hold partials over disjoint lane sets, so every lane ends with the
// op over all 64; with a commutative op both lanes of a pair compute the same bits, so all lanes
// agree.  Take / put convert the reduced type to and from 64-bit words.
template <class T, class Get, class Put, class Op>
__device__ __forceinline__ T wave_allreduce(T v, Get get, Put put, Op op) {
  v = op(v, put(lane_dpp_u64<0xB1>(get(v))));
  v = op(v, put(lane_dpp_u64<0x4E>(get(v))));
  v = op(v, put(lane_dpp_u64<0x141>(get(v))));
  v = op(v, put(lane_dpp_u64<0x140>(get(v))));
  uint64_t a, b;
  lane_swap_u64<16>(get(v), a, b);
  v = op(put(a), put(b));
  lane_swap_u64<32>(get(v), a, b);
  return op(put(a), put(b));
}
// Inclusive prefix sum over the wave's 64 lanes by DPP (row shifts, then the row broadcasts of lane
// 15 and 31): exact, no LDS crossbar.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return v;
}
__device__ __forceinline__ uint64_t d_bits(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ double d_from(uint64_t b) { return __longlong_as_double((long long)b); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ long long wave_sum_i(long long v) {
  return wave_allreduce(v, [](long long x) { return (uint64_t)x; }, [](uint64_t b) { return (long long)b; },
                        [](long long x, long long y) { return x + y; });
}
// Butterfly all-reduce of a double-double.  Each step keeps the pair unnormalised: two_sum of the
// high parts (exact: s + e = a + b) and the low parts plus e added plainly; one two_sum renormalises
// after the last step.  8 fp64 adds per step instead of dd_add's 26 -- in the premat and HRS kernels
// the reductions were about two thirds of all fp64 adds (profiles/r06w_c5c) -- with an error of
// order 2^-100 of the sum's magnitude.  Every step is symmetric in the two operands (two_sum's
// error term is exact, the plain adds commute), so all lanes hold the same bits unless a sum
// overflows.
__device__ __forceinline__ DD dd_fold_step(DD a, DD b) {   // unnormalised: renormalise at the end
  const DD s = two_sum(a.hi, b.hi);
  return DD{s.hi, (a.lo + b.lo) + s.lo};
}
__device__ __forceinline__ DD wave_sum_dd(DD v) {
  // a DD is two words: the exchanges move hi and lo alike
  v = dd_fold_step(v, DD{d_from(lane_dpp_u64<0xB1>(d_bits(v.hi))), d_from(lane_dpp_u64<0xB1>(d_bits(v.lo)))});
  v = dd_fold_step(v, DD{d_from(lane_dpp_u64<0x4E>(d_bits(v.hi))), d_from(lane_dpp_u64<0x4E>(d_bits(v.lo)))});
  v = dd_fold_step(v, DD{d_from(lane_dpp_u64<0x141>(d_bits(v.hi))), d_from(lane_dpp_u64<0x141>(d_bits(v.lo)))});
  v = dd_fold_step(v, DD{d_from(lane_dpp_u64<0x140>(d_bits(v.hi))), d_from(lane_dpp_u64<0x140>(d_bits(v.lo)))});
  uint64_t ah, bh, al, bl;
  lane_swap_u64<16>(d_bits(v.hi), ah, bh);
  lane_swap_u64<16>(d_bits(v.lo), al, bl);
  v = dd_fold_step(DD{d_from(ah), d_from(al)}, DD{d_from(bh), d_from(bl)});
  lane_swap_u64<32>(d_bits(v.hi), ah, bh);
  lane_swap_u64<32>(d_bits(v.lo), al, bl);
  v = dd_fold_step(DD{d_from(ah), d_from(al)}, DD{d_from(bh), d_from(bl)});
  return two_sum(v.hi, v.lo);
}
__device__ __forceinline__ double wave_min(double v) {
  return wave_allreduce(v, d_bits, d_from, [](double x, double y) { return fmin(x, y); });
}
__device__ __forceinline__ double wave_max(double v) {
  return wave_allreduce(v, d_bits, d_from, [](double x, double y) { return fmax(x, y); });
}
// The per-wave partials of one sum (hi at h[0..nw), lo at l[0..nw)) folded in wave order with the
// same step: the workgroup kernels' last reduction stage, one thread per sum.
template <int NW>
__device__ __forceinline__ DD fold_waves_dd(const double* h, const double* l) {
  DD a{h[0], l[0]};
#pragma unroll
  for (int w = 1; w < NW; ++w) a = dd_fold_step(a, DD{h[w], l[w]});
  return two_sum(a.hi, a.lo);
}

// Workgroup sums of NV doubles; result broadcast to every thread. Scratch: NV*DCOR_WAVES.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) scratch[i * DCOR_WAVES + wv] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < DCOR_WAVES; ++w) s += scratch[i * DCOR_WAVES + w];
    v[i] = s;
  }
  __syncthreads();
}

template <int NV, int NW = DCOR_WAVES>
__device__ __forceinline__ void block_sum_dd(DD (&v)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum_dd(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      scratch[(2 * i) * NW + wv] = v[i].hi;
      scratch[(2 * i + 1) * NW + wv] = v[i].lo;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = fold_waves_dd<NW>(scratch + (2 * i) * NW, scratch + (2 * i + 1) * NW);
  }
  __syncthreads();
}

__device__ __forceinline__ long long block_sum_i(long long v, long long* scratch) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum_i(v);
  if (lane == 0) scratch[wv] = v;
  __syncthreads();
  long long s = 0;
#pragma unroll
  for (int w = 0; w < DCOR_WAVES; ++w) s += scratch[w];
  __syncthreads();
  return s;
}

// ------------------------------------------------------------- mixquant
// R: sort(x)[pos] (0-based pos) with NaN dropped (ver-cor-subG.R:12, vert-cor.R:47).
// Radix select over keys held in registers (VPT per thread): an order-preserving
// uint64 map of each double (NaN -> all ones, above +inf; absent slots likewise), then
// 8-bit digits from the top: a 256-bin LDS histogram of the keys still matching the
// prefix, a block scan to find the digit holding rank pos, stop when that bin holds
// one key.  No sort, no key array in LDS: ~3 passes for 2000 keys.
#define SEL_VPT 8  // MIX_MAX / DCOR_BLOCK
#define SEL_CAND 256  // candidates ranked directly by value_select
struct SelScratch {
  uint32_t hist[256];
  uint32_t wtot[DCOR_WAVES];
  uint32_t sel[3];
  int nan_cnt;
  int ncand;
  unsigned long long key;
  double mm[2 * DCOR_WAVES];
  double cand[SEL_CAND];
};

__device__ __forceinline__ unsigned long long sel_key(double v) {
  if (v != v) return ~0ull;
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double sel_unkey(unsigned long long k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// All threads call; every thread gets the result.  valid = keys that are not NaN/absent.
__device__ __forceinline__ double reg_select(const unsigned long long (&key)[SEL_VPT], int pos,
                                             int valid, SelScratch* sc) {
  if (pos < 0 || pos >= valid) return dnan();  // uniform
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned long long prefix = 0, mask = 0;
  uint32_t k = (uint32_t)pos;
  for (int shift = 56; shift >= 0; shift -= 8) {
    sc->hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SEL_VPT; ++s)
      if ((key[s] & mask) == prefix) atomicAdd(&sc->hist[(key[s] >> shift) & 255], 1u);
    __syncthreads();
    const uint32_t h = sc->hist[tid];
    const uint32_t inc = wave_incl_scan_u32(h);
    if (lane == 63) sc->wtot[wv] = inc;
    __syncthreads();
    uint32_t base = 0;
#pragma unroll
    for (int w = 0; w < DCOR_WAVES; ++w) base += (w < wv) ? sc->wtot[w] : 0u;
    const uint32_t ex = base + inc - h;
    if (h != 0 && k >= ex && k < ex + h) { sc->sel[0] = (uint32_t)tid; sc->sel[1] = k - ex; sc->sel[2] = h; }
    __syncthreads();
    const uint32_t bin = sc->sel[0], cnt = sc->sel[2];
    k = sc->sel[1];
    prefix |= (unsigned long long)bin << shift;
    mask |= 0xFFull << shift;
    if (cnt == 1 && shift > 0) {  // unique key left under this prefix
#pragma unroll
      for (int s = 0; s < SEL_VPT; ++s)
        if ((key[s] & mask) == prefix) sc->key = key[s];
      __syncthreads();
      const unsigned long long r = sc->key;
      __syncthreads();
      return sel_unkey(r);
    }
  }
  __syncthreads();
  return sel_unkey(prefix);
}

// Order statistic by value binning: sort(valid v)[pos] for v held SEL_VPT per thread (NaN =
// absent / NA, counted in `valid` by the caller).  Keys map to 256 bins by the monotone
// non-decreasing b(v) = min(floor((v - min) * 256 / (max - min)), 255), so the bin where the
// cumulative count crosses pos holds the answer; its few keys (~nsim/100 for mixquant draws)
// are ranked directly.  One histogram pass with little atomic contention instead of the radix
// passes (whose top digit piles every key of a narrow range into one or two bins).  Falls
// back to reg_select for non-finite ranges or a crowded bin.  All threads call.
__device__ __forceinline__ double value_select(const double (&v)[SEL_VPT], int pos, int valid,
                                               SelScratch* sc) {
  if (pos < 0 || pos >= valid) return dnan();  // uniform
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double lo = __longlong_as_double(0x7FF0000000000000LL), hi = -lo;
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s)
    if (v[s] == v[s]) { lo = fmin(lo, v[s]); hi = fmax(hi, v[s]); }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if (lane == 0) { sc->mm[wv] = lo; sc->mm[DCOR_WAVES + wv] = hi; }
  sc->hist[tid] = 0;
  if (tid == 0) sc->ncand = 0;
  __syncthreads();
#pragma unroll
  for (int w = 0; w < DCOR_WAVES; ++w) { lo = fmin(lo, sc->mm[w]); hi = fmax(hi, sc->mm[DCOR_WAVES + w]); }
  if (!(hi > lo)) {                      // every valid key equal (pos < valid >= 1)
    __syncthreads();
    return lo;
  }
  const double scale = 256.0 / (hi - lo);
  if (!(scale > 0.0) || !(scale < __longlong_as_double(0x7FF0000000000000LL)) ||
      !((hi - lo) < __longlong_as_double(0x7FF0000000000000LL))) {
    __syncthreads();
    unsigned long long key[SEL_VPT];
#pragma unroll
    for (int s = 0; s < SEL_VPT; ++s) key[s] = sel_key(v[s]);
    return reg_select(key, pos, valid, sc);
  }
  int bin[SEL_VPT];
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s) {
    bin[s] = -1;
    if (v[s] == v[s]) {
      const double t = (v[s] - lo) * scale;
      bin[s] = t < 255.0 ? (int)t : 255;
      atomicAdd(&sc->hist[bin[s]], 1u);
    }
  }
  __syncthreads();
  const uint32_t h = sc->hist[tid];
  const uint32_t inc = wave_incl_scan_u32(h);
  if (lane == 63) sc->wtot[wv] = inc;
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (int w = 0; w < DCOR_WAVES; ++w) base += (w < wv) ? sc->wtot[w] : 0u;
  const uint32_t ex = base + inc - h;
  const uint32_t k = (uint32_t)pos;
  if (h != 0 && k >= ex && k < ex + h) { sc->sel[0] = (uint32_t)tid; sc->sel[1] = k - ex; sc->sel[2] = h; }
  __syncthreads();
  const int b = (int)sc->sel[0];
  const uint32_t kk = sc->sel[1], cnt = sc->sel[2];
  if (cnt > SEL_CAND) {  // crowded bin: radix select over all keys (uniform branch)
    __syncthreads();
    unsigned long long key[SEL_VPT];
#pragma unroll
    for (int s = 0; s < SEL_VPT; ++s) key[s] = sel_key(v[s]);
    return reg_select(key, pos, valid, sc);
  }
#pragma unroll
  for (int s = 0; s < SEL_VPT; ++s)
    if (bin[s] == b) sc->cand[atomicAdd(&sc->ncand, 1)] = v[s];
  __syncthreads();
  if ((uint32_t)tid < cnt) {  // rank = #smaller + #equal at a lower slot (ties broken by slot)
    const double x = sc->cand[tid];
    uint32_t r = 0;
    for (uint32_t j = 0; j < cnt; ++j) {
      const double y = sc->cand[j];
      r += (y < x) || (y == x && j < (uint32_t)tid);
    }
    if (r == kk) sc->mm[0] = x;
  }
  __syncthreads();
  const double res = sc->mm[0];
  __syncthreads();
  return res;
}


// ---------------------------------------------------- wave-level order statistic
// One wavefront per replicate (the epilogue kernels): no workgroup barriers, so the four
// waves of a workgroup finish four replicates independently.  Same value-binning scheme as
// value_select: a min/max reduction, a 256-bin LDS histogram of the active keys, the bin
// holding rank k is either ranked directly (<= 64 keys) or becomes the new active set
// (iterate; each round removes at least one distinct value).  Infinite keys are peeled off
// first.  Lanes of one wave see each other's LDS writes after wave_sync (in-order LDS).
struct WaveSel {
  uint32_t hist[256];
  double cand[64];
  int ncand;
  int pad;
  double res;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ int wave_sum_int(int v) {
  v += (int)lane_dpp_u32<0xB1>((uint32_t)v);
  v += (int)lane_dpp_u32<0x4E>((uint32_t)v);
  v += (int)lane_dpp_u32<0x141>((uint32_t)v);
  v += (int)lane_dpp_u32<0x140>((uint32_t)v);
  uint32_t a, b;
  lane_swap_u32<16>((uint32_t)v, a, b);
  v = (int)(a + b);
  lane_swap_u32<32>((uint32_t)v, a, b);
  return (int)(a + b);
}

// Monotone bin of v in [0, 255] for the active range [lo, hi]: by value when the range is
// representable ((v - lo) * 256 / (hi - lo), computed on halves so it cannot overflow), else by
// the order-preserving integer key of the double (tiny subnormal ranges).
struct BinMap {
  double lo, scale;
  unsigned long long klo;
  int sh;
  bool by_value;
  __device__ __forceinline__ int operator()(double v) const {
    if (by_value) {
      const double t = (0.5 * v - 0.5 * lo) * scale;
      return t < 255.0 ? (int)t : 255;
    }
    return (int)((sel_key(v) - klo) >> sh);
  }
};

// sort(active keys)[pos] (0-based) over VPL <= 32 keys per lane; NaN keys are never active.
template <int VPL>
__device__ __forceinline__ double wave_select(const double (&v)[VPL], int pos, WaveSel* ws) {
  static_assert(VPL <= 32, "active keys are a 32-bit mask per lane");
  const int lane = threadIdx.x & 63;
  const double INF = __longlong_as_double(0x7FF0000000000000LL);
  uint32_t act = 0;
#pragma unroll
  for (int s = 0; s < VPL; ++s) act |= (v[s] == v[s] ? 1u : 0u) << s;
  const int nact = wave_sum_int(__popc(act));
  int k = pos;
  if (k < 0 || k >= nact) return dnan();
  {  // peel -inf / +inf keys (binning needs a finite range)
    uint32_t mlo = 0, mhi = 0;
#pragma unroll
    for (int s = 0; s < VPL; ++s) {
      mlo |= (v[s] == -INF ? 1u : 0u) << s;
      mhi |= (v[s] == INF ? 1u : 0u) << s;
    }
    const int nlo = wave_sum_int(__popc(mlo)), nhi = wave_sum_int(__popc(mhi));
    if (k < nlo) return -INF;
    if (k >= nact - nhi) return INF;
    act &= ~(mlo | mhi);
    k -= nlo;
  }
  for (int iter = 0; iter < 80; ++iter) {
    double lo = INF, hi = -INF;
#pragma unroll
    for (int s = 0; s < VPL; ++s)
      if ((act >> s) & 1u) { lo = fmin(lo, v[s]); hi = fmax(hi, v[s]); }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (!(hi > lo)) return lo;  // every active key equal
    BinMap bm;
    bm.lo = lo;
    const double h = 0.5 * hi - 0.5 * lo;
    bm.scale = 128.0 / h;
    bm.by_value = (h > 0.0) && (bm.scale < INF);
    bm.klo = sel_key(lo);
    {
      const unsigned long long d = sel_key(hi) - bm.klo;
      const int bits = 64 - __clzll((long long)d);
      bm.sh = bits > 8 ? bits - 8 : 0;
    }
    // every active key's bin, once per round, packed 4 per register (the round's three uses read
    // these: computing bm() at each use kept both mappings' temporaries live, ~180 VGPRs); the
    // mapping is wave-uniform, so one branch picks it for all keys
    uint32_t pk[(VPL + 3) / 4];
#pragma unroll
    for (int q = 0; q < (VPL + 3) / 4; ++q) pk[q] = 0u;
    if (bm.by_value) {
#pragma unroll
      for (int s = 0; s < VPL; ++s) {
        const double t = (0.5 * v[s] - 0.5 * lo) * bm.scale;
        const uint32_t b = t < 255.0 ? (uint32_t)(int)t : 255u;
        pk[s >> 2] |= (((act >> s) & 1u) ? b : 0u) << (8 * (s & 3));
      }
    } else {
#pragma unroll
      for (int s = 0; s < VPL; ++s) {
        const uint32_t b = (uint32_t)((sel_key(v[s]) - bm.klo) >> bm.sh);
        pk[s >> 2] |= (((act >> s) & 1u) ? (b & 255u) : 0u) << (8 * (s & 3));
      }
    }
    auto bin = [&](int s) -> int { return (int)((pk[s >> 2] >> (8 * (s & 3))) & 255u); };
#pragma unroll
    for (int q = 0; q < 4; ++q) ws->hist[4 * lane + q] = 0u;
    if (lane == 0) ws->ncand = 0;
    wave_sync();
#pragma unroll
    for (int s = 0; s < VPL; ++s)
      if ((act >> s) & 1u) atomicAdd(&ws->hist[bin(s)], 1u);
    wave_sync();
    uint32_t hb[4], s4 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { hb[q] = ws->hist[4 * lane + q]; s4 += hb[q]; }
    const uint32_t inc = wave_incl_scan_u32(s4);
    const uint32_t ex = inc - s4;
    int B = -1;
    uint32_t cnt = 0, kk = 0;
    if ((uint32_t)k >= ex && (uint32_t)k < inc) {
      uint32_t base = ex;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (B < 0 && (uint32_t)k < base + hb[q]) { B = 4 * lane + q; cnt = hb[q]; kk = (uint32_t)k - base; }
        base += hb[q];
      }
    }
    const int owner = __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(B >= 0)) - 1);
    B = __builtin_amdgcn_readlane(B, owner);
    cnt = __builtin_amdgcn_readlane(cnt, owner);
    kk = __builtin_amdgcn_readlane(kk, owner);
    if (cnt <= 64) {  // rank the bin's keys directly
#pragma unroll
      for (int s = 0; s < VPL; ++s)
        if (((act >> s) & 1u) && bin(s) == B) ws->cand[atomicAdd(&ws->ncand, 1)] = v[s];
      wave_sync();
      if ((uint32_t)lane < cnt) {
        const double x = ws->cand[lane];
        uint32_t r = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const double y = ws->cand[j];
          r += (y < x) || (y == x && j < (uint32_t)lane);
        }
        if (r == kk) ws->res = x;
      }
      wave_sync();
      const double res = ws->res;
      wave_sync();
      return res;
    }
    uint32_t keep = 0;  // the crowded bin becomes the active set
#pragma unroll
    for (int s = 0; s < VPL; ++s) keep |= (bin(s) == B ? 1u : 0u) << s;
    act &= keep;
    k = (int)kk;
  }
  return dnan();
}


// The same order statistic over keys kept in LDS (keys[lane + 64 s], s < VPL; NaN = absent):
// only the per-round bins (8 bits a key, packed) and the active mask live in registers, so an
// epilogue that generates its keys and selects runs at 4-5 waves per SIMD instead of the 2 the
// register-resident select allows (its 16 keys and their per-round temporaries take ~170 VGPRs).
struct WaveSelL {
  uint32_t hist[256];
  double cand[64];
  int ncand;
  int pad;
  double res;
};

template <int VPL>
__device__ __forceinline__ double wave_select_lds(const double* kv, int pos, WaveSelL* ws) {
  static_assert(VPL <= 32, "active keys are a 32-bit mask per lane");
  const int lane = threadIdx.x & 63;
  const double INF = __longlong_as_double(0x7FF0000000000000LL);
  auto key = [&](int s) -> double { return kv[lane + 64 * s]; };
  uint32_t act = 0;
#pragma unroll
  for (int s = 0; s < VPL; ++s) { const double x = key(s); act |= (x == x ? 1u : 0u) << s; }
  const int nact = wave_sum_int(__popc(act));
  int k = pos;
  if (k < 0 || k >= nact) return dnan();
  {  // peel -inf / +inf keys (binning needs a finite range)
    uint32_t mlo = 0, mhi = 0;
#pragma unroll
    for (int s = 0; s < VPL; ++s) {
      const double x = key(s);
      mlo |= (x == -INF ? 1u : 0u) << s;
      mhi |= (x == INF ? 1u : 0u) << s;
    }
    const int nlo = wave_sum_int(__popc(mlo)), nhi = wave_sum_int(__popc(mhi));
    if (k < nlo) return -INF;
    if (k >= nact - nhi) return INF;
    act &= ~(mlo | mhi);
    k -= nlo;
  }
  for (int iter = 0; iter < 80; ++iter) {
    double lo = INF, hi = -INF;
#pragma unroll
    for (int s = 0; s < VPL; ++s)
      if ((act >> s) & 1u) { const double x = key(s); lo = fmin(lo, x); hi = fmax(hi, x); }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if (!(hi > lo)) return lo;  // every active key equal
    const double h = 0.5 * hi - 0.5 * lo;
    const double scale = 128.0 / h;
    const bool by_value = (h > 0.0) && (scale < INF);
    const unsigned long long klo = sel_key(lo);
    int sh;
    {
      const unsigned long long d = sel_key(hi) - klo;
      const int bits = 64 - __clzll((long long)d);
      sh = bits > 8 ? bits - 8 : 0;
    }
    uint32_t pk[(VPL + 3) / 4];
#pragma unroll
    for (int q = 0; q < (VPL + 3) / 4; ++q) pk[q] = 0u;
    if (by_value) {   // the BinMap of wave_select, one uniform branch per round
#pragma unroll
      for (int s = 0; s < VPL; ++s) {
        const double t = (0.5 * key(s) - 0.5 * lo) * scale;
        const uint32_t b = t < 255.0 ? (uint32_t)(int)t : 255u;
        pk[s >> 2] |= (((act >> s) & 1u) ? b : 0u) << (8 * (s & 3));
      }
    } else {
#pragma unroll
      for (int s = 0; s < VPL; ++s) {
        const uint32_t b = (uint32_t)((sel_key(key(s)) - klo) >> sh);
        pk[s >> 2] |= (((act >> s) & 1u) ? (b & 255u) : 0u) << (8 * (s & 3));
      }
    }
    auto bin = [&](int s) -> int { return (int)((pk[s >> 2] >> (8 * (s & 3))) & 255u); };
#pragma unroll
    for (int q = 0; q < 4; ++q) ws->hist[4 * lane + q] = 0u;
    if (lane == 0) ws->ncand = 0;
    wave_sync();
#pragma unroll
    for (int s = 0; s < VPL; ++s)
      if ((act >> s) & 1u) atomicAdd(&ws->hist[bin(s)], 1u);
    wave_sync();
    uint32_t hb[4], s4 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { hb[q] = ws->hist[4 * lane + q]; s4 += hb[q]; }
    const uint32_t inc = wave_incl_scan_u32(s4);
    const uint32_t ex = inc - s4;
    int B = -1;
    uint32_t cnt = 0, kk = 0;
    if ((uint32_t)k >= ex && (uint32_t)k < inc) {
      uint32_t base = ex;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (B < 0 && (uint32_t)k < base + hb[q]) { B = 4 * lane + q; cnt = hb[q]; kk = (uint32_t)k - base; }
        base += hb[q];
      }
    }
    const int owner = __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(B >= 0)) - 1);
    B = __builtin_amdgcn_readlane(B, owner);
    cnt = __builtin_amdgcn_readlane(cnt, owner);
    kk = __builtin_amdgcn_readlane(kk, owner);
    if (cnt <= 64) {  // rank the bin's keys directly
#pragma unroll
      for (int s = 0; s < VPL; ++s)
        if (((act >> s) & 1u) && bin(s) == B) ws->cand[atomicAdd(&ws->ncand, 1)] = key(s);
      wave_sync();
      if ((uint32_t)lane < cnt) {
        const double x = ws->cand[lane];
        uint32_t r = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const double y = ws->cand[j];
          r += (y < x) || (y == x && j < (uint32_t)lane);
        }
        if (r == kk) ws->res = x;
      }
      wave_sync();
      const double res = ws->res;
      wave_sync();
      return res;
    }
    uint32_t keep = 0;  // the crowded bin becomes the active set
#pragma unroll
    for (int s = 0; s < VPL; ++s) keep |= (bin(s) == B ? 1u : 0u) << s;
    act &= keep;
    k = (int)kk;
  }
  return dnan();
}

}  // namespace dcor
