// dcor_fused.hip -- fused Monte-Carlo kernels (the hot path): Philox DGP -> clip ->
// reduce -> Laplace -> NI + INT estimate + CI, one 256-thread workgroup per replicate.
//
// Nothing of a replicate's input is materialised in HBM except, for the one-pass sign
// kernel, a 2-byte record per sample (k_sign_pass1 / k_sign_pass2).  The DGP is a template parameter
// so the sample loops are straight-line code.  fp64 throughout (R `double`).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "dcor_common.h"

namespace dcor {

// ------------------------------------------------------------- generators
// Sample i of a replicate from the draw-site contract of include/dcor.h.
template <int DGP> struct Dgp;

// Where a DGP's sign-family INT flips come from (vert-cor.R:175).
enum { FLIP_SITE = 0, FLIP_SPARE24 = 1, FLIP_SPARE32 = 2 };

template <> struct Dgp<DCOR_DGP_GAUSSIAN> {  // MASS::mvrnorm (vert-cor.R:389-394), 1 sample/block
  // Sample i: block (i, rep, DGP_A) = (w0, w1, w2, w3); the ziggurat normals z1 = zig(w0, w2 &
  // 0xffff), z2 = zig(w1, w2 >> 16) (dcor_device.h), x = mu + A z; the sign family's INT flip is
  // w3 < ceil(p 2^32).
  static constexpr int flip_src = FLIP_SPARE32;
  // sample i from its DGP_A block w (= draw(i, rep, DGP_A))
  static __device__ __forceinline__ void from_block(const DgpConst& g, uint32_t i, uint32_t rep, uint32_t k0,
                                                    uint32_t k1, const U4& w, double& x, double& y,
                                                    const double2* zt = nullptr) {
    const double z1 = zig_draw(i, 0u, rep, k0, k1, w.w0, w.w2 & 0xffffu, zt);
    const double z2 = zig_draw(i, 1u, rep, k0, k1, w.w1, w.w2 >> 16, zt);
    mvn_z(z1, z2, g.mu0, g.mu1, g.a00, g.a01, g.a10, g.a11, &x, &y);
  }
  // The same sample for the slow-sample drains, where (nearly) every lane has one normal off the
  // fast path: the lanes run ONE divergent zig_slow loop between them -- each for its own slow
  // normal, z1 or z2 -- instead of one loop for z1 and one for z2; a sample with both normals slow
  // (about 1 in 55000) runs z2's after.  Same draws, same values as from_block.
  static __device__ __forceinline__ void from_block_slow(const DgpConst& g, uint32_t i, uint32_t rep,
                                                         uint32_t k0, uint32_t k1, const U4& w, double& x,
                                                         double& y, const double2* zt) {
    const uint32_t H1 = w.w2 & 0xffffu, H2 = w.w2 >> 16;
    const double2 t1 = zig_entry(zt, H1 >> 5), t2 = zig_entry(zt, H2 >> 5);
    double z1 = fma(zig_d(w.w0, zig_y_lo(H1)), t1.x, -t1.x);
    double z2 = fma(zig_d(w.w1, zig_y_lo(H2)), t2.x, -t2.x);
    const bool ok1 = fabs(z1) < t1.y, ok2 = fabs(z2) < t2.y;
    if (!ok1 || !ok2) {
      const uint32_t wh = ok1 ? 1u : 0u;
      const double zs = zig_slow(i, wh, rep, k0, k1, ok1 ? w.w1 : w.w0, ok1 ? H2 : H1, zt);
      if (ok1) z2 = zs; else z1 = zs;
      if (!ok1 && !ok2) z2 = zig_slow(i, 1u, rep, k0, k1, w.w1, H2, zt);
    }
    mvn_z(z1, z2, g.mu0, g.mu1, g.a00, g.a01, g.a10, g.a11, &x, &y);
  }
  static __device__ __forceinline__ void one_w3(const DgpConst& g, uint32_t i, uint32_t rep,
                                                uint32_t k0, uint32_t k1, double& x, double& y,
                                                uint32_t& w3) {
    const U4 w = draw(i, rep, DCOR_SITE_DGP_A, k0, k1);
    from_block(g, i, rep, k0, k1, w, x, y);
    w3 = w.w3;
  }
  static __device__ __forceinline__ void one(const DgpConst& g, uint32_t i, uint32_t rep,
                                             uint32_t k0, uint32_t k1, double& x, double& y) {
    uint32_t w3;
    one_w3(g, i, rep, k0, k1, x, y, w3);
  }
  static __device__ __forceinline__ void quad(const DgpConst& g, uint32_t i0, uint32_t rep,
                                              uint32_t k0, uint32_t k1, double* x, double* y) {
#pragma unroll
    for (int q = 0; q < 4; ++q) one(g, i0 + q, rep, k0, k1, x[q], y[q]);
  }
  static __device__ __forceinline__ double lap(uint32_t i, uint32_t rep, uint32_t k0, uint32_t k1) {
    const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
    return unit_laplace(u53(v.w2, v.w3));
  }
};

template <> struct Dgp<DCOR_DGP_BERNOULLI> {  // gen_bernoulli (vert-cor.R:78-98), 2 samples/block
  // Sample words (wa, wb) = (w0, w1) or (w2, w3) of block i/2: u < 0.5 is the top bit of wa
  // (wa < 2^31, exact); v < thr is the low 24 bits of wa against ceil(thr 2^24) (|bias| <
  // 2^-24); the sign family's INT flip is wb >> 8 against ceil(p 2^24).
  static constexpr int flip_src = FLIP_SPARE24;
  static __device__ __forceinline__ bool xbit(uint32_t wa) { return wa < 0x80000000u; }
  static __device__ __forceinline__ bool ybit(const DgpConst& g, uint32_t wa, bool xb) {
    return (wa & 0xFFFFFFu) < (xb ? g.T1_24 : g.T0_24);
  }
  static __device__ __forceinline__ void from_words(const DgpConst& g, uint32_t wa, double& x,
                                                    double& y) {
    const bool xb = xbit(wa);
    x = xb ? 1.0 : 0.0;
    y = ybit(g, wa, xb) ? 1.0 : 0.0;
  }
  static __device__ __forceinline__ void one_u24(const DgpConst& g, uint32_t i, uint32_t rep,
                                                 uint32_t k0, uint32_t k1, double& x, double& y,
                                                 uint32_t& u24) {
    const U4 w = draw(i >> 1, rep, DCOR_SITE_DGP_A, k0, k1);
    const uint32_t wa = (i & 1) ? w.w2 : w.w0, wb = (i & 1) ? w.w3 : w.w1;
    from_words(g, wa, x, y);
    u24 = wb >> 8;
  }
  static __device__ __forceinline__ void one(const DgpConst& g, uint32_t i, uint32_t rep,
                                             uint32_t k0, uint32_t k1, double& x, double& y) {
    uint32_t u24;
    one_u24(g, i, rep, k0, k1, x, y, u24);
  }
  static __device__ __forceinline__ void quad_u24(const DgpConst& g, uint32_t i0, uint32_t rep,
                                                  uint32_t k0, uint32_t k1, double* x, double* y,
                                                  uint32_t* u24) {
    const U4 a = draw(i0 >> 1, rep, DCOR_SITE_DGP_A, k0, k1);
    const U4 b = draw((i0 >> 1) + 1, rep, DCOR_SITE_DGP_A, k0, k1);
    from_words(g, a.w0, x[0], y[0]);
    from_words(g, a.w2, x[1], y[1]);
    from_words(g, b.w0, x[2], y[2]);
    from_words(g, b.w2, x[3], y[3]);
    u24[0] = a.w1 >> 8; u24[1] = a.w3 >> 8; u24[2] = b.w1 >> 8; u24[3] = b.w3 >> 8;
  }
  static __device__ __forceinline__ void quad(const DgpConst& g, uint32_t i0, uint32_t rep,
                                              uint32_t k0, uint32_t k1, double* x, double* y) {
    uint32_t u24[4];
    quad_u24(g, i0, rep, k0, k1, x, y, u24);
  }
  static __device__ __forceinline__ double lap(uint32_t i, uint32_t rep, uint32_t k0, uint32_t k1) {
    const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
    return unit_laplace(u53(v.w2, v.w3));
  }
};

template <> struct Dgp<DCOR_DGP_BOUNDED_FACTOR> {  // gen_bounded_factor (ver-cor-subG.R:141-154)
  static constexpr int flip_src = FLIP_SITE;
  static __device__ __forceinline__ void one_lap(const DgpConst& g, uint32_t i, uint32_t rep,
                                                 uint32_t k0, uint32_t k1, double& x, double& y,
                                                 double* lap) {
    const U4 w = draw(i, rep, DCOR_SITE_DGP_A, k0, k1);
    const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
    const double U = -g.cU + g.cU2 * u53(w.w0, w.w1);
    x = U + (-g.cE + g.cE2 * u53(w.w2, w.w3));
    y = U + (-g.cE + g.cE2 * u53(v.w0, v.w1));
    if (lap) *lap = unit_laplace(u53(v.w2, v.w3));
  }
  static __device__ __forceinline__ void one(const DgpConst& g, uint32_t i, uint32_t rep,
                                             uint32_t k0, uint32_t k1, double& x, double& y) {
    one_lap(g, i, rep, k0, k1, x, y, nullptr);
  }
  static __device__ __forceinline__ void quad(const DgpConst& g, uint32_t i0, uint32_t rep,
                                              uint32_t k0, uint32_t k1, double* x, double* y) {
#pragma unroll
    for (int q = 0; q < 4; ++q) one(g, i0 + q, rep, k0, k1, x[q], y[q]);
  }
};

template <> struct Dgp<DCOR_DGP_MIX_GAUSSIAN> {  // gen_mix_gaussian (ver-cor-subG.R:113-133)
  static constexpr int flip_src = FLIP_SITE;
  // One DGP_A block: Box-Muller from the top 52 bits of (w0,w1), (w2,w3); the component label
  // from the 24 bits Box-Muller leaves unused (low 12 of w1 and of w3): u24 < ceil(pi 2^24)
  // (exact for pi = .5, the R default; |bias| < 2^-24 otherwise).  Row shuffling
  // (sample.int, :131) leaves the law of an iid mixture sample unchanged, so samples are
  // drawn iid.  pmax(pmin(., 1), -1) last (:132).
  static __device__ __forceinline__ void one(const DgpConst& g, uint32_t i, uint32_t rep,
                                             uint32_t k0, uint32_t k1, double& x, double& y) {
    const U4 w = draw(i, rep, DCOR_SITE_DGP_A, k0, k1);
    double r, s, cs;
    normal_polar(w, &r, &s, &cs);
    const uint32_t u24 = ((w.w1 & 0xFFFu) << 12) | (w.w3 & 0xFFFu);
    const int c = u24 < g.T24 ? 1 : 0;   // label ~ rbinom(1, pi_mix): 1 -> component 1
    const double mx = c ? g.xmu[1][0] : g.xmu[0][0], my = c ? g.xmu[1][1] : g.xmu[0][1];
    const double a00 = c ? g.xa[1][0] : g.xa[0][0], a01 = c ? g.xa[1][1] : g.xa[0][1];
    const double a10 = c ? g.xa[1][2] : g.xa[0][2], a11 = c ? g.xa[1][3] : g.xa[0][3];
    mvn_polar(r, s, cs, mx, my, a00, a01, a10, a11, &x, &y);
    x = rclip_fin(x, 1.0);
    y = rclip_fin(y, 1.0);
  }
  static __device__ __forceinline__ void quad(const DgpConst& g, uint32_t i0, uint32_t rep,
                                              uint32_t k0, uint32_t k1, double* x, double* y) {
#pragma unroll
    for (int q = 0; q < 4; ++q) one(g, i0 + q, rep, k0, k1, x[q], y[q]);
  }
  static __device__ __forceinline__ double lap(uint32_t i, uint32_t rep, uint32_t k0, uint32_t k1) {
    const U4 v = draw(i, rep, DCOR_SITE_DGP_B, k0, k1);
    return unit_laplace(u53(v.w2, v.w3));
  }
};

// Sub-G needs the sample and its local Laplace (DGP_B words 2,3).
template <int DGP>
__device__ __forceinline__ void sample_lap(const DgpConst& g, uint32_t i, uint32_t rep, uint32_t k0,
                                           uint32_t k1, double& x, double& y, double& l) {
  if constexpr (DGP == DCOR_DGP_BOUNDED_FACTOR) {
    Dgp<DGP>::one_lap(g, i, rep, k0, k1, x, y, &l);
  } else {
    Dgp<DGP>::one(g, i, rep, k0, k1, x, y);
    l = Dgp<DGP>::lap(i, rep, k0, k1);
  }
}

__device__ __forceinline__ uint32_t word(const U4& w, uint32_t q) {
  return q == 0 ? w.w0 : (q == 1 ? w.w1 : (q == 2 ? w.w2 : w.w3));
}

struct FlipGen {  // sign-family INT flips, 4 per Philox block (SITE_FLIP), cached per block
  uint32_t cidx;
  U4 cw;
  __device__ __forceinline__ int get(uint32_t i, uint32_t rep, uint32_t k0, uint32_t k1,
                                     uint64_t p) {
    const uint32_t bi = i >> 2;
    if (bi != cidx) { cw = draw(bi, rep, DCOR_SITE_FLIP, k0, k1); cidx = bi; }
    return ((uint64_t)word(cw, i & 3) < p) ? 1 : -1;  // 2*S - 1 (vert-cor.R:175-179)
  }
};

// mixquant inside the workgroup: keys = z + c*l from Philox, then the order statistic.
__device__ __forceinline__ double mixquant_fused(const MixConst& mx, double c, uint32_t rep,
                                                 uint32_t k0, uint32_t k1, SelScratch* sc) {
  if (threadIdx.x == 0) sc->nan_cnt = 0;
  __syncthreads();
  double val[SEL_VPT];
  int nn = 0;
#pragma unroll
  for (int s = 0; s < SEL_VPT / 2; ++s) {
    const int b = threadIdx.x + s * DCOR_BLOCK;  // Philox block b -> elements 2b, 2b+1
    val[2 * s] = val[2 * s + 1] = dnan();
    if (2 * b < mx.nsim) {
      const U4 wz = draw((uint32_t)b, rep, DCOR_SITE_MIX_Z, k0, k1);
      const U4 wl = draw((uint32_t)b, rep, DCOR_SITE_MIX_L, k0, k1);
      double z0, z1;
      normal_pair(wz, &z0, &z1);
      val[2 * s] = z0 + c * unit_laplace(u53(wl.w0, wl.w1));
      nn += (val[2 * s] != val[2 * s]);
      if (2 * b + 1 < mx.nsim) {
        val[2 * s + 1] = z1 + c * unit_laplace(u53(wl.w2, wl.w3));
        nn += (val[2 * s + 1] != val[2 * s + 1]);
      }
    }
  }
  if (nn) atomicAdd(&sc->nan_cnt, nn);
  __syncthreads();
  return value_select(val, mx.pos, mx.nsim - sc->nan_cnt, sc);
}

__device__ __forceinline__ void scalar_laplace(uint32_t rep, uint32_t k0, uint32_t k1, double* lap) {
  if (threadIdx.x < 5) {  // SITE_SCALAR blocks 0..4: NI mu/m2 X, NI mu/m2 Y, INT ..., Z
    const U4 w = draw((uint32_t)threadIdx.x, rep, DCOR_SITE_SCALAR, k0, k1);
    lap[2 * threadIdx.x] = unit_laplace(u53(w.w0, w.w1));
    lap[2 * threadIdx.x + 1] = unit_laplace(u53(w.w2, w.w3));
  }
}

// Wave-level mixquant from Philox (one replicate per wave): the same elements as
// mixquant_fused, VPL keys per lane, written to the wave's LDS and selected there.
template <int VPL>
struct WaveMix {
  double keys[64 * VPL];
  WaveSelL sel;
};

template <int VPL>
__device__ __forceinline__ double wave_mixquant_fused(const MixConst& mx, double c, uint32_t rep,
                                                      uint32_t k0, uint32_t k1, WaveMix<VPL>* ws) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < VPL / 2; ++s) {
    const int b = lane + 64 * s;  // Philox block b -> elements 2b, 2b+1
    double v0 = dnan(), v1 = dnan();
    if (2 * b < mx.nsim) {
      const U4 wz = draw((uint32_t)b, rep, DCOR_SITE_MIX_Z, k0, k1);
      const U4 wl = draw((uint32_t)b, rep, DCOR_SITE_MIX_L, k0, k1);
      double z0, z1;
      normal_pair(wz, &z0, &z1);
      v0 = z0 + c * unit_laplace(u53(wl.w0, wl.w1));
      if (2 * b + 1 < mx.nsim) v1 = z1 + c * unit_laplace(u53(wl.w2, wl.w3));
    }
    ws->keys[lane + 64 * (2 * s)] = v0;
    ws->keys[lane + 64 * (2 * s + 1)] = v1;
  }
  wave_sync();
  return wave_select_lds<VPL>(ws->keys, mx.pos, &ws->sel);
}

// INT epilogue + CI write shared by the sign kernels (vert-cor.R:281-313).
__device__ __forceinline__ void sign_finish(const SignConst& c, uint32_t rep, DD sT, DD sT2,
                                            long long core, bool any_ni, bool any_int,
                                            const double* lap, SelScratch* sel,
                                            dcor_rep_out* dst) {
  double o[6];
  ni_sign_result(c, sT, sT2, any_ni, o);
  double rho, eta, se, cstar;
  int_sign_point(c, core, lap[8], rho, eta, se, cstar);
  double w;
  if (c.mode_normal)
    w = mixquant_fused(c.mix, cstar, rep, c.k0, c.k1, sel) * se;
  else
    w = c.w_laplace;
  o[3] = rho;
  o[4] = sin(M_PI / 2.0 * rmax(eta - w, -1.0));
  o[5] = sin(M_PI / 2.0 * rmin(eta + w, 1.0));
  if (any_int) o[3] = o[4] = o[5] = dnan();
  if (threadIdx.x == 0) *dst = dcor_rep_out{o[0], o[1], o[2], o[3], o[4], o[5]};
}

// ======================================== fused sign family, one pass (hot) ===
// Pass 1 generates each sample once: the DP-mean sums of clip(x), clip(y) (vert-cor.R:
// 328-340) and a 2-byte record per sample in a per-replicate slab -- monotone 7-bit codes of
// clip(x) (bits 0-6) and clip(y) (bits 8-14) and the INT flip bit S (bit 7); bit 15 is 0.  The
// code map q (below) is monotone non-decreasing, so q(xc) != q(mu) proves sign(xc - mu); pass 2
// decides every sign from codes and regenerates only samples whose code ties a threshold's code.
// Results equal the two-pass algorithm's exactly.  Each thread generates groups of 4 consecutive
// samples (8-B slab stores).
// q(v) = unorm16(fma(float(v), inv, nb)) >> 9 per coordinate, inv = 1 / (2 R), nb = -base inv:
// every step (round to float, fma with inv > 0, v_cvt_pknorm_u16_f32's clamp to [0, 1] and round
// to nearest, the shift) is monotone non-decreasing, which is all the sign decision needs.  Both
// 16-bit unorms come from one v_pk_fma_f32 and one v_cvt_pknorm_u16_f32 (a NaN codes as 0; a NaN
// threshold is flagged); one v_perm_b32 takes two samples' high bytes, and a shift and mask make
// the 7-bit codes of a record pair.  128 levels per coordinate over the window (prepare_cell) put
// about 1e-3 of the headline's records on a threshold's code; pass 2 recomputes those batches
// exactly, deferred (sign_pass2_core).  Round 4's 4-byte records with 15-bit codes took twice the
// slab bytes and twice pass 2's decision work (packed 16-bit compares).
__device__ __forceinline__ int sgnq(uint32_t q, uint32_t qm) { return (q > qm) - (q < qm); }
typedef unsigned short dcor_u16x2 __attribute__((ext_vector_type(2)));
typedef float dcor_f32x2 __attribute__((ext_vector_type(2)));
// the 16-bit unorms of (x, y), x in the low half
__device__ __forceinline__ uint32_t code16_pair(double x, double y, float ix, float iy, float bx, float by) {
  const dcor_f32x2 v = {(float)x, (float)y};
  const dcor_f32x2 t = __builtin_elementwise_fma(v, dcor_f32x2{ix, iy}, dcor_f32x2{bx, by});
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_u16(t.x, t.y));
}
// the same from two scalar fmas (fma rounds exactly either way): the thresholds' form, which keeps
// the kernel-argument fields out of a vector build
__device__ __forceinline__ uint32_t code16_pair_s(double x, double y, float ix, float iy, float bx, float by) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_u16(fmaf((float)x, ix, bx), fmaf((float)y, iy, by)));
}
// one record from a unorm pair and its flip (0 or 0x80)
__device__ __forceinline__ uint32_t rec_of(uint32_t P, uint32_t fl) {
  return ((P >> 9) & 0x7fu) | ((P >> 17) & 0x7f00u) | fl;
}
// two records in one word: sample a in the low half
__device__ __forceinline__ uint32_t rec_pair(uint32_t Pa, uint32_t Pb, uint32_t fla, uint32_t flb) {
  const uint32_t hb = __builtin_amdgcn_perm(Pb, Pa, 0x07050301u);   // high bytes: xa, ya, xb, yb
  return ((hb >> 1) & 0x7f7f7f7fu) | fla | (flb << 16);
}

template <int DGP>
__device__ __forceinline__ void exact_signs(const SignConst& c, const SignStd& s, uint32_t i,
                                            uint32_t rep, int& nx, int& ny, int& ix, int& iy,
                                            bool& bad_ni, bool& bad_int) {
  double x, y;
  Dgp<DGP>::one(c.g, i, rep, c.k0, c.k1, x, y);
  const double xc = rclip_fin(x, c.L), yc = rclip_fin(y, c.L);
  nx = sgn_std(xc, s.muNx, s.sdNx, bad_ni);
  ny = sgn_std(yc, s.muNy, s.sdNy, bad_ni);
  ix = sgn_std(xc, s.muIx, s.sdIx, bad_int);
  iy = sgn_std(yc, s.muIy, s.sdIy, bad_int);
}

// Pass 1: replicate `rep` -> its slab (n records) and its clipped sums (SIGN_SUMS doubles:
// sum clip(x) as double-double {hi, lo}, a second-moment slot, the same for y).  The sums of
// clip(x), clip(y) decide the private centres, hence every sign (vert-cor.R:335-347), so they
// are compensated: each thread adds its group of 4 samples plainly and folds the group sum into
// a TwoSum accumulator; the workgroup reduction is double-double.
// The second moments are not accumulated: mean(clip(x)^2) enters the reference only through
// sd_priv = sqrt(max(m2 + noise - mu^2, 1e-12)) (vert-cor.R:339-347), and only signs of
// (clip(x) - mu) / sd_priv are used (:218, :277).  For any finite mean(x^2) in [0, L^2], sd_priv
// is positive and finite (signs = signs of clip(x) - mu), or +Inf / NaN exactly when the noise
// terms overflow -- the same for every such value -- so the slot carries 0 and every sign, hence
// every result, is unchanged.
// Gaussian DGP in pass 1: the ziggurat's fast path inline; a sample with a normal that misses it
// (0.85 % of samples) is queued in a per-wave LDS list and generated in full later by the whole
// wave at once (zig_slow would otherwise run under divergence nearly every iteration).  The
// queued sample's record is rewritten and its clipped values replace its placeholder's in the
// sums at the drain.
// Pass 1 folds two sample groups' plain sums per compensated add (one TwoSum per 8 samples); pass 2
// (m = 8) pair-groups the T sums of a thread's two batches in flight.  Measured (round 4): 11 and 4 us
// per headline chunk against per-group / per-batch sums.
// Slab layout: record i of a replicate is u16 i of its slab (two records per 32-bit word).
// (Measured and dropped in round 4, with 4-B records: a wave-contiguous half-batch layout for
// m = 8, pass 2 181 vs 177 us; non-temporal slab stores and loads, +-0.)
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
// a group of 4 records (i0 % 4 == 0): one 8-B store of two record pairs
__device__ __forceinline__ void slab_st_group(uint32_t* slab, uint32_t i0, uint32_t r01, uint32_t r23) {
  *reinterpret_cast<uint2*>(slab + (i0 >> 1)) = make_uint2(r01, r23);
}
__device__ __forceinline__ void slab_st1(uint32_t* slab, uint32_t i, uint32_t r) {
  reinterpret_cast<uint16_t*>(slab)[i] = (uint16_t)r;
}
__device__ __forceinline__ uint4 slab_ld4(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }
// 16 B from a 4-B aligned word (global_load_dwordx4 takes dword alignment)
__device__ __forceinline__ uint4 slab_ld4a(const uint32_t* p) {
  const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// The Gaussian DGP's ziggurat fast path for one sample's Philox block (pass 1 and the drain
// compute it alike): the clipped sample, true = both normals took the fast path (otherwise the
// values are a finite placeholder in [-L, L] that pass 1 adds and the drain takes out again).
__device__ __forceinline__ bool gauss_fast_xy(const SignConst& c, const double2* zt, const U4& w, double& xc,
                                              double& yc) {
  const double2 t1 = zt[zig_j1(w.w2)], t2 = zt[zig_j2(w.w2)];
  const double z1 = fma(zig_d(w.w0, zig_y1(w.w2)), t1.x, -t1.x);
  const double z2 = fma(zig_d(w.w1, zig_y2(w.w2)), t2.x, -t2.x);
  const bool ok = ((int)(fabs(z1) < t1.y) & (int)(fabs(z2) < t2.y)) != 0;
  double x, y;
  mvn_z(z1, z2, c.g.mu0, c.g.mu1, c.g.a00, c.g.a01, c.g.a10, c.g.a11, &x, &y);
  xc = rclip_fin(x, c.L);
  yc = rclip_fin(y, c.L);
  return ok;
}
// The INT flip of a sample's 32-bit word, u < flipT (flipT <= 2^32), as the record's bit 7.
__device__ __forceinline__ uint32_t sign_flip7(const SignConst& c, uint32_t u) {
  return (c.flipT != 0 && u <= (uint32_t)(c.flipT - 1u)) ? 0x80u : 0u;
}
// A sample's slab record (u16): the codes of (clip(x), clip(y)) and its INT flip.
__device__ __forceinline__ uint32_t sign_record(const SignConst& c, double xc, double yc, uint32_t u) {
  return rec_of(code16_pair(xc, yc, c.cinv_xf, c.cinv_yf, c.cnb_xf, c.cnb_yf), sign_flip7(c, u));
}

// Per-wave slow-normal queue (the wave-per-replicate pass 1): a loop step adds at most 256 entries
// per wave (about 0.85 % of a wave's samples are queued); it drains at DCOR_DRAIN_AT (or, with 0,
// above ZQ_CAP - 256), so it never holds more than DCOR_DRAIN_AT - 1 + 256 entries.  384: the
// workgroup's LDS (38.9 KB with the 32 KB layer table) fits four workgroups per CU.
#ifndef DCOR_ZQ_CAP
#define DCOR_ZQ_CAP 384
#endif
#define ZQ_CAP DCOR_ZQ_CAP
// DCOR_DRAIN_AT > 0: a wave drains whole 64-entry rounds of its queue as soon as it holds
// DCOR_DRAIN_AT entries (the rest stays queued for later), so its regenerations interleave with
// the other waves' hot loops instead of all coinciding at the replicates' ends.  Measured (round 4,
// headline, one box, two runs each): pass 1 506-511 us per chunk at 64, 510-511 at 128, 517-535
// at 256, 514-519 draining at the end (0); 2.85e6-2.86e6 replicates/s against 2.81e6-2.83e6.
// The drain order only moves the low bits of the compensated sums.
#ifndef DCOR_DRAIN_AT
#define DCOR_DRAIN_AT 64
#endif
static_assert(ZQ_CAP >= 256 && (DCOR_DRAIN_AT == 0 || DCOR_DRAIN_AT - 1 + 256 <= ZQ_CAP), "slow-sample queue bound");

// WAVE = false: one 256-thread workgroup per replicate; WAVE = true: one wave per replicate (the
// caller's workgroup has loaded the ziggurat table `zt` into LDS once for all its replicates).
// Slow samples (Gaussian DGP): both forms regenerate them inside the kernel, 64 at a time, from a
// per-wave LDS list zq: the workgroup form fills it from a register of pend bits every four loop
// steps (ballot compaction, no atomics); the wave form through an LDS atomic counter zqn.
// CEIL (Gaussian workgroup form only; a measurement kernel, never a result): the same hot loop with
// its memory side removed -- no slab store, no slow-sample list or regeneration; an empty asm consumes the records
// and the pending masks, so the compiler keeps every instruction that computes them.  Its time is
// the loop's own VALU-issue ceiling (dcor_diag_sign_pass, bench.py roofline.issue_frac).  CEIL = 2
// keeps the slab stores only, CEIL = 3 the slow-sample list and its regenerations only (the cost of each).
template <int DGP, bool WAVE, int CEIL = 0>
__device__ __forceinline__ void sign_pass1_core(const SignConst& c, uint32_t rep,
                                                uint32_t* __restrict__ slab,
                                                double* __restrict__ sums_out, const double2* zt,
                                                uint32_t* zq, uint32_t* zqn) {
  constexpr int NT = WAVE ? 64 : DCOR_BLOCK;
  const int tid = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  DD sx{0.0, 0.0}, sy{0.0, 0.0};
  const float cix = c.cinv_xf, ciy = c.cinv_yf, cbx = c.cnb_xf, cby = c.cnb_yf;
  // the INT flip from its 32-bit word: u < flipT (flipT <= 2^32) as a 32-bit compare, bit 7
  const uint32_t ftm1 = (uint32_t)(c.flipT - 1u), fbit = c.flipT != 0 ? 0x80u : 0u;
  auto record_w = [&](double xc, double yc, uint32_t u) { return sign_record(c, xc, yc, u); };
  // each thread runs its groups in increasing order; the partial last group (n % 4) is the last
  // group of its thread
  const int64_t nfull = c.n / 4;
  if constexpr (DGP == DCOR_DGP_GAUSSIAN) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    auto fast_xy = [&](const U4& w, double& xc, double& yc) -> bool { return gauss_fast_xy(c, zt, w, xc, yc); };
    // Every valid sample enters the group sums, a queued one with its placeholder: the drain
    // takes the placeholder out and adds the true values (both compensated), so the hot loop
    // selects nothing.  The group's plain sums are added into (hx, hy); the caller folds them
    // into the compensated sums, once per two groups.
    // The group's slow samples (pend bit q: sample i0 + q) are queued by the caller (enqueue),
    // outside the lanes' divergent group branch.
    auto group = [&](int64_t g4, auto full_tag, double& hx, double& hy, uint32_t& pend) {
      constexpr bool FULL = decltype(full_tag)::value;
      const uint32_t i0 = (uint32_t)(4 * g4);
      uint32_t P[4], fl[4];
      pend = 0;
      double gx, gy;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const U4 w = draw(i0 + q, rep, DCOR_SITE_DGP_A, c.k0, c.k1);
        double xc, yc;
        const bool ok = fast_xy(w, xc, yc);
        const bool valid = FULL || (int64_t)(i0 + q) < c.n;
        const double ax = valid ? xc : 0.0, ay = valid ? yc : 0.0;
        gx = q == 0 ? ax : gx + ax;
        gy = q == 0 ? ay : gy + ay;
        pend |= (valid && !ok) ? (1u << q) : 0u;
        P[q] = code16_pair(xc, yc, cix, ciy, cbx, cby);
        fl[q] = w.w3 <= ftm1 ? fbit : 0u;
      }
      hx += gx;
      hy += gy;
      const uint32_t r01 = rec_pair(P[0], P[1], fl[0], fl[1]), r23 = rec_pair(P[2], P[3], fl[2], fl[3]);
      if constexpr (CEIL == 1 || CEIL == 3)
        asm volatile("" ::"v"(r01), "v"(r23));
      if constexpr (CEIL == 1 || CEIL == 2) {
        asm volatile("" ::"v"(pend));
        if constexpr (CEIL == 1) return;
      }
      if constexpr (CEIL == 0 || CEIL == 2) {
        if (FULL) {
          slab_st_group(slab, i0, r01, r23);
        } else {
          for (int q = 0; q < 4; ++q) if ((int64_t)(i0 + q) < c.n) slab_st1(slab, i0 + q, rec_of(P[q], fl[q]));
        }
      }
    };
    // Queue one group's slow samples (pend bit q: sample i0 + q; 0 in lanes without a group), one
    // LDS atomic per group.  (Measured against: one atomic per two-group step with the drain test
    // taken from the reservations -- its drain threshold has to be 512 lower, so the queue drains
    // more often, 513 vs 497 us for the queue-only ceiling; ballot-allocated slots, 535 vs 523 us.)
    auto enqueue = [&](uint32_t pend, uint32_t i0) {
      if constexpr (CEIL == 1 || CEIL == 2) {
        asm volatile("" ::"v"(pend));
        return;
      }
      if (pend) {
        uint32_t pos = atomicAdd(zqn, (uint32_t)__popc(pend));
        for (; pend; pend &= pend - 1u) zq[pos++] = i0 + (uint32_t)(__ffs(pend) - 1);
      }
    };
    auto full = [&]() {
      return (CEIL == 0 || CEIL == 3) &&
             __builtin_amdgcn_readfirstlane(*zqn) > (DCOR_DRAIN_AT > 0 ? DCOR_DRAIN_AT - 1 : ZQ_CAP - 256);
    };
    // the whole wave, converged: each lane takes queued samples lane, lane + 64, ...
    // part: the loop's early drains take the queue's top 64 floor(cnt / 64) entries; the final
    // drain takes all
    auto drain = [&](bool part) {
      if constexpr (CEIL == 1 || CEIL == 2) return;
      const uint32_t cnt = __builtin_amdgcn_readfirstlane(*zqn);
      const uint32_t keep = (DCOR_DRAIN_AT > 0 && part) ? (cnt & 63u) : 0u;
      if (cnt == keep) return;
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the placeholder records have landed
      for (uint32_t k = keep + (uint32_t)lane; k < cnt; k += 64) {
        const uint32_t i = zq[k];
        const U4 w = draw(i, rep, DCOR_SITE_DGP_A, c.k0, c.k1);   // one block: placeholder and sample
        double px, py;
        fast_xy(w, px, py);
        ks_acc(sx, -px);
        ks_acc(sy, -py);
        double x, y;
        const uint32_t w3 = w.w3;
        // the table from LDS in the workgroup kernel (the wave kernel keeps the global table: the
        // LDS pointer costs it six VGPRs and a wave per SIMD)
        Dgp<DGP>::from_block_slow(c.g, i, rep, c.k0, c.k1, w, x, y, WAVE ? nullptr : zt);
        const double xc = rclip_fin(x, c.L), yc = rclip_fin(y, c.L);
        ks_acc(sx, xc);
        ks_acc(sy, yc);
        if constexpr (CEIL == 3) {
          const uint32_t r = record_w(xc, yc, w3);
          asm volatile("" ::"v"(r));
        } else {
          slab_st1(slab, i, record_w(xc, yc, w3));
        }
      }
      wave_sync();
      if (lane == 0) *zqn = keep;
      wave_sync();
    };
    // two groups per step (wave groups b + lane and b + NT + lane), one compensated fold of their
    // plain 8-sample sums: half the TwoSum chains of a fold per group (the low bits of the sums
    // differ from per-group folds; the private centres they decide are unchanged in practice)
    if constexpr (!WAVE) {
      // Slow samples: the step's two pend nibbles enter a per-lane byte shift register; every four
      // steps the wave compacts the register's set bits into its LDS list -- each lane hands over one
      // bit per sub-round (ballot + mbcnt slots, the count wave-uniform) -- and regenerates 64 at a
      // time, every lane busy, between its hot-loop steps (so the regenerations of a CU's waves
      // interleave with the others' hot loops instead of coinciding at the replicates' ends).
      // Each regeneration takes the placeholder out of and the true value into the lane's sums (one
      // compensated add of their difference per coordinate) and rewrites the record.
      uint32_t acc = 0, s4 = 0, q = 0, cnt = 0;
      auto fix = [&](uint32_t i) {
        const U4 w = draw(i, rep, DCOR_SITE_DGP_A, c.k0, c.k1);   // one block: placeholder and sample
        double px, py, x, y;
        fast_xy(w, px, py);
        Dgp<DGP>::from_block_slow(c.g, i, rep, c.k0, c.k1, w, x, y, zt);
        const double xc = rclip_fin(x, c.L), yc = rclip_fin(y, c.L);
        ks_acc(sx, xc - px);
        ks_acc(sy, yc - py);
        const uint32_t r = record_w(xc, yc, w.w3);
        if constexpr (CEIL == 3) asm volatile("" ::"v"(r));
        else slab_st1(slab, i, r);
      };
      // (Measured, round 5, headline, one box: the regenerations cost about 40 us of pass 1's ~494
      // per chunk -- without them 454 -- at about 430 VALU instructions per 64-entry flush, 4.5 % of
      // the kernel's VALU count.  Two entries per lane, their slow normals in one attempt loop so
      // each lane runs two independent chains: 494-497 us, no gain, so the flush is VALU-bound, not
      // latency-bound.  Dropping the vmcnt(0) below: no gain either.)
      auto flush = [&](uint32_t upto) {   // regenerate the list's top `upto` entries
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0), lgkmcnt(0): placeholders stored, list in LDS
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < upto) fix(zq[cnt - upto + (uint32_t)lane]);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        cnt -= upto;
      };
      // bit (byte 3 - t, nibble h, bit j) of a quad word whose first step's groups start at g0: step
      // t of the quad, group g0 + 2 NT t + h NT + lane; tail: the n % 4 group's bit j
      auto take = [&](uint32_t word, int64_t g0, bool tail) {   // every lane, converged
        while (__ballot(word != 0u)) {
          const bool has = word != 0u;
          uint32_t idx = 0;
          if (has) {
            const uint32_t bit = (uint32_t)(__ffs(word) - 1);
            const int64_t g = g0 + (int64_t)(2 * NT) * (3 - (bit >> 3)) + ((bit & 4u) ? NT : 0) + lane;
            idx = tail ? (uint32_t)(4 * nfull) + bit : (uint32_t)(4 * g) + (bit & 3u);
            word &= word - 1u;
          }
          const uint64_t bal = __ballot(has);
          if (has)
            zq[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = idx;
          cnt += (uint32_t)__popcll(bal);
          if (cnt >= 64u) flush(64u);
        }
      };
      auto quad_word = [&](uint32_t word) {
        if constexpr (CEIL == 1 || CEIL == 2)
          asm volatile("" ::"v"(word));
        else
          take(word, 64 * (int64_t)wv + (int64_t)(2 * NT) * (4 * (int64_t)q), false);
        ++q;
      };
      for (int64_t b = 64 * wv; b < nfull; b += 2 * NT) {  // trip count uniform per wave
        double hx = 0.0, hy = 0.0;
        uint32_t pa = 0, pb = 0;
        if (b + lane < nfull) group(b + lane, std::true_type(), hx, hy, pa);
        if (b + NT + lane < nfull) group(b + NT + lane, std::true_type(), hx, hy, pb);
        ks_acc(sx, hx);
        ks_acc(sy, hy);
        acc = (acc << 8) | pa | (pb << 4);
        if (++s4 == 4) {
          quad_word(acc);
          acc = 0;
          s4 = 0;
        }
      }
      if (s4) quad_word(acc << (8 * (4 - s4)));   // the partial last quad, left-aligned
      // the partial last group (n % 4)
      const bool last = (c.n & 3) && tid == (int)(nfull % NT);
      uint32_t pt = 0;
      if (last) {
        double hx = 0.0, hy = 0.0;
        group(nfull, std::false_type(), hx, hy, pt);
        ks_acc(sx, hx);
        ks_acc(sy, hy);
      }
      if constexpr (CEIL == 0 || CEIL == 3) {
        take(pt, 0, true);
        if (cnt) flush(cnt);
      }
    } else {
    for (int64_t b = 0; b < nfull; b += 2 * NT) {  // trip count uniform per wave
      double hx = 0.0, hy = 0.0;
      uint32_t pa = 0, pb = 0;
      if (b + lane < nfull) group(b + lane, std::true_type(), hx, hy, pa);
      enqueue(pa, (uint32_t)(4 * (b + lane)));
      if (full()) drain(true);
      if (b + NT + lane < nfull) group(b + NT + lane, std::true_type(), hx, hy, pb);
      enqueue(pb, (uint32_t)(4 * (b + NT + lane)));
      if (full()) drain(true);
      ks_acc(sx, hx);
      ks_acc(sy, hy);
    }
    {  // the partial last group (n % 4), converged around its enqueue
      double hx = 0.0, hy = 0.0;
      uint32_t pa = 0;
      const bool last = (c.n & 3) && tid == (int)(nfull % NT);
      if (last) group(nfull, std::false_type(), hx, hy, pa);
      enqueue(pa, (uint32_t)(4 * nfull));   // the final drain follows
      if (last) {
        ks_acc(sx, hx);
        ks_acc(sy, hy);
      }
    }
    drain(false);
    }
  } else {
    static_assert(CEIL == 0, "the ceiling kernel runs the Gaussian loop");
    // group g4 = samples 4 g4 .. 4 g4 + 3; FULL: all four exist (the hot loop has no guards)
    auto group = [&](int64_t g4, auto full_tag) {
      constexpr bool FULL = decltype(full_tag)::value;
      const uint32_t i0 = (uint32_t)(4 * g4);
      double x[4], y[4];
      uint32_t fl[4];  // INT flip bits (vert-cor.R:175), in bit 7
      if constexpr (Dgp<DGP>::flip_src == FLIP_SPARE24) {
        uint32_t u24[4];
        Dgp<DGP>::quad_u24(c.g, i0, rep, c.k0, c.k1, x, y, u24);
#pragma unroll
        for (int q = 0; q < 4; ++q) fl[q] = u24[q] < c.flipT24 ? 0x80u : 0u;
      } else {
        const U4 fw = draw((uint32_t)g4, rep, DCOR_SITE_FLIP, c.k0, c.k1);
        Dgp<DGP>::quad(c.g, i0, rep, c.k0, c.k1, x, y);
#pragma unroll
        for (int q = 0; q < 4; ++q) fl[q] = word(fw, q) <= ftm1 ? fbit : 0u;
      }
      uint32_t P[4];
      double gx = 0.0, gy = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double xc = rclip_fin(x[q], c.L), yc = rclip_fin(y[q], c.L);
        if (FULL || (int64_t)(i0 + q) < c.n) { gx += xc; gy += yc; }
        P[q] = code16_pair(xc, yc, cix, ciy, cbx, cby);
      }
      ks_acc(sx, gx);
      ks_acc(sy, gy);
      if (FULL) {
        slab_st_group(slab, i0, rec_pair(P[0], P[1], fl[0], fl[1]), rec_pair(P[2], P[3], fl[2], fl[3]));
      } else {
        for (int q = 0; q < 4; ++q) if ((int64_t)(i0 + q) < c.n) slab_st1(slab, i0 + q, rec_of(P[q], fl[q]));
      }
    };
    for (int64_t g4 = tid; g4 < nfull; g4 += NT) group(g4, std::true_type());
    if ((c.n & 3) && tid == (int)(nfull % NT)) group(nfull, std::false_type());
  }
  DD d2[2] = {sx, sy};
  if constexpr (WAVE) {
    d2[0] = wave_sum_dd(d2[0]);
    d2[1] = wave_sum_dd(d2[1]);
  } else {
    __shared__ double red[16 * DCOR_WAVES];
    block_sum_dd<2>(d2, red);
  }
  if (tid == 0) {
    sums_out[0] = d2[0].hi; sums_out[1] = d2[0].lo; sums_out[2] = 0.0;
    sums_out[3] = d2[1].hi; sums_out[4] = d2[1].lo; sums_out[5] = 0.0;
  }
}

// slab: the replicate's records (sign_item_words)
template <int DGP, int CEIL = 0>
__device__ __forceinline__ void sign_pass1_body(const SignConst& c, uint32_t rep,
                                                uint32_t* __restrict__ slab,
                                                double* __restrict__ sums_out) {
  if constexpr (DGP == DCOR_DGP_GAUSSIAN) {
    constexpr int ZTN = 2 * DCOR_ZIG_N;
    __shared__ double2 zt[ZTN];
    __shared__ uint32_t zl[DCOR_WAVES][128];   // each wave's slow-sample list
    const int tid = threadIdx.x;
    for (int e = tid; e < ZTN; e += DCOR_BLOCK)
      zt[e] = make_double2(dcor_zig_tab[e][0], dcor_zig_tab[e][1]);
    __syncthreads();
    sign_pass1_core<DGP, false, CEIL>(c, rep, slab, sums_out, zt, zl[tid >> 6], nullptr);
  } else {
    sign_pass1_core<DGP, false>(c, rep, slab, sums_out, nullptr, nullptr, nullptr);
  }
}

// Minimum waves per SIMD the one-pass kernels are compiled for (register budget 512 / w).
#ifndef DCOR_P1_WPE
#define DCOR_P1_WPE 1
#endif
#ifndef DCOR_P2_WPE
#define DCOR_P2_WPE 4
#endif
template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK, DCOR_P1_WPE) void k_sign_pass1(SignConst c,
                                                           uint32_t* __restrict__ scratch,
                                                           double* __restrict__ sums) {
  sign_pass1_body<DGP>(c, (uint32_t)(c.rep_begin + blockIdx.x),
                       scratch + (size_t)blockIdx.x * sign_item_words(c.n, DGP), sums + SIGN_SUMS * (size_t)blockIdx.x);
}
// The pass-1 ceiling (CEIL above): same grid, registers and occupancy target as k_sign_pass1.
template <int CM>
__global__ __launch_bounds__(DCOR_BLOCK, DCOR_P1_WPE) void k_sign_pass1_ceil(SignConst c,
                                                                         uint32_t* __restrict__ scratch,
                                                                         double* __restrict__ sums) {
  sign_pass1_body<DCOR_DGP_GAUSSIAN, CM>(c, (uint32_t)(c.rep_begin + blockIdx.x),
                                         scratch + (size_t)blockIdx.x * sign_item_words(c.n, DCOR_DGP_GAUSSIAN),
                                         sums + SIGN_SUMS * (size_t)blockIdx.x);
}


// The private centres and scales from pass 1's sums (vert-cor.R:335-344): mean(xc) is the
// double-double sum divided by n, rounded once.
__device__ __forceinline__ void sign_std_from_pass1(const SignConst& c, const double* sums,
                                                    const double lap[8], SignStd& s) {
  const double mx = dd_div_d(DD{sums[0], sums[1]}, c.nd).hi;
  const double my = dd_div_d(DD{sums[3], sums[4]}, c.nd).hi;
  priv_std_from_means(c, mx, sums[2] / c.nd, my, sums[5] / c.nd, lap, s);
}

// Per-replicate partial results handed from pass 2 to the epilogue.
struct SignPartial {
  double sT[2], sT2[2];  // double-double sum of T_j and T_j^2 (vert-cor.R:233-239)
  long long core;        // sum of (2S-1) sign(X) sign(Y) (vert-cor.R:178-183)
  long long flags;       // bit 0: NI saw NaN, bit 1: INT saw NaN; bits 8-: tie batches (k_sign_pass2)
};
static_assert(sizeof(SignPartial) == SIGN_PARTIAL_BYTES, "dcor_engine.h SIGN_PARTIAL_BYTES");

// Pass 2: signs from the codes (exact regeneration on a code tie), batch counts, NI
// Laplace, T sums and the INT flip sum.  Lean: the mixquant/CI epilogue is its own kernel.
// The reduced per-replicate results of pass 2 (every lane / thread holds them).
struct P2Result {
  DD sT, sT2;
  long long core;
  bool bad_ni, bad_int;
  double lapz;   // SITE_SCALAR block 4's first draw: the INT estimate's Z (vert-cor.R:188)
  long long ties;  // NI batches that took the exact fix-up (workgroup form only; 0 in the wave form)
};

// The 10 SITE_SCALAR draws of one replicate in every lane of a wave (lanes 0-4 draw, shuffles).
__device__ __forceinline__ void scalar_laplace_wave(uint32_t rep, uint32_t k0, uint32_t k1,
                                                    double (&lap)[10]) {
  const int lane = threadIdx.x & 63;
  double a = 0.0, b = 0.0;
  if (lane < 5) {
    const U4 w = draw((uint32_t)lane, rep, DCOR_SITE_SCALAR, k0, k1);
    a = unit_laplace(u53(w.w0, w.w1));
    b = unit_laplace(u53(w.w2, w.w3));
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    lap[2 * q] = __shfl(a, q, 64);
    lap[2 * q + 1] = __shfl(b, q, 64);
  }
}

// WAVE = false: one 256-thread workgroup per replicate (barriers, LDS reductions); WAVE = true:
// one wave per replicate (wave reductions only) -- the same arithmetic per batch and sample.
// CEIL (m = 8 only; a measurement kernel, never a result): the decision loop with each thread's
// first two batches' records loaded once and then held in registers (an empty asm redefines them
// every step, so nothing is hoisted), and no tie fix-up (1e-4 of samples): the loop's own
// VALU-issue ceiling without the slab stream (dcor_diag_sign_pass, bench.py roofline.issue_frac).
// pbuf: the calling wave's piece buffer (64 c.pieces words of LDS) when c.pieces > 0; tq: its
// tie-deferral queue (TQ words of LDS).
#define TQ 256
template <int DGP, bool WAVE, bool CEIL = false, bool ONLY8 = false>
__device__ __forceinline__ P2Result sign_pass2_core(const SignConst& c, uint32_t rep,
                                                    const uint32_t* __restrict__ slab,
                                                    const double* __restrict__ sums_in,
                                                    const double2* lt, uint32_t* pbuf, uint32_t* tq) {
  constexpr int NT = WAVE ? 64 : DCOR_BLOCK;   // threads sharing the replicate
  const int tid = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  double lap[10];
  if constexpr (WAVE) {
    scalar_laplace_wave(rep, c.k0, c.k1, lap);
  } else {
    __shared__ double lap_s[10];
    scalar_laplace(rep, c.k0, c.k1, lap_s);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 10; ++q) lap[q] = lap_s[q];
  }
  SignStd s;
  {
    double l8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) l8[q] = lap[q];
    sign_std_from_pass1(c, sums_in, l8, s);
  }
  const bool thr_nan = (s.muNx != s.muNx) || (s.muNy != s.muNy) || (s.muIx != s.muIx) ||
                       (s.muIy != s.muIy) || (s.sdNx != s.sdNx) || (s.sdNy != s.sdNy) ||
                       (s.sdIx != s.sdIx) || (s.sdIy != s.sdIy);
  // sign(d/sd) == sign(d) needs sd < 2^900 (no underflow of the quotient); else exact path.
  const bool force_exact = !(s.sdNx < 0x1p900 && s.sdNy < 0x1p900 && s.sdIx < 0x1p900 &&
                             s.sdIy < 0x1p900);
  // threshold codes (the records' map), and as the four bytes (x, y, x, y) of a record pair
  const uint32_t TN = code16_pair_s(s.muNx, s.muNy, c.cinv_xf, c.cinv_yf, c.cnb_xf, c.cnb_yf);
  const uint32_t TI = code16_pair_s(s.muIx, s.muIy, c.cinv_xf, c.cinv_yf, c.cnb_xf, c.cnb_yf);
  const uint32_t qNx = (TN & 0xffffu) >> 9, qNy = TN >> 25, qIx = (TI & 0xffffu) >> 9, qIy = TI >> 25;
  const uint32_t TN4 = (qNx | (qNy << 8)) * 0x00010001u, TI4 = (qIx | (qIy << 8)) * 0x00010001u;
  const uint32_t TN4p = TN4 + 0x01010101u, TI4p = TI4 + 0x01010101u;
  const uint16_t* __restrict__ s16 = reinterpret_cast<const uint16_t*>(slab);
  bool bad_ni = thr_nan, bad_int = thr_nan;
  DD sT{0.0, 0.0}, sT2{0.0, 0.0};
  long long core = 0;
  int ties = 0;   // batches whose codes tie a threshold (diagnostic: dcor_diag_sign_ties)
  // One record's exact signs: from the codes unless a code ties a threshold's (then the sample is
  // regenerated, exact_signs).  Adds its NI signs to (cx, cy) and its INT term to cc.
  auto exact_rec = [&](int64_t i, uint32_t w, int& cx, int& cy, int& cc, bool& bni) {
    const uint32_t qx = w & 0x7fu, qy = (w >> 8) & 0x7fu;
    const int f = (w & 0x80u) ? 1 : -1;
    int nx, ny, ix, iy;
    if (force_exact || qx == qNx || qy == qNy || qx == qIx || qy == qIy) {
      exact_signs<DGP>(c, s, (uint32_t)i, rep, nx, ny, ix, iy, bni, bad_int);
    } else {
      nx = qx < qNx ? -1 : 1;
      ny = qy < qNy ? -1 : 1;
      ix = qx < qIx ? -1 : 1;
      iy = qy < qIy ? -1 : 1;
    }
    cx += nx;
    cy += ny;
    cc += f * ix * iy;
  };
  // Two records (one word) by SWAR: g = w | 0x80 per byte, g - T per byte has bit 7 = (q >= t) with
  // no borrow between bytes (0x80 + q - t >= 1), and g - (T + 1) has it = (q > t): the two differ
  // exactly on a tie.  neg counts (q < t) per byte (x0, y0, x1, y1); the INT bit of each record is
  // px ^ py ^ S (bits 7, 23 of dI ^ dI >> 8 ^ w), +1 when set.  13 full-rate operations and one
  // v_bcnt for two records.
  auto word2 = [&](uint32_t w, uint32_t& neg, uint32_t& pc, uint32_t& tie) {
    const uint32_t g = w | 0x80808080u;
    const uint32_t dN = g - TN4, dN1 = g - TN4p, dI = g - TI4, dI1 = g - TI4p;
    tie |= (dN ^ dN1) | (dI ^ dI1);
    neg += (~dN >> 7) & 0x01010101u;
    pc += (uint32_t)__popc((dI ^ (dI >> 8) ^ w) & 0x00800080u);
  };
  // mean of m signs = count / m (exact quotient for the configs' m); a power-of-two m divides by
  // an exact multiply.  M8: the headline geometry, m = 8 known at compile time.
  auto batch_T = [&](int64_t j, int cx, int cy, auto m8_tag) {
    constexpr bool M8 = decltype(m8_tag)::value;
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);   // vert-cor.R:230-231
    double mx, my;
    if constexpr (M8) {
      mx = (double)cx * 0.125;
      my = (double)cy * 0.125;
    } else {
      mx = c.md_pow2 ? (double)cx * c.inv_md : (double)cx / c.md;
      my = c.md_pow2 ? (double)cy * c.inv_md : (double)cy / c.md;
    }
    const double xt = mx + c.bx * unit_laplace_t(u53(w.w0, w.w1), lt);
    const double yt = my + c.by * unit_laplace_t(u53(w.w2, w.w3), lt);
    const double T = (M8 ? 8.0 : c.md) * xt * yt;                        // vert-cor.R:233
    ks_acc(sT, T);  // compensated (error ~ k 2^-106): the T mean / sd inputs
    ks_acc(sT2, T * T);
  };
  // T_j alone (no accumulation): the pair-grouped form below
  auto batch_T_val = [&](int64_t j, int cx, int cy) -> double {
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);   // vert-cor.R:230-231
    const double xt = (double)cx * 0.125 + c.bx * unit_laplace_t(u53(w.w0, w.w1), lt);
    const double yt = (double)cy * 0.125 + c.by * unit_laplace_t(u53(w.w2, w.w3), lt);
    return 8.0 * xt * yt;                                                 // vert-cor.R:233
  };
  // Tie deferral.  A batch whose codes tie a threshold (about 1e-3 of records at the headline's 128
  // code levels) is not fixed up inside the loop, where every lane would wait for its regeneration:
  // its index goes to the wave's LDS queue (ballot + mbcnt slots, the count wave-uniform) and the
  // whole wave recomputes queued batches exactly, one per lane (exact_rec over its m records, then
  // its T), once per loop trip when a next trip could overflow the queue (a trip of the m = 8 and
  // piece loops queues at most 128 batches, of the unit loop 64 per batch end) and after the loop:
  // one inlined copy of the recomputation per loop.  Callers defer at wave-uniform points.  Which batches tie depends on the replicate alone, so a replicate's bits
  // do not depend on the launch; the code window moves only the order of the T sums.
  const int lane = (int)(threadIdx.x & 63);
  uint32_t tqn = 0;
  auto drain_ties = [&]() {
    if (tqn == 0) return;
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the queue's entries are in LDS
    __builtin_amdgcn_wave_barrier();
    for (uint32_t e0 = 0; e0 < tqn; e0 += 64) {   // uniform trips
      const uint32_t e = e0 + (uint32_t)lane;
      const bool has = e < tqn;
      const int64_t j = has ? (int64_t)tq[e] : 0;
      const int64_t i0 = j * c.m;
      int cx = 0, cy = 0, cc = 0;
      // records decided by their codes first; the tied ones (m <= 64) are regenerated afterwards one
      // per lane per round, every lane's regeneration in the same pass -- in record order, a round
      // per record position, nearly every lane would wait for some other lane's regeneration
      uint64_t tmask = 0;
      if (has) {
#pragma unroll 1
        for (int r = 0; r < c.m; ++r) {
          const uint32_t w = s16[i0 + r];
          const uint32_t qx = w & 0x7fu, qy = (w >> 8) & 0x7fu;
          if (c.m <= 64 && (force_exact || qx == qNx || qy == qNy || qx == qIx || qy == qIy))
            tmask |= 1ull << r;
          else
            exact_rec(i0 + r, w, cx, cy, cc, bad_ni);
        }
      }
      while (__ballot(tmask != 0)) {
        if (tmask) {
          const int r = __ffsll((long long)tmask) - 1;
          tmask &= tmask - 1;
          exact_rec(i0 + r, s16[i0 + r], cx, cy, cc, bad_ni);
        }
      }
      if (has) {
        core += cc;
        batch_T(j, cx, cy, std::false_type());
        ++ties;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    tqn = 0;
  };
  auto defer = [&](bool tie, int64_t j) -> bool {
    const uint64_t bal = __ballot(tie);
    if (bal) {
      if (tie)
        tq[tqn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] =
            (uint32_t)j;
      tqn += (uint32_t)__popcll(bal);
    }
    return tie;
  };
  auto drain_if_full = [&](uint32_t per_trip) {
    if (tqn > TQ - per_trip) drain_ties();
  };
  if (ONLY8 || c.m == 8) {
    // headline geometry: one thread = one batch = one 16-B load (8 records), decided by word2.
    auto decide = [&](const uint4& v, int& cx, int& cy, int& cc) -> bool {
      uint32_t neg = 0, pc = 0, tie = 0;
      word2(v.x, neg, pc, tie);
      word2(v.y, neg, pc, tie);
      word2(v.z, neg, pc, tie);
      word2(v.w, neg, pc, tie);
      const uint32_t t = neg + (neg >> 16);      // x0 + x1 in byte 0, y0 + y1 in byte 1
      cx = 8 - 2 * (int)(t & 0xffu);
      cy = 8 - 2 * (int)((t >> 8) & 0xffu);
      cc = 2 * (int)pc - 8;
      if constexpr (CEIL) {
        asm volatile("" : "+v"(tie));
        cc += (int)(tie & 1u);
        return false;
      }
      return (tie & 0x80808080u) != 0 || force_exact;
    };
    // Two batches in flight per thread in two register sets, used in place (a move of a register
    // with a load pending waits for the load): batch j is decided while j + NT loads, j + 2 NT is
    // issued into j's registers, then j + NT is decided.  The trip count is uniform per wave; loads
    // past the last batch re-read it, and batches past it are dropped.
    auto load = [&](int64_t jj, uint4& v) {
      if constexpr (CEIL) {
        asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
      } else {
        const int64_t jc = jj < c.k ? jj : c.k - 1;
        v = slab_ld4(slab + 4 * jc);
      }
    };
    if (c.k > 0) {
      const int64_t base = tid - lane;       // the wave's first batch
      uint4 a, b;
      {
        const int64_t ja = tid < c.k ? tid : c.k - 1, jb = tid + NT < c.k ? tid + NT : c.k - 1;
        a = slab_ld4(slab + 4 * ja);
        __builtin_amdgcn_sched_barrier(0);
        b = slab_ld4(slab + 4 * jb);
        __builtin_amdgcn_sched_barrier(0);
      }
      for (int64_t jw = base; jw < c.k; jw += 2 * NT) {   // uniform per wave
        const int64_t j = jw + lane, jb = j + NT;
        const bool va = j < c.k, vb = jb < c.k;
        int cxa, cya, cca, cxb, cyb, ccb;
        const bool ta = decide(a, cxa, cya, cca);
        load(j + 2 * NT, a);
        __builtin_amdgcn_sched_barrier(0);  // keep j + NT's decisions after j + 2 NT's loads
        const bool tb = decide(b, cxb, cyb, ccb);
        load(j + 3 * NT, b);
        __builtin_amdgcn_sched_barrier(0);
        // defer() is called by every lane (its ballot and the queue count are wave-wide)
        const bool fa = defer(va && ta, j);
        const bool fb = defer(vb && tb, jb);
        const bool da = va && !fa, db = vb && !fb;
        core += (da ? cca : 0) + (db ? ccb : 0);
        // the two batches' T and T^2 added plainly, the pair sums compensated: half the TwoSum
        // chains (the low bits differ from per-batch sums, within the oracle's 1e-12); a batch
        // dropped here (past the end or deferred) adds 0
        const double Ta = da ? batch_T_val(j, cxa, cya) : 0.0;
        const double Tb = db ? batch_T_val(jb, cxb, cyb) : 0.0;
        ks_acc(sT, Ta + Tb);
        ks_acc(sT2, Ta * Ta + Tb * Tb);
        drain_if_full(128u);
      }
    }
  } else if constexpr (!CEIL && !ONLY8) {
    // m % 8 == 0, 16 <= m <= 248 (the grids' 32, C4's 200): 16-B pieces of 8 records.  A replicate's
    // batches go in rounds of 64 (waves take rounds wv, wv + 4, ...); in a round the wave's lanes
    // read 64 consecutive pieces at a time (1 KB, coalesced -- lane-per-batch loads would touch 64
    // cache lines per instruction at m = 32), decide their 8 records by word2 and store the piece's
    // packed counts (x negatives, y negatives, INT bits, tie) to the wave's LDS buffer; then lane L
    // adds batch L's P = m / 8 piece words and finishes the batch (deferred on a tie, else T).
    if (c.pieces > 0) {
      const uint32_t P = (uint32_t)c.pieces, m = (uint32_t)c.m;
      const int wv0 = WAVE ? 0 : (int)(threadIdx.x >> 6);
      constexpr int NWV = WAVE ? 1 : DCOR_WAVES;
      const int64_t rounds = (c.k + 63) / 64, npc = c.k * (int64_t)P;
      auto piece = [&](const uint4& v) -> uint32_t {
        uint32_t neg = 0, pc = 0, tie = 0;
        word2(v.x, neg, pc, tie);
        word2(v.y, neg, pc, tie);
        word2(v.z, neg, pc, tie);
        word2(v.w, neg, pc, tie);
        const uint32_t t = neg + (neg >> 16);
        return (t & 0xffffu) | (pc << 16) | ((tie & 0x80808080u) != 0 ? 0x01000000u : 0u);
      };
      // the wave's pieces as one stream of steps (its rounds wv0, wv0 + NWV, ..., P steps each),
      // two register sets used in place and loaded two steps ahead across round ends
      const int64_t my_rounds = rounds > wv0 ? (rounds - wv0 + NWV - 1) / NWV : 0;
      const int64_t nsteps = my_rounds * (int64_t)P;
      int64_t lt_ = 0;
      uint32_t lit = 0;
      auto load_next = [&](uint4& v) {
        const int64_t pc = (wv0 + NWV * lt_) * 64 * (int64_t)P + (int64_t)lit * 64 + lane;
        v = slab_ld4(slab + 4 * (pc < npc ? pc : npc - 1));
        if (++lit == P) { lit = 0; ++lt_; }
      };
      int64_t dt = 0;     // the decision cursor's round (of this wave) and piece
      uint32_t dit = 0;
      auto step = [&](const uint4& v) {
        pbuf[dit * 64 + (uint32_t)lane] = piece(v);
        if (++dit < P) return;
        // the round's pieces are in: lane L finishes batch 64 rd + L
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        uint32_t sum = 0;
        for (uint32_t q = 0; q < P; ++q) sum += pbuf[(uint32_t)lane * P + q];
        __builtin_amdgcn_s_waitcnt(0xC07F);   // read before the next round overwrites the buffer
        __builtin_amdgcn_wave_barrier();
        const int64_t j = (wv0 + NWV * dt) * 64 + lane;
        const bool ok = j < c.k;
        if (!defer(ok && ((sum >> 24) != 0 || force_exact), j) && ok) {
          core += 2 * (int)((sum >> 16) & 0xffu) - (int)m;
          batch_T(j, (int)m - 2 * (int)(sum & 0xffu), (int)m - 2 * (int)((sum >> 8) & 0xffu), std::false_type());
        }
        dit = 0;
        ++dt;
      };
      if (nsteps > 0) {
        uint4 a, b;
        load_next(a);
        __builtin_amdgcn_sched_barrier(0);
        load_next(b);
        __builtin_amdgcn_sched_barrier(0);
        // an odd step count runs one step past the end: it writes a buffer word no round reads
        for (int64_t st = 0; st < nsteps; st += 2) {
          step(a);
          load_next(a);
          __builtin_amdgcn_sched_barrier(0);
          step(b);
          load_next(b);
          __builtin_amdgcn_sched_barrier(0);
          drain_if_full(128u);
        }
      }
    } else if (c.m <= 252) {
      // any other m <= 252 (the reference grids' 11): a stream of 16-B units.  Batch j's records
      // [j m, j m + m) are read from the 4-B aligned record j m & ~1 on, U = ceil((m + (m & 1)) / 8)
      // units, four units in flight in four register sets used in place (the loop waits vmcnt(3));
      // a record outside the batch (a leading one when j m is odd, trailing ones in the last unit) is
      // replaced by PAD = (127, 127), flip 0: no negatives, INT bit 0, and a tie only with a threshold
      // coded 127, which the exact recomputation settles.  The loop runs a multiple of four units
      // with a uniform trip count per wave; units past the thread's last batch are dropped.
      const uint32_t m = (uint32_t)c.m, U = (m + (m & 1u) + 7u) >> 3;
      const uint32_t per_trip = 64u * (U >= 4u ? 1u : (U >= 2u ? 2u : 4u));   // batch ends per 4 units
      const int64_t rounds = (c.k + NT - 1 - (tid - lane)) / NT;   // this wave's batch rounds (uniform)
      const int64_t nu = rounds > 0 ? ((rounds * (int64_t)U) + 3) & ~(int64_t)3 : 0;
      constexpr uint32_t PAD = 0x7f7f7f7fu;
      int64_t rl = 0;
      uint32_t ul = 0;
      auto load_next = [&](uint4& v) {
        const int64_t jj = tid + NT * rl;
        const int64_t jc = jj < c.k ? jj : c.k - 1;
        const int64_t s0 = (jc * (int64_t)m) & ~(int64_t)1;     // even record: 4-B aligned
        v = slab_ld4a(slab + (s0 >> 1) + 4 * ul);
        if (++ul == U) { ul = 0; ++rl; }
      };
      int64_t rd = 0;
      uint32_t ud = 0, neg = 0, pc = 0, tie = 0;
      auto step = [&](const uint4& v) {
        const int64_t j = tid + NT * rd;
        const uint32_t lead = (uint32_t)((j * (int64_t)m) & 1);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if (ud == 0) w[0] = lead ? ((w[0] & 0xffff0000u) | (PAD & 0xffffu)) : w[0];
        const bool last = ud + 1u == U;
        if (last) {
          // records r >= nv of the unit are past the batch: PAD halves from bit 16 nv on
          const uint32_t nv = m + lead - 8u * ud;       // 1 .. 8
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int sh = 16 * (int)nv - 32 * k;       // invalid bits from `sh` on in word k
            const uint32_t M = sh <= 0 ? 0xffffffffu : (sh >= 32 ? 0u : (0xffffffffu << sh));
            w[k] = (w[k] & ~M) | (PAD & M);
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) word2(w[k], neg, pc, tie);
        if (last) {
          const bool ok = j < c.k;
          const uint32_t t = neg + (neg >> 16);
          if (!defer(ok && ((tie & 0x80808080u) != 0 || force_exact), j) && ok) {
            core += 2 * (int)pc - (int)m;
            batch_T(j, (int)m - 2 * (int)(t & 0xffu), (int)m - 2 * (int)((t >> 8) & 0xffu), std::false_type());
          }
          neg = pc = tie = 0;
          ud = 0;
          ++rd;
        } else {
          ++ud;
        }
      };
      if (nu > 0) {
        uint4 u0, u1, u2, u3;
        load_next(u0);
        __builtin_amdgcn_sched_barrier(0);
        load_next(u1);
        __builtin_amdgcn_sched_barrier(0);
        load_next(u2);
        __builtin_amdgcn_sched_barrier(0);
        load_next(u3);
        __builtin_amdgcn_sched_barrier(0);
        for (int64_t t = 0; t < nu; t += 4) {
          step(u0);
          load_next(u0);
          __builtin_amdgcn_sched_barrier(0);
          step(u1);
          load_next(u1);
          __builtin_amdgcn_sched_barrier(0);
          step(u2);
          load_next(u2);
          __builtin_amdgcn_sched_barrier(0);
          step(u3);
          load_next(u3);
          __builtin_amdgcn_sched_barrier(0);
          drain_if_full(per_trip);
        }
      }
    } else {
      // m > 252 (byte counters would overflow): record by record, exactly
      for (int64_t j = tid; j < c.k; j += NT) {
        int cx = 0, cy = 0, cc = 0;
        const int64_t i0 = j * c.m;
        for (int r = 0; r < c.m; ++r) exact_rec(i0 + r, s16[i0 + r], cx, cy, cc, bad_ni);
        core += cc;
        batch_T(j, cx, cy, std::false_type());
      }
    }
  }
  if constexpr (!CEIL) drain_ties();
  for (int64_t i = c.k * c.m + tid; !CEIL && i < c.n; i += NT) {  // tail: INT only
    int dx = 0, dy = 0, cc = 0;
    bool ignore = false;  // NI never reads the tail
    exact_rec(i, s16[i], dx, dy, cc, ignore);
    core += cc;
  }
  P2Result r;
  r.lapz = lap[8];
  r.ties = 0;
  if constexpr (WAVE) {
    r.sT = wave_sum_dd(sT);
    r.sT2 = wave_sum_dd(sT2);
    r.core = wave_sum_i(core);
    r.bad_ni = __ballot(bad_ni) != 0;
    r.bad_int = __ballot(bad_int) != 0;
  } else {
    __shared__ double red[16 * DCOR_WAVES];
    __shared__ long long redi[DCOR_WAVES];
    DD d2[2] = {sT, sT2};
    block_sum_dd<2>(d2, red);
    r.sT = d2[0];
    r.sT2 = d2[1];
    r.core = block_sum_i(core, redi);
    const long long nbad = block_sum_i((bad_ni ? 1LL : 0LL) + (bad_int ? (1LL << 20) : 0LL) +
                                       ((long long)ties << 40), redi);
    r.bad_ni = (nbad & 0xFFFFF) != 0;
    r.bad_int = ((nbad >> 20) & 0xFFFFF) != 0;
    r.ties = nbad >> 40;
  }
  return r;
}

// The calling wave's piece buffer in the launch's dynamic LDS (sign_piece_lds): 64 `stride` words
// per wave of the workgroup.
extern __shared__ uint32_t dcor_pbuf_dyn[];
__device__ __forceinline__ uint32_t* wave_pbuf(int stride) {
  return dcor_pbuf_dyn + (size_t)(threadIdx.x >> 6) * 64u * (uint32_t)stride;
}

template <int DGP, bool CEIL = false, bool M8 = false>
__device__ __forceinline__ void sign_pass2_body(const SignConst& c, uint32_t rep,
                                                const uint32_t* __restrict__ slab,
                                                const double* __restrict__ sums_in,
                                                SignPartial* __restrict__ part_out) {
  __shared__ double2 lt[256];
  __shared__ uint32_t tq[DCOR_WAVES][TQ];
  log_tab_to_lds(lt, DCOR_BLOCK);
  __syncthreads();
  const P2Result r = sign_pass2_core<DGP, false, CEIL, M8>(c, rep, slab, sums_in, lt, wave_pbuf(c.pieces),
                                                       tq[threadIdx.x >> 6]);
  if (threadIdx.x == 0) {
    SignPartial p;
    p.sT[0] = r.sT.hi; p.sT[1] = r.sT.lo; p.sT2[0] = r.sT2.hi; p.sT2[1] = r.sT2.lo;
    p.core = r.core;
    p.flags = (r.bad_ni ? 1 : 0) | (r.bad_int ? 2 : 0) | (r.ties << 8);
    *part_out = p;
  }
}



// M8: a cell with m = 8 (the headline geometry) gets an instantiation holding the m = 8 decision
// loop only, so the other batch-size loops' registers do not weigh on its allocation (the generic
// instantiation spilled 8 VGPRs at 4 waves per SIMD); the m = 8 code path is the same either way.
template <int DGP, bool M8 = false>
__global__ __launch_bounds__(DCOR_BLOCK, DCOR_P2_WPE) void k_sign_pass2(SignConst c,
                                                           const uint32_t* __restrict__ scratch,
                                                           const double* __restrict__ sums,
                                                           SignPartial* __restrict__ part) {
  sign_pass2_body<DGP, false, M8>(c, (uint32_t)(c.rep_begin + blockIdx.x),
                       scratch + (size_t)blockIdx.x * sign_item_words(c.n, DGP),
                       sums + SIGN_SUMS * (size_t)blockIdx.x, part + blockIdx.x);
}
// The pass-2 ceiling (CEIL above, m = 8): same grid as k_sign_pass2, compiled for 4 waves per SIMD
// (its register-held records would otherwise take it to 3) and launched at k_sign_pass2's occupancy.
__global__ __launch_bounds__(DCOR_BLOCK, 4) void k_sign_pass2_ceil(SignConst c,
                                                                         const uint32_t* __restrict__ scratch,
                                                                         const double* __restrict__ sums,
                                                                         SignPartial* __restrict__ part) {
  sign_pass2_body<DCOR_DGP_GAUSSIAN, true>(c, (uint32_t)(c.rep_begin + blockIdx.x),
                                           scratch + (size_t)blockIdx.x * sign_item_words(c.n, DCOR_DGP_GAUSSIAN),
                                           sums + SIGN_SUMS * (size_t)blockIdx.x, part + blockIdx.x);
}

// The INT side and the record of one replicate from its pass-2 result, one wave: NI estimate/CI,
// INT estimate, mixquant, INT CI (vert-cor.R:233-254, 186-194, 281-313).
template <int VPL>
__device__ __forceinline__ void sign_finish_wave(const SignConst& c, uint32_t rep, const P2Result& p,
                                                 dcor_rep_out* dst, WaveMix<VPL>* ws) {
  const int lane = threadIdx.x & 63;
  double o[6];
  ni_sign_result(c, p.sT, p.sT2, p.bad_ni, o);
  double rho, eta, se, cstar;
  int_sign_point(c, p.core, p.lapz, rho, eta, se, cstar);
  double w;
  if (c.mode_normal)
    w = wave_mixquant_fused<VPL>(c.mix, cstar, rep, c.k0, c.k1, ws) * se;
  else
    w = c.w_laplace;
  o[3] = rho;
  o[4] = sin(M_PI / 2.0 * rmax(eta - w, -1.0));
  o[5] = sin(M_PI / 2.0 * rmin(eta + w, 1.0));
  if (p.bad_int) o[3] = o[4] = o[5] = dnan();
  if (lane == 0) *dst = dcor_rep_out{o[0], o[1], o[2], o[3], o[4], o[5]};
}

// Wave-per-replicate epilogue (four replicates per workgroup, no workgroup barriers) from the
// SignPartial a workgroup-per-replicate pass 2 left.
template <int VPL>
__device__ __forceinline__ void sign_epilogue_wave(const SignConst& c, uint32_t rep,
                                                   const SignPartial& sp, dcor_rep_out* dst,
                                                   WaveMix<VPL>* ws) {
  const U4 wz = draw(4u, rep, DCOR_SITE_SCALAR, c.k0, c.k1);  // SCALAR block 4: Z (vert-cor.R:188)
  P2Result p;
  p.lapz = unit_laplace(u53(wz.w0, wz.w1));
  p.sT = DD{sp.sT[0], sp.sT[1]};
  p.sT2 = DD{sp.sT2[0], sp.sT2[1]};
  p.core = sp.core;
  p.bad_ni = (sp.flags & 1) != 0;
  p.bad_int = (sp.flags & 2) != 0;
  sign_finish_wave<VPL>(c, rep, p, dst, ws);
}

// ---- small cells (n <= SIGN_W_NMAX): one wave per replicate for both passes ------------------
// The pass 2 + epilogue wave kernels: the tie queue (TQ words) lives in the wave's select histogram,
// which the epilogue fills only after pass 2 has drained the queue, and the NI Laplace log table is
// read from global memory (L1/L2) instead of a 4-KB LDS copy: 39 KB of LDS per 4-wave workgroup, four
// workgroups per CU instead of three.  Measured (round 6, one box): VG 3.98e7 against 3.80e7 with the
// LDS copy, C1 1.59e7 against 1.45e7.
static_assert(TQ == 256, "the tie queue aliases WaveSelL::hist");
#define P2E_LOG_TABLE(lt) const double2* lt = reinterpret_cast<const double2*>(dcor_log8_tab)
#ifndef DCOR_P2E_WPE
#define DCOR_P2E_WPE 4  // waves per SIMD the pass 2 + epilogue wave kernel is compiled for (the
                        // mixture DGP's: 3, its sampler needs more than 128 VGPRs)
#endif
// At the reference grids' n (1000-12000) a 256-thread workgroup per replicate spends much of
// its time in per-replicate fixed work -- the ziggurat table load, the scalar draws, the
// barriers of its reductions.  Here pass 1 runs in persistent workgroups that load the table
// once and give each wave one replicate at a time, and pass 2 and the epilogue are one wave
// per replicate with wave reductions only.  Same per-sample and per-batch arithmetic as the
// workgroup kernels; the sums are folded in a different (wave) order.
template <int DGP>
__device__ __forceinline__ void pass1_w_setup(double2* zt, uint32_t* zqn) {
  if constexpr (DGP == DCOR_DGP_GAUSSIAN) {
    for (int e = threadIdx.x; e < 2 * DCOR_ZIG_N; e += DCOR_BLOCK)
      zt[e] = make_double2(dcor_zig_tab[e][0], dcor_zig_tab[e][1]);
    if (threadIdx.x < DCOR_WAVES) zqn[threadIdx.x] = 0u;
  }
  __syncthreads();
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_pass1_w(SignConst c, int64_t nreps,
                                                             uint32_t* __restrict__ scratch,
                                                             double* __restrict__ sums) {
  __shared__ double2 zt[DGP == DCOR_DGP_GAUSSIAN ? 2 * DCOR_ZIG_N : 1];
  __shared__ uint32_t zq[DCOR_WAVES][DGP == DCOR_DGP_GAUSSIAN ? ZQ_CAP : 1];
  __shared__ uint32_t zqn[DCOR_WAVES];
  pass1_w_setup<DGP>(zt, zqn);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + wv; r < nreps; r += (int64_t)gridDim.x * DCOR_WAVES)
    sign_pass1_core<DGP, true>(c, (uint32_t)(c.rep_begin + r), scratch + (size_t)r * sign_item_words(c.n, DGP),
                               sums + SIGN_SUMS * (size_t)r, zt, zq[wv], &zqn[wv]);
}

// Pass 2 alone, one wave per replicate, writing the SignPartial the wave epilogue reads.
template <int DGP>
__device__ __forceinline__ void sign_pass2_wave_part(const SignConst& c, uint32_t rep, const uint32_t* slab,
                                                     const double* sums_in, SignPartial* part_out,
                                                     const double2* lt, int pstride, uint32_t* tq) {
  const P2Result r = sign_pass2_core<DGP, true>(c, rep, slab, sums_in, lt, wave_pbuf(pstride), tq);
  if ((threadIdx.x & 63) == 0) {
    SignPartial p;
    p.sT[0] = r.sT.hi; p.sT[1] = r.sT.lo; p.sT2[0] = r.sT2.hi; p.sT2[1] = r.sT2.lo;
    p.core = r.core;
    p.flags = (r.bad_ni ? 1 : 0) | (r.bad_int ? 2 : 0) | (r.ties << 8);
    *part_out = p;
  }
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_pass2_w(SignConst c, int64_t nreps,
                                                             const uint32_t* __restrict__ scratch,
                                                             const double* __restrict__ sums,
                                                             SignPartial* __restrict__ part, int pstride) {
  __shared__ double2 lt[256];
  __shared__ uint32_t tq[DCOR_WAVES][TQ];
  log_tab_to_lds(lt, DCOR_BLOCK);
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (r >= nreps) return;
  sign_pass2_wave_part<DGP>(c, (uint32_t)(c.rep_begin + r), scratch + (size_t)r * sign_item_words(c.n, DGP),
                            sums + SIGN_SUMS * (size_t)r, part + r, lt, pstride, tq[threadIdx.x >> 6]);
}

template <int DGP, int VPL>
__global__ __launch_bounds__(DCOR_BLOCK, DGP == DCOR_DGP_MIX_GAUSSIAN ? 3 : DCOR_P2E_WPE) void k_sign_p2e_w(SignConst c, int64_t nreps,
                                                           const uint32_t* __restrict__ scratch,
                                                           const double* __restrict__ sums,
                                                           dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  P2E_LOG_TABLE(lt);
  const int wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + __builtin_amdgcn_readfirstlane(wv);
  if (r >= nreps) return;  // whole waves only
  const uint32_t rep = (uint32_t)(c.rep_begin + r);
  // the piece buffer lives in the wave's mixquant keys, which the epilogue fills only after pass 2
  static_assert(sizeof(wsel[0].keys) >= 64 * SIGN_PIECES_MAX * sizeof(uint32_t), "piece buffer");
  const P2Result p = sign_pass2_core<DGP, true>(c, rep, scratch + (size_t)r * sign_item_words(c.n, DGP),
                                                sums + SIGN_SUMS * (size_t)r, lt,
                                                reinterpret_cast<uint32_t*>(wsel[wv].keys), wsel[wv].sel.hist);
  sign_finish_wave<VPL>(c, rep, p, out + r, &wsel[wv]);
}

template <int VPL>
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_epilogue_w(SignConst c, int64_t nreps,
                                                                const SignPartial* __restrict__ part,
                                                                dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  const int wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + wv;
  if (r >= nreps) return;  // whole waves only
  sign_epilogue_wave<VPL>(c, (uint32_t)(c.rep_begin + r), part[r], out + r, &wsel[wv]);
}

// Epilogue: NI estimate/CI, INT estimate, mixquant, INT CI (vert-cor.R:233-254, 186-194, 281-313).
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_epilogue(SignConst c,
                                                              const SignPartial* __restrict__ part,
                                                              dcor_rep_out* out) {
  __shared__ double lap[10];
  __shared__ SelScratch sel;
  const uint32_t rep = (uint32_t)(c.rep_begin + blockIdx.x);
  scalar_laplace(rep, c.k0, c.k1, lap);
  __syncthreads();
  const SignPartial p = part[blockIdx.x];
  sign_finish(c, rep, DD{p.sT[0], p.sT[1]}, DD{p.sT2[0], p.sT2[1]}, p.core, (p.flags & 1) != 0,
              (p.flags & 2) != 0, lap, &sel, out + blockIdx.x);
}

static inline void launch_sign_epilogue(const SignConst& c, int64_t nr, const SignPartial* part,
                                        dcor_rep_out* out, hipStream_t st) {
  const int block_epi = [] {
    const char* v = dcor::variant("DCOR_EPILOGUE");
    return v && std::strcmp(v, "block") == 0;
  }();
  const unsigned gw = (unsigned)((nr + DCOR_WAVES - 1) / DCOR_WAVES);
  if (block_epi)
    hipLaunchKernelGGL(k_sign_epilogue, dim3((unsigned)nr), dim3(DCOR_BLOCK), 0, st, c, part, out);
  else if (c.mix.nsim <= 1024)
    hipLaunchKernelGGL(k_sign_epilogue_w<16>, dim3(gw), dim3(DCOR_BLOCK), 0, st, c, nr, part, out);
  else
    hipLaunchKernelGGL(k_sign_epilogue_w<32>, dim3(gw), dim3(DCOR_BLOCK), 0, st, c, nr, part, out);
}

// ================================ Bernoulli sign family: bit planes (hot, exact) ===
// gen_bernoulli (vert-cor.R:78-98) yields X, Y in {0, 1}, so clip(X) takes two values and
// every sign is one of two per threshold: s0 = sign((clip(0) - mu)/sd), s1 = sign((clip(1)
// - mu)/sd) (vert-cor.R:343-347), evaluated once per replicate with the exact rule.  The
// replicate reduces to counts: pass A generates each sample once into three bit planes
// (X, Y, flip) in a per-replicate slab (0.375 B/sample) and popcounts the INT combination
// totals; pass B gives each NI batch its popcounts (vert-cor.R:226-229).  Results equal
// the per-sample algorithm's exactly.  One kernel per replicate chunk, then the epilogue.
// Plane word w covers samples [64w, 64w + 64); a wave's 256-sample chunk is 4 words, built
// from 12 ballots (lane l holds samples 4l..4l+3) by a 4-way bit interleave on the SALU.
__device__ __forceinline__ uint64_t part1by3(uint64_t x) {
  x &= 0xFFFFull;
  x = (x ^ (x << 24)) & 0x000000FF000000FFull;
  x = (x ^ (x << 12)) & 0x000F000F000F000Full;
  x = (x ^ (x << 6)) & 0x0303030303030303ull;
  x = (x ^ (x << 3)) & 0x1111111111111111ull;
  return x;
}
__device__ __forceinline__ uint64_t interleave4(const uint64_t (&b)[4], int q) {
  const int sh = 16 * q;
  return part1by3(b[0] >> sh) | (part1by3(b[1] >> sh) << 1) | (part1by3(b[2] >> sh) << 2) |
         (part1by3(b[3] >> sh) << 3);
}

// Pass A of one thread for the four samples of group g4 (< ngrp): X, Y and flip bits
// (Dgp<BERNOULLI>::one_u24; bit q = sample 4 g4 + q).
__device__ __forceinline__ void bern_gen4(const SignConst& c, uint32_t rep, int64_t g4,
                                          uint32_t& xb, uint32_t& yb, uint32_t& fb) {
  xb = yb = fb = 0;
  const uint32_t i0 = (uint32_t)(4 * g4);
  const U4 a = draw(i0 >> 1, rep, DCOR_SITE_DGP_A, c.k0, c.k1);
  const U4 b = draw((i0 >> 1) + 1, rep, DCOR_SITE_DGP_A, c.k0, c.k1);
  const uint32_t wa[4] = {a.w0, a.w2, b.w0, b.w2}, wb[4] = {a.w1, a.w3, b.w1, b.w3};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if ((int64_t)i0 + q < c.n) {
      const bool x1 = Dgp<DCOR_DGP_BERNOULLI>::xbit(wa[q]);
      const bool y1 = Dgp<DCOR_DGP_BERNOULLI>::ybit(c.g, wa[q], x1);
      xb |= (uint32_t)x1 << q;
      yb |= (uint32_t)y1 << q;
      fb |= (uint32_t)((wb[q] >> 8) < c.flipT24) << q;
    }
  }
}

// Wave-uniform counts of one 256-sample chunk (ballots of the lanes' 4 sample bits) and its
// sample-ordered plane words (interleave4).
struct BernCounts { long long n1x, n1y, n11, fx, fy, f11, ft; };
__device__ __forceinline__ void bern_ballots(uint32_t xb, uint32_t yb, uint32_t fb, BernCounts& t,
                                             uint64_t (&BX)[4], uint64_t (&BY)[4],
                                             uint64_t (&BF)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    BX[q] = __ballot((xb >> q) & 1u);
    BY[q] = __ballot((yb >> q) & 1u);
    BF[q] = __ballot((fb >> q) & 1u);
    t.n1x += __popcll(BX[q]);
    t.n1y += __popcll(BY[q]);
    t.n11 += __popcll(BX[q] & BY[q]);
    t.fx += __popcll(BF[q] & BX[q]);
    t.fy += __popcll(BF[q] & BY[q]);
    t.f11 += __popcll(BF[q] & BX[q] & BY[q]);
    t.ft += __popcll(BF[q]);
  }
}

// Thresholds (vert-cor.R:322-348), the two signs per threshold, the INT flip sum from the
// combination counts (vert-cor.R:175-183) and the NaN flags.
struct BernSigns {
  int sN0x, sN1x, sN0y, sN1y;
  bool bN0x, bN1x, bN0y, bN1y;
  bool bad_ni, bad_int;
  long long core;
};
__device__ __forceinline__ BernSigns bern_signs(const SignConst& c, const BernCounts& t,
                                                const double (&l8)[8]) {
  BernSigns r;
  const double c0 = rclip_fin(0.0, c.L), c1 = rclip_fin(1.0, c.L);
  int sI0x, sI1x, sI0y, sI1y;
  bool bI0x = false, bI1x = false, bI0y = false, bI1y = false;
  r.bN0x = r.bN1x = r.bN0y = r.bN1y = false;
  r.bad_ni = r.bad_int = false;
  if (c.normalise) {
    const double nd = c.nd;
    const double n0x = nd - (double)t.n1x, n0y = nd - (double)t.n1y;
    double v[4];
    v[0] = (double)t.n1x * c1 + n0x * c0;
    v[1] = (double)t.n1x * (c1 * c1) + n0x * (c0 * c0);
    v[2] = (double)t.n1y * c1 + n0y * c0;
    v[3] = (double)t.n1y * (c1 * c1) + n0y * (c0 * c0);
    SignStd st;
    priv_std_from_sums(c, v, l8, st);
    const bool thr_nan = (st.muNx != st.muNx) || (st.muNy != st.muNy) || (st.muIx != st.muIx) ||
                         (st.muIy != st.muIy) || (st.sdNx != st.sdNx) || (st.sdNy != st.sdNy) ||
                         (st.sdIx != st.sdIx) || (st.sdIy != st.sdIy);
    r.bad_ni = r.bad_int = thr_nan;
    r.sN0x = sgn_std(c0, st.muNx, st.sdNx, r.bN0x); r.sN1x = sgn_std(c1, st.muNx, st.sdNx, r.bN1x);
    r.sN0y = sgn_std(c0, st.muNy, st.sdNy, r.bN0y); r.sN1y = sgn_std(c1, st.muNy, st.sdNy, r.bN1y);
    sI0x = sgn_std(c0, st.muIx, st.sdIx, bI0x); sI1x = sgn_std(c1, st.muIx, st.sdIx, bI1x);
    sI0y = sgn_std(c0, st.muIy, st.sdIy, bI0y); sI1y = sgn_std(c1, st.muIy, st.sdIy, bI1y);
  } else {  // signs of the raw values (vert-cor.R:172-173, 226-227)
    r.sN0x = r.sN0y = sI0x = sI0y = 0;
    r.sN1x = r.sN1y = sI1x = sI1y = 1;
  }
  const long long N10 = t.n1x - t.n11, N01 = t.n1y - t.n11, N00 = (long long)c.n - t.n1x - t.n1y + t.n11;
  const long long F10 = t.fx - t.f11, F01 = t.fy - t.f11, F00 = t.ft - t.fx - t.fy + t.f11;
  r.core = (long long)(sI1x * sI1y) * (2 * t.f11 - t.n11) + (long long)(sI1x * sI0y) * (2 * F10 - N10) +
           (long long)(sI0x * sI1y) * (2 * F01 - N01) + (long long)(sI0x * sI0y) * (2 * F00 - N00);
  r.bad_int |= (bI1x && t.n1x > 0) || (bI0x && t.n1x < c.n) || (bI1y && t.n1y > 0) ||
               (bI0y && t.n1y < c.n);
  return r;
}

// NI batch j from the plane popcounts (vert-cor.R:226-239).
__device__ __forceinline__ void bern_batch(const SignConst& c, const BernSigns& sg,
                                           const uint64_t* PX, const uint64_t* PY, int64_t j,
                                           uint32_t rep, DD& sT, DD& sT2, bool& bad_ni) {
  const int64_t a = j * c.m, b = a + c.m;
  const int64_t wa = a >> 6, wb = (b - 1) >> 6;
  int cx1 = 0, cy1 = 0;
  for (int64_t w = wa; w <= wb; ++w) {
    uint64_t mask = ~0ull;
    if (w == wa) mask &= ~0ull << (a & 63);
    if (w == wb) mask &= ~0ull >> (63 - ((b - 1) & 63));
    cx1 += __popcll(PX[w] & mask);
    cy1 += __popcll(PY[w] & mask);
  }
  const int cx0 = c.m - cx1, cy0 = c.m - cy1;
  bad_ni |= (sg.bN1x && cx1) || (sg.bN0x && cx0) || (sg.bN1y && cy1) || (sg.bN0y && cy0);
  const int cx = sg.sN1x * cx1 + sg.sN0x * cx0, cy = sg.sN1y * cy1 + sg.sN0y * cy0;
  const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);   // vert-cor.R:230-231
  const double xt = (double)cx / c.md + c.bx * unit_laplace(u53(w.w0, w.w1));
  const double yt = (double)cy / c.md + c.by * unit_laplace(u53(w.w2, w.w3));
  const double T = c.md * xt * yt;                                     // vert-cor.R:233
  dd_acc(sT, T);
  dd_acc(sT2, T * T);
}

__device__ __forceinline__ void sign_bern_body(const SignConst& c, uint32_t rep,
                                               uint64_t* __restrict__ planes,
                                               SignPartial* __restrict__ part_out) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[8 * DCOR_WAVES];
  __shared__ double lap[10];
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t nw = 4 * ((c.n + 255) / 256);  // plane words per replicate
  scalar_laplace(rep, c.k0, c.k1, lap);
  // ---- pass A: generate, ballot into plane words, count (wave-uniform counters)
  BernCounts t{0, 0, 0, 0, 0, 0, 0};
  const int64_t ngrp = (c.n + 3) / 4;
  const int64_t ngrp_pad = (ngrp + DCOR_BLOCK - 1) / DCOR_BLOCK * DCOR_BLOCK;
  for (int64_t g4 = tid; g4 < ngrp_pad; g4 += DCOR_BLOCK) {  // whole waves stay converged
    uint32_t xb = 0, yb = 0, fb = 0;
    if (g4 < ngrp) bern_gen4(c, rep, g4, xb, yb, fb);
    uint64_t BX[4], BY[4], BF[4];
    bern_ballots(xb, yb, fb, t, BX, BY, BF);
    const int64_t w0 = (g4 - lane) / 16;  // first plane word of this wave's chunk
    if (lane < 12 && w0 < nw) {
      const int q = lane & 3, pl = lane >> 2;
      const uint64_t v = pl == 0 ? interleave4(BX, q) : (pl == 1 ? interleave4(BY, q) : interleave4(BF, q));
      planes[(size_t)pl * nw + w0 + q] = v;
    }
  }
  // block totals (one lane per wave contributes its wave-uniform counters)
  long long cnt[7] = {t.n1x, t.n1y, t.n11, t.fx, t.fy, t.f11, t.ft};
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 7; ++q) redi[8 * (tid >> 6) + q] = cnt[q];
  }
  __syncthreads();  // also orders the plane stores before pass B (workgroup scope)
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    long long v = 0;
#pragma unroll
    for (int w = 0; w < DCOR_WAVES; ++w) v += redi[8 * w + q];
    cnt[q] = v;
  }
  const BernCounts tot{cnt[0], cnt[1], cnt[2], cnt[3], cnt[4], cnt[5], cnt[6]};
  double l8[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) l8[q] = lap[q];
  const BernSigns sg = bern_signs(c, tot, l8);
  // ---- pass B: NI batches from plane popcounts
  bool bad_ni = sg.bad_ni;
  DD sT{0.0, 0.0}, sT2{0.0, 0.0};
  for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) bern_batch(c, sg, planes, planes + nw, j, rep, sT, sT2, bad_ni);
  DD d2[2] = {sT, sT2};
  block_sum_dd<2>(d2, red);
  const long long nbad = block_sum_i(bad_ni ? 1LL : 0LL, redi);
  if (tid == 0) {
    SignPartial p;
    p.sT[0] = d2[0].hi; p.sT[1] = d2[0].lo; p.sT2[0] = d2[1].hi; p.sT2[1] = d2[1].lo;
    p.core = sg.core;
    p.flags = (nbad ? 1 : 0) | (sg.bad_int ? 2 : 0);
    *part_out = p;
  }
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_bern(SignConst c, uint64_t* __restrict__ scratch,
                                                          SignPartial* __restrict__ part) {
  const int64_t nw = 4 * ((c.n + 255) / 256);
  sign_bern_body(c, (uint32_t)(c.rep_begin + blockIdx.x),
                 scratch + (size_t)blockIdx.x * 3 * (size_t)nw, part + blockIdx.x);
}

// Wave-per-replicate form for n <= BERN_W_NMAX: the planes of a replicate (3 x n/8 B) stay
// in LDS, four replicates per workgroup run without workgroup barriers, so many more
// replicates are in flight per CU (the per-replicate fixed work -- scalar Laplace,
// thresholds, reductions -- is latency that the other waves hide).
#define BERN_W_NMAX 16384
#define BERN_W_WORDS (4 * (BERN_W_NMAX / 256))
__device__ __forceinline__ void sign_bern_wave(const SignConst& c, uint32_t rep,
                                               uint64_t (*pls)[BERN_W_WORDS],
                                               SignPartial* __restrict__ part_out) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = 4 * ((c.n + 255) / 256);
  // scalar Laplace blocks 0..3 (NI / INT mu, m2 of X, Y): lane q < 4 draws block q
  double la = 0.0, lb = 0.0;
  if (lane < 4) {
    const U4 w = draw((uint32_t)lane, rep, DCOR_SITE_SCALAR, c.k0, c.k1);
    la = unit_laplace(u53(w.w0, w.w1));
    lb = unit_laplace(u53(w.w2, w.w3));
  }
  double l8[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) { l8[2 * q] = __shfl(la, q, 64); l8[2 * q + 1] = __shfl(lb, q, 64); }
  // ---- pass A
  BernCounts t{0, 0, 0, 0, 0, 0, 0};
  const int64_t ngrp = (c.n + 3) / 4;
  for (int64_t g0 = 0; g0 < ngrp; g0 += 64) {
    const int64_t g4 = g0 + lane;
    uint32_t xb = 0, yb = 0, fb = 0;
    if (g4 < ngrp) bern_gen4(c, rep, g4, xb, yb, fb);
    uint64_t BX[4], BY[4], BF[4];
    bern_ballots(xb, yb, fb, t, BX, BY, BF);
    const int64_t w0 = g0 / 16;
    if (lane < 12 && w0 + (lane & 3) < nw) {
      const int q = lane & 3, pl = lane >> 2;
      pls[pl][w0 + q] = pl == 0 ? interleave4(BX, q) : (pl == 1 ? interleave4(BY, q) : interleave4(BF, q));
    }
  }
  wave_sync();  // plane words written by lanes 0..11 are read by every lane below
  const BernSigns sg = bern_signs(c, t, l8);
  bool bad_ni = sg.bad_ni;
  DD sT{0.0, 0.0}, sT2{0.0, 0.0};
  for (int64_t j = lane; j < c.k; j += 64) bern_batch(c, sg, pls[0], pls[1], j, rep, sT, sT2, bad_ni);
  sT = wave_sum_dd(sT);
  sT2 = wave_sum_dd(sT2);
  const bool any_bad = __ballot(bad_ni) != 0;
  if (lane == 0) {
    SignPartial p;
    p.sT[0] = sT.hi; p.sT[1] = sT.lo; p.sT2[0] = sT2.hi; p.sT2[1] = sT2.lo;
    p.core = sg.core;
    p.flags = (any_bad ? 1 : 0) | (sg.bad_int ? 2 : 0);
    *part_out = p;
  }
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_bern_w(SignConst c, int64_t nreps,
                                                            SignPartial* __restrict__ part) {
  __shared__ uint64_t pls[DCOR_WAVES][3][BERN_W_WORDS];
  const int wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + wv;
  if (r >= nreps) return;  // whole waves only
  sign_bern_wave(c, (uint32_t)(c.rep_begin + r), pls[wv], part + r);
}

// ============================= fused sign family, regenerate (two-pass, A/B) ===
// The direct two-pass algorithm: pass 2 regenerates every sample.  Used for
// normalise = FALSE (signs against 0: pass 1 is skipped, so it is one pass) and as the
// A/B reference for k_sign_fused_codes (DCOR_SIGN_KERNEL=regen).
template <int DGP>
__device__ __forceinline__ void sign_fused_body(const SignConst& c, uint32_t rep, dcor_rep_out* dst) {
  __shared__ double red[16 * DCOR_WAVES];
  __shared__ long long redi[DCOR_WAVES];
  __shared__ double lap[10];
  __shared__ SelScratch sel;
  const int tid = threadIdx.x;
  scalar_laplace(rep, c.k0, c.k1, lap);
  // the same compensated sums as k_sign_pass1 (groups of 4, TwoSum, double-double reduction;
  // no second moments, see sign_pass1_body)
  DD sx{0.0, 0.0}, sy{0.0, 0.0};
  if (c.normalise) {
    for (int64_t g4 = tid; 4 * g4 < c.n; g4 += DCOR_BLOCK) {
      double x[4], y[4];
      Dgp<DGP>::quad(c.g, (uint32_t)(4 * g4), rep, c.k0, c.k1, x, y);
      double gx = 0.0, gy = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (4 * g4 + q < c.n) {
          gx += rclip_fin(x[q], c.L);
          gy += rclip_fin(y[q], c.L);
        }
      }
      ks_acc(sx, gx);
      ks_acc(sy, gy);
    }
  }
  DD d2s[2] = {sx, sy};
  block_sum_dd<2>(d2s, red);
  SignStd s;
  {
    double l8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) l8[q] = lap[q];
    const double sums[6] = {d2s[0].hi, d2s[0].lo, 0.0, d2s[1].hi, d2s[1].lo, 0.0};
    sign_std_from_pass1(c, sums, l8, s);
  }
  FlipGen fl;
  fl.cidx = 0xffffffffu;
  bool bad_ni = false, bad_int = false;
  DD sT{0.0, 0.0}, sT2{0.0, 0.0};
  long long core = 0;
  auto signs = [&](uint32_t i, int& nx, int& ny, int& ix, int& iy, bool& bni, int& flip) {
    double x, y;
    if constexpr (Dgp<DGP>::flip_src == FLIP_SPARE24) {
      uint32_t u24;
      Dgp<DGP>::one_u24(c.g, i, rep, c.k0, c.k1, x, y, u24);
      flip = u24 < c.flipT24 ? 1 : -1;
    } else if constexpr (Dgp<DGP>::flip_src == FLIP_SPARE32) {
      uint32_t w3;
      Dgp<DGP>::one_w3(c.g, i, rep, c.k0, c.k1, x, y, w3);
      flip = ((uint64_t)w3 < c.flipT) ? 1 : -1;
    } else {
      Dgp<DGP>::one(c.g, i, rep, c.k0, c.k1, x, y);
      flip = fl.get(i, rep, c.k0, c.k1, c.flipT);
    }
    if (c.normalise) {
      const double xc = rclip_fin(x, c.L), yc = rclip_fin(y, c.L);
      nx = sgn_std(xc, s.muNx, s.sdNx, bni);
      ny = sgn_std(yc, s.muNy, s.sdNy, bni);
      ix = sgn_std(xc, s.muIx, s.sdIx, bad_int);
      iy = sgn_std(yc, s.muIy, s.sdIy, bad_int);
    } else {
      bool b = false;
      nx = ix = sgn_raw(x, b);
      ny = iy = sgn_raw(y, b);
      bni |= b;
      bad_int |= b;
    }
  };
  for (int64_t j = tid; j < c.k; j += DCOR_BLOCK) {
    int cx = 0, cy = 0;
    const int64_t i0 = j * c.m;
    for (int r = 0; r < c.m; ++r) {
      const uint32_t i = (uint32_t)(i0 + r);
      int nx, ny, ix, iy, flip;
      signs(i, nx, ny, ix, iy, bad_ni, flip);
      cx += nx; cy += ny;
      core += flip * ix * iy;
    }
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);
    const double xt = (double)cx / c.md + c.bx * unit_laplace(u53(w.w0, w.w1));
    const double yt = (double)cy / c.md + c.by * unit_laplace(u53(w.w2, w.w3));
    const double T = c.md * xt * yt;
    dd_acc(sT, T);
    dd_acc(sT2, T * T);
  }
  for (int64_t i = c.k * c.m + tid; i < c.n; i += DCOR_BLOCK) {
    int nx, ny, ix, iy, flip;
    bool ignore = false;
    signs((uint32_t)i, nx, ny, ix, iy, ignore, flip);
    core += flip * ix * iy;
  }
  DD d2[2] = {sT, sT2};
  block_sum_dd<2>(d2, red);
  core = block_sum_i(core, redi);
  const long long nbad = block_sum_i((bad_ni ? 1LL : 0LL) + (bad_int ? (1LL << 20) : 0LL), redi);
  sign_finish(c, rep, d2[0], d2[1], core, (nbad & 0xFFFFF) != 0, (nbad >> 20) != 0, lap, &sel, dst);
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_sign_fused(SignConst c, dcor_rep_out* out) {
  sign_fused_body<DGP>(c, (uint32_t)(c.rep_begin + blockIdx.x), out + blockIdx.x);
}

// ===================================================== fused sub-G family ===
// correlation_NI_subG + ci_INT_subG (ver-cor-subG.R:25-108): single pass (the clip
// thresholds are data-independent).  Each thread owns whole contiguous batches.
// WAVE = false: one 256-thread workgroup per replicate; WAVE = true: one wave per replicate (cells
// with n <= SUBG_W_NMAX, the reference grid's sizes), wave reductions and the wave mixquant.
template <int DGP, bool WAVE, int VPL = 16>
__device__ __forceinline__ void subg_fused_core(const SubgConst& c, uint32_t rep, dcor_rep_out* dst,
                                                SelScratch* sel, WaveMix<VPL>* ws) {
  constexpr int NT = WAVE ? 64 : DCOR_BLOCK;
  const int tid = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  double lapz;
  {
    const U4 w = draw(4u, rep, DCOR_SITE_SCALAR, c.k0, c.k1);   // uniform: every thread draws it
    lapz = unit_laplace(u53(w.w0, w.w1));
  }
  DD sP{0, 0}, sT{0, 0}, sT2{0, 0}, sU{0, 0}, sU2{0, 0};
  auto uc_of = [&](double x, double y, double l) {
    const double S = c.sender_is_X ? x : y, O = c.sender_is_X ? y : x;
    return rclip_fin((rclip_fin(S, c.ls) + c.bs * l) * O, c.lr);          // ver-cor-subG.R:88-90
  };
  auto int_term = [&](double x, double y, double l) {
    const double Uc = uc_of(x, y, l);
    ks_acc(sU, Uc);  // compensated sums (error ~ n 2^-106): the mean / sd of Uc
    ks_acc(sU2, Uc * Uc);
  };
  // two samples' INT terms added plainly and the pair sum compensated: half the TwoSum chains of
  // per-term sums (as the HRS kernels do), sums that differ from per-term ones in the low bits only
  auto int_term2 = [&](double U0, double U1) {
    ks_acc(sU, U0 + U1);
    ks_acc(sU2, U0 * U0 + U1 * U1);
  };
  for (int64_t j = tid; j < c.k; j += NT) {
    double sx = 0.0, sy = 0.0;
    const int64_t i0 = j * c.m;
    int r = 0;
    for (; r + 1 < c.m; r += 2) {
      double x0, y0, l0, x1, y1, l1;
      sample_lap<DGP>(c.g, (uint32_t)(i0 + r), rep, c.k0, c.k1, x0, y0, l0);
      sample_lap<DGP>(c.g, (uint32_t)(i0 + r + 1), rep, c.k0, c.k1, x1, y1, l1);
      sx += rclip_fin(x0, c.l1);                                         // :33
      sy += rclip_fin(y0, c.l2);                                         // :34
      sx += rclip_fin(x1, c.l1);
      sy += rclip_fin(y1, c.l2);
      int_term2(uc_of(x0, y0, l0), uc_of(x1, y1, l1));
    }
    if (r < c.m) {
      double x, y, l;
      sample_lap<DGP>(c.g, (uint32_t)(i0 + r), rep, c.k0, c.k1, x, y, l);
      sx += rclip_fin(x, c.l1);
      sy += rclip_fin(y, c.l2);
      int_term(x, y, l);
    }
    const U4 w = draw((uint32_t)j, rep, DCOR_SITE_NI_LAP, c.k0, c.k1);
    const double mx = c.md_pow2 ? sx * c.inv_md : sx / c.md;            // exact for m = 2^e
    const double my = c.md_pow2 ? sy * c.inv_md : sy / c.md;
    const double xt = mx + c.bx * unit_laplace(u53(w.w0, w.w1));        // :48
    const double yt = my + c.by * unit_laplace(u53(w.w2, w.w3));        // :49
    ks_acc(sP, xt * yt);
    const double T = c.md * xt * yt;                                     // :55
    ks_acc(sT, T);
    ks_acc(sT2, T * T);
  }
  for (int64_t i = c.k * c.m + tid; i < c.n; i += NT) {
    double x, y, l;
    sample_lap<DGP>(c.g, (uint32_t)i, rep, c.k0, c.k1, x, y, l);
    int_term(x, y, l);
  }
  DD d5[5] = {sP, sT, sT2, sU, sU2};
  if constexpr (WAVE) {
#pragma unroll
    for (int q = 0; q < 5; ++q) d5[q] = wave_sum_dd(d5[q]);
  } else {
    __shared__ double red[16 * DCOR_WAVES];
    block_sum_dd<5>(d5, red);
  }
  double o[6];
  ni_subg_result(c, d5[0], d5[1], d5[2], o);
  const DD mU = dd_div_d(d5[3], c.nd);
  const double rho = (mU.hi + mU.lo) + c.s_central * lapz;             // :91
  const double sd = sqrt(dd_var(d5[3], d5[4], c.nd));
  const double se_norm = sqrt(sd * sd + c.sn2x2);                      // :99
  const double cstar = 2.0 / (c.sqrt_n * sd * c.eps_r);                // :100
  double q;
  if constexpr (WAVE) q = wave_mixquant_fused<VPL>(c.mix, cstar, rep, c.k0, c.k1, ws);
  else q = mixquant_fused(c.mix, cstar, rep, c.k0, c.k1, sel);
  const double width = q * se_norm / c.sqrt_n;                         // :101
  o[3] = rho;
  o[4] = rmax(rho - width, -1.0);
  o[5] = rmin(rho + width, 1.0);
  if (tid == 0) *dst = dcor_rep_out{o[0], o[1], o[2], o[3], o[4], o[5]};
}

template <int DGP>
__device__ __forceinline__ void subg_fused_body(const SubgConst& c, uint32_t rep, dcor_rep_out* dst) {
  __shared__ SelScratch sel;
  subg_fused_core<DGP, false, 16>(c, rep, dst, &sel, nullptr);
}

template <int DGP, int VPL>
__global__ __launch_bounds__(DCOR_BLOCK) void k_subg_fused_w(SubgConst c, int64_t nreps, dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  const int wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + __builtin_amdgcn_readfirstlane(wv);
  if (r >= nreps) return;  // whole waves only
  subg_fused_core<DGP, true, VPL>(c, (uint32_t)(c.rep_begin + r), out + r, nullptr, &wsel[wv]);
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_subg_fused(SubgConst c, dcor_rep_out* out) {
  subg_fused_body<DGP>(c, (uint32_t)(c.rep_begin + blockIdx.x), out + blockIdx.x);
}

// ================================================== batched grid kernels ===
// The same bodies over a work-item table (dcor_grid_launch): workgroup (or wave) w runs item
// items[w] with the constants of cells[item.cell].  Both index loads are uniform, so the
// constants are scalar loads as with a kernel argument.
template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_pass1(const SignConst* __restrict__ cells,
                                                                const GridItem* __restrict__ items,
                                                                uint32_t* __restrict__ scratch,
                                                                double* __restrict__ sums) {
  const GridItem it = items[blockIdx.x];
  sign_pass1_body<DGP>(cells[it.cell], it.rep, scratch + it.scratch, sums + SIGN_SUMS * (size_t)blockIdx.x);
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK, DCOR_P2_WPE) void k_grid_sign_pass2(const SignConst* __restrict__ cells,
                                                                const GridItem* __restrict__ items,
                                                                const uint32_t* __restrict__ scratch,
                                                                const double* __restrict__ sums,
                                                                SignPartial* __restrict__ part) {
  const GridItem it = items[blockIdx.x];
  sign_pass2_body<DGP>(cells[it.cell], it.rep, scratch + it.scratch,
                       sums + SIGN_SUMS * (size_t)blockIdx.x, part + blockIdx.x);
}

// wave w of the launch = item w; the index is made wave-uniform (SGPR) for the table loads
__device__ __forceinline__ int64_t wave_item() {
  return (int64_t)blockIdx.x * DCOR_WAVES + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

template <int VPL>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_epilogue(const SignConst* __restrict__ cells,
                                                                   const GridItem* __restrict__ items,
                                                                   int64_t nitems,
                                                                   const SignPartial* __restrict__ part,
                                                                   dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  const int64_t r = wave_item();
  if (r >= nitems) return;  // whole waves only
  const GridItem it = items[r];
  sign_epilogue_wave<VPL>(cells[it.cell], it.rep, part[r], out + it.out, &wsel[threadIdx.x >> 6]);
}

// Small cells (n <= SIGN_W_NMAX): wave-per-replicate pass 1 (persistent workgroups) and pass 2 +
// epilogue over the work items.
template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_pass1_w(const SignConst* __restrict__ cells,
                                                                  const GridItem* __restrict__ items,
                                                                  int64_t nitems,
                                                                  uint32_t* __restrict__ scratch,
                                                                  double* __restrict__ sums) {
  __shared__ double2 zt[DGP == DCOR_DGP_GAUSSIAN ? 2 * DCOR_ZIG_N : 1];
  __shared__ uint32_t zq[DCOR_WAVES][DGP == DCOR_DGP_GAUSSIAN ? ZQ_CAP : 1];
  __shared__ uint32_t zqn[DCOR_WAVES];
  pass1_w_setup<DGP>(zt, zqn);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (int64_t r = (int64_t)blockIdx.x * DCOR_WAVES + wv; r < nitems; r += (int64_t)gridDim.x * DCOR_WAVES) {
    const GridItem it = items[r];
    sign_pass1_core<DGP, true>(cells[it.cell], it.rep, scratch + it.scratch, sums + SIGN_SUMS * (size_t)r,
                               zt, zq[wv], &zqn[wv]);
  }
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_pass2_w(const SignConst* __restrict__ cells,
                                                                  const GridItem* __restrict__ items,
                                                                  int64_t nitems,
                                                                  const uint32_t* __restrict__ scratch,
                                                                  const double* __restrict__ sums,
                                                                  SignPartial* __restrict__ part, int pstride) {
  __shared__ double2 lt[256];
  __shared__ uint32_t tq[DCOR_WAVES][TQ];
  log_tab_to_lds(lt, DCOR_BLOCK);
  __syncthreads();
  const int64_t r = wave_item();
  if (r >= nitems) return;
  const GridItem it = items[r];
  sign_pass2_wave_part<DGP>(cells[it.cell], it.rep, scratch + it.scratch, sums + SIGN_SUMS * (size_t)r, part + r,
                            lt, pstride, tq[threadIdx.x >> 6]);
}

template <int DGP, int VPL>
__global__ __launch_bounds__(DCOR_BLOCK, DGP == DCOR_DGP_MIX_GAUSSIAN ? 3 : DCOR_P2E_WPE) void k_grid_sign_p2e_w(const SignConst* __restrict__ cells,
                                                                const GridItem* __restrict__ items,
                                                                int64_t nitems,
                                                                const uint32_t* __restrict__ scratch,
                                                                const double* __restrict__ sums,
                                                                dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  P2E_LOG_TABLE(lt);
  const int64_t r = wave_item();
  if (r >= nitems) return;  // whole waves only
  const GridItem it = items[r];
  const SignConst& c = cells[it.cell];
  // the piece buffer lives in the wave's mixquant keys, which the epilogue fills only after pass 2
  const P2Result p = sign_pass2_core<DGP, true>(c, it.rep, scratch + it.scratch, sums + SIGN_SUMS * (size_t)r, lt,
                                                reinterpret_cast<uint32_t*>(wsel[threadIdx.x >> 6].keys),
                                                wsel[threadIdx.x >> 6].sel.hist);
  sign_finish_wave<VPL>(c, it.rep, p, out + it.out, &wsel[threadIdx.x >> 6]);
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_regen(const SignConst* __restrict__ cells,
                                                                const GridItem* __restrict__ items,
                                                                dcor_rep_out* out) {
  const GridItem it = items[blockIdx.x];
  sign_fused_body<DGP>(cells[it.cell], it.rep, out + it.out);
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_bern(const SignConst* __restrict__ cells,
                                                               const GridItem* __restrict__ items,
                                                               uint64_t* __restrict__ scratch,
                                                               SignPartial* __restrict__ part) {
  const GridItem it = items[blockIdx.x];
  sign_bern_body(cells[it.cell], it.rep, scratch + it.scratch, part + blockIdx.x);
}

__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_sign_bern_w(const SignConst* __restrict__ cells,
                                                                 const GridItem* __restrict__ items,
                                                                 int64_t nitems,
                                                                 SignPartial* __restrict__ part) {
  __shared__ uint64_t pls[DCOR_WAVES][3][BERN_W_WORDS];
  const int64_t r = wave_item();
  if (r >= nitems) return;
  const GridItem it = items[r];
  sign_bern_wave(cells[it.cell], it.rep, pls[threadIdx.x >> 6], part + r);
}

template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_subg(const SubgConst* __restrict__ cells,
                                                          const GridItem* __restrict__ items,
                                                          dcor_rep_out* out) {
  const GridItem it = items[blockIdx.x];
  subg_fused_body<DGP>(cells[it.cell], it.rep, out + it.out);
}

// Work items of one chunk launch from its pieces: workgroup p writes piece p's items.
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_expand(const GridPiece* __restrict__ pieces,
                                                            GridItem* __restrict__ items) {
  const GridPiece pc = pieces[blockIdx.x];
  for (uint64_t t = threadIdx.x; t < pc.count; t += DCOR_BLOCK)
    items[pc.item0 + t] = GridItem{pc.cell, pc.rep0 + (uint32_t)t, pc.scr0 + t * pc.scr_stride, pc.out0 + t};
}

template <int DGP, int VPL>
__global__ __launch_bounds__(DCOR_BLOCK) void k_grid_subg_w(const SubgConst* __restrict__ cells,
                                                            const GridItem* __restrict__ items,
                                                            int64_t nitems, dcor_rep_out* out) {
  __shared__ WaveMix<VPL> wsel[DCOR_WAVES];
  const int64_t r = wave_item();
  if (r >= nitems) return;  // whole waves only
  const GridItem it = items[r];
  subg_fused_core<DGP, true, VPL>(cells[it.cell], it.rep, out + it.out, nullptr, &wsel[threadIdx.x >> 6]);
}

// ============================================================ launchers ===
static inline int last_err() { return (int)hipGetLastError(); }

int launch_grid_expand(const GridPiece* pieces, int64_t npieces, GridItem* items, void* stream) {
  if (npieces <= 0) return 0;
  hipLaunchKernelGGL(k_grid_expand, dim3((unsigned)npieces), dim3(DCOR_BLOCK), 0, (hipStream_t)stream,
                     pieces, items);
  return last_err();
}

static inline unsigned wave_groups(int64_t n) { return (unsigned)((n + DCOR_WAVES - 1) / DCOR_WAVES); }

static void launch_grid_epilogue(const SignConst* cells, const GridItem* items, int64_t nitems,
                                 const SignPartial* part, int vpl32, dcor_rep_out* out, hipStream_t st) {
  if (vpl32)
    hipLaunchKernelGGL(k_grid_sign_epilogue<32>, dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st,
                       cells, items, nitems, part, out);
  else
    hipLaunchKernelGGL(k_grid_sign_epilogue<16>, dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st,
                       cells, items, nitems, part, out);
}

template <int DGP>
static void grid_codes_t(const SignConst* cells, const GridItem* items, int64_t nitems,
                         uint32_t* scratch, double* sums, SignPartial* part, int pmax, hipStream_t st) {
  hipLaunchKernelGGL(k_grid_sign_pass1<DGP>, dim3((unsigned)nitems), dim3(DCOR_BLOCK), 0, st, cells,
                     items, scratch, sums);
  hipLaunchKernelGGL(k_grid_sign_pass2<DGP>, dim3((unsigned)nitems), dim3(DCOR_BLOCK), sign_piece_lds(pmax), st,
                     cells, items, scratch, sums, part);
}

int launch_grid_sign_codes(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                           uint32_t* scratch, double* sums, SignPartial* part, int vpl32, int pmax,
                           dcor_rep_out* out, void* stream) {
  if (nitems <= 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  switch (dgp) {
    case DCOR_DGP_GAUSSIAN: grid_codes_t<DCOR_DGP_GAUSSIAN>(cells, items, nitems, scratch, sums, part, pmax, st); break;
    case DCOR_DGP_BERNOULLI: grid_codes_t<DCOR_DGP_BERNOULLI>(cells, items, nitems, scratch, sums, part, pmax, st); break;
    case DCOR_DGP_MIX_GAUSSIAN: grid_codes_t<DCOR_DGP_MIX_GAUSSIAN>(cells, items, nitems, scratch, sums, part, pmax, st); break;
    default: grid_codes_t<DCOR_DGP_BOUNDED_FACTOR>(cells, items, nitems, scratch, sums, part, pmax, st);
  }
  launch_grid_epilogue(cells, items, nitems, part, vpl32, out, st);
  return last_err();
}

// persistent pass-1 workgroups: at most 8 per CU of the largest part (256 CUs)
static inline unsigned persistent_groups(int64_t nitems) {
  const unsigned g = wave_groups(nitems);
  return g < 2048u ? g : 2048u;
}

// Small cells: pass 2 and the epilogue fused into one wave kernel (default; VG 3.35e7 vs 3.25e7
// replicates/s with the two kernels, r03c), or DCOR_SIGN_P2E=0 for the pass-2 wave kernel + the
// wave epilogue kernel.
static bool p2e_fused() {
  const bool v = [] {
    const char* e = dcor::variant("DCOR_SIGN_P2E");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return v;
}

template <int DGP>
static void grid_codes_w_t(const SignConst* cells, const GridItem* items, int64_t nitems, uint32_t* scratch,
                           double* sums, int vpl32, int pmax, dcor_rep_out* out, hipStream_t st) {
  hipLaunchKernelGGL(k_grid_sign_pass1_w<DGP>, dim3(persistent_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells,
                     items, nitems, scratch, sums);
  const size_t lds = sign_piece_lds(pmax);
  if (!p2e_fused()) {
    SignPartial* part = reinterpret_cast<SignPartial*>(sums + SIGN_SUMS * nitems);
    hipLaunchKernelGGL(k_grid_sign_pass2_w<DGP>, dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), lds, st, cells,
                       items, nitems, scratch, sums, part, pmax);
    launch_grid_epilogue(cells, items, nitems, part, vpl32, out, st);
    return;
  }
  if (vpl32)
    hipLaunchKernelGGL((k_grid_sign_p2e_w<DGP, 32>), dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells,
                       items, nitems, scratch, sums, out);
  else
    hipLaunchKernelGGL((k_grid_sign_p2e_w<DGP, 16>), dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells,
                       items, nitems, scratch, sums, out);
}

int launch_grid_sign_codes_w(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                             uint32_t* scratch, double* sums, int vpl32, int pmax, dcor_rep_out* out,
                             void* stream) {
  if (nitems <= 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  switch (dgp) {
    case DCOR_DGP_GAUSSIAN: grid_codes_w_t<DCOR_DGP_GAUSSIAN>(cells, items, nitems, scratch, sums, vpl32, pmax, out, st); break;
    case DCOR_DGP_BERNOULLI: grid_codes_w_t<DCOR_DGP_BERNOULLI>(cells, items, nitems, scratch, sums, vpl32, pmax, out, st); break;
    case DCOR_DGP_MIX_GAUSSIAN: grid_codes_w_t<DCOR_DGP_MIX_GAUSSIAN>(cells, items, nitems, scratch, sums, vpl32, pmax, out, st); break;
    default: grid_codes_w_t<DCOR_DGP_BOUNDED_FACTOR>(cells, items, nitems, scratch, sums, vpl32, pmax, out, st);
  }
  return last_err();
}

int launch_grid_sign_regen(int dgp, const SignConst* cells, const GridItem* items, int64_t nitems,
                           dcor_rep_out* out, void* stream) {
  if (nitems <= 0) return 0;
  const dim3 g((unsigned)nitems), b(DCOR_BLOCK);
  const hipStream_t st = (hipStream_t)stream;
  switch (dgp) {
    case DCOR_DGP_GAUSSIAN: hipLaunchKernelGGL(k_grid_sign_regen<DCOR_DGP_GAUSSIAN>, g, b, 0, st, cells, items, out); break;
    case DCOR_DGP_BERNOULLI: hipLaunchKernelGGL(k_grid_sign_regen<DCOR_DGP_BERNOULLI>, g, b, 0, st, cells, items, out); break;
    case DCOR_DGP_MIX_GAUSSIAN: hipLaunchKernelGGL(k_grid_sign_regen<DCOR_DGP_MIX_GAUSSIAN>, g, b, 0, st, cells, items, out); break;
    default: hipLaunchKernelGGL(k_grid_sign_regen<DCOR_DGP_BOUNDED_FACTOR>, g, b, 0, st, cells, items, out);
  }
  return last_err();
}

int launch_grid_sign_bern(bool wave, const SignConst* cells, const GridItem* items, int64_t nitems,
                          uint64_t* scratch, SignPartial* part, int vpl32, dcor_rep_out* out,
                          void* stream) {
  if (nitems <= 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  if (wave)
    hipLaunchKernelGGL(k_grid_sign_bern_w, dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells,
                       items, nitems, part);
  else
    hipLaunchKernelGGL(k_grid_sign_bern, dim3((unsigned)nitems), dim3(DCOR_BLOCK), 0, st, cells, items,
                       scratch, part);
  launch_grid_epilogue(cells, items, nitems, part, vpl32, out, st);
  return last_err();
}

template <int DGP>
static void grid_subg_w_t(const SubgConst* cells, const GridItem* items, int64_t nitems, int vpl32,
                          dcor_rep_out* out, hipStream_t st) {
  if (vpl32)
    hipLaunchKernelGGL((k_grid_subg_w<DGP, 32>), dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells, items,
                       nitems, out);
  else
    hipLaunchKernelGGL((k_grid_subg_w<DGP, 16>), dim3(wave_groups(nitems)), dim3(DCOR_BLOCK), 0, st, cells, items,
                       nitems, out);
}

int launch_grid_subg_w(int dgp, const SubgConst* cells, const GridItem* items, int64_t nitems, int vpl32,
                       dcor_rep_out* out, void* stream) {
  if (nitems <= 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  switch (dgp) {
    case DCOR_DGP_GAUSSIAN: grid_subg_w_t<DCOR_DGP_GAUSSIAN>(cells, items, nitems, vpl32, out, st); break;
    case DCOR_DGP_BERNOULLI: grid_subg_w_t<DCOR_DGP_BERNOULLI>(cells, items, nitems, vpl32, out, st); break;
    case DCOR_DGP_MIX_GAUSSIAN: grid_subg_w_t<DCOR_DGP_MIX_GAUSSIAN>(cells, items, nitems, vpl32, out, st); break;
    default: grid_subg_w_t<DCOR_DGP_BOUNDED_FACTOR>(cells, items, nitems, vpl32, out, st);
  }
  return last_err();
}

int launch_grid_subg(int dgp, const SubgConst* cells, const GridItem* items, int64_t nitems,
                     dcor_rep_out* out, void* stream) {
  if (nitems <= 0) return 0;
  const dim3 g((unsigned)nitems), b(DCOR_BLOCK);
  const hipStream_t st = (hipStream_t)stream;
  switch (dgp) {
    case DCOR_DGP_GAUSSIAN: hipLaunchKernelGGL(k_grid_subg<DCOR_DGP_GAUSSIAN>, g, b, 0, st, cells, items, out); break;
    case DCOR_DGP_BERNOULLI: hipLaunchKernelGGL(k_grid_subg<DCOR_DGP_BERNOULLI>, g, b, 0, st, cells, items, out); break;
    case DCOR_DGP_MIX_GAUSSIAN: hipLaunchKernelGGL(k_grid_subg<DCOR_DGP_MIX_GAUSSIAN>, g, b, 0, st, cells, items, out); break;
    default: hipLaunchKernelGGL(k_grid_subg<DCOR_DGP_BOUNDED_FACTOR>, g, b, 0, st, cells, items, out);
  }
  return last_err();
}

template <int DGP>
static int launch_sign_t(const SignConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  hipLaunchKernelGGL(k_sign_fused<DGP>, dim3((unsigned)reps), dim3(DCOR_BLOCK), 0,
                     (hipStream_t)stream, c, out);
  return last_err();
}

int launch_sign_fused(const SignConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  switch (c.g.dgp) {
    case DCOR_DGP_GAUSSIAN: return launch_sign_t<DCOR_DGP_GAUSSIAN>(c, reps, out, stream);
    case DCOR_DGP_BERNOULLI: return launch_sign_t<DCOR_DGP_BERNOULLI>(c, reps, out, stream);
    case DCOR_DGP_MIX_GAUSSIAN: return launch_sign_t<DCOR_DGP_MIX_GAUSSIAN>(c, reps, out, stream);
    default: return launch_sign_t<DCOR_DGP_BOUNDED_FACTOR>(c, reps, out, stream);
  }
}

// Replicate chunks alternate between the caller's stream and an auxiliary stream, each
// with its own slab, so pass 2 (memory-latency bound) of one chunk runs beside pass 1
// (VALU bound) of the next.
template <int DGP>
static int launch_codes_t(SignConst c, int64_t reps, int64_t chunk, const CodesBufs& bf,
                          dcor_rep_out* out, void* stream) {
  const int64_t rep0 = c.rep_begin;
  const bool two = reps > chunk && bf.lib[0] != nullptr;
  hipStream_t st[2] = {(hipStream_t)stream, (hipStream_t)stream};
  bool waited[2] = {true, true};  // this stream's `out` writers are ordered after the caller's work
  if (two) {
    st[0] = (hipStream_t)bf.lib[0];
    st[1] = (hipStream_t)bf.lib[1];
    if (hipEventRecord((hipEvent_t)bf.ev_entry, (hipStream_t)stream) != hipSuccess) return last_err();
    for (int b = 0; b < 2; ++b) {
      waited[b] = !bf.cross;
      if (!bf.cross && hipStreamWaitEvent(st[b], (hipEvent_t)bf.ev_entry, 0) != hipSuccess) return last_err();
    }
  }
  auto before_out = [&](int b) -> int {  // the first kernel writing `out` on stream b
    if (waited[b]) return 0;
    waited[b] = true;
    return hipStreamWaitEvent(st[b], (hipEvent_t)bf.ev_entry, 0) != hipSuccess ? last_err() : 0;
  };
  int64_t t = 0;
  for (int64_t r = 0; r < reps; r += chunk, ++t) {
    const int64_t nr = (reps - r < chunk) ? reps - r : chunk;
    const int b = two ? (int)(t & 1) : 0;
    c.rep_begin = rep0 + r;
    if (c.n <= SIGN_W_NMAX) {   // small cells: the wave-per-replicate kernels (as the grid runs them)
      hipLaunchKernelGGL(k_sign_pass1_w<DGP>, dim3(persistent_groups(nr)), dim3(DCOR_BLOCK), 0, st[b], c, nr,
                         bf.slab[b], bf.sums[b]);
      if (int e = before_out(b)) return e;
      const size_t lds = sign_piece_lds(c.pieces);
      if (!p2e_fused()) {
        SignPartial* part = reinterpret_cast<SignPartial*>(bf.sums[b] + SIGN_SUMS * chunk);
        hipLaunchKernelGGL(k_sign_pass2_w<DGP>, dim3(wave_groups(nr)), dim3(DCOR_BLOCK), lds, st[b], c, nr,
                           bf.slab[b], bf.sums[b], part, c.pieces);
        launch_sign_epilogue(c, nr, part, out + r, st[b]);
      } else if (c.mix.nsim > 1024)
        hipLaunchKernelGGL((k_sign_p2e_w<DGP, 32>), dim3(wave_groups(nr)), dim3(DCOR_BLOCK), 0, st[b], c, nr,
                           bf.slab[b], bf.sums[b], out + r);
      else
        hipLaunchKernelGGL((k_sign_p2e_w<DGP, 16>), dim3(wave_groups(nr)), dim3(DCOR_BLOCK), 0, st[b], c, nr,
                           bf.slab[b], bf.sums[b], out + r);
      if (int e = last_err()) return e;
      continue;
    }
    SignPartial* part = reinterpret_cast<SignPartial*>(bf.sums[b] + SIGN_SUMS * chunk);
    hipLaunchKernelGGL(k_sign_pass1<DGP>, dim3((unsigned)nr), dim3(DCOR_BLOCK), 0, st[b], c,
                       bf.slab[b], bf.sums[b]);
    if (c.m == 8)
      hipLaunchKernelGGL((k_sign_pass2<DGP, true>), dim3((unsigned)nr), dim3(DCOR_BLOCK), 0, st[b], c,
                         bf.slab[b], bf.sums[b], part);
    else
      hipLaunchKernelGGL(k_sign_pass2<DGP>, dim3((unsigned)nr), dim3(DCOR_BLOCK), sign_piece_lds(c.pieces), st[b], c,
                         bf.slab[b], bf.sums[b], part);
    if (int e = before_out(b)) return e;
    launch_sign_epilogue(c, nr, part, out + r, st[b]);
    if (int e = last_err()) return e;
  }
  if (two) {  // the caller's stream continues after both library streams
    for (int b = 0; b < 2; ++b) {
      if (hipEventRecord((hipEvent_t)bf.ev_end[b], st[b]) != hipSuccess) return last_err();
      if (hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)bf.ev_end[b], 0) != hipSuccess) return last_err();
    }
  }
  return 0;
}

int launch_sign_fused_codes(const SignConst& c, int64_t reps, int64_t chunk, const CodesBufs& bf,
                            dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  switch (c.g.dgp) {
    case DCOR_DGP_GAUSSIAN: return launch_codes_t<DCOR_DGP_GAUSSIAN>(c, reps, chunk, bf, out, stream);
    case DCOR_DGP_BERNOULLI: return launch_codes_t<DCOR_DGP_BERNOULLI>(c, reps, chunk, bf, out, stream);
    case DCOR_DGP_MIX_GAUSSIAN: return launch_codes_t<DCOR_DGP_MIX_GAUSSIAN>(c, reps, chunk, bf, out, stream);
    default: return launch_codes_t<DCOR_DGP_BOUNDED_FACTOR>(c, reps, chunk, bf, out, stream);
  }
}

// Dynamic LDS that brings kernel `ceil`'s workgroups per CU down to kernel `real`'s (256 threads).
static int occupancy_pad(const void* real, const void* ceil, size_t* pad) {
  int want = 0, have = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&want, real, DCOR_BLOCK, 0) != hipSuccess) return last_err();
  for (*pad = 0;; *pad += 256) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&have, ceil, DCOR_BLOCK, *pad) != hipSuccess) return last_err();
    if (have <= want || *pad > 64 * 1024) return 0;
  }
}

// One pass of the one-pass sign path over `reps` replicates as a single chunk on `stream`, for
// timing (dcor_diag_sign_pass): 1 pass 1, 2 pass 2 (with the slow-sample drain), 3 the epilogue; 11 / 12 the pass-1 / pass-2
// ceilings (Gaussian DGP, m = 8) at the real passes' occupancy, 13 the pass-1 ceiling at its own.  slab / sums / part / out as launch_codes_t lays them out.
int launch_sign_diag(const SignConst& c, int64_t reps, int which, uint32_t* slab, double* sums,
                     void* part_v, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  SignPartial* part = reinterpret_cast<SignPartial*>(part_v);
  const hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)reps), b(DCOR_BLOCK);
  switch (which) {
    case 1:
      switch (c.g.dgp) {
        case DCOR_DGP_GAUSSIAN: hipLaunchKernelGGL(k_sign_pass1<DCOR_DGP_GAUSSIAN>, g, b, 0, st, c, slab, sums); break;
        case DCOR_DGP_MIX_GAUSSIAN: hipLaunchKernelGGL(k_sign_pass1<DCOR_DGP_MIX_GAUSSIAN>, g, b, 0, st, c, slab, sums); break;
        default: hipLaunchKernelGGL(k_sign_pass1<DCOR_DGP_BOUNDED_FACTOR>, g, b, 0, st, c, slab, sums);
      }
      break;
    case 2:
      switch (c.g.dgp) {
        case DCOR_DGP_GAUSSIAN:
          if (c.m == 8) hipLaunchKernelGGL((k_sign_pass2<DCOR_DGP_GAUSSIAN, true>), g, b, 0, st, c, slab, sums, part);
          else hipLaunchKernelGGL(k_sign_pass2<DCOR_DGP_GAUSSIAN>, g, b, sign_piece_lds(c.pieces), st, c, slab, sums, part);
          break;
        case DCOR_DGP_MIX_GAUSSIAN: hipLaunchKernelGGL(k_sign_pass2<DCOR_DGP_MIX_GAUSSIAN>, g, b, sign_piece_lds(c.pieces), st, c, slab, sums, part); break;
        default: hipLaunchKernelGGL(k_sign_pass2<DCOR_DGP_BOUNDED_FACTOR>, g, b, sign_piece_lds(c.pieces), st, c, slab, sums, part);
      }
      break;
    case 3: launch_sign_epilogue(c, reps, part, out, st); break;
    case 11: case 13: {
      // 11: at pass 1's occupancy (pass 1 holds more VGPRs and LDS than its ceiling); 13: its own
      size_t pad = 0;
      if (which == 11) {
        const int e = occupancy_pad((const void*)k_sign_pass1<DCOR_DGP_GAUSSIAN>, (const void*)k_sign_pass1_ceil<1>, &pad);
        if (e) return e;
      }
      hipLaunchKernelGGL(k_sign_pass1_ceil<1>, g, b, pad, st, c, slab, sums);
      break;
    }
    case 14: case 15: {   // the ceiling plus the slab stores / plus the slow-normal queue
      size_t pad = 0;
      const void* k = which == 14 ? (const void*)k_sign_pass1_ceil<2> : (const void*)k_sign_pass1_ceil<3>;
      const int e = occupancy_pad((const void*)k_sign_pass1<DCOR_DGP_GAUSSIAN>, k, &pad);
      if (e) return e;
      if (which == 14) hipLaunchKernelGGL(k_sign_pass1_ceil<2>, g, b, pad, st, c, slab, sums);
      else hipLaunchKernelGGL(k_sign_pass1_ceil<3>, g, b, pad, st, c, slab, sums);
      break;
    }
    case 12: {
      size_t pad = 0;
      const int e = occupancy_pad((const void*)k_sign_pass2<DCOR_DGP_GAUSSIAN, true>, (const void*)k_sign_pass2_ceil, &pad);
      if (e) return e;
      hipLaunchKernelGGL(k_sign_pass2_ceil, g, b, pad, st, c, slab, sums, part);
      break;
    }
    default: return (int)hipErrorInvalidValue;
  }
  return last_err();
}

int launch_sign_bern(SignConst c, int64_t reps, int64_t chunk, uint64_t* scratch,
                     SignPartial* part, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  const int64_t rep0 = c.rep_begin;
  for (int64_t r = 0; r < reps; r += chunk) {
    const int64_t nr = (reps - r < chunk) ? reps - r : chunk;
    c.rep_begin = rep0 + r;
    if (c.n <= BERN_W_NMAX)
      hipLaunchKernelGGL(k_sign_bern_w, dim3((unsigned)((nr + DCOR_WAVES - 1) / DCOR_WAVES)),
                         dim3(DCOR_BLOCK), 0, (hipStream_t)stream, c, nr, part);
    else
      hipLaunchKernelGGL(k_sign_bern, dim3((unsigned)nr), dim3(DCOR_BLOCK), 0, (hipStream_t)stream,
                         c, scratch, part);
    launch_sign_epilogue(c, nr, part, out + r, (hipStream_t)stream);
    if (int e = last_err()) return e;
  }
  return 0;
}

// The cell's DGP samples (Dgp<DGP>::one, the full draw contract): X, Y [reps][n].
template <int DGP>
__global__ __launch_bounds__(DCOR_BLOCK) void k_dgp(DgpConst g, uint32_t k0, uint32_t k1,
                                                   int64_t rep_begin, int64_t n, double* X,
                                                   double* Y) {
  const int64_t i = (int64_t)blockIdx.x * DCOR_BLOCK + threadIdx.x;
  if (i >= n) return;
  double x, y;
  Dgp<DGP>::one(g, (uint32_t)i, (uint32_t)(rep_begin + blockIdx.y), k0, k1, x, y);
  X[blockIdx.y * n + i] = x;
  Y[blockIdx.y * n + i] = y;
}

int launch_dgp(const DgpConst& g, uint32_t k0, uint32_t k1, int64_t rep_begin, int64_t reps,
               int64_t n, double* X, double* Y, void* stream) {
  if (reps <= 0 || n <= 0) return 0;
  const dim3 gr((unsigned)((n + DCOR_BLOCK - 1) / DCOR_BLOCK), (unsigned)reps), b(DCOR_BLOCK);
  const hipStream_t st = (hipStream_t)stream;
  switch (g.dgp) {
    case DCOR_DGP_GAUSSIAN: hipLaunchKernelGGL(k_dgp<DCOR_DGP_GAUSSIAN>, gr, b, 0, st, g, k0, k1, rep_begin, n, X, Y); break;
    case DCOR_DGP_BERNOULLI: hipLaunchKernelGGL(k_dgp<DCOR_DGP_BERNOULLI>, gr, b, 0, st, g, k0, k1, rep_begin, n, X, Y); break;
    case DCOR_DGP_MIX_GAUSSIAN: hipLaunchKernelGGL(k_dgp<DCOR_DGP_MIX_GAUSSIAN>, gr, b, 0, st, g, k0, k1, rep_begin, n, X, Y); break;
    default: hipLaunchKernelGGL(k_dgp<DCOR_DGP_BOUNDED_FACTOR>, gr, b, 0, st, g, k0, k1, rep_begin, n, X, Y);
  }
  return last_err();
}

template <int DGP>
static void subg_w_t(const SubgConst& c, int64_t reps, dcor_rep_out* out, hipStream_t st) {
  if (c.mix.nsim > 1024)
    hipLaunchKernelGGL((k_subg_fused_w<DGP, 32>), dim3(wave_groups(reps)), dim3(DCOR_BLOCK), 0, st, c, reps, out);
  else
    hipLaunchKernelGGL((k_subg_fused_w<DGP, 16>), dim3(wave_groups(reps)), dim3(DCOR_BLOCK), 0, st, c, reps, out);
}

int launch_subg_fused(const SubgConst& c, int64_t reps, dcor_rep_out* out, void* stream) {
  if (reps <= 0) return 0;
  if (c.n <= SUBG_W_NMAX) {   // small cells: one wave per replicate (as the grid runs them)
    const hipStream_t st = (hipStream_t)stream;
    switch (c.g.dgp) {
      case DCOR_DGP_GAUSSIAN: subg_w_t<DCOR_DGP_GAUSSIAN>(c, reps, out, st); break;
      case DCOR_DGP_BERNOULLI: subg_w_t<DCOR_DGP_BERNOULLI>(c, reps, out, st); break;
      case DCOR_DGP_MIX_GAUSSIAN: subg_w_t<DCOR_DGP_MIX_GAUSSIAN>(c, reps, out, st); break;
      default: subg_w_t<DCOR_DGP_BOUNDED_FACTOR>(c, reps, out, st);
    }
    return last_err();
  }
  const dim3 g((unsigned)reps), b(DCOR_BLOCK);
  switch (c.g.dgp) {
    case DCOR_DGP_GAUSSIAN:
      hipLaunchKernelGGL(k_subg_fused<DCOR_DGP_GAUSSIAN>, g, b, 0, (hipStream_t)stream, c, out); break;
    case DCOR_DGP_BERNOULLI:
      hipLaunchKernelGGL(k_subg_fused<DCOR_DGP_BERNOULLI>, g, b, 0, (hipStream_t)stream, c, out); break;
    case DCOR_DGP_MIX_GAUSSIAN:
      hipLaunchKernelGGL(k_subg_fused<DCOR_DGP_MIX_GAUSSIAN>, g, b, 0, (hipStream_t)stream, c, out); break;
    default:
      hipLaunchKernelGGL(k_subg_fused<DCOR_DGP_BOUNDED_FACTOR>, g, b, 0, (hipStream_t)stream, c, out);
  }
  return last_err();
}

}  // namespace dcor
