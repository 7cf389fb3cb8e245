"""Generate distributed-correlation_amd/csrc/dcor_tables.h: the tables and coefficients of the
engine's division-free log and table-driven sincospi (part of the draw-transform contract;
shared verbatim by the gfx950 kernels and the CPU oracle, like the Philox constants).

log(x), x positive normal:  x = 2^k z, z in [0.6875, 1.375) (offset 0x3fe6...), table
index i = 8 bits below the offset (dcor_log8_tab), r = fma(z, invc_i, -1), log x = k ln2 +
logc_i + log1p(r), log1p by its degree-6 Taylor polynomial (|r| < 2^-9, truncation r^7/7 <
2^-56.8 |r|).  The two intervals that touch 1.0 use c = 1, so log is exact-relative near 1.

sincospi(t), t in [0, 2]:  j = rint(64 t), d = (64 t - j) pi/64, |d| <= pi/128;
sin(pi t) = S_j cos d + C_j sin d, cos(pi t) = C_j cos d - S_j sin d, with S_j, C_j =
sin, cos(pi j / 64) and degree-7 / degree-6 Taylor polynomials in d (truncation d^8/8! <
3.3e-18).

Ziggurat (the Gaussian DGP's normals, Marsaglia & Tsang 2000 with 1024 layers): f(x) =
exp(-x^2/2); r solves the layer recursion X[1] = r, X[i+1] = f^-1(v / X[i] + f(X[i])) with the
top layer closing at f(0) = 1 (v = r f(r) + int_r^inf f, X[0] = v / f(r), X[1024] = 0).
dcor_zig_tab[2L + s] = {(-1)^s X[L], X[L+1]} (the signed strip width and the fast-accept bound);
dcor_zig_wedge[L] = {f(X[L]), f(X[L+1]) - f(X[L])}.  Computed with mpmath at 50 digits.

The R-stream mode's accurate log (csrc/dcor_rstream.h) uses the 7-bit table dcor_log_tab with
log(c) as a double-double (dcor_log_tab_lo) and its own log1p tail.

Values are computed in 60-digit decimal arithmetic and rounded once to double.
Usage: python scripts/gen_transcendental_tables.py
"""
import os
from decimal import Decimal, getcontext

getcontext().prec = 60
PI = Decimal("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "distributed-correlation_amd", "csrc", "dcor_tables.h")


def dbl(d: Decimal) -> float:
    return float(format(d, ".55e"))  # correctly rounded decimal -> double


def hx(v: float) -> str:
    return v.hex()


def exact(v: float) -> Decimal:
    return Decimal(v)  # exact binary value


def sin_cos(x: Decimal):
    s, c, term, k = Decimal(0), Decimal(0), Decimal(1), 0
    # term = x^k / k!
    while True:
        if k % 4 == 0:
            c += term
        elif k % 4 == 1:
            s += term
        elif k % 4 == 2:
            c -= term
        else:
            s -= term
        k += 1
        term = term * x / k
        if abs(term) < Decimal(10) ** -70:
            break
    return s, c


def log_table():
    rows = []
    for i in range(128):
        # tmp = ix - 0x3fe6 << 48; i = (tmp >> 45) & 127 -> z interval
        if i < 80:   # z in [0.6875, 1): width 2^-8
            a = Decimal("0.6875") + Decimal(i) / 256
            b = a + Decimal(1) / 256
        else:        # z in [1, 1.375): width 2^-7
            a = Decimal(1) + Decimal(i - 80) / 128
            b = a + Decimal(1) / 128
        c = Decimal(1) if i in (79, 80) else (a + b) / 2
        invc = dbl(1 / c)
        lg = -exact(invc).ln()
        logc = dbl(lg)
        rows.append((invc, logc, float(a), float(b), dbl(lg - exact(logc))))
    return rows


def log8_table():
    rows = []
    for i in range(256):
        # tmp = ix - 0x3fe6 << 48; i = (tmp >> 44) & 255 -> z interval
        if i < 160:  # z in [0.6875, 1): width 2^-9
            a = Decimal("0.6875") + Decimal(i) / 512
            b = a + Decimal(1) / 512
        else:        # z in [1, 1.375): width 2^-8
            a = Decimal(1) + Decimal(i - 160) / 256
            b = a + Decimal(1) / 256
        c = Decimal(1) if i in (159, 160) else (a + b) / 2
        invc = dbl(1 / c)
        rows.append((invc, dbl(-exact(invc).ln()), float(a), float(b)))
    return rows


ZIG_N = 1024


def zig_tables():
    import mpmath as mp
    mp.mp.dps = 50
    f = lambda x: mp.e ** (-x * x / 2)
    finv = lambda y: mp.sqrt(-2 * mp.log(y))
    tail = lambda r: mp.sqrt(mp.pi / 2) * mp.erfc(r / mp.sqrt(2))

    def build(r):
        v = r * f(r) + tail(r)
        X = [v / f(r), r]
        for _ in range(2, ZIG_N):
            y = v / X[-1] + f(X[-1])
            if y >= 1:
                return None, v
            X.append(finv(y))
        return X, v

    def close(r):  # > 0: r too small (the layers overshoot f(0) = 1)
        X, v = build(r)
        return 1 if X is None else v / X[-1] + f(X[-1]) - 1

    lo, hi = mp.mpf(3), mp.mpf(5)
    for _ in range(200):
        mid = (lo + hi) / 2
        if close(mid) > 0:
            lo = mid
        else:
            hi = mid
    X, v = build(hi)
    X.append(mp.mpf(0))
    tab = []
    for L in range(ZIG_N):
        xl, xn = float(X[L]), float(X[L + 1])
        tab += [(xl, xn), (-xl, xn)]
    wedge = [(float(f(X[L])), float(f(X[L + 1]) - f(X[L]))) for L in range(ZIG_N)]
    r = float(X[1])
    return r, float(v), tab, wedge


def main():
    ln2 = Decimal(2).ln()
    ln2_hi = float.fromhex("0x1.62e42fefa3800p-1")          # 42 significant bits: k * ln2_hi exact
    ln2_lo = dbl(ln2 - exact(ln2_hi))
    lp = [dbl(Decimal((-1) ** (k + 1)) / k) for k in range(2, 9)]      # log1p: c2 .. c8
    pi64 = PI / 64
    pi64_hi = float.fromhex(float(pi64).hex()[:12] + "p" + float(pi64).hex().split("p")[1])
    pi64_lo = dbl(pi64 - exact(pi64_hi))
    fact = lambda n: Decimal(1) if n < 2 else n * fact(n - 1)
    sc_s = [dbl(Decimal((-1) ** ((k - 1) // 2)) / fact(k)) for k in (3, 5, 7)]
    sc_c = [dbl(Decimal((-1) ** (k // 2)) / fact(k)) for k in (2, 4, 6, 8)]
    scp = []
    for j in range(129):
        s, c = sin_cos(PI * j / 64)
        scp.append((dbl(s), dbl(c)))
    rows = log_table()
    L = ["/* dcor_tables.h -- GENERATED by scripts/gen_transcendental_tables.py; do not edit.",
         " * Tables and coefficients of the engine's division-free log and table-driven sincospi",
         " * (the draw-transform contract; shared by the gfx950 kernels and the CPU oracle). */",
         "#ifndef DCOR_TABLES_H", "#define DCOR_TABLES_H", "",
         "#ifndef DCOR_TABLE_ATTR", "#define DCOR_TABLE_ATTR", "#endif", "",
         f"#define DCOR_LN2_HI {hx(ln2_hi)}", f"#define DCOR_LN2_LO {hx(ln2_lo)}"]
    for k, v in zip(range(2, 9), lp):
        if k <= 6:
            L.append(f"#define DCOR_LOG1P_C{k} {hx(v)}")
    for k in range(3, 11):  # R-stream log: log1p tail r^3 (c3 + c4 r + ... + c10 r^7)
        L.append(f"#define DCOR_RS_LOG1P_C{k} {hx(dbl(Decimal((-1) ** (k + 1)) / k))}")
    L += [f"#define DCOR_PI64_HI {hx(pi64_hi)}", f"#define DCOR_PI64_LO {hx(pi64_lo)}"]
    for k, v in zip((3, 5, 7), sc_s):
        L.append(f"#define DCOR_SIN_S{k} {hx(v)}")
    for k, v in zip((2, 4, 6, 8), sc_c):
        if k <= 6:
            L.append(f"#define DCOR_COS_C{k} {hx(v)}")
    L += ["", "/* R-stream log: {1/c, -log(1/c)} per z interval (index = 7 bits of x - 0x3fe6 << 48) */",
          "DCOR_TABLE_ATTR static const double dcor_log_tab[128][2] = {"]
    for invc, logc, a, b, _ in rows:
        L.append(f"  {{{hx(invc)}, {hx(logc)}}},  /* z in [{a:.8f}, {b:.8f}) */")
    L += ["};", "", "/* the draws' log: {1/c, -log(1/c)} per z interval (index = 8 bits of x - 0x3fe6 << 48) */",
          "DCOR_TABLE_ATTR static const double dcor_log8_tab[256][2] = {"]
    for invc, logc, a, b in log8_table():
        L.append(f"  {{{hx(invc)}, {hx(logc)}}},  /* z in [{a:.9f}, {b:.9f}) */")
    L += ["};", "", "/* -log(1/c) - logc_hi: the low half of a double-double log(c) (R-stream log) */",
          "DCOR_TABLE_ATTR static const double dcor_log_tab_lo[128] = {"]
    for row in rows:
        L.append(f"  {hx(row[4])},")
    L += ["};", "", "/* {sin(pi j / 64), cos(pi j / 64)}, j = 0 .. 128 */",
          "DCOR_TABLE_ATTR static const double dcor_sincospi_tab[129][2] = {"]
    for s, c in scp:
        L.append(f"  {{{hx(s)}, {hx(c)}}},")
    zr, zv, ztab, zwedge = zig_tables()
    L += ["};", "", f"/* ziggurat normal, {ZIG_N} layers (v = {zv!r}) */", f"#define DCOR_ZIG_N {ZIG_N}",
          f"#define DCOR_ZIG_R {hx(zr)}", f"#define DCOR_ZIG_RINV {hx(1.0 / zr)}",
          "/* {(-1)^s X[L], X[L+1]} at 2L + s */",
          f"DCOR_TABLE_ATTR static const double dcor_zig_tab[{2 * ZIG_N}][2] = {{"]
    for a, b in ztab:
        L.append(f"  {{{hx(a)}, {hx(b)}}},")
    L += ["};", "", "/* {f(X[L]), f(X[L+1]) - f(X[L])}, f(x) = exp(-x^2/2) */",
          f"DCOR_TABLE_ATTR static const double dcor_zig_wedge[{ZIG_N}][2] = {{"]
    for a, b in zwedge:
        L.append(f"  {{{hx(a)}, {hx(b)}}},")
    L += ["};", "", "#endif /* DCOR_TABLES_H */", ""]
    open(OUT, "w").write("\n".join(L))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
