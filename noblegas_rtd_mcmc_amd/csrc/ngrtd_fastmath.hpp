// ngrtd_fastmath.hpp -- exp/log in float64 for the per-(walker, well) likelihood path.
//
// OCML's f64 exp/log are double-double compensated (~0.5 ulp, ~60-80 instructions each);
// the CE + Student-t + prior block of one unit calls them ~20 times, and FP64 VALU issue
// is what bounds the log-prob kernel.  These are table-driven (64-entry 2^(j/64) and
// 65-entry log(1 + i/64) tables, hi + lo, in LDS) with short Taylor polynomials on FMAs:
// <= 1 ulp over the full double range (tests/test_fastmath_cpu.py measures against 80-bit
// long double), far inside the 1e-12 parity bar.  Special values follow IEEE/libm:
// exp(NaN)=NaN, exp(+-inf)=inf/0, log(x<0)=NaN, log(0)=-inf, log(inf)=inf, subnormals.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "ngrtd_fmtab.hpp"

namespace ngrtd {

#define NGRTD_FM __host__ __device__ __forceinline__

// Lookup tables (ngrtd_fmtab.hpp): kernels read them from LDS -- every kernel that
// evaluates fexp/flog (or anything built on them) runs fm_lds_init() and a barrier first --
// and host code from the constant array, so host and device execute the same arithmetic.
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ double g_fm_lds[kFmTabDoubles];
#define NGRTD_FMT g_fm_lds
#else
#define NGRTD_FMT kFmTab
#endif

__device__ __forceinline__ void fm_lds_init() {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int i = threadIdx.x; i < kFmTabDoubles; i += blockDim.x) g_fm_lds[i] = kFmTab[i];
#endif
}

// a * b + c for a compile-time constant c (the addend of a Horner step).  On the device
// the constant goes to an SGPR pair (s_mov) and the step is one VOP3 v_fma_f64 reading it;
// left to the compiler, the addend was materialised into the destination VGPRs (2 v_mov
// per step, full-rate VALU work) for a v_fmac_f64.  Same IEEE fma either way.
NGRTD_FM double fma_k(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NGRTD_NO_FMA_K)   // (NGRTD_NO_FMA_K: A/B builds)
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
#else
    return fma(a, b, c);
#endif
}

NGRTD_FM unsigned fm_hi(double x) {
    unsigned long long b;
    __builtin_memcpy(&b, &x, 8);
    return (unsigned)(b >> 32);
}
NGRTD_FM double fm_with_hi(double x, unsigned hi) {
    unsigned long long b;
    __builtin_memcpy(&b, &x, 8);
    b = (b & 0xFFFFFFFFull) | ((unsigned long long)hi << 32);
    double r;
    __builtin_memcpy(&r, &b, 8);
    return r;
}

// e^x: x = (64 m + j) ln2/64 + r, |r| <= ln2/128; e^x = 2^m 2^(j/64) e^r with 2^(j/64) as
// hi + lo from the table and e^r - 1 by its Taylor series to r^6/720 (truncation
// < 3e-20).  <= 1 ulp (tests/test_fastmath_cpu.py).  NaN -> NaN, overflow -> inf,
// underflow -> 0 / subnormal.
NGRTD_FM double fexp(double x) {
    const double L64E = 92.332482616893656;              // 64 / ln 2
    const double L2HI = 6.93147180369123816490e-01 / 64; // (k ln2/64 exact for |k| < 2^21)
    const double L2LO = 1.90821492927058770002e-10 / 64;
    const double xc = fmin(fmax(x, -800.0), 800.0);
    const double kd = rint(xc * L64E);
    double r = fma(-kd, L2HI, xc);
    r = fma(-kd, L2LO, r);
    double q = 1.0 / 720.0;
    q = fma_k(q, r, 1.0 / 120.0);
    q = fma_k(q, r, 1.0 / 24.0);
    q = fma_k(q, r, 1.0 / 6.0);
    q = fma_k(q, r, 0.5);
    const double p = fma(r * r, q, r);                   // e^r - 1
    const int k = (int)kd;
    const int j = k & 63;
    const double th = NGRTD_FMT[2 * j], tl = NGRTD_FMT[2 * j + 1];
    const double res = ldexp(th + fma(th, p, tl), k >> 6);
    return (x == x) ? res : x;
}

// 10^y = e^(y ln10) with y ln10 carried as a double-double (ph + pl) through the argument
// reduction, so r is exact to ~2^-61 and the result is fexp's table/polynomial evaluation
// of e^r: < 0.51 ulp (correctly rounded in all but ~1% of cases), against NumPy's
// np.power(10.0, y) (tests/test_fastmath_cpu.py).  The frac_inf_diff advective grid
// tadv = logspace(...) needs this accuracy: t_ret = tp - tadv cancels.
NGRTD_FM double fexp10(double y) {
    const double LN10 = 2.302585092994046;
    const double LN10_LO = -2.1707562233822494e-16;      // ln10 - LN10
    const double L64E = 92.332482616893656;
    const double L2HI = 6.93147180369123816490e-01 / 64;
    const double L2LO = 1.90821492927058770002e-10 / 64;
    const double yc = fmin(fmax(y, -350.0), 350.0);
    const double ph = yc * LN10;
    const double pl = fma(yc, LN10, -ph) + yc * LN10_LO;
    const double kd = rint(ph * L64E);
    double r = fma(-kd, L2HI, ph);
    r = fma(-kd, L2LO, r) + pl;
    double q = 1.0 / 5040.0;
    q = fma_k(q, r, 1.0 / 720.0);
    q = fma_k(q, r, 1.0 / 120.0);
    q = fma_k(q, r, 1.0 / 24.0);
    q = fma_k(q, r, 1.0 / 6.0);
    q = fma_k(q, r, 0.5);
    const double p = fma(r * r, q, r);                   // e^r - 1
    const int k = (int)kd;
    const int j = k & 63;
    const double th = NGRTD_FMT[2 * j], tl = NGRTD_FMT[2 * j + 1];
    const double res = ldexp(th + fma(th, p, tl), k >> 6);
    return (y == y) ? res : y;
}

// log x: x = 2^e m, m in [1 - 2^-7, 2 - 2^-7) taken from the bit pattern, c_i = 1 + i/64
// the nearest table point, r = (m - c_i) / c_i (m - c_i exact, |r| < 2^-7); log x = e ln2 + log c_i +
// log1p(r), log1p by its Taylor series to r^8/8 (truncation < 2e-20).  <= 1 ulp.
// log(0) = -inf, log(x < 0) = NaN, log(inf) = inf, subnormals scaled by 2^54 first.
NGRTD_FM double flog(double x) {
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    const bool sub = x < 2.2250738585072014e-308;
    const double xs = sub ? x * 18014398509481984.0 : x;    // 2^54
    const unsigned hi = fm_hi(xs);
    const int i64 = (int)(((hi >> 13) & 127) + 1) >> 1;      // nearest 1/64: 0..64
    // i = 64 (m within 2^-7 of 2) is taken as m/2 next to c_0 = 1 with e + 1, so that
    // x just below 1 gives log x = log1p(r) with no cancellation against e ln2
    const bool wrap = i64 == 64;
    const int i = wrap ? 0 : i64;
    const int e = (int)((hi >> 20) & 0x7FF) - 1023 - (sub ? 54 : 0) + (wrap ? 1 : 0);
    const double m = fm_with_hi(xs, (hi & 0x000FFFFFu) | (wrap ? 0x3FE00000u : 0x3FF00000u));
    const double ci = fm_with_hi(0.0, 0x3FF00000u | ((unsigned)i << 14));   // 1 + i/64, from bits
    const double f = m - ci;
    const double r = f * NGRTD_FMT[2 * kFmExpN + 3 * i];
    double q = -0.125;
    q = fma_k(q, r, 1.0 / 7.0);
    q = fma_k(q, r, -1.0 / 6.0);
    q = fma_k(q, r, 0.2);
    q = fma_k(q, r, -0.25);
    q = fma_k(q, r, 1.0 / 3.0);
    q = fma_k(q, r, -0.5);
    const double l1p = fma(r * r, q, r);
    const double ed = (double)e;
    const double t1 = fma(ed, LN2_HI, NGRTD_FMT[2 * kFmExpN + 3 * i + 1]);
    const double t2 = fma(ed, LN2_LO, NGRTD_FMT[2 * kFmExpN + 3 * i + 2]) + l1p;
    double res = t1 + t2;
    if (x == 0.0) res = -__builtin_inf();
    if (!(x >= 0.0)) res = __builtin_nan("");
    if (x == __builtin_inf()) res = x;
    return res;
}

// flog for arguments the caller knows to be positive, normal and finite (a product of
// factors >= 1, a product of Beta factors >= 1e-280): the same arithmetic as flog on them --
// the same bits -- without the subnormal scaling and the special-value selects (~17 VALU
// instructions fewer); any other argument gives an unspecified value.
NGRTD_FM double flog_pn(double x) {
#ifdef NGRTD_NO_FLOG_PN   // (A/B builds: the general flog)
    return flog(x);
#endif
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    const unsigned hi = fm_hi(x);
    const int i64 = (int)(((hi >> 13) & 127) + 1) >> 1;
    const bool wrap = i64 == 64;
    const int i = wrap ? 0 : i64;
    const int e = (int)((hi >> 20) & 0x7FF) - 1023 + (wrap ? 1 : 0);
    const double m = fm_with_hi(x, (hi & 0x000FFFFFu) | (wrap ? 0x3FE00000u : 0x3FF00000u));
    const double ci = fm_with_hi(0.0, 0x3FF00000u | ((unsigned)i << 14));
    const double f = m - ci;
    const double r = f * NGRTD_FMT[2 * kFmExpN + 3 * i];
    double q = -0.125;
    q = fma_k(q, r, 1.0 / 7.0);
    q = fma_k(q, r, -1.0 / 6.0);
    q = fma_k(q, r, 0.2);
    q = fma_k(q, r, -0.25);
    q = fma_k(q, r, 1.0 / 3.0);
    q = fma_k(q, r, -0.5);
    const double l1p = fma(r * r, q, r);
    const double ed = (double)e;
    const double t1 = fma(ed, LN2_HI, NGRTD_FMT[2 * kFmExpN + 3 * i + 1]);
    const double t2 = fma(ed, LN2_LO, NGRTD_FMT[2 * kFmExpN + 3 * i + 2]) + l1p;
    return t1 + t2;
}
// ... and for 0 as well (log(0) = -inf): 1 - x for x in [0, 1] is 0 or >= 2^-53
NGRTD_FM double flog_z(double x) {
    const double r = flog_pn(x);
    return x == 0.0 ? -__builtin_inf() : r;
}

// expm1(x) = 2^k (e^r - 1) + (2^k - 1), x = k ln2 + r, |r| <= ln2/2: e^r - 1 by its Taylor
// series to r^14/14! (truncation < 2e-19 relative), then ONE fma with the exact 2^k - 1
// (|k| <= 57 below), so there is no cancellation for small |x| and <= 2 ulp everywhere
// (tests/test_fastmath_cpu.py).  x <= -40 rounds to -1 exactly; NaN/inf as libm.
NGRTD_FM double fexpm1(double x) {
    const double LOG2E = 1.4426950408889634074;
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    const double kd = rint(fmin(fmax(x, -40.0), 40.0) * LOG2E);
    double r = fma(-kd, LN2_HI, x);
    r = fma(-kd, LN2_LO, r);
    double p = 1.0 / 87178291200.0;
    p = fma_k(p, r, 1.0 / 6227020800.0);
    p = fma_k(p, r, 1.0 / 479001600.0);
    p = fma_k(p, r, 1.0 / 39916800.0);
    p = fma_k(p, r, 1.0 / 3628800.0);
    p = fma_k(p, r, 1.0 / 362880.0);
    p = fma_k(p, r, 1.0 / 40320.0);
    p = fma_k(p, r, 1.0 / 5040.0);
    p = fma_k(p, r, 1.0 / 720.0);
    p = fma_k(p, r, 1.0 / 120.0);
    p = fma_k(p, r, 1.0 / 24.0);
    p = fma_k(p, r, 1.0 / 6.0);
    p = fma_k(p, r, 0.5);
    const double em = fma(r * r, p, r);                     // e^r - 1
    const double t = ldexp(1.0, (int)kd);                   // exact, |kd| <= 58
    double res = (kd == 0.0) ? em : fma(t, em, t - 1.0);
    if (x > 40.0) res = fexp(x) - 1.0;                      // e^x >= 2^57: the -1 is below 1 ulp
    if (x < -40.0) res = -1.0;
    return (x != x) ? x : res;
}

}  // namespace ngrtd
