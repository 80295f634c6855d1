// ngrtd_fastmath.hpp -- exp/log in float64 for the per-(walker, well) likelihood path.
//
// OCML's f64 exp/log are double-double compensated (~0.5 ulp, ~60-80 instructions each);
// the CE + Student-t + prior block of one unit calls them ~30 times, which made that
// block VALU-bound.  These are the classic single-precision-free reductions with a short
// polynomial (Horner on FMAs): max error <= 2 ulp over the full double range
// (tests/test_fastmath_cpu.py measures it against 80-bit long double), far inside the
// 1e-12 parity bar.  Special values follow IEEE/libm: exp(NaN)=NaN, exp(+-inf)=inf/0,
// log(x<0)=NaN, log(0)=-inf, log(inf)=inf, subnormals handled via frexp/ldexp.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace ngrtd {

#define NGRTD_FM __host__ __device__ __forceinline__

NGRTD_FM double fexp(double x) {
    const double LOG2E = 1.4426950408889634074;
    const double LN2_HI = 6.93147180369123816490e-01;   // 0x3fe62e42fee00000 (k*LN2_HI exact)
    const double LN2_LO = 1.90821492927058770002e-10;
    const double k = rint(x * LOG2E);
    double r = fma(-k, LN2_HI, x);
    r = fma(-k, LN2_LO, r);                               // |r| <= ln2/2 + tiny
    // e^r, Taylor to r^13/13! (truncation < 4e-18 relative at |r| = 0.347)
    double p = 1.0 / 6227020800.0;
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    // 2^k with k in [-1075, 1024]: split so each ldexp factor stays representable
    const int ki = (int)fmax(fmin(k, 2100.0), -2100.0);
    const int k1 = ki / 2;
    double res = ldexp(ldexp(p, k1), ki - k1);
    if (x > 709.782712893384) res = __builtin_inf();
    if (x < -745.1332191019412) res = 0.0;
    return (x != x) ? x : res;
}

NGRTD_FM double flog(double x) {
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    int e;
    double m = frexp(x, &e);                              // x = m 2^e, m in [0.5, 1)
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;                                   // m in [sqrt(1/2), sqrt(2))
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f / (2.0 + f);                       // |s| <= 0.1716
    const double s2 = s * s;
    // log(m) = 2 atanh(s) = 2s (1 + s^2/3 + s^4/5 + ...), truncated after s^24/25
    double q = 1.0 / 25.0;
    q = fma(q, s2, 1.0 / 23.0);
    q = fma(q, s2, 1.0 / 21.0);
    q = fma(q, s2, 1.0 / 19.0);
    q = fma(q, s2, 1.0 / 17.0);
    q = fma(q, s2, 1.0 / 15.0);
    q = fma(q, s2, 1.0 / 13.0);
    q = fma(q, s2, 1.0 / 11.0);
    q = fma(q, s2, 1.0 / 9.0);
    q = fma(q, s2, 1.0 / 7.0);
    q = fma(q, s2, 1.0 / 5.0);
    q = fma(q, s2, 1.0 / 3.0);
    const double hs = s * s2 * q;                         // 2s - f + ... computed as f - 2s*... below
    // log(m) = 2s + 2 s^3 q  ; write 2s = f - s f (exactly: 2s = f - s*f since s(2+f) = f)
    const double lm = fma(-s, f, f) + 2.0 * hs;
    const double ed = (double)e;
    double res = fma(ed, LN2_HI, fma(ed, LN2_LO, lm));
    if (x == 0.0) res = -__builtin_inf();
    if (x < 0.0 || x != x) res = __builtin_nan("");
    if (x == __builtin_inf()) res = x;
    return res;
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
    p = fma(p, r, 1.0 / 6227020800.0);
    p = fma(p, r, 1.0 / 479001600.0);
    p = fma(p, r, 1.0 / 39916800.0);
    p = fma(p, r, 1.0 / 3628800.0);
    p = fma(p, r, 1.0 / 362880.0);
    p = fma(p, r, 1.0 / 40320.0);
    p = fma(p, r, 1.0 / 5040.0);
    p = fma(p, r, 1.0 / 720.0);
    p = fma(p, r, 1.0 / 120.0);
    p = fma(p, r, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    const double em = fma(r * r, p, r);                     // e^r - 1
    const double t = ldexp(1.0, (int)kd);                   // exact, |kd| <= 58
    double res = (kd == 0.0) ? em : fma(t, em, t - 1.0);
    if (x > 40.0) res = fexp(x) - 1.0;                      // e^x >= 2^57: the -1 is below 1 ulp
    if (x < -40.0) res = -1.0;
    return (x != x) ? x : res;
}

}  // namespace ngrtd
