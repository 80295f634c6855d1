// ngrtd_math.hpp -- scalar float64 building blocks shared by the gfx950 kernels.
//
// CE model: utils/noble_gas_utils.py.  Every expression keeps the reference's operation
// order (Python evaluates left to right) so that per-element results agree to ~1 ulp per
// transcendental call; x**2 is x*x (pow(x,2) is exact), x**3 is x*x*x (<= 1 ulp).
// Log densities: PyMC3 3.11.2 StudentT/Beta/Normal/Uniform/HalfNormal .logp (the
// reference's third-party likelihood), each "bound" to -inf outside its support.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "ngrtd_fastmath.hpp"

#define NGRTD_HD __host__ __device__ __forceinline__

namespace ngrtd {

constexpr double kNegInf = -__builtin_inf();
constexpr double kPi = 3.141592653589793;
// -1 * np.log(0.5): the numerator of thalf_2_lambda (convolution_integral_utils.py:146-152)
constexpr double kLn2Ref = 0.6931471805599453;

// Dry-air mole fractions, noble_gas_utils.py:38-73 (He, Ne, Ar, Kr, Xe)
struct GasCoef {
    double z;               // atm_std
    double A0, A1, A2, A3;  // solubility, :138-142
    double G1, G2, G3;      // Setchenow, :145-149
};

NGRTD_HD GasCoef gas_coef(int g) {
    switch (g) {
    case 0: return {5.24e-6, -0.00953, 0.107722, 0.001969, -0.043825, -10.081, 15.1068, 4.8127};
    case 1: return {1.818e-5, -7.259, 6.95, -1.3826, 0.0538, -11.9556, 18.4062, 5.5464};
    case 2: return {9.34e-3, -9.52, 8.83, -1.8959, 0.0698, -10.6951, 16.7513, 4.9551};
    case 3: return {1.14e-6, -6.292, 5.612, -0.8881, -0.0458, -9.9787, 15.7619, 4.6181};
    default: return {8.7e-8, -3.902, 2.439, 0.3863, -0.221, -14.5524, 22.5255, 6.7513};
    }
}

// lapse_rate(), noble_gas_utils.py:103-113 -- GPa
NGRTD_HD double lapse_rate(double E) {
    return pow(1 - .0065 * E / 288.15, 5.2561) * 0.000101325;
}

// vapor_pressure(), :184-199 -- Antoine equation, GPa (NaN T takes the else branch)
NGRTD_HD double vapor_pressure(double T) {
    double A, B, C;
    if (T <= 99.0) { A = 8.07131; B = 1730.63; C = 233.426; }
    else           { A = 8.14019; B = 1810.94; C = 244.485; }
    double P = pow(10.0, A - (B / (C + T)));
    P = P / 760. * 101325;
    return P / 1.0e9;
}

// ---- likelihood-path variants (one call per (walker, well) in the batched log-prob).
// OCML's pow/exp10/log1p are double-double accurate (~0.5 ulp) and several times the cost
// of exp/log.  Here 10**y = exp(y ln10) and b**c = exp(c log b): the argument rounding
// adds |y ln10| * 2^-53 (< 3e-15 for the CE ranges) relative error -- far inside the
// 1e-12 parity bar (DESIGN.md 'Numerics').
constexpr double kLn10 = 2.302585092994045684;
NGRTD_HD double exp10_fast(double y) { return fexp(y * kLn10); }
NGRTD_HD double lapse_rate_fast(double E) {
    // (1 - .0065 E / 288.15)^5.2561 for E in [-500, 4500] m: degree-9 polynomial in
    // x = (E - 2000) / 2500, the 50-digit Chebyshev interpolant in monomial form
    // (tools/fit_lapse.py: <= 2.7e-16 relative in double Horner) -- 9 FMAs for a log and an
    // exp.  Elsewhere (and NaN) exp(5.2561 log(.)), .0065 E / 288.15 folded (<= 1 ulp).
    const double x = (E - 2000.0) * (1.0 / 2500.0);
    if (fabs(x) <= 1.0) {
        double b = 0x1.009c0d260cdd0p-48;
        b = fma_k(b, x, 0x1.bd2da15efea83p-43);
        b = fma_k(b, x, 0x1.0de2196582d5ep-36);
        b = fma_k(b, x, 0x1.4ff1690d5a15dp-29);
        b = fma_k(b, x, -0x1.0449a1098ab8bp-20);
        b = fma_k(b, x, 0x1.121ddef15cb4bp-14);
        b = fma_k(b, x, -0x1.0128f0b9dc6d6p-9);
        b = fma_k(b, x, 0x1.f57ab080e12f8p-6);
        b = fma_k(b, x, -0x1.f2c43bdf3c9eep-3);
        b = fma_k(b, x, 0x1.91b05cf635860p-1);
        return b * 0.000101325;
    }
    return fexp(5.2561 * flog(1 - E * (.0065 / 288.15))) * 0.000101325;
}
NGRTD_HD double vapor_pressure_fast(double T) {
    double A, B, C;
    if (T <= 99.0) { A = 8.07131; B = 1730.63; C = 233.426; }
    else           { A = 8.14019; B = 1810.94; C = 244.485; }
    // P / 760 * 101325 / 1e9 as one multiply by the folded constant (<= 2 ulp)
    return exp10_fast(A - (B / (C + T))) * (101325. / 760. / 1.0e9);
}

// Antoine coefficients of vapor_pressure() for T (NaN T takes the else branch), and the
// pressure from them with B / (C + T) given as B * rcp, rcp = 1 / (C + T) (<= 3 ulp).
NGRTD_HD void antoine(double T, double& A, double& B, double& C) {
    const bool lo = T <= 99.0;
    A = lo ? 8.07131 : 8.14019;
    B = lo ? 1730.63 : 1810.94;
    C = lo ? 233.426 : 244.485;
}
NGRTD_HD double vapor_pressure_rcp(double A, double B, double rcp) {
    return exp10_fast(A - B * rcp) * (101325. / 760. / 1.0e9);
}

// r_i = 1 / d_i for i < n with ONE division (the running products, one reciprocal of
// the last, then back-substitution: 3(n-1) multiplies; each r_i within ~3(n-1)/2 ulp).
// FP64 division is 11 VALU instructions on gfx950.  When some |d_i| lies outside
// [2^-200, 2^200] -- zero, inf, NaN, subnormal or extreme values, where products could
// leave the normal range or IEEE division's special values differ -- every r_i is a plain
// division instead (a divergent branch that in-range data never takes).
template <int n>
NGRTD_HD void batch_recip(const double* d, double* r) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < n; ++i) {
        const unsigned e = (fm_hi(d[i]) >> 20) & 0x7FFu;          // biased exponent
        ok &= e - (1023u - 200u) <= 400u;
    }
    if (ok) {
        double p[n];
        p[0] = d[0];
#pragma unroll
        for (int i = 1; i < n; ++i) p[i] = p[i - 1] * d[i];
        double inv = 1.0 / p[n - 1];
#pragma unroll
        for (int i = n - 1; i > 0; --i) {
            r[i] = inv * p[i - 1];
            inv *= d[i];
        }
        r[0] = inv;
    } else {
#pragma unroll
        for (int i = 0; i < n; ++i) r[i] = 1.0 / d[i];
    }
}

// Setchenow salting factor of solubility(), :154-159.  With S = 0 this is exp(0*s) = 1
// unless s is not finite (T_k <= 0), exactly as the reference.
NGRTD_HD double setchenow_gamma(const GasCoef& c, double T, double S, double T_k) {
    if (T < 65.) {
        const double setch = c.G1 + (c.G2 / (.01 * T_k)) + (c.G3 * log(.01 * T_k));
        return exp(S * setch);
    }
    return 1.;
}

// solubility(gas), :117-180 -- Henry coefficient K [GPa]
NGRTD_HD double solubility(int g, double T, double S) {
    const GasCoef c = gas_coef(g);
    const double T_k = T + 273.15;
    const double gamma = setchenow_gamma(c, T, S, T_k);
    const double x = .001 * T_k;
    const double x2 = x * x, x3 = x * x * x;
    if (g == 0) {
        const double ln_F_He = c.A0 + (c.A1 / x) + (c.A2 / x2) + (c.A3 / x3);
        const double F = exp(ln_F_He);
        const double Frac_He_gas = 5.24e-6 / 9.31e-3;
        const GasCoef ar = gas_coef(2);
        const double X_Ar_water = 1. / (exp(ar.A0 + (ar.A1 / x) + (ar.A2 / x2) + (ar.A3 / x3))) * 9.31e-3;
        const double X_he_water = F * Frac_He_gas * X_Ar_water;
        const double K_h = 5.24e-6 / X_he_water;
        return gamma * K_h;
    }
    const double ln_K = c.A0 + (c.A1 / x) + (c.A2 / x2) + (c.A3 / x3);
    return gamma * exp(ln_K);
}

// equil_conc_dry()[gas], :216-232 (T < 0 -> -9999 sentinel)
NGRTD_HD double equil_conc_dry(int g, double T, double P, double Pv, double K) {
    const double p_i = gas_coef(g).z * (P - Pv);
    const double x_i = p_i / K;
    return (T < 0.0) ? -9999.0 : x_i * (22414. / 18.);
}

// equil_conc()[gas], :202-213 (wet pressure)
NGRTD_HD double equil_conc(int g, double P, double K) {
    const double p_i = gas_coef(g).z * P;
    const double x_i = p_i / K;
    return x_i * (22414. / 18.);
}

// ce_exc()[gas] excess-air part, :247-248
NGRTD_HD double ce_excess(int g, double Ae, double F, double C_eq) {
    const double z_i = gas_coef(g).z;
    return ((1 - F) * Ae * z_i) / (1 + ((F * Ae * z_i) / C_eq));
}

// ---------------------------------------------------------------- log densities
// lgamma(x + 1/2) - lgamma(x) for x > 0, without two general lgamma() calls (the
// StudentT normaliser needs only this difference).  Shift x up by 12 with the recurrence
// lgamma(y+1) = lgamma(y) + log(y):
//   D(x) = D(x + 12) - log(P(x) / Q(x)),  P = prod_{k<12} (x + k + 1/2),  Q = prod_{k<12} (x + k),
// then the asymptotic series at y = x + 12 >= 12
//   D(y) = 1/2 log y + sum_{m>=1} (2^(1-2m) - 2) B_2m / (2m (2m-1) y^(2m-1))
// (Bernoulli numbers B_2m), truncated after y^-13: the first omitted term is < 5e-18.
// P and Q are degree-12 polynomials with exactly representable positive coefficients,
// evaluated by Horner (12 FMAs each, relative error <= 12 ulp for x > 0) -- no per-step
// selects, so the lanes of a wavefront never diverge.  x >= 1e6 skips the shift (P, Q
// would overflow near 1e25; the series alone is already exact there).
NGRTD_HD void shift12(double x, double& P, double& Q) {
    P = 1.0;
    P = fma(P, x, 72.0);
    P = fma(P, x, 2304.5);
    P = fma(P, x, 43230.0);
    P = fma(P, x, 527486.4375);
    P = fma(P, x, 4391541.0);
    P = fma(P, x, 25442216.9375);
    P = fma(P, x, 102636393.75);
    P = fma(P, x, 283508825.74609375);
    P = fma(P, x, 516212165.90625);
    P = fma(P, x, 576705198.5332031);
    P = fma(P, x, 343464997.1484375);
    P = fma(P, x, 77205601.37329102);
    Q = 1.0;
    Q = fma(Q, x, 66.0);
    Q = fma(Q, x, 1925.0);
    Q = fma(Q, x, 32670.0);
    Q = fma(Q, x, 357423.0);
    Q = fma(Q, x, 2637558.0);
    Q = fma(Q, x, 13339535.0);
    Q = fma(Q, x, 45995730.0);
    Q = fma(Q, x, 105258076.0);
    Q = fma(Q, x, 150917976.0);
    Q = fma(Q, x, 120543840.0);
    Q = fma(Q, x, 39916800.0);
    Q = Q * x;
    const bool sh = x < 1.0e6;
    P = sh ? P : 1.0;
    Q = sh ? Q : 1.0;
}
// asymptotic tail  sum_m (...) r^(2m-1),  r = 1/y
NGRTD_HD double lgamma_half_tail(double r) {
    const double r2 = r * r;
    double t = -5461.0 / 425984.0;
    t = fma(t, r2, 691.0 / 180224.0);
    t = fma(t, r2, -31.0 / 18432.0);
    t = fma(t, r2, 17.0 / 14336.0);
    t = fma(t, r2, -1.0 / 640.0);
    t = fma(t, r2, 1.0 / 192.0);
    t = fma(t, r2, -0.125);
    return t * r;
}
NGRTD_HD double lgamma_half_diff(double x) {
    double P, Q;
    shift12(x, P, Q);
    const double y = (x < 1.0e6) ? x + 12.0 : x;
    return 0.5 * flog(y) + lgamma_half_tail(1.0 / y) - flog(P / Q);
}

// StudentT.logp, summed over observations that share nu: the caller adds
//   st_const(nu) + st_term(x, mu, sigma, nu)
// st_const = lgamma((nu+1)/2) - lgamma(nu/2), as PyMC3 writes it.
NGRTD_HD double st_const(double nu) {
    return lgamma_half_diff(nu / 2.0);
}
NGRTD_HD double st_term(double x, double mu, double sigma, double nu) {
    const double lam = 1.0 / (sigma * sigma);
    const double d = x - mu;
    const double v = 0.5 * log(lam / (nu * kPi)) - (nu + 1.0) / 2.0 * log1p(lam * (d * d) / nu);
    return (lam > 0 && nu > 0 && sigma > 0) ? v : kNegInf;
}

// Beta.logp with small integer exponents (a-1, b-1 in 0..4, e.g. Beta(2,2), Beta(2,4)):
// (a-1) log x + (b-1) log1p(-x) = log(x^(a-1) (1-x)^(b-1)) -- one log instead of two.
// ia/ib < 0 selects the general two-log form.
NGRTD_HD double ipow_small(double v, int k) {
    // k in 0..7: branch-free selects, no loop
    const double v2 = v * v;
    const double lo = (k & 1) ? v : 1.0;
    const double hi = (k & 2) ? v2 : 1.0;
    const double r = lo * hi;
    return (k & 4) ? r * (v2 * v2) : r;
}
NGRTD_HD double beta_logp_fast(double x, double a, double b, double betaln_ab, int ia, int ib) {
    double lp;
    if (ia >= 0 && ib >= 0) {
        lp = flog(ipow_small(x, ia) * ipow_small(1 - x, ib)) - betaln_ab;
    } else {
        // log1p(-x) as log(1 - x): absolute error <= 2^-53 (parity bar is absolute on logp)
        const double t1 = (a == 1.0) ? 0.0 : (a - 1) * flog(x);
        const double t2 = (b == 1.0) ? 0.0 : (b - 1) * flog(1 - x);
        lp = t1 + t2 - betaln_ab;
    }
    return (x >= 0 && x <= 1) ? lp : kNegInf;
}

// StudentT sum over n observations sharing nu (one likelihood block of a unit):
//   sum_j [ lgamma((nu+1)/2) - lgamma(nu/2) + 0.5 log(lam_j/(nu pi)) - (nu+1)/2 log1p(z_j) ]
// with z_j = lam_j (x_j - mu_j)^2 / nu, evaluated as
//   n * c0 + sum_j 0.5 log lam_j - (nu+1)/2 * log(prod_j (1 + z_j)),
//   c0 = lgamma((nu+1)/2) - lgamma(nu/2) - 0.5 log(nu pi) in ONE log (see lgamma_half_diff),
// i.e. 2 logs per block instead of 3 + n, and 2 divisions (1/(y P), 1/nu) instead of n + 3.  log(1 + z) vs log1p(z) differs by < 2^-53 per
// factor.  Very large z (z >= 1e38, inf, NaN) take a per-observation log path so the
// product cannot overflow (the T < 0 sentinel -9999 gives z ~ 1e28: still one log).  hll_sum = sum_j 0.5 log lam_j (host precomputed).
// Student-t normaliser c0(nu) = lgamma((nu+1)/2) - lgamma(nu/2) - log(pi nu)/2, exact form
// (~50 FP64 operations, one division and one log).
NGRTD_HD double st_c0_exact(double nu, double inu) {
    const double x = nu / 2.0;
    double P, Q;
    shift12(x, P, Q);
    const double y = (x < 1.0e6) ? x + 12.0 : x;
    const double iyP = 1.0 / (y * P);               // one division for 1/y and Q/P
    const double qp = (Q * y) * iyP;
    return 0.5 * flog(y * qp * qp * (inu * (1.0 / kPi))) + lgamma_half_tail(P * iyP);
}

// c0(nu) from a per-plan piecewise polynomial (ngrtd.hip c0_build): kC0Sub pieces per
// binary octave of nu, over the octaves [2^e0, 2^(e0 + np/kC0Sub)) spanned by the nu
// priors' supports, kC0N monomial coefficients per piece in x = 8 (m - c_j), where m in
// [1, 2) is nu's significand and c_j = 1 + (2j + 1)/8 the centre of piece j (x in [-1, 1),
// exact in binary).  c0 is analytic up to its poles at nu = 0, -1, ...; every piece sits at
// >= 9 half-widths from nu = 0 whatever the octave, so one degree fits every scale.  The
// host validates the table against lgammal (kC0Tol) and the kernel evaluates 11 FMAs
// instead of st_c0_exact.  Returns the piece, or -1 for nu outside the table -- NaN, inf,
// <= 0 and subnormal nu land there through the exponent field alone.
constexpr int kC0N = 12, kC0Sub = 4, kC0MaxPieces = 64;
NGRTD_HD int c0_piece(double nu, int e0, int np, double& x) {
    const unsigned hi = fm_hi(nu);
    const int j = (int)((hi >> 18) & 3u);
    const int p = ((int)(hi >> 20) - 1023 - e0) * kC0Sub + j;    // sign bit -> p >= 4096
    const double m = fm_with_hi(nu, (hi & 0x000FFFFFu) | 0x3FF00000u);
    x = (m - (1.125 + 0.25 * j)) * 8.0;
    return (unsigned)p < (unsigned)np ? p : -1;
}
NGRTD_HD double c0_poly(const double* t, double x) {
    double b = t[kC0N - 1];
#pragma unroll
    for (int k = kC0N - 2; k >= 0; --k) b = fma_k(b, x, t[k]);
    return b;
}
// table view: t = [np][kC0N] coefficients (null: exact everywhere)
struct C0Tab {
    const double* t;
    int32_t e0, np;
};

// (inu = 1 / nu, from the caller's batched reciprocals)
template <int NMAX>
NGRTD_HD double st_block_inu(int n, const double* obs, const double* mu, const double* lam, double hll_sum,
                             double nu, double inu, C0Tab c0t) {
    double c0;
    double cx;
    const int cp = c0t.t ? c0_piece(nu, c0t.e0, c0t.np, cx) : -1;
    c0 = c0t.t ? c0_poly(c0t.t + (cp >= 0 ? cp : 0) * kC0N, cx) : 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
    // the exact normaliser behind a wave-uniform branch (nu outside the table: a proposal past
    // its prior's support), so that waves without such a lane never evaluate it
    if (__any(cp < 0))
#endif
        if (cp < 0) c0 = st_c0_exact(nu, inu);
    // unrolled over NMAX constant slots (slots j >= n masked; their loads clamp to n - 1)
    double prod = 1.0;
    bool big = false, ok = nu > 0;
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
        const int jj = j < n ? j : n - 1;
        const double d = obs[jj] - mu[j];
        const double z = lam[jj] * (d * d) * inu;
        const bool on = j < n;
        prod *= on ? (1.0 + z) : 1.0;
        big |= on && !(z < 1.0e38);      // (1 + 1e38)^8 < DBL_MAX: the product cannot overflow
        ok &= !on || lam[jj] > 0;
    }
    double Lg;
    if (!big) {
        // prod >= 1 (finite) whenever the block is in bounds (nu > 0, lam > 0); else the result
        // is -inf whatever Lg is
        Lg = flog_pn(prod);
    } else {
        // inf/NaN z or z >= 1e38: one log per factor (log(1 + z) = log1p(z) + O(2^-53))
        Lg = 0.0;
        for (int j = 0; j < n; ++j) {
            const double d = obs[j] - mu[j];
            Lg += flog(1.0 + lam[j] * (d * d) * inu);
        }
    }
    const double v = (double)n * c0 + hll_sum - (nu + 1.0) / 2.0 * Lg;
    return ok ? v : kNegInf;
}
template <int NMAX>
NGRTD_HD double st_block(int n, const double* obs, const double* mu, const double* lam, double hll_sum,
                         double nu, C0Tab c0t = C0Tab{nullptr, 0, 0}) {
    return st_block_inu<NMAX>(n, obs, mu, lam, hll_sum, nu, 1.0 / nu, c0t);
}

// Beta.logp with precomputed betaln(a, b)
NGRTD_HD double beta_logp(double x, double a, double b, double betaln_ab) {
    const double t1 = (a == 1.0) ? 0.0 : (a - 1) * log(x);
    const double t2 = (b == 1.0) ? 0.0 : (b - 1) * log1p(-x);
    const double lp = t1 + t2 - betaln_ab;
    return (x >= 0 && x <= 1) ? lp : kNegInf;
}
NGRTD_HD double normal_logp(double x, double mu, double tau, double log_tau_2pi) {
    const double d = x - mu;
    return (-tau * (d * d) + log_tau_2pi) / 2.0;
}
NGRTD_HD double uniform_logp(double x, double lo, double hi, double neg_log_width) {
    return (x >= lo && x <= hi) ? neg_log_width : kNegInf;
}
NGRTD_HD double halfnormal_logp(double x, double tau, double half_log_tau_2_pi) {
    return (x >= 0) ? -0.5 * tau * (x * x) + half_log_tau_2_pi : kNegInf;
}
// PyMC3 default transforms' log|Jacobian| (logodds / interval / log)
NGRTD_HD double jac_logodds(double x) { return log(x) + log1p(-x); }
// The Interval transform's log-Jacobian log(x - a) + log(b - x) - log(b - a) as ONE table log of
// the product (<= ((b - a) / 2)^2, no overflow; x = a or b gives -inf as the sum does) plus
// nlw = -log(b - a) from the plan (three OCML logs before: ~1.1 us per c4 launch).
NGRTD_HD double jac_interval(double x, double a, double b, double nlw) { return flog((x - a) * (b - x)) + nlw; }

}  // namespace ngrtd
