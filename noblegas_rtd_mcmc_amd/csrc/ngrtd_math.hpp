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

#define NGRTD_HD __host__ __device__ __forceinline__

namespace ngrtd {

constexpr double kNegInf = -__builtin_inf();
constexpr double kPi = 3.141592653589793;

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
// StudentT.logp, summed over observations that share nu: the caller adds
//   st_const(nu) + st_term(x, mu, sigma, nu)
NGRTD_HD double st_const(double nu) {
    return lgamma((nu + 1.0) / 2.0) - lgamma(nu / 2.0);
}
NGRTD_HD double st_term(double x, double mu, double sigma, double nu) {
    const double lam = 1.0 / (sigma * sigma);
    const double d = x - mu;
    const double v = 0.5 * log(lam / (nu * kPi)) - (nu + 1.0) / 2.0 * log1p(lam * (d * d) / nu);
    return (lam > 0 && nu > 0 && sigma > 0) ? v : kNegInf;
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
NGRTD_HD double jac_interval(double x, double a, double b) { return log(x - a) + log(b - x) - log(b - a); }

}  // namespace ngrtd
