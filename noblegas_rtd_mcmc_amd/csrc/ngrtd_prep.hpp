// ngrtd_prep.hpp -- gfx950 kernels of the prep-stage ensemble propagation (SURVEY.md §8f
// rank 2): the CE posterior ensemble pushed through to tracer observations.
//
//   he_comps_kernel  ng_parse(obs, Ae, F, E, T).He_comps(Rterr)  utils/noble_gas_utils.py:394-422
//   cfc_corr_kernel  cfc_ce_corr / sf6_ce_corr methods           utils/cfc_utils.py:25-306
//
// Both are elementwise over ensemble members (age_modeling_mcmc.prep.py:247-397 runs
// them 50 000 x wells x passes, one Python object per member).  One lane per member;
// parameters are read and results written structure-of-arrays, so every wave issues
// 512-B coalesced loads and stores: HBM-bound (algorithmic bytes per member in DESIGN.md).
// The arithmetic keeps the reference's association order (Python evaluates left to right,
// -ffp-contract=off), like ngrtd_math.hpp.
#pragma once
#include <hip/hip_runtime.h>
#include "ngrtd_math.hpp"
#include "../../include/ngrtd.h"

namespace ngrtd {

// ------------------------------------------------------------------- He_comps
struct HeCompsArgs {
    const double *He4, *He3, *Ae, *F, *E, *T, *Rterr;
    double Rterr_c;        // used when Rterr == nullptr (the constant-Rterr passes, prep.py:341)
    int64_t n;
    double* out;           // [NGRTD_HE_NOUT][n]
};

// noble_gas_fun(gases=['He'], E, T, Ae, F, P='lapse_rate') (:76-113), S = 0.0, then the
// mass balance of :400-421.  Restated for one pass over the member with the per-unit
// rewrites of ce_model_s0 (ngrtd_kernels.hpp): table-driven fexp/flog
// instead of OCML pow/exp (<= 1-2 ulp), ln K in Horner form of 1/x (one division), and
// K_He = K_Ar / F_He exactly as the reference's chain of ratios
// (5.24e-6 / (F (5.24e-6/9.31e-3) (9.31e-3 / K_Ar))), so x_He = gamma p_He exp(ln F - ln K_Ar);
// the Setchenow factor exp(0 * setch) is 1, or NaN when T < 65 and T_k <= 0.  Each rewrite
// moves a result by a few ulp; He4_ter / He4_del / He3_tu then inherit them relative to
// their cancelling operands (tests/test_gpu_prep.py).
NGRTD_HD void he_comps(double He4_obs, double He3_obs, double Ae, double F, double E, double T, double Rterr,
                       double o[NGRTD_HE_NOUT]) {
    const double P = lapse_rate_fast(E);
    double A, B, Cc;
    if (T <= 99.0) { A = 8.07131; B = 1730.63; Cc = 233.426; }
    else           { A = 8.14019; B = 1810.94; Cc = 244.485; }
    const double Pv = fexp10(A - (B / (Cc + T))) * (101325. / 760. / 1.0e9);
    const double T_k = T + 273.15;
    const double ix = 1.0 / (.001 * T_k);
    const double gamma = (T < 65. && !(T_k > 0.0)) ? __builtin_nan("") : 1.0;
    const GasCoef he = gas_coef(NGRTD_HE), ar = gas_coef(NGRTD_AR);
    const double lnF = fma(fma(fma(he.A3, ix, he.A2), ix, he.A1), ix, he.A0);
    const double lnAr = fma(fma(fma(ar.A3, ix, ar.A2), ix, ar.A1), ix, ar.A0);
    const double e = gamma * fexp(lnF - lnAr);                          // 1 / K_He
    const double z = he.z;
    const double He4_eq = ((z * P) * e) * (22414. / 18.);               // equil_conc()['He'], :202-213
    const double ceq = (T < 0.0) ? -9999.0 : ((z * (P - Pv)) * e) * (22414. / 18.);   // :216-232
    const double ex = ((1 - F) * Ae * z) * ceq / (ceq + F * Ae * z);     // ce_exc excess, :247-248
    const double He4_atm = ex + ceq;                                     // ce_exc(True)['He']
    const double He4_ter = He4_obs - He4_atm;                            // :405
    const double He4_del = 100 * (He4_ter / He4_atm);                   // :408
    // 3He mass balance, :414-421: Ratm = 1.384e-6, CF = 4.021e14/(1-S) with S = 0
    const double Ratm = 1.384e-6;
    const double CF = 4.021e14 / (1 - 0.0);
    const double He3_trit = He3_obs - (He4_obs - He4_ter) * Ratm + He4_eq * Ratm * (1 - 0.983) - He4_ter * Rterr;
    o[NGRTD_HE_EQ] = He4_eq;
    o[NGRTD_HE_ATM] = He4_atm;
    o[NGRTD_HE_TER] = He4_ter;
    o[NGRTD_HE_DEL] = He4_del;
    o[NGRTD_HE_TU] = He3_trit * CF;
}

__global__ void __launch_bounds__(256) he_comps_kernel(const HeCompsArgs a) {
    fm_lds_init();
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    double o[NGRTD_HE_NOUT];
    he_comps(a.He4[i], a.He3[i], a.Ae[i], a.F[i], a.E[i], a.T[i], a.Rterr ? a.Rterr[i] : a.Rterr_c, o);
#pragma unroll
    for (int k = 0; k < NGRTD_HE_NOUT; ++k) a.out[(int64_t)k * a.n + i] = o[k];
}

// ------------------------------------------------------------ CFC / SF6 correction
// utils/cfc_utils.py: vapor_pressure_atm (:34-51, :181-196) and lapse_rate_atm (:53-62,
// :198-206), both in atm, through the table-driven fexp10 / fexp / flog (<= 1-2 ulp against
// libm pow; the parity bar is 1e-12).
NGRTD_HD double vapor_pressure_atm(double T) {
    double A, B, C;
    if (T <= 99.0) { A = 8.07131; B = 1730.63; C = 233.426; }
    else           { A = 8.14019; B = 1810.94; C = 244.485; }
    // mmHg -> Pa -> GPa -> atm (P/760.*101325, /1.0e9, /0.000101325) as ONE multiply by
    // the folded constant: <= 3 ulp from the reference's three roundings
    return fexp10(A - (B / (C + T))) * (101325. / 760. / 1.0e9 / 0.000101325);
}
NGRTD_HD double lapse_rate_atm(double E) { return fexp(5.2561 * flog(1 - E * (.0065 / 288.15))); }

// Bullister solubility coefficients [a1, a2, a3, b1, b2, b3]: cfc_dict (:74) and
// solubility_sf6 (:214-219); index = enum ngrtd_cfc_species
NGRTD_HD void cfc_coef(int sp, double c[6]) {
    switch (sp) {
    case NGRTD_CFC11:  c[0] = -136.2685; c[1] = 206.1150; c[2] = 57.2805; c[3] = -.148598; c[4] = 0.095114; c[5] = -0.0163396; break;
    case NGRTD_CFC12:  c[0] = -124.4395; c[1] = 185.4299; c[2] = 51.6383; c[3] = -0.149779; c[4] = 0.094668; c[5] = -0.0160043; break;
    case NGRTD_CFC113: c[0] = -136.129; c[1] = 206.475; c[2] = 55.8957; c[3] = -0.02754; c[4] = 0.006033; c[5] = 0; break;
    default:           c[0] = -98.7264000; c[1] = 142.803; c[2] = 38.8746; c[3] = 0.0268696; c[4] = -0.0334407; c[5] = 0.0070843; break;
    }
}
// per-member terms of solubility_cfc (:64-84) / solubility_sf6 (:208-221) shared by the
// species: 100 / T_k, log(T_k / 100), T_k / 100 (the reference recomputes them per species)
struct CfcT {
    double r100, lg, r;
};
NGRTD_HD CfcT cfc_t(double T) {
    const double T_k = T + 273.15;
    const double r = T_k * 0.01;                  // T_k / 100 (<= 1 ulp)
    return {100 / T_k, flog(r), r};
}
// K [mol atm^-1 kg^-1]
NGRTD_HD double solubility_cfc(int sp, const CfcT& t, double S) {
    double c[6];
    cfc_coef(sp, c);
    return fexp(c[0] + c[1] * t.r100 + c[2] * t.lg + S * (c[3] + c[4] * t.r + c[5] * (t.r * t.r)));
}

struct CfcArgs {
    int32_t what, ns;
    int32_t sp[NGRTD_MAX_CFC];
    const double *E, *T, *Ae, *F, *S, *P, *x;   // x: [ns][n] (C_meas or z_i); P: self.P (ce_exc only)
    int64_t n;
    double* out;                                 // [ns][n] ([n] for the pressure entries)
};

// Ae is self.Ae, ccSTP/kg (the constructor's Ae*1000., :30, :176); P_da / P_vapor per member
// (am = Ae / 22414.1, Ae over the molar volume: the same per species, formed once per member)
NGRTD_HD double cfc_value(int what, int sp, const CfcT& t, double P_da, double P_vapor, double Ae, double F,
                          double S, double Pself, double x, double am) {
    const bool sf6 = (sp == NGRTD_SF6);
    const double Ki = solubility_cfc(sp, t, S);
    if (what == NGRTD_CFC_SOLUBILITY) return Ki;
    if (what == NGRTD_CFC_EQUIL_AIR) {           // equil_air_conc_cfc :86-106 / _sf6 :229-249
        // (x + x F am / KP) / (KP + am) over one denominator: x (KP + F am) / (KP (KP + am)),
        // one division instead of two (a few ulp; parity bar 1e-12)
        const double KP = Ki * P_da;
        const double z = (x * (KP + F * am)) / (KP * (KP + am));
        return sf6 ? z * 0.001 : z;
    }
    if (what == NGRTD_CFC_EQUIL_AQ) {            // equil_aq_conc_cfc :108-124 / _sf6 :264-278
        const double C = Ki * x * P_da;
        return sf6 ? C / 0.001 : C;
    }
    // ce_exc_conc_cfc :126-142 / _sf6 :280-296 (uses self.P as last set by lapse_rate_atm)
    const double C_eq = Ki * x * (Pself - P_vapor);
    const double Aem = Ae / 22414 / 1e-12;
    const double num = (1 - F) * Aem * (x * 1e-12);
    const double den = 1 + F * Aem * ((x * 1e-12 / C_eq));
    return sf6 ? 1000 * num / den : num / den;
}

__global__ void __launch_bounds__(256) cfc_corr_kernel(const CfcArgs a) {
    fm_lds_init();
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const double E = a.E ? a.E[i] : 0.0;
    const double T = a.T ? a.T[i] : 0.0;
    if (a.what == NGRTD_CFC_LAPSE_RATE_ATM) { a.out[i] = lapse_rate_atm(E); return; }
    const double P_vapor = vapor_pressure_atm(T);
    if (a.what == NGRTD_CFC_VAPOR_PRESSURE_ATM) { a.out[i] = P_vapor; return; }
    const double Ae = a.Ae ? a.Ae[i] : 0.0;
    const double F = a.F ? a.F[i] : 0.0;
    const double S = a.S ? a.S[i] : 0.0;
    const double P = a.P ? a.P[i] : 0.0;
    const bool need_pda = a.what == NGRTD_CFC_EQUIL_AIR || a.what == NGRTD_CFC_EQUIL_AQ;
    const double P_da = need_pda ? lapse_rate_atm(E) - P_vapor : 0.0;
    const CfcT t = cfc_t(T);
    const double am = Ae / 22414.1;
    for (int j = 0; j < a.ns; ++j) {
        const double x = a.x ? a.x[(int64_t)j * a.n + i] : 0.0;
        a.out[(int64_t)j * a.n + i] = cfc_value(a.what, a.sp[j], t, P_da, P_vapor, Ae, F, S, P, x, am);
    }
}

}  // namespace ngrtd
