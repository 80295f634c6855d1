// ngrtd_kernels.hip -- gfx950 (CDNA4, wave64) kernels of the CE + RTD log-likelihood.
//
// The RTD convolution (utils/convolution_integral_utils.py:155-340) is evaluated per
// (walker, well) "unit" without materialising the N-long weight vector g(tp):
//
//   conc = sum_k C_k g_k d_k / sum_k g_k          (g normalised by its sum, :270)
//
// For the piston model this is a lookup at argmin|tp - tau| (:180).  For the two
// geometric models (exponential :184, exp_pist_flow :189-190) the weights are
// g_k ~ exp(-beta tp_k) on a yearly grid, so sum_k C_k q^k is a polynomial in
// q = exp(-beta) evaluated by Horner's rule: ONE fused multiply-add per age per channel
// instead of the reference's two exp() per age.  The decay exp(-lambda tp) of a tracer
// with a fixed half-life is folded into its channel table on the host (A_k = C_k d_k),
// the normaliser sum_k q^k has the closed form expm1(-beta n)/expm1(-beta), and Horner
// chains are restarted every LDS slice sub-range (<= a few hundred ages) and rescaled by
// an exactly computed exp(), which bounds the rounding growth to a few hundred ulp
// (parity bar: rtol 1e-12).  The dispersion model (:192-196) has no such
// structure and evaluates the reference formula per age.
//
// Work mapping: a wave owns 64*R units (lane = unit, R units per lane for register reuse
// of each LDS coefficient read); the NW waves of a block split the age axis, share the
// channel table slice through LDS, and are reduced through LDS in a fixed order
// (deterministic, no atomics).
#pragma once
#include <hip/hip_runtime.h>
#include "ngrtd_device.hpp"
#include "ngrtd_math.hpp"
#include "../../include/ngrtd.h"

// A translation unit that uses only the logp_fused_kernel template (ngrtd_dz.hip) defines
// NGRTD_FUSED_ONLY: the header's plain kernels then have internal linkage there and do not
// collide with ngrtd.hip's definitions at link time.
#ifdef NGRTD_FUSED_ONLY
#define NGRTD_KLINK static
#else
#define NGRTD_KLINK
#endif

namespace ngrtd {

// Section-timing probe (tools/section_probe.py builds a separate library with
// -DNGRTD_SECTION_PROBE): lane 0 of every wave of logp_fused_kernel records the shader
// clock (s_memtime) at fixed points.  Compiled out of the product library.
#ifdef NGRTD_SECTION_PROBE
// slots 0-7: the log-prob sections; 8-15: a DEMetropolisZ step's (the last step of a launch)
constexpr int kProbeSlots = 16;
__device__ unsigned long long g_probe[8192 * kProbeSlots];
#define NGRTD_PROBE(k)                                                                        \
    do {                                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
        if ((threadIdx.x & 63) == 0)                                                          \
            g_probe[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kProbeSlots + (k)] = t_; \
    } while (0)
#else
#define NGRTD_PROBE(k) do {} while (0)
#endif

// ------------------------------------------------------------------ CE forward
struct CeArgs {
    int32_t what, p_mode, G;
    int32_t gas[kMaxGas];
    const double *E, *T, *Ae, *F, *P, *S;
    int64_t n;
    double* out;
};

NGRTD_KLINK __global__ void __launch_bounds__(256) ce_forward_kernel(const CeArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const double E = a.E ? a.E[i] : 0.0;
    const double T = a.T ? a.T[i] : 0.0;
    const double S = a.S ? a.S[i] : 0.0;
    double P;
    if (a.p_mode == NGRTD_P_LAPSE_RATE) P = lapse_rate(E);
    else if (a.p_mode == NGRTD_P_1ATM) P = 0.000101325;
    else P = a.P[i];
    if (a.what == NGRTD_CE_PRESSURE) { a.out[i] = P; return; }
    const double Pv = vapor_pressure(T);
    if (a.what == NGRTD_CE_VAPOR_PRESSURE) { a.out[i] = Pv; return; }
    const double Ae = a.Ae ? a.Ae[i] : 0.0;
    const double F = a.F ? a.F[i] : 0.0;
    for (int j = 0; j < a.G; ++j) {
        const int g = a.gas[j];
        const double K = solubility(g, T, S);
        double v;
        switch (a.what) {
        case NGRTD_CE_SOLUBILITY: v = K; break;
        case NGRTD_CE_EQUIL: v = equil_conc(g, P, K); break;
        case NGRTD_CE_EQUIL_DRY: v = equil_conc_dry(g, T, P, Pv, K); break;
        case NGRTD_CE_EXC_EXCESS: v = ce_excess(g, Ae, F, equil_conc_dry(g, T, P, Pv, K)); break;
        default: {
            const double ceq = equil_conc_dry(g, T, P, Pv, K);
            v = ce_excess(g, Ae, F, ceq) + ceq;
        }
        }
        a.out[i * a.G + j] = v;
    }
}

// ------------------------------------------------------------- RTD helpers
// exp_pist_flow mask, :189: first k with tp_k >= tau*(1-(1/eta)); N if none.
__device__ __forceinline__ int epm_first(double thr, double tp0, double dtp, int N) {
    if (tp0 >= thr) return 0;
    if (!(thr == thr)) return N;
    double kk = ceil(thr - dtp);
    if (kk < 1.0) kk = 1.0;
    if (kk > (double)N) return N;
    int k = (int)kk;
    while (k < N && !((double)k + dtp >= thr)) ++k;
    while (k > 1 && ((double)(k - 1) + dtp >= thr)) --k;
    return k;
}

// piston, :179-181: FIRST index of min |tp - tau| (numpy argmin semantics, NaN -> 0).
__device__ __forceinline__ int piston_index(double tau, double tp0, double dtp, int N) {
    if (!(fabs(tau) < 1.0e15)) {
        int best = 0;
        double bd = fabs(tp0 - tau);
        if (bd != bd) return 0;
        for (int k = 1; k < N; ++k) {
            const double d = fabs(((double)k + dtp) - tau);
            if (d < bd) { bd = d; best = k; }
        }
        return best;
    }
    int best = 0;
    double bd = fabs(tp0 - tau);
    const double kf = floor(tau - dtp);
    // |tp_k - tau| is unimodal in k: the k >= 1 minimum is at floor/ceil(tau - dtp),
    // clamped into [1, N-1] (tau past either end of the grid)
    const int k0 = (kf < 1.0) ? 1 : (kf > (double)(N - 1) ? N - 1 : (int)kf);
    for (int k = k0 - 1; k <= k0 + 2; ++k) {
        if (k < 1 || k >= N) continue;
        const double d = fabs(((double)k + dtp) - tau);
        if (d < bd) { bd = d; best = k; }
    }
    return best;
}

__device__ __forceinline__ int wave_min_int(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ double theta_or(const RtdArgs& a, int row, int64_t u, double dflt) {
    return row >= 0 ? a.theta[(int64_t)row * a.U + u] : dflt;
}

// ------------------------------------------------------------ RTD kernel
// Template: R units per lane, C channels (table columns; CP = padded row length).
template <int R, int C, bool LAMW>
__global__ void __launch_bounds__(256) rtd_conc_kernel(const RtdArgs a) {
    constexpr int CP = (C + 1) & ~1;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int NW = blockDim.x >> 6;
    const int N = a.N;
    const int64_t ubase = (int64_t)blockIdx.x * 64 * R;

    int64_t u[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        u[r] = ubase + r * 64 + lane;
        valid[r] = u[r] < a.U;
        if (!valid[r]) u[r] = a.U - 1;   // clamp for loads; never stored
    }
    // per-unit decay from the CFC12 half-life role (run_age_mcmc_utils.py:107-109)
    double lamw[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (LAMW) {
            const double th = a.thalf_a * a.theta[(int64_t)a.row_thalf * a.U + u[r]] + a.thalf_b;
            lamw[r] = (th != 0.0) ? -1 * log(0.5) / th : 0.0;   // thalf_2_lambda, :150
        } else {
            lamw[r] = 0.0;
        }
    }

    for (int comp = 0; comp < 2; ++comp) {
        const int mod = a.mod[comp];
        if (mod == MOD_NONE) break;
        double tau[R], beta[R], q0[R], qw[R], Dv[R];
        int f[R], m[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            tau[r] = theta_or(a, a.row_tau[comp], u[r], 0.0);
            Dv[r] = (mod == MOD_DISP) ? theta_or(a, a.row_D[comp], u[r], 0.0) : 0.0;
            if (mod == MOD_EXP) {
                beta[r] = 1. / tau[r];
                f[r] = 0;
            } else if (mod == MOD_EPM) {
                const double eta = theta_or(a, a.row_eta[comp], u[r], 0.0);
                beta[r] = eta / tau[r];
                f[r] = epm_first(tau[r] * (1 - (1 / eta)), a.tp0, a.dtp, N);
            } else {
                beta[r] = 0.0;
                f[r] = 0;
            }
            m[r] = f[r] > 1 ? f[r] : 1;
            q0[r] = exp(-beta[r]);
            qw[r] = LAMW ? exp(-(beta[r] + lamw[r])) : q0[r];
        }

        // ---- age loop: partial sums per unit (geometric: Y_c; dispersion: num_c, den)
        double tot[R][C + 1];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c <= C; ++c) tot[r][c] = 0.0;

        if (mod != MOD_PISTON) {
            const int LW = a.LW;
            const int SL = LW * NW;
            int mmin = N;
#pragma unroll
            for (int r = 0; r < R; ++r) mmin = (valid[r] && m[r] < mmin) ? m[r] : mmin;
            mmin = wave_min_int(mmin);
            for (int s0 = 0; s0 < N; s0 += SL) {
                // stage table rows [s0, s0+SL) into LDS (coalesced 16-byte copies)
                __syncthreads();
                {
                    const int rows = (N - s0) < SL ? (N - s0) : SL;
                    const int n2 = rows * CP / 2;
                    const double2* src = reinterpret_cast<const double2*>(a.tab + (int64_t)s0 * CP);
                    double2* dst = reinterpret_cast<double2*>(smem);
                    for (int i = threadIdx.x; i < n2; i += blockDim.x) dst[i] = src[i];
                }
                __syncthreads();
                const int klo0 = s0 + wave * LW;
                const int khi = (klo0 + LW) < N ? (klo0 + LW) : N;
                if (mod == MOD_DISP) {
                    for (int k = klo0; k < khi; ++k) {
                        const double* row = smem + (k - s0) * CP;
                        double av[C];
#pragma unroll
                        for (int c = 0; c < C; ++c) av[c] = row[c];
                        const double tp = (k == 0) ? a.tp0 : ((double)k + a.dtp);
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const double D = Dv[r];
                            const double x = tp / tau[r];
                            const double f1 = (1. / tau[r]) / (sqrt(4. * kPi * D * x));
                            const double f2 = (1. / x) * exp(-1. * (((1. - x) * (1. - x)) / (4. * D * x)));
                            const double w = f1 * f2;
                            const double wd = LAMW ? w * exp(-lamw[r] * tp) : w;
                            tot[r][C] += w;
#pragma unroll
                            for (int c = 0; c < C; ++c) tot[r][c] = fma(av[c], a.chan_lamw[c] ? wd : w, tot[r][c]);
                        }
                    }
                } else {
                    // geometric: ages k >= max(1, m); Horner top-down over [klo, khi)
                    const int klo = klo0 > mmin ? klo0 : mmin;
                    if (klo < khi) {
                        double q[R][C];
#pragma unroll
                        for (int r = 0; r < R; ++r)
#pragma unroll
                            for (int c = 0; c < C; ++c) q[r][c] = (LAMW && a.chan_lamw[c]) ? qw[r] : q0[r];
                        double acc[R][C];
#pragma unroll
                        for (int r = 0; r < R; ++r)
#pragma unroll
                            for (int c = 0; c < C; ++c) acc[r][c] = 0.0;
                        if (mod == MOD_EPM) {
                            for (int k = khi - 1; k >= klo; --k) {
                                const double* row = smem + (k - s0) * CP;
                                double av[C];
#pragma unroll
                                for (int c = 0; c < C; ++c) av[c] = row[c];
#pragma unroll
                                for (int r = 0; r < R; ++r) {
                                    const bool on = k >= m[r];
#pragma unroll
                                    for (int c = 0; c < C; ++c) {
                                        const double t = fma(acc[r][c], q[r][c], av[c]);
                                        acc[r][c] = on ? t : acc[r][c];
                                    }
                                }
                            }
                        } else {
#pragma unroll 4
                            for (int k = khi - 1; k >= klo; --k) {
                                const double* row = smem + (k - s0) * CP;
                                double av[C];
#pragma unroll
                                for (int c = 0; c < C; ++c) av[c] = row[c];
#pragma unroll
                                for (int r = 0; r < R; ++r)
#pragma unroll
                                    for (int c = 0; c < C; ++c) acc[r][c] = fma(acc[r][c], q[r][c], av[c]);
                            }
                        }
                        // rescale the sub-range partial to the unit's base index m
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const int e = klo > m[r] ? klo : m[r];
                            if (e < khi) {
                                const double de = (double)(e - m[r]);
                                const double s_0 = exp(-beta[r] * de);
                                const double s_w = LAMW ? exp(-(beta[r] + lamw[r]) * de) : s_0;
#pragma unroll
                                for (int c = 0; c < C; ++c)
                                    tot[r][c] = fma((LAMW && a.chan_lamw[c]) ? s_w : s_0, acc[r][c], tot[r][c]);
                            }
                        }
                    }
                }
            }
            // ---- fixed-order cross-wave reduction through LDS
            __syncthreads();
            double* comb = smem;
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int c = 0; c <= C; ++c)
                    comb[(((wave * R) + r) * (C + 1) + c) * 64 + lane] = tot[r][c];
            __syncthreads();
            if (wave == 0) {
                for (int w = 1; w < NW; ++w)
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int c = 0; c <= C; ++c)
                            tot[r][c] += comb[(((w * R) + r) * (C + 1) + c) * 64 + lane];
            }
        }

        // ---- finalize: per tracer concentration of this component (wave 0)
        if (wave == 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!valid[r]) continue;
                double num[C];
                double den;
                if (mod == MOD_PISTON) {
                    const int ix = piston_index(tau[r], a.tp0, a.dtp, N);
                    const double tp = (ix == 0) ? a.tp0 : ((double)ix + a.dtp);
                    const double dw = LAMW ? exp(-lamw[r] * tp) : 1.0;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        const double v = a.tab[(int64_t)ix * CP + c];
                        num[c] = a.chan_lamw[c] ? v * dw : v;
                    }
                    den = 1.0;
                } else if (mod == MOD_DISP) {
#pragma unroll
                    for (int c = 0; c < C; ++c) num[c] = tot[r][c];
                    den = tot[r][C];
                } else {
                    const int fr = f[r], mr = m[r];
                    const double tpm = (double)mr + a.dtp;
                    const double s01 = (fr == 0) ? exp(-beta[r] * ((1.0 + a.dtp) - a.tp0)) : 1.0;
                    const int n = N - mr;
                    const double G = (n > 0) ? expm1(-beta[r] * (double)n) / expm1(-beta[r]) : 0.0;
                    den = ((fr == 0) ? 1.0 : 0.0) + s01 * G;
                    const double dw0 = LAMW ? exp(-lamw[r] * a.tp0) : 1.0;
                    const double dwm = LAMW ? exp(-lamw[r] * tpm) : 1.0;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        const double y = tot[r][c];
                        const double base = (fr == 0) ? a.tab[c] * (a.chan_lamw[c] ? dw0 : 1.0) : 0.0;
                        num[c] = base + s01 * (a.chan_lamw[c] ? dwm : 1.0) * y;
                    }
                }
                // tracer concentrations: (A + J B) / den, then the BMM mix and SF6 factor
                const double fmix = (comp == 0) ? theta_or(a, a.row_f1, u[r], 1.0)
                                                : 1 - theta_or(a, a.row_f1, u[r], 1.0);
                double Jw = 0.0;
                if (a.row_J >= 0) {
                    const double jv = a.theta[(int64_t)a.row_J * a.U + u[r]];
                    Jw = a.J_is_log10 ? pow(10.0, jv) : jv;
                }
                for (int t = 0; t < a.K; ++t) {
                    double sA = 0.0, sB = 0.0;
                    bool hasB = false;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        if (a.chan_tracer[c] != t) continue;
                        if (a.chan_isB[c]) { sB = num[c]; hasB = true; }
                        else sA = num[c];
                    }
                    double cc;
                    if (hasB) {
                        const double J = (a.row_J >= 0) ? Jw : a.tr_J[t];
                        cc = (sA + J * sB) / den;
                    } else {
                        cc = sA / den;
                    }
                    double* dst = a.conc + (int64_t)t * a.U + u[r];
                    double cout = (comp == 0) ? fmix * cc : (*dst + fmix * cc);
                    const bool last = (comp == 1) || (a.mod[1] == MOD_NONE);
                    if (last && a.mod[1] == MOD_NONE) cout = cout + 0.0 * 0.0;   // f2 * cout2, :154
                    if (last && a.tr_sf6[t] && a.row_lamsf6 >= 0)
                        cout *= (1 + a.theta[(int64_t)a.row_lamsf6 * a.U + u[r]]);
                    *dst = cout;
                }
            }
        }
    }
}

// ------------------------------------------------- per-unit CE + likelihood
// CE concentrations of one (walker, well) for the likelihood gases, with S = 0 (the
// reference models never pass a salinity).  noble_gas_utils.py:117-253 restated for the
// per-unit path with one division per gas instead of ~7:
//  * Setchenow factor exp(0 * setch) (:154-156) is 1 whenever setch is finite, NaN
//    otherwise; for T < 65 setch is finite iff T_k > 0 (T_k = T + 273.15 is never a positive
//    value small enough for G2 / (.01 T_k) to overflow), so gamma needs no exp/log;
//  * ln K = A0 + A1/x + A2/x^2 + A3/x^3 is evaluated by Horner in 1/x (one reciprocal for
//    all gases), and x_i = p_i / K = gamma p_i exp(-ln K) (gamma is 1 or NaN);
//  * He (:161-176): K_He = exp(ln K_Ar - ln F_He) exactly as the reference's chain of
//    ratios, so x_He = gamma p_He exp(ln F_He - ln K_Ar);
//  * ce_excess (1-F) Ae z / (1 + F Ae z / C_eq) = (1-F) Ae z C_eq / (C_eq + F Ae z).
// Each rewrite moves a result by a few ulp of ln K (|ln K| < 30 on the CE ranges): far
// inside the 1e-12 parity bar (tests/test_gpu_parity.py checks against the reference).
__device__ __forceinline__ double lnK_horner(const GasCoef& c, double ix) {
    return fma(fma(fma(c.A3, ix, c.A2), ix, c.A1), ix, c.A0);
}
__device__ __forceinline__ void ce_model_s0(const UnitArgs& a, double T, double P, double Ae, double F,
                                            double* mod) {
    const double T_k = T + 273.15;
    // the Antoine denominator C + T and .001 T_k share one division (batch_recip)
    double vA, vB, vC;
    antoine(T, vA, vB, vC);
    const double dv[2] = {vC + T, .001 * T_k};
    double rv[2];
    batch_recip<2>(dv, rv);
    const double Pv = vapor_pressure_rcp(vA, vB, rv[0]);
    const double ix = rv[1];
    const double gamma = (T < 65. && !(T_k > 0.0)) ? __builtin_nan("") : 1.0;
    const double dP = P - Pv;
    const double lnAr = lnK_horner(gas_coef(2), ix);
    const double FA = F * Ae, ImFA = (1 - F) * Ae;
    const bool neg = T < 0.0;
    double ceq[kMaxGas], den[kMaxGas], rd[kMaxGas];
#pragma unroll
    for (int j = 0; j < kMaxGas; ++j) {
        const double lnK = fma(fma(fma(a.gA3[j], ix, a.gA2[j]), ix, a.gA1[j]), ix, a.gA0[j]);
        const double e = fexp(a.g_he[j] ? lnK - lnAr : -lnK);
        ceq[j] = neg ? -9999.0 : (gamma * (a.gz[j] * dP) * e) * (22414. / 18.);
        den[j] = ceq[j] + FA * a.gz[j];
    }
    batch_recip<kMaxGas>(den, rd);                  // the 5 excess-air denominators: one division
#pragma unroll
    for (int j = 0; j < kMaxGas; ++j) {
        const double ex = ((ImFA * a.gz[j]) * ceq[j]) * rd[j];
        mod[j] = ex + ceq[j];
    }
}

// log-prob contribution of one (walker, well) unit that depends on theta only: priors,
// CE model + likelihood, RTD priors (the RTD likelihood is added by unit_like_rtd).
// Sum of all Beta-prior log densities of a unit (and their logodds Jacobians):
//   sum_i [(a_i-1) log x_i + (b_i-1) log(1-x_i) - betaln(a_i, b_i)]
// as ONE log of the product of the integer-exponent factors plus one log per non-integer
// exponent (c4: 4 logs instead of 9).  -inf when any x_i is outside [0, 1] (or NaN), as
// PyMC3's bound.  A product below 1e-280 (x within ~1e-40 of 0 or 1) redoes the sum
// term by term so that it cannot underflow.  Differs from the term-by-term sum by a few
// ulp of the largest log (the logp parity bar is atol 1e-9).
// theta values of a unit loaded ahead of use (logp_fused_kernel issues these loads before
// its first barrier so their latency overlaps it): the 6 CE rows, tau1 and the RTD nu
struct ThetaPre {
    double ce[6];
    double tau1, nub;
};

// The per-well data a kernel staged in LDS (UnitArgs::wd_src copied to its LDS block), passed
// beside the UnitArgs the unit functions read every other field from.  The multi-step
// DEMetropolisZ instances read UnitArgs through the opaque kernarg pointer: a per-step copy of
// the whole struct with these pointers redirected parked its scalars in VGPR lanes (round 4:
// ~660 v_readlane / 212 v_writelane in the step loop); with the view each field is loaded where
// it is used.  Null: the UnitArgs' own pointers.
struct WdView {
    const double *ce_obs, *ce_lam, *ce_hll_sum, *ce_Emin, *rtd_obs, *rtd_lam, *rtd_hll_sum, *c0_tab;
};

__device__ __forceinline__ void theta_preload(const UnitArgs& a, int64_t u, ThetaPre& t) {
#pragma unroll
    for (int i = 0; i < 6; ++i) t.ce[i] = a.ce_on ? a.theta[(int64_t)a.row_ce[i] * a.U + u] : 0.0;
    t.tau1 = a.rtd_on ? a.theta[(int64_t)a.row_tau1 * a.U + u] : 0.0;
    t.nub = a.rtd_on ? a.theta[(int64_t)a.row_nu * a.U + u] : 0.0;
}

// x of Beta slot i (beta slots follow the host order: CE Ae, F, E, b, nu, then RTD nu,
// then thalf_cfc -- ngrtd.hip add_beta) from the preloaded values when available
// `full`: compile-time promise (literal true, inlined) that the plan has the CE and RTD
// blocks, priors and likelihoods and no Jacobians -- the joint workload -- so that every
// flag test folds away and the unit's work is one straight-line block for the scheduler.
__device__ __forceinline__ double beta_x(const UnitArgs& a, int64_t u, int i, const ThetaPre* pre, bool full) {
    const bool ce_on = full || a.ce_on, rtd_on = full || a.rtd_on;
    if (pre) {
        if (ce_on && i < 5) return pre->ce[i < 3 ? i : i + 1];
        if (rtd_on && i == (ce_on ? 5 : 0)) return pre->nub;
    }
    return a.theta[(int64_t)a.bt_row[i] * a.U + u];
}

// The reference's own Beta priors as compile-time exponent sets (REFB: every FULL instance of
// logp_fused_kernel, the joint plan with the reference's priors): CE Ae (2, 2), F (2, 2), E (2, 4),
// b (2, 2.5), nu (2, 0.1) (noble_gas_mcmc.py:224-226, 237, 249), the RTD nu (2, 0.1) and, with
// the sampled CFC12 half-life, thalf_cfc (2, 2) (run_age_mcmc_utils.py:333-335), in the host's
// slot order (ngrtd.hip add_beta, whose split into integer parts and non-integer coefficients
// the expressions below restate): sets 0 / 1 bare / with the logodds Jacobians (every exponent
// + 1), 2 / 3 the same with thalf_cfc.  With the exponents known the integer powers need no
// selects and the non-integer terms no uniform branches; the arithmetic -- and so every bit --
// is the runtime loop's (A/B: 11.95 -> 11.37 us per c4 launch, profiles/r04i_refb_ab.txt).
struct BetaExp {
    int n;
    int ia[kMaxBeta], ib[kMaxBeta];
    double fa[kMaxBeta], fb[kMaxBeta];
};
constexpr BetaExp kRefBeta[4] = {
    {6, {1, 1, 1, 1, 1, 1, 0}, {1, 1, 3, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0},
     {0, 0, 0, 2.5 - 1, 0.1 - 1, 0.1 - 1, 0}},
    {6, {2, 2, 2, 2, 2, 2, 0}, {2, 2, 4, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0},
     {0, 0, 0, (2.5 - 1) + 1.0, (0.1 - 1) + 1.0, (0.1 - 1) + 1.0, 0}},
    {7, {1, 1, 1, 1, 1, 1, 1}, {1, 1, 3, 0, 0, 0, 1}, {0, 0, 0, 0, 0, 0, 0},
     {0, 0, 0, 2.5 - 1, 0.1 - 1, 0.1 - 1, 0}},
    {7, {2, 2, 2, 2, 2, 2, 2}, {2, 2, 4, 0, 0, 0, 2}, {0, 0, 0, 0, 0, 0, 0},
     {0, 0, 0, (2.5 - 1) + 1.0, (0.1 - 1) + 1.0, (0.1 - 1) + 1.0, 0}}};

template <int REFB = 0>
__device__ __forceinline__ double beta_block(const UnitArgs& a, int64_t u, const ThetaPre* pre = nullptr,
                                             bool full = false) {
    constexpr BetaExp E = REFB ? kRefBeta[REFB - 1] : BetaExp{};
    const int n = REFB ? E.n : a.bt_n;
    auto IA = [&](int i) { return REFB ? E.ia[i] : a.bt_ia[i]; };
    auto IB = [&](int i) { return REFB ? E.ib[i] : a.bt_ib[i]; };
    auto FA = [&](int i) { return REFB ? E.fa[i] : a.bt_fa[i]; };
    auto FB = [&](int i) { return REFB ? E.fb[i] : a.bt_fb[i]; };
    double pint = 1.0, lsum = 0.0;
    bool inb = true;
    double xs[kMaxBeta];
#pragma unroll
    for (int i = 0; i < kMaxBeta; ++i) {
        if (i < n) {
            const double x = beta_x(a, u, i, pre, full);
            xs[i] = x;
            inb &= (x >= 0 && x <= 1);
            pint *= ipow_small(x, IA(i)) * ipow_small(1 - x, IB(i));
            if (FA(i) != 0.0) lsum += FA(i) * flog(x);
            // (1 - x for x in [0, 1]: 0 or >= 2^-53; x outside makes the sum -inf anyway)
            if (FB(i) != 0.0) lsum += FB(i) * flog_z(1 - x);
        }
    }
    // (a normal number: <= 1 in bounds; out of bounds the sum is -inf).  The term-by-term
    // fallback sits behind a wave-uniform branch: as a per-lane branch the compiler evaluated
    // its logs in every lane (9 full logs per unit with the compile-time exponents).  A lane
    // out of bounds needs no fallback (its sum is -inf): in the natural-space sampler a
    // proposal past a Beta variable's [0, 1] made the product negative and sent the wave
    // through it.
    double lint = flog_pn(pint);
    const bool small = inb && !(pint >= 1e-280);
    if (__builtin_expect(__any(small), 0)) {
        double lt = 0.0;
#pragma unroll
        for (int i = 0; i < kMaxBeta; ++i) {
            if (i < n) {
                if (IA(i)) lt += (double)IA(i) * flog(xs[i]);
                if (IB(i)) lt += (double)IB(i) * flog(1 - xs[i]);
            }
        }
        lint = small ? lt : lint;
    }
    return inb ? (lint + lsum) - a.bt_betaln : kNegInf;
}

// full_jac: compile-time promise (with full) that the plan also carries the PyMC3
// transform Jacobians -- the transformed-space sampler's log-prob (sampler.py)
// REFB: the plan's Beta slots are the reference's (kRefBeta[REFB - 1]; FULL instances only)
template <int REFB = 0>
__device__ __forceinline__ double unit_logp_theta(const UnitArgs& a, int64_t u, int l,
                                                  const ThetaPre* pre = nullptr, bool full = false,
                                                  bool full_jac = false, const WdView* wv = nullptr) {
    const bool want_like = full || (a.flags & NGRTD_WANT_LIKE);
    const bool want_prior = full || (a.flags & NGRTD_WANT_PRIOR);
    const bool jac = full ? full_jac : (a.flags & NGRTD_WANT_JACOBIAN) != 0;
    double lp = 0.0;
    if (want_prior) lp += beta_block<REFB>(a, u, pre, full);
    if (full || a.ce_on) {
        double p[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = pre ? pre->ce[i] : a.theta[(int64_t)a.row_ce[i] * a.U + u];
        if (want_prior) lp += normal_logp(p[3], a.m_mu, a.m_tau, a.m_log_tau_2pi);
        if (want_like || (!full && a.ce_out)) {
            // noble_gas_mcmc.py:229-250 parameter mapping, then ce_exc_wrapper (:205-213)
            const double Emin = (wv ? wv->ce_Emin : a.ce_Emin)[l];
            const double Ae_log = p[0] * (a.logA_max - a.logA_min) + a.logA_min;
            const double F_log = p[1] * (a.logF_max - a.logF_min) + a.logF_min;
            const double E = p[2] * (a.E_max - Emin) + Emin;
            const double b = p[4] * (a.b_max - a.b_min) + a.b_min;
            const double nu = p[5] * (a.nu_max - a.nu_min) + a.nu_min;
            const double dm[2] = {p[3], nu};        // 1/m and the Student-t 1/nu: one division
            double rm[2];
            batch_recip<2>(dm, rm);
            const double T = (E - b) * rm[0];
            double mod[kMaxGas];
            ce_model_s0(a, T, lapse_rate_fast(E), exp10_fast(Ae_log), exp10_fast(F_log), mod);
            if (!full && a.ce_out)
                for (int j = 0; j < a.G; ++j) a.ce_out[(int64_t)j * a.U + u] = mod[j];
            if (want_like)
                lp += st_block_inu<kMaxGas>(a.G, (wv ? wv->ce_obs : a.ce_obs) + l * a.G, mod,
                                             (wv ? wv->ce_lam : a.ce_lam) + l * a.G, (wv ? wv->ce_hll_sum : a.ce_hll_sum)[l],
                                             nu, rm[1], C0Tab{wv ? wv->c0_tab : a.c0_tab, a.c0_e0, a.c0_np});
        }
    }
    if (full || a.rtd_on) {
        const double tau1 = pre ? pre->tau1 : a.theta[(int64_t)a.row_tau1 * a.U + u];
        if (want_prior) {
            lp += uniform_logp(tau1, a.tau1_lo, a.tau1_hi, a.tau1_nlw);
            if (jac) lp += jac_interval(tau1, a.tau1_lo, a.tau1_hi, a.tau1_nlw);
#define NGRTD_UNIF(row, lo, hi, nlw)                                                   \
    if (a.row >= 0) {                                                                  \
        const double x = a.theta[(int64_t)a.row * a.U + u];                            \
        lp += uniform_logp(x, a.lo, a.hi, a.nlw);                                      \
        if (jac) lp += jac_interval(x, a.lo, a.hi, a.nlw);                             \
    }
            NGRTD_UNIF(row_tau2, tau2_lo, tau2_hi, tau2_nlw)
            NGRTD_UNIF(row_f1, f1_lo, f1_hi, f1_nlw)
            NGRTD_UNIF(row_eta1, eta1_lo, eta1_hi, eta1_nlw)
            NGRTD_UNIF(row_eta2, eta2_lo, eta2_hi, eta2_nlw)
            NGRTD_UNIF(row_D1, D1_lo, D1_hi, D1_nlw)
            NGRTD_UNIF(row_D2, D2_lo, D2_hi, D2_nlw)
#undef NGRTD_UNIF
            if (a.row_J >= 0) lp += normal_logp(a.theta[(int64_t)a.row_J * a.U + u], a.J_mu, a.J_tau, a.J_log_tau_2pi);
            if (a.row_lamsf6 >= 0) {
                const double x = a.theta[(int64_t)a.row_lamsf6 * a.U + u];
                lp += halfnormal_logp(x, a.ls_tau, a.ls_half_log);
                if (jac) lp += flog(x);
            }
        }
    }
    return lp;
}

// Student-t likelihood of the unit's K model concentrations (run_age_mcmc_utils.py:292-296)
// (NMAX: compile-time bound on K -- the single-launch kernel passes its channel count,
// K <= C since every tracer owns at least one channel)
// (inu: 1 / nu when the caller has it from batched reciprocals)
template <int NMAX = kMaxTracer>
__device__ __forceinline__ double unit_like_rtd(const UnitArgs& a, int64_t u, int l, const double* conc,
                                                const ThetaPre* pre = nullptr, bool full = false,
                                                const double* inu = nullptr, const WdView* wv = nullptr) {
    if (!full && (!a.rtd_on || !(a.flags & NGRTD_WANT_LIKE))) return 0.0;
    const double nub = pre ? pre->nub : a.theta[(int64_t)a.row_nu * a.U + u];
    const double nu = nub * (a.rnu_max - a.rnu_min) + a.rnu_min;
    return st_block_inu<NMAX>(a.K, (wv ? wv->rtd_obs : a.rtd_obs) + l * a.K, conc, (wv ? wv->rtd_lam : a.rtd_lam) + l * a.K,
                              (wv ? wv->rtd_hll_sum : a.rtd_hll_sum)[l], nu, inu ? *inu : 1.0 / nu,
                              C0Tab{wv ? wv->c0_tab : a.c0_tab, a.c0_e0, a.c0_np});
}

// full log-prob contribution of one unit (same addition order as the reference's sum)
__device__ __forceinline__ double unit_logp(const UnitArgs& a, int64_t u, const double* conc) {
    const int l = (int)(u / a.W);
    return unit_logp_theta(a, u, l) + unit_like_rtd(a, u, l, conc);
}

NGRTD_KLINK __global__ void __launch_bounds__(256) unit_logp_kernel(const UnitArgs a) {
    fm_lds_init();
    __syncthreads();
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= a.U) return;
    double conc[kMaxTracer];
    if (a.rtd_on)
        for (int t = 0; t < a.K; ++t) conc[t] = a.conc[(int64_t)t * a.U + u];
    a.ulogp[u] = unit_logp(a, u, conc);
}

// Per-unit log-prob AND the per-walker sum over wells in one launch (L <= 512): a block
// owns WB walkers x LS >= L well slots, one unit per thread; the wells of each walker are
// then added in well order through LDS (deterministic, no atomics, no second launch).
NGRTD_KLINK __global__ void __launch_bounds__(512) unit_walker_kernel(const UnitArgs a, int32_t WB, int32_t LS,
                                                          double* __restrict__ logp) {
    extern __shared__ __attribute__((aligned(16))) double part[];   // [LS][WB]
    fm_lds_init();
    __syncthreads();
    const int wl = threadIdx.x % WB, l = threadIdx.x / WB;
    const int64_t w = (int64_t)blockIdx.x * WB + wl;
    double s = 0.0;
    if (w < a.W && l < a.L) {
        const int64_t u = (int64_t)l * a.W + w;
        double conc[kMaxTracer];
        if (a.rtd_on)
            for (int t = 0; t < a.K; ++t) conc[t] = a.conc[(int64_t)t * a.U + u];
        s = unit_logp(a, u, conc);
    }
    part[l * WB + wl] = s;
    __syncthreads();
    if (l == 0 && w < a.W) {
        double tot = part[wl];
        for (int i = 1; i < a.L; ++i) tot += part[i * WB + wl];
        logp[w] = tot;
    }
}

// ------------------------------------------- exponential RTD on the matrix cores
// Single-component exponential model (convolution_integral_utils.py:184) with every decay
// folded into the channel table, so that for unit u (q = exp(-1/tau_u))
//   Y_c(u) = sum_{j=0}^{n-1} A_{c,1+j} q^j ,   n = N - 1,
// and conc = (tab_{c,0} + s01 Y_c) / (1 + s01 G) as in rtd_conc_kernel.  The ages j are cut
// into S = 4 * SG segments of Lseg (a multiple of 4) ages, j = s*Lseg + 4*step + kq, and
//   Y_c = sum_s q^(s*Lseg) P_{c,s},   P_{c,s} = sum_step sum_kq A_{c,1+j} q^(4*step+kq)
// is a GEMM: rows = (c, s), columns = 16 units, K = 4 ages per v_mfma_f64_16x16x4f64.
// Lane l of a wave supplies
//   B[kq = l>>4][col = l&15] = q_col^(4*step + kq)     (ONE register per 16-unit tile)
//   A[row = l&15][kq = l>>4] of row tile rt           (fragment table, staged in LDS)
// and each B feeds R row tiles (R MFMAs per VALU multiply B *= q^4; the f64 VALU and MFMA
// share one pipe on gfx950, so that ratio bounds the loop).  Row i of tile rt is group
// g = 4*rt + (i>>2), segment slot i&3, i.e. lane (tq = l>>4) accumulates segments
// s = 4m + tq of channel c = g % C (m = g / C) in element (g&3) of accumulator rt: the
// segment sum runs in registers (Horner in q^(4 Lseg)) and the 4 lanes of a column are
// added with two cross-lane shuffles.  With `fuse`, the epilogue also evaluates the CE
// model, both Student-t likelihoods and the priors of the unit (unit_logp).
typedef double ngrtd_v4d __attribute__((ext_vector_type(4)));

constexpr int kMfmaLdsBytes = 64 * 1024;   // fragment bytes staged in LDS at a time
// 16-unit column tiles per wave (accumulators: 8 * NT * R VGPRs) and waves per block
__host__ __device__ constexpr int mfma_tiles(int C) { return mfma_rows(C) <= 5 ? 4 : 2; }
__host__ __device__ constexpr int mfma_waves(int C) { return 16 / mfma_tiles(C); }   // 256 units per block
__host__ __device__ constexpr int mfma_chunk_steps(int C) { return kMfmaLdsBytes / (mfma_rows(C) * 64 * 8); }
constexpr int kMfmaUnitsPerBlock = 256;

// One wave's share of the matrix-core RTD: NT column tiles of 16 units (unit of lane
// column `col` in tile t given by uoff[t]).  init() sets the powers, steps() runs the
// MFMA recurrence over fragments already staged in LDS (callable chunk after chunk),
// finish() forms the per-tile channel sums Y_c (identical in the 4 lanes of a column).
// NTT: tiles held at once (default all of the wave's tiles; 1 = one tile per pass, 40
// accumulator VGPRs at C = 5, for callers with a tight register budget).
template <int C, int NTT = mfma_tiles(C)>
struct MfmaWave {
    static constexpr int R = mfma_rows(C), SG = mfma_groups_per_chan(C), NT = NTT;
    double beta[NT], q4[NT], pw[NT];
    ngrtd_v4d acc[NT][R];

    __device__ __forceinline__ void init(const RtdArgs& a, const int64_t* uoff) {
        const double* tau_row = a.theta + (int64_t)a.row_tau[0] * a.U;
        double tau[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) tau[t] = tau_row[uoff[t]];
        init_tau(tau);
    }
    // ... from the tiles' tau values (the column's unit, tile t)
    __device__ __forceinline__ void init_tau(const double* tau) {
        const int tq = (threadIdx.x & 63) >> 4;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            beta[t] = 1. / tau[t];
            const double q = fexp(-beta[t]);
            const double q2 = q * q;
            q4[t] = q2 * q2;
            pw[t] = (tq == 0) ? 1.0 : (tq == 1) ? q : (tq == 2) ? q2 : q2 * q;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[t][r] = ngrtd_v4d{0.0, 0.0, 0.0, 0.0};
        }
    }
    __device__ __forceinline__ void steps(const double* __restrict__ fr, int nsteps) {
        const double* f = fr + (threadIdx.x & 63);
        for (int step = 0; step < nsteps; ++step, f += R * 64) {
            double A[R];
#pragma unroll
            for (int r = 0; r < R; ++r) A[r] = f[r * 64];
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r)
                    acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[r], pw[t], acc[t][r], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
        }
    }
    // segment sums: lane (tq, col) of tile t holds P_{c, 4m+tq} for all c, m
    __device__ __forceinline__ void finish(const RtdArgs& a, double (*y)[C]) const {
        const int tq = (threadIdx.x & 63) >> 4;
        const double Lseg = (double)a.Lseg;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const double Q = fexp(-beta[t] * Lseg);
            const double Q2 = Q * Q, Q4 = Q2 * Q2;
            const double Qt = (tq == 0) ? 1.0 : (tq == 1) ? Q : (tq == 2) ? Q2 : Q2 * Q;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                double v = 0.0;
#pragma unroll
                for (int m = SG - 1; m >= 0; --m) {
                    const int g = c + C * m;
                    v = fma(v, Q4, acc[t][g >> 2][g & 3]);
                }
                v *= Qt;
                v += __shfl_xor(v, 16);
                v += __shfl_xor(v, 32);
                y[t][c] = v;
            }
        }
    }
};

// ---------------------------------------------- Chebyshev surrogate (see ngrtd_device.hpp)
// Piece of tau and its local coordinate x in [-1, 1]; -1 when tau is not covered (tau < 1/2
// or NaN).  Host and device run this same code (the host validates the table with it).
// OCT0 / OCTS: the binary octaves [2^OCT0, 2^(OCT0 + OCTS)) the pieces split, then the tail.
template <int OCT0, int OCTS>
__host__ __device__ __forceinline__ int cheb_piece_t(double tau, double& x) {
    static_assert(OCT0 + OCTS == kChebOct0 + kChebOcts, "one tail piece for every table");
    constexpr double lo = OCT0 >= 0 ? (double)(1ull << OCT0) : 1.0 / (double)(1ull << -OCT0);
    if (!(tau >= lo)) return -1;
    const unsigned hi = fm_hi(tau);
    const int e = (int)(hi >> 20) - 1023;          // tau > 0: sign bit clear
    if (e >= OCT0 + OCTS) {                        // tau >= 2^18, inf
        const double sv = 1.0 / tau;
        x = sv * (2.0 / kChebSHi) - 1.0;
        return kChebSub * OCTS;
    }
    const int j = (int)((hi >> 18) & 3u);
    const double m = fm_with_hi(tau, (hi & 0x000FFFFFu) | 0x3FF00000u);
    x = (m - (1.125 + 0.25 * j)) * 8.0;
    return (e - OCT0) * kChebSub + j;
}
__host__ __device__ __forceinline__ int cheb_piece(double tau, double& x) {
    return cheb_piece_t<kChebOct0, kChebOcts>(tau, x);
}
// the exp_pist_flow block-tail tables: tau' >= 2^kEpmOct0 (ngrtd_device.hpp)
__host__ __device__ __forceinline__ int epm_piece(double tau, double& x) {
    return cheb_piece_t<kEpmOct0, kEpmOcts>(tau, x);
}

// Surrogate sums of C channels at x from one piece's coefficients [kChebN][CP]: the
// Chebyshev fit in monomial form (cheb_build), evaluated by Horner -- one FMA per
// coefficient and channel.
// PIPE (device only): software-pipelined two rows ahead, with each row's results pinned
// ("+v") behind a compiler memory barrier, so at most three rows of coefficients are live
// in registers -- otherwise the scheduler issues all kChebN rows' LDS loads up front
// (12 C doubles, 144 VGPRs at C = 6), which caps occupancy at 2 waves/SIMD.
template <int C, bool PIPE = false>
__host__ __device__ __forceinline__ void cheb_sums(const double* pc, int CP, double x, double* y) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (PIPE) {   // rows k (cur) and k-1 (nxt) in registers, row k-2 in flight
        double b[C], nxt[C];
#pragma unroll
        for (int c = 0; c < C; ++c) b[c] = pc[(kChebN - 1) * CP + c];
#pragma unroll
        for (int c = 0; c < C; ++c) nxt[c] = pc[(kChebN - 2) * CP + c];
#pragma unroll
        for (int k = kChebN - 2; k >= 0; --k) {
            double nn[C];
            if (k >= 1) {
#pragma unroll
                for (int c = 0; c < C; ++c) nn[c] = pc[(k - 1) * CP + c];
            }
#pragma unroll
            for (int c = 0; c < C; ++c) b[c] = fma(b[c], x, nxt[c]);
#pragma unroll
            for (int c = 0; c < C; ++c) asm volatile("" : "+v"(b[c]));
            asm volatile("" ::: "memory");
            if (k >= 1) {
#pragma unroll
                for (int c = 0; c < C; ++c) nxt[c] = nn[c];
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) y[c] = b[c];
        return;
    }
#endif
#pragma unroll
    for (int c = 0; c < C; ++c) y[c] = pc[(kChebN - 1) * CP + c];
#pragma unroll
    for (int k = kChebN - 2; k >= 0; --k) {
        const double* row = pc + k * CP;
#pragma unroll
        for (int c = 0; c < C; ++c) y[c] = fma(y[c], x, row[c]);
    }
}

// Numerators num_c = A_{c,0} + s01 Y_c and the reciprocal normaliser 1 / (1 + s01 G) ->
// tracer concentrations of unit u (rtd_conc_kernel's combination step): per tracer
// (A + J B) / den, the BMM mix and the SF6 factor (run_age_mcmc_utils.py:154-161).
// num2: the second BMM component's numerators, rden2 its reciprocal normaliser (a piston's
// is g.sum() = 1, convolution_integral_utils.py:178-181, 270): cout = f1 cout1 + f2 cout2 with
// f2 = 1 - f1 (the Deterministic of run_age_mcmc_utils.py:304).
template <int C, bool ST = false>
__device__ __forceinline__ void unit_conc(const RtdArgs& a, int64_t u, const double* num, double rden,
                                          double* conc, const double* num2 = nullptr, double rden2 = 1.0) {
    const double fmix = (a.row_f1 >= 0) ? a.theta[(int64_t)a.row_f1 * a.U + u] : 1.0;
    double Jw = 0.0;
    if (a.row_J >= 0) {
        const double jv = a.theta[(int64_t)a.row_J * a.U + u];
        Jw = a.J_is_log10 ? fexp10(jv) : jv;   // (<= 0.51 ulp: the J of 4He accumulation, 10**J)
    }
    // ST (dz_chain_kernel, whose theta view is a modified local copy of a): t < C -- every tracer
    // owns at least one channel, K <= C -- unrolled with compile-time tracer indices, so that
    // the copy's arrays are indexed statically and the copy stays in registers (a runtime index
    // put it in scratch).  The plain kernels keep the runtime loop (unrolled, their kernarg
    // arrays went to ~250 spilled SGPRs).
    auto tracer = [&](int t) {
        double sA = 0.0, sB = 0.0, sA2 = 0.0, sB2 = 0.0;
        bool hasB = false;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (a.chan_tracer[c] != t) continue;
            if (a.chan_isB[c]) { sB = num[c]; hasB = true; if (num2) sB2 = num2[c]; }
            else { sA = num[c]; if (num2) sA2 = num2[c]; }
        }
        const double J = (a.row_J >= 0) ? Jw : a.tr_J[t];
        const double cc = hasB ? (sA + J * sB) * rden : sA * rden;
        double cout;
        if (num2) {
            const double cc2 = (hasB ? (sA2 + J * sB2) : sA2) * rden2;
            cout = fmix * cc + (1 - fmix) * cc2;
        } else {
            cout = fmix * cc + 0.0 * 0.0;   // f1*cout1 + f2*cout2, run_age_mcmc_utils.py:154
        }
        if (a.tr_sf6[t] && a.row_lamsf6 >= 0) cout *= (1 + a.theta[(int64_t)a.row_lamsf6 * a.U + u]);
        conc[t] = cout;
    };
    if constexpr (ST) {
#pragma unroll
        for (int t = 0; t < C; ++t)
            if (t < a.K) tracer(t);
    } else {
        if (a.conc_ident) {
            // tracer t owns exactly channel t (the plan's table order; K = C): no channel search,
            // the same expressions as tracer(t) with one channel (the SF6 factor as a select:
            // x * 1.0 is x, so the bits are the branch's)
            const double sf = (a.row_lamsf6 >= 0) ? 1 + a.theta[(int64_t)a.row_lamsf6 * a.U + u] : 1.0;
#pragma unroll
            for (int t = 0; t < C; ++t) {
                const bool isB = a.chan_isB[t] != 0;
                const double J = (a.row_J >= 0) ? Jw : a.tr_J[t];
                const double sA = isB ? 0.0 : num[t], sB = isB ? num[t] : 0.0;
                const double cc = isB ? (sA + J * sB) * rden : sA * rden;
                double cout;
                if (num2) {
                    const double sA2 = isB ? 0.0 : num2[t], sB2 = isB ? num2[t] : 0.0;
                    const double cc2 = (isB ? (sA2 + J * sB2) : sA2) * rden2;
                    cout = fmix * cc + (1 - fmix) * cc2;
                } else {
                    cout = fmix * cc + 0.0 * 0.0;
                }
                conc[t] = cout * (a.tr_sf6[t] ? sf : 1.0);
            }
            return;
        }
        for (int t = 0; t < a.K; ++t) tracer(t);
    }
}

// Piston second component (BMM, convolution_integral_utils.py:178-181): the channel-table
// row at the FIRST argmin |tp - tau2| -- a lookup, no age loop.
// LW: channel 0 decays per unit (the sampled CFC12 half-life, decay constant lam): its row
// value times exp(-lam tp_ix) (convolution_integral_utils.py:316, g * exp(-lamba tp)).
template <int C, bool LW = false>
__device__ __forceinline__ void piston_num_tau(const RtdArgs& a, double tau2, double* num2, double lam = 0.0) {
    const int ix = piston_index(tau2, a.tp0, a.dtp, a.N);
#pragma unroll
    for (int c = 0; c < C; ++c) num2[c] = a.tab[(int64_t)ix * a.CP + c];
    if (LW) num2[0] *= fexp(-lam * (ix == 0 ? a.tp0 : (double)ix + a.dtp));
}
template <int C, bool LW = false>
__device__ __forceinline__ void piston_num(const RtdArgs& a, int64_t u, double* num2, double lam = 0.0) {
    piston_num_tau<C, LW>(a, a.theta[(int64_t)a.row_tau[1] * a.U + u], num2, lam);
}

// The sampled CFC12 half-life (run_age_mcmc_utils.py:107-109, savenum with a 2) as the
// single-launch kernel carries it (LW instances): the plan puts the CFC12 channel first and
// leaves it undecayed, so that for a unit with decay constant lam = ln2 / t_half
// (thalf_2_lambda, convolution_integral_utils.py:146-152) and exponential weights e^(-tp/tau)
// the decayed numerator sum_k C_k e^(-tp_k / tau) e^(-lam tp_k) is
//   e^(-lam tp_0) (C_0 + Z_0(tau_eff)),   1 / tau_eff = 1 / tau + lam,
// with Z_0 the SAME channel function the surrogate fits (a function of one variable); the
// normaliser stays a function of tau.  One reciprocal gives both lam and tau_eff:
// tau_eff = tau t / (t + ln2 tau).
struct LwDecay {
    double lam, teff;
};
__device__ __forceinline__ LwDecay lw_decay(const RtdArgs& a, double tau, double thx) {
    const double th = a.thalf_a * thx + a.thalf_b;                // t_half = 5 + 30 Beta (:334)
    const double d[2] = {th, th + kLn2Ref * tau};
    double r[2];
    batch_recip<2>(d, r);
    return LwDecay{kLn2Ref * r[0], (tau * th) * r[1]};
}

// The reference's exponential weights g = (1/tau) exp(-tp/tau) / sum(...) (:184, :270)
// are NaN for every age when exp overflows for some age (inf / inf), when every weight
// underflows to 0 (0 / 0), and for tau = 0 or NaN; otherwise finite.  -tp/tau is monotone
// in tp, so its extremes are at tp_0 and tp_{N-1}.
// tau = +-inf: 1/tau = 0 makes every weight 0 (0 / 0 as well).
__device__ __forceinline__ bool exp_rtd_nan(const RtdArgs& a, double tau) {
    const double tpN = (a.N > 1) ? (double)(a.N - 1) + a.dtp : a.tp0;
    const double x0 = (-a.tp0) / tau, xN = (-tpN) / tau;
    const double xmax = x0 > xN ? x0 : xN;
    return !(tau == tau) || tau == 0.0 || !(fabs(tau) <= 1.7976931348623157e308) || !(xmax == xmax) ||
           xmax > 709.782712893384 || xmax < -745.1332191019412;
}

// Exact channel sums Y_c (matrix-core path) -> concentrations: the normaliser
// 1 + s01 G with G = sum_{j<n} q^j = expm1(-beta n) / expm1(-beta) in closed form.
// LW: channel 0 decays per unit (lw_decay): yw = its exact sum Y_0 at tau_eff (bw = 1 / tau_eff)
// and lam, numerator e^(-lam tp_0) (C_0 + s01(bw) yw).
template <int C, bool LW = false, bool ST = false>
__device__ __forceinline__ void mfma_unit_conc(const RtdArgs& a, int64_t u, double bu, const double* yy,
                                               double* conc, const double* num2 = nullptr, double lam = 0.0,
                                               double yw = 0.0, double bw = 0.0) {
    const int n = a.N - 1;
    const double d01 = (1.0 + a.dtp) - a.tp0;
    const double s01 = fexp(-bu * d01);
    const double G = (n > 0) ? fexpm1(-bu * (double)n) / fexpm1(-bu) : 0.0;
    const double rden = 1.0 / (1.0 + s01 * G);     // one division for the K tracers (<= 1 ulp)
    double num[C];
#pragma unroll
    for (int c = 0; c < C; ++c) num[c] = a.tab0[c] + s01 * yy[c];
    if (LW) num[0] = fexp(-lam * a.tp0) * (a.tab0[0] + fexp(-bw * d01) * yw);
    unit_conc<C, ST>(a, u, num, rden, conc, num2);    // (num2: the piston component of a BMM)
    const double tau = a.theta[(int64_t)a.row_tau[0] * a.U + u];
    if (exp_rtd_nan(a, tau)) {
#pragma unroll
        for (int t = 0; t < kMaxTracer; ++t)
            if (t < a.K) conc[t] = __builtin_nan("");
    }
}

// lanes with tq = t finish the units of tile t: select that tile's sums
template <int C>
__device__ __forceinline__ void mfma_pick_tile(const double (*y)[C], const double* beta, double* yy, double& bu) {
    constexpr int NT = mfma_tiles(C);
    const int tq = (threadIdx.x & 63) >> 4;
    bu = 0.0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        if (t == tq) {
            bu = beta[t];
#pragma unroll
            for (int c = 0; c < C; ++c) yy[c] = y[t][c];
        }
    }
}

template <int C>
__global__ void __launch_bounds__(64 * mfma_waves(C)) rtd_exp_mfma_kernel(const RtdArgs a, const UnitArgs ua,
                                                                         int32_t fuse) {
    constexpr int R = mfma_rows(C), NT = mfma_tiles(C), NW = mfma_waves(C);
    constexpr int CHUNK = mfma_chunk_steps(C);
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int col = lane & 15, tq = lane >> 4;
    const int64_t u0 = ((int64_t)blockIdx.x * NW + wave) * (16 * NT);
    const int64_t Umax = a.U - 1;
    fm_lds_init();
    __syncthreads();
    int64_t uoff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int64_t u = u0 + 16 * t + col;
        uoff[t] = u < Umax ? u : Umax;
    }
    MfmaWave<C> mw;
    mw.init(a, uoff);
    for (int c0 = 0; c0 < a.nsteps; c0 += CHUNK) {
        const int cn = (a.nsteps - c0) < CHUNK ? (a.nsteps - c0) : CHUNK;
        if (c0 > 0) __syncthreads();
        // fragments of steps [c0, c0 + cn): cn * R * 512 contiguous bytes
        const double2* src = reinterpret_cast<const double2*>(a.frag + (int64_t)c0 * R * 64);
        double2* dst = reinterpret_cast<double2*>(lds);
        for (int i = threadIdx.x; i < cn * R * 32; i += 64 * NW) dst[i] = src[i];
        __syncthreads();
        mw.steps(lds, cn);
    }
    double y[NT][C];
    mw.finish(a, y);
    if (tq >= NT) return;
    double yy[C], bu;
    mfma_pick_tile<C>(y, mw.beta, yy, bu);
    const int64_t u = u0 + 16 * tq + col;
    if (u > Umax) return;
    double conc[kMaxTracer];
    mfma_unit_conc<C>(a, u, bu, yy, conc);
    if (a.conc)
        for (int t = 0; t < a.K; ++t) a.conc[(int64_t)t * a.U + u] = conc[t];
    if (fuse) ua.ulogp[u] = unit_logp(ua, u, conc);
}

// The whole batched log-prob in ONE launch (exponential single-component RTD with
// C <= 5 channels, L <= 512; FULL: the joint CE + RTD plan with priors and likelihoods).  A block of 8 waves owns WB = 512 / L walkers x all L wells
// (block-local unit i = l * WB + w'); lane `lane` of wave `wave` owns unit
// i = 64 * wave + lane for all of its work:
//  1. the theta-only part: CE model + likelihood and all priors (the surrogate table's
//     global loads, issued first into registers, land meanwhile);
//  2. the channel sums Y_c(tau) from the Chebyshev surrogate (a.cheb, staged in LDS; about
//     C * 2 * kChebN FP64 ops per unit instead of C * (N - 1) FMAs).  A wave with a lane
//     whose tau the surrogate does not cover (tau < 1/2, NaN) evaluates the exact sums of
//     all 4 of its 16-unit tiles on the matrix cores instead (MfmaWave; fragments read
//     from global memory / L2, the exact path of rtd_exp_mfma_kernel); so does every wave
//     when the plan has no validated surrogate (a.cheb == nullptr);
//  3. the unit's concentrations and RTD Student-t likelihood.
// Per-walker sums over wells run through LDS: for WB a power of two <= 64, lane
// (g, w') of wave 0 adds wells g, g + 64/WB, ... in order and the 64/WB partials are
// combined by a fixed xor-shuffle tree; otherwise WB lanes add the L wells in order.
// Both orders are fixed (deterministic, no atomics).
// ------------------------------------------------------------- device DE-MC
// Counter-based RNG: splitmix64 finaliser.  Per step one key = mix(mix(seed) + step);
// stream s of the step is mix(key + s) (1: partners, 2: proposal noise, 3: accept), and
// draw i of a stream is mix(stream + i).  Uniforms lie in (0, 1) exclusive of both ends.
__host__ __device__ __forceinline__ uint64_t rng_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t demc_key(uint64_t seed, uint64_t step) {
    return rng_mix(rng_mix(seed) + step);
}
// Step j of a multi-step DEMetropolisZ launch (DemcAccept::Sched): ngrtd_demcz_run's
// per-step bookkeeping -- every step but the call's first appends its state (the previous
// step's q_new) at the current history length; stop_tuning drops the oldest drop * (len - lo)
// entries at step n_tune (after that step's append); tune() after the decision of a step
// whose successor is a multiple of tune_interval below n_tune.
__host__ __device__ __forceinline__ DzStep dz_step(const DemcAccept::Sched& c, int64_t j) {
    DzStep r;
    const int64_t s = c.s0 + j;
    r.key = demc_key(c.seed, (uint64_t)s);
    r.len = c.h_len0 + (c.append0 ? j + 1 : j);
    r.at = (c.append0 || j > 0) ? r.len - 1 : -1;
    r.lo = c.h_lo0;
    if (c.n_tune > 0 && c.s0 <= c.n_tune && c.n_tune <= s) {
        const int64_t jd = c.n_tune - c.s0;
        const int64_t lend = c.h_len0 + (c.append0 ? jd + 1 : jd);
        r.lo += (int64_t)(c.drop * (double)(lend - c.h_lo0));
    }
    r.it = r.len - r.lo;
    const int64_t next = s + 1;
    r.tune_now = (c.tune_target != NGRTD_TUNE_NONE && next < c.n_tune && next % c.tune_interval == 0) ? 1 : 0;
    return r;
}
__host__ __device__ __forceinline__ double rng_unit(uint64_t h) {
    return ((double)(h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

// PyMC3 3.11.2 step_methods/metropolis.py tune(): multiplicative update from the
// acceptance rate of the last tune interval.
__host__ __device__ __forceinline__ double pymc3_tune(double scale, double acc_rate) {
    if (acc_rate < 0.001) return scale * 0.1;
    if (acc_rate < 0.05) return scale * 0.5;
    if (acc_rate < 0.2) return scale * 0.9;
    if (acc_rate > 0.95) return scale * 10.0;
    if (acc_rate > 0.75) return scale * 2.0;
    if (acc_rate > 0.5) return scale * 1.1;
    return scale;
}

// Metropolis decision of chain w (PyMC3 metrop_select, step_methods/arraystep.py: accept
// iff mr = logp(x*) - logp(x) is finite and log(u) < mr), applied to lp[w]; one thread per
// chain.  Then the chain's tuning counter and, at the end of a tune interval, its lamb or
// scaling (DEMetropolisZ.astep: tuned at the start of the next step from the interval's
// acceptance rate, counter reset).  Returns the decision.
// Chain index w of the per-chain arrays, random-stream id rid (joint chains: chain0 + w;
// per-well chains: the unit's cid, dz_cid).
// The acceptances of the calling lanes, counted with ONE atomic per wave (an integer count:
// order-independent; one atomic per accepted per-well chain serialised ~10^5 atomics on one
// address per step).
__device__ __forceinline__ void count_accepts(unsigned long long* n, bool acc) {
    const unsigned long long act = __ballot(1), m = __ballot(acc);
    if (m && (int)__lane_id() == __ffsll((long long)act) - 1) atomicAdd(n, (unsigned long long)__popcll(m));
}
// li: the chain's index in the logs (log_off + li), which may differ from w (per-well chains
// in the multi-step launch keep their state arrays walker-major).
// count: add the decision to d.n_acc here (per wave); the per-well multi-step launch counts
// per block itself (one atomic per block: same-address atomics serialise in L2, and one per
// wave cost ~10 us per c4 step).
// The chain's lp / lamb / scaling / tuning counter at index w of the arrays given (d's own
// global arrays, or the multi-step launch's LDS copies, DemcAccept::state_lds; the tuning
// state exists iff d.n_acc_tune does); acc_out: the decision array, stored iff store_acc.
// (Flags rather than null tests: a null test of an LDS-derived generic pointer miscompiles.)
// The accept draw's log: log(u) of the (key, rid) stream (a function of the step and the
// chain only, so the multi-step launch takes it before the step's log-prob is known).
// (flog: table-driven, <= 1 ulp; the torch restatement takes the same function through
// ngrtd_fm_log, so the chains stay bitwise equal.  Every kernel that decides runs
// fm_lds_init() and a barrier first.)
// (rng_unit lies in [2^-54, 1 - 2^-54]: flog_pn gives flog's bits there)
__device__ __forceinline__ double demc_logu(uint64_t key, uint64_t rid) {
    return flog_pn(rng_unit(rng_mix(rng_mix(key + 3) + rid)));
}
template <class F64P, class I32P>
__device__ __forceinline__ bool demc_decide_at_u(const DemcAccept& d, F64P lpa, F64P lamb, F64P scal, I32P nat,
                                                 int32_t* acc_out, bool store_acc, int64_t w, double logu,
                                                 double lp_prop, int32_t tune_now, int64_t log_off, int64_t li,
                                                 bool count) {
    const double cur = lpa[w];
    const double mr = lp_prop - cur;
    const bool acc = __builtin_isfinite(mr) && logu < mr;
    if (store_acc) acc_out[w] = acc;
    if (acc) lpa[w] = lp_prop;
    if (count && d.n_acc) count_accepts(d.n_acc, acc);
    if (d.n_acc_tune) {
        int32_t na = nat[w] + (acc ? 1 : 0);
        if (tune_now) {
            const double rate = (double)na / (double)d.tune_interval;
            if (d.tune_target == 2) lamb[w] = pymc3_tune(lamb[w], rate);
            else if (d.tune_target == 1) scal[w] = pymc3_tune(scal[w], rate);
            na = 0;
        }
        nat[w] = na;
    }
    if (d.acc_log) d.acc_log[log_off + li] = (uint8_t)acc;
    if (d.lp_log) d.lp_log[log_off + li] = acc ? lp_prop : cur;
    if (d.ar_log) d.ar_log[log_off + li] = exp(mr);
    return acc;
}
template <class F64P, class I32P>
__device__ __forceinline__ bool demc_decide_at(const DemcAccept& d, F64P lpa, F64P lamb, F64P scal, I32P nat,
                                               int32_t* acc_out, bool store_acc, int64_t w, uint64_t rid,
                                               double lp_prop, uint64_t key, int32_t tune_now, int64_t log_off,
                                               int64_t li, bool count) {
    return demc_decide_at_u(d, lpa, lamb, scal, nat, acc_out, store_acc, w, demc_logu(key, rid), lp_prop, tune_now,
                            log_off, li, count);
}
__device__ __forceinline__ bool demc_decide(const DemcAccept& d, int64_t w, uint64_t rid, double lp_prop,
                                            uint64_t key, int32_t tune_now, int64_t log_off, int64_t li,
                                            bool count = true) {
    return demc_decide_at(d, d.lp, d.lamb, d.scaling, d.n_acc_tune, d.acc, true, w, rid, lp_prop, key, tune_now,
                          log_off, li, count);
}
__device__ __forceinline__ bool demc_decide(const DemcAccept& d, int64_t w, uint64_t rid, double lp_prop,
                                            uint64_t key, int32_t tune_now, int64_t log_off) {
    return demc_decide(d, w, rid, lp_prop, key, tune_now, log_off, w);
}
__device__ __forceinline__ bool demc_decide(const DemcAccept& d, int64_t w, double lp_prop, uint64_t key,
                                            int32_t tune_now, int64_t log_off) {
    return demc_decide(d, w, (uint64_t)(d.chain0 + w), lp_prop, key, tune_now, log_off);
}
__device__ __forceinline__ bool demc_decide(const DemcAccept& d, int64_t w, double lp_prop) {
    return demc_decide(d, w, lp_prop, d.key, d.tune_now, 0);
}
// Per-well chains: the random-stream id of unit (walker w, well l) -- the same in a run of
// all L wells and in a run of well l alone (well0 = l), and in any walker-block shard.  It
// keys the unit's proposal noise and its accept draw; the partner indices are keyed by the
// walker (every well of a walker draws the same indices, each into its own history), so
// each well's chain is still exactly a DEMetropolisZ chain.
__host__ __device__ __forceinline__ uint64_t dz_cid(int64_t well0, int64_t l, int64_t Wg, int64_t chain0, int64_t w) {
    return (uint64_t)(well0 + l) * (uint64_t)Wg + (uint64_t)(chain0 + w);
}
// ... and the noise element of its parameter row p (rows of one chain are contiguous)
constexpr int kPwRowStride = 32;   // >= NGRTD_ROLE_COUNT
__host__ __device__ __forceinline__ uint64_t dz_pw_elem(uint64_t cid, int p) {
    return cid * (uint64_t)kPwRowStride + (uint64_t)p;
}

// accept after the generic kernels: one thread per walker decides and copies the
// walker's P*L proposal rows into the state (coalesced across the walkers of a wave)
NGRTD_KLINK __global__ void __launch_bounds__(256) demc_accept_kernel(const DemcAccept d, const double* __restrict__ lp_prop,
                                                          int64_t W, int64_t R) {
    fm_lds_init();                           // flog (demc_logu)
    __syncthreads();
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    if (demc_decide(d, w, lp_prop[w])) {
        for (int64_t r = 0; r < R; ++r) d.x[r * W + w] = d.prop[r * W + w];
        if (d.xu)
            for (int64_t r = 0; r < R; ++r) d.xu[r * W + w] = d.prop_u[r * W + w];
    }
}

// PyMC3 3.11 transforms (pymc3/distributions/transforms.py) backward(u): LogOdds
// invlogit(u, 0) = 1 / (1 + exp(-u)); Interval s b + (1 - s) a with s = sigmoid(u); Log exp(u).
// exp is the table-driven fexp (<= 1 ulp, a third of OCML's instructions: the transformed
// DEMetropolisZ step evaluates one per parameter row); sampler.Transform calls this same
// function on the device (ngrtd_pymc3_backward), so the chains agree bitwise.  Kernels that
// call it run fm_lds_init() and a barrier first (the host reads the constant table).
__host__ __device__ __forceinline__ double pymc3_backward(int kind, double a, double b, double u) {
    if (kind == NGRTD_TR_LOGODDS) return 1.0 / (1.0 + fexp(-u));
    if (kind == NGRTD_TR_INTERVAL) {
        const double s = 1.0 / (1.0 + fexp(-u));
        return s * b + (1.0 - s) * a;
    }
    if (kind == NGRTD_TR_LOG) return fexp(u);
    return u;
}
// The same values with ONE exp call and selects (straight-line: what an unrolled loop
// over the parameter rows wants); bitwise equal to pymc3_backward.
__device__ __forceinline__ double pymc3_backward_sel(int kind, double a, double b, double u) {
    const double ex = fexp(kind == NGRTD_TR_LOG ? u : -u);
    const double s = 1.0 / (1.0 + ex);
    const double iv = s * b + (1.0 - s) * a;
    return kind == NGRTD_TR_LOGODDS ? s : kind == NGRTD_TR_INTERVAL ? iv : kind == NGRTD_TR_LOG ? ex : u;
}

// Partners of chain w for the step keyed `key` (DEMetropolisZ.astep: iz1 = randint(it),
// iz2 = randint(it) redrawn until != iz1 -- i.e. uniform over the it - 1 others):
// iz1 = floor(u1 it), iz2 = floor(u2 (it - 1)), +1 when >= iz1.  it >= 2.
__host__ __device__ __forceinline__ void demcz_partners(uint64_t key, uint64_t w, uint64_t it, uint64_t& iz1,
                                                        uint64_t& iz2) {
    const uint64_t hp = rng_mix(rng_mix(key + 1) + w);
    iz1 = ((hp >> 32) * it) >> 32;
    iz2 = ((hp & 0xFFFFFFFFull) * (it - 1)) >> 32;
    iz2 += (iz2 >= iz1) ? 1 : 0;
}

// DEMetropolisZ proposal of every chain (pymc3 DEMetropolisZ.astep):
//   x* = x + lamb_w (Z_w[iz1] - Z_w[iz2]) + eps,  eps = U(-1, 1) S_r scaling_w per row
// (noise only while the history has < 2 entries), the history append of the current state
// x (the previous step's q_new) into entry append_at, and -- transformed chains -- the
// natural-space copy backward(x*) the log-prob reads.
// Layouts: theta / proposals are [R][W] (walkers contiguous: what the log-prob kernel
// reads coalesced); the history is CHAIN-major, entry e of chain w at (e W + w) R: a
// partner state is one contiguous R * 8-byte run (4 KiB at c4), so the two random
// partner reads per chain hit whole DRAM pages instead of R scattered lines.  A block
// owns a tile of kZTileW chains x kZTileR rows and transposes through LDS: x rows are read
// (and proposals written) 128 B per row, history rows 1 KiB per chain.
constexpr int kZTileW = 16, kZTileR = 128, kZThreads = 256;
constexpr int kZPer = kZTileW * kZTileR / kZThreads;   // tile elements per thread (8)
NGRTD_KLINK __global__ void __launch_bounds__(kZThreads) demcz_propose_kernel(const DemczArgs d) {
    fm_lds_init();                                    // fexp (pymc3_backward), behind the barrier below
    __shared__ double xs[kZTileW][kZTileR + 1];       // chain-major tiles (+1: no bank conflicts)
    __shared__ double ps[kZTileW][kZTileR + 1];
    __shared__ double px[kZTileW][kZTileR + 1];
    const int64_t W = d.W, R = d.R;
    const int64_t w0 = (int64_t)blockIdx.x * kZTileW, r0 = (int64_t)blockIdx.y * kZTileR;
    const int nw = (int)((W - w0) < kZTileW ? (W - w0) : kZTileW);
    const int nr = (int)((R - r0) < kZTileR ? (R - r0) : kZTileR);
    const int t = threadIdx.x;
    // chain-major mapping: thread -> (chain j, rows i0 + 16 k); row-major: (row t / 16 + 16 k, chain t % 16)
    const int j = t / kZTileW, i0 = t % kZTileW;
    const int jr = t % kZTileW, ir = t / kZTileW;
    const bool jv = j < nw;
    const int64_t w = w0 + j;
    const size_t entry = (size_t)W * R;
    // ONE memory round trip: the partner indices need only the random key, so the x tile
    // (row-major) and both partner runs (chain-major) are loaded together
    const bool de = d.propose && d.it > 1;
    int64_t e1 = -1, e2 = -1;
    if (de && jv) {
        uint64_t iz1, iz2;
        demcz_partners(d.key, (uint64_t)(d.chain0 + w), (uint64_t)d.it, iz1, iz2);
        e1 = d.lo + (int64_t)iz1;
        e2 = d.lo + (int64_t)iz2;
    }
    double xr[kZPer], z1v[kZPer], z2v[kZPer];
#pragma unroll
    for (int k = 0; k < kZPer; ++k) {
        const int i = ir + kZTileW * k;
        xr[k] = (i < nr && jr < nw) ? d.x[(r0 + i) * W + w0 + jr] : 0.0;
    }
    if (de && jv) {
        const double* z1 = d.hist + (size_t)e1 * entry + (size_t)w * R + r0;
        const double* z2 = d.hist + (size_t)e2 * entry + (size_t)w * R + r0;
#pragma unroll
        for (int k = 0; k < kZPer; ++k) {
            const int i = i0 + kZTileW * k;
            z1v[k] = i < nr ? z1[i] : 0.0;
            z2v[k] = i < nr ? z2[i] : 0.0;
        }
    }
#pragma unroll
    for (int k = 0; k < kZPer; ++k) {
        const int i = ir + kZTileW * k;
        if (i < nr && jr < nw) xs[jr][i] = xr[k];
    }
    __syncthreads();
    // history append (contiguous R-runs per chain)
    if (d.append_at >= 0 && jv) {
        double* dst = d.hist + (size_t)d.append_at * entry + (size_t)w * R + r0;
#pragma unroll
        for (int k = 0; k < kZPer; ++k) {
            const int i = i0 + kZTileW * k;
            if (i < nr) dst[i] = xs[j][i];
        }
    }
    if (!d.propose) return;
    if (jv) {
        const double lamb = d.lamb[w], sc = d.scaling[w];
        const uint64_t ke = rng_mix(d.key + 2);
        // an entry appended by this block in this launch: its values are x itself
        const bool c1 = e1 == d.append_at, c2 = e2 == d.append_at;
#pragma unroll
        for (int k = 0; k < kZPer; ++k) {
            const int i = i0 + kZTileW * k;
            if (i >= nr) continue;
            const double x = xs[j][i];
            double y = x;
            if (de) {
                const double a1 = c1 ? x : z1v[k], a2 = c2 ? x : z2v[k];
                y = x + lamb * (a1 - a2);
            }
            // element stream: row-major over (row, GLOBAL chain) -- a shard draws its chains' numbers
            const uint64_t e = (uint64_t)(r0 + i) * (uint64_t)d.Wg + (uint64_t)(d.chain0 + w);
            const double u2 = 2.0 * rng_unit(rng_mix(ke + e)) - 1.0;
            const double eps = (d.S ? u2 * d.S[r0 + i] : u2) * sc;
            const double v = y + eps;
            ps[j][i] = v;
            if (d.prop_x) {       // transformed chains: the natural-space value the log-prob reads
                const int pr = (int)((r0 + i) / d.L);
                px[j][i] = pymc3_backward(d.tr_kind[pr], d.tr_a[pr], d.tr_b[pr], v);
            }
        }
    }
    __syncthreads();
    // proposals back to [R][W], 128 B per row
#pragma unroll
    for (int k = 0; k < kZPer; ++k) {
        const int i = ir + kZTileW * k;
        if (i < nr && jr < nw) {
            d.prop[(r0 + i) * W + w0 + jr] = ps[jr][i];
            if (d.prop_x) d.prop_x[(r0 + i) * W + w0 + jr] = px[jr][i];
        }
    }
}

// sampler.Transform.backward / the torch restatement's accept draws on the device: the same
// pymc3_backward / flog the DEMetropolisZ kernels evaluate (ngrtd_pymc3_backward, ngrtd_fm_log)
struct TrRows {
    int32_t kind[kRoleCount];
    double a[kRoleCount], b[kRoleCount];
};
NGRTD_KLINK __global__ void __launch_bounds__(256) pymc3_backward_kernel(const double* __restrict__ u,
                                                                         double* __restrict__ x, int64_t n, int32_t P,
                                                                         int64_t inner, const TrRows t) {
    fm_lds_init();
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int p = (int)((i / inner) % P);
    x[i] = pymc3_backward(t.kind[p], t.a[p], t.b[p], u[i]);
}
NGRTD_KLINK __global__ void __launch_bounds__(256) fm_log_kernel(const double* __restrict__ in, double* __restrict__ out,
                                                                 int64_t n) {
    fm_lds_init();
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = flog(in[i]);
}

// out[p][b][a] = in[p][a][b] for p < P (a < A, b < B): the caller's [P][L][W] state into the
// multi-step DEMetropolisZ launch's walker-major [P][W][L] and back (and, per-well chains,
// the per-chain arrays [L][W] <-> [W][L]).  32 x 32 LDS tiles.
template <class T>
__device__ __forceinline__ void dz_layout_body(T (*t)[33], const T* __restrict__ in, T* __restrict__ out, int64_t A,
                                               int64_t B) {
    const int64_t p = blockIdx.z;
    const int64_t a0 = (int64_t)blockIdx.y * 32, b0 = (int64_t)blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const T* src = in + p * A * B;
    T* dst = out + p * A * B;
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
        const int64_t a = a0 + ty + k, b = b0 + tx;
        if (a < A && b < B) t[ty + k][tx] = src[a * B + b];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
        const int64_t b = b0 + ty + k, a = a0 + tx;
        if (a < A && b < B) dst[b * A + a] = t[tx][ty + k];
    }
}
NGRTD_KLINK __global__ void __launch_bounds__(256) dz_layout_kernel(const double* __restrict__ in,
                                                                    double* __restrict__ out, int64_t A, int64_t B) {
    __shared__ double t[32][33];
    dz_layout_body<double>(t, in, out, A, B);
}
NGRTD_KLINK __global__ void __launch_bounds__(256) dz_layout_i32_kernel(const int32_t* __restrict__ in,
                                                                        int32_t* __restrict__ out, int64_t A, int64_t B) {
    __shared__ int32_t t[32][33];
    dz_layout_body<int32_t>(t, in, out, A, B);
}

constexpr int kDzMaxP = 12;          // parameter rows of a single-launch DEMetropolisZ step
#ifndef NGRTD_DZ_PREFETCH
#define NGRTD_DZ_PREFETCH 1
#endif
constexpr bool kDzPrefetch = NGRTD_DZ_PREFETCH != 0;   // partner rows one step ahead (dz_partner_rows)
#ifndef NGRTD_DZ_TR_BRANCH
#define NGRTD_DZ_TR_BRANCH 1
#endif
#ifndef NGRTD_DZ_PF_STEP
#define NGRTD_DZ_PF_STEP 2
#endif
// 2: each role prefetches and stages its parity's rows; 1: the theta lanes all of them.
// Per-well chains stage from the theta lanes only (their RTD waves carry the longer log-prob
// body, so the step's critical path loses the RTD waves' staging: A/B 17.5-18.2 -> 16.9-17.1 us
// transformed, 15.7-15.8 -> 15.2-15.3 us natural, profiles/r04y_dz_pfstep_ab.txt); joint
// chains keep the split (1 was 0.15 us slower there).
#ifndef NGRTD_DZ_PF_STEP_PW
#define NGRTD_DZ_PF_STEP_PW 1
#endif
constexpr int kDzPfStep = NGRTD_DZ_PF_STEP;
constexpr int kDzPfStepPw = NGRTD_DZ_PF_STEP_PW;
constexpr int kFusedUnitsDz = 512;   // = kFusedUnits (units per logp_fused_kernel block)

// One element of a DEMetropolisZ proposal, the arithmetic of demcz_propose_kernel (bitwise):
// x + lamb (z1 - z2) + eps, eps = U(-1, 1) S_r scaling from the (row, global chain) stream.
// e: the noise element (row-major (row, global chain) for joint chains, dz_pw_elem for
// per-well chains); r: the theta row p L + l (the index of S).
// x* = x + lamb (z1 - z2) + U(-1, 1) S_r scaling (no DE term while the history has < 2
// entries); sr = S_r when has_s.
__device__ __forceinline__ double dz_value_core(bool de, double x, double z1, double z2, double lamb, double sc,
                                               uint64_t ke, uint64_t e, bool has_s, double sr) {
    const double y = de ? x + lamb * (z1 - z2) : x;
    const double u2 = 2.0 * rng_unit(rng_mix(ke + e)) - 1.0;
    const double eps = (has_s ? u2 * sr : u2) * sc;
    return y + eps;
}
template <class A>
__device__ __forceinline__ double dz_value_e(const A& d, bool de, double x, double z1, double z2, double lamb,
                                            double sc, uint64_t ke, uint64_t e, int64_t r) {
    return dz_value_core(de, x, z1, z2, lamb, sc, ke, e, d.S != nullptr, d.S ? d.S[r] : 1.0);
}
__device__ __forceinline__ double dz_value(const DemcAccept& d, bool de, double x, double z1, double z2, double lamb,
                                          double sc, uint64_t ke, int64_t r, int64_t chain) {
    return dz_value_e(d, de, x, z1, z2, lamb, sc, ke, (uint64_t)r * (uint64_t)d.Wg + (uint64_t)chain, r);
}

// Per-well chains (DemczArgs::per_well), the proposal step of plans without a single-launch
// instance: one thread per unit c = l W + w (theta's [L][W] order: the state / proposal
// rows [P][L][W] are read and written coalesced), noise and accept draws of the unit's
// own stream (dz_cid), partner indices of the walker, the joint chains' history layout.  The
// arithmetic of dz_stage's per-well branch (bitwise).
// Per-well chains: unit c's history append (append_at) and proposal (demcz_propose_pw_kernel's
// body; also run right after the accept step by demc_accept_propose_pw_kernel)
__device__ __forceinline__ void demcz_propose_pw_unit(const DemczArgs& d, int64_t c) {
    const int64_t W = d.W, U = d.W * d.L;
    const int64_t l = c / W, w = c % W;
    const int P = d.P;
    const uint64_t cid = dz_cid(d.well0, l, d.Wg, d.chain0, w);
    // the joint chains' history layout: entry e of walker w at (e W + w) R, row p L + l
    const size_t entry = (size_t)U * P, base = (size_t)w * P * d.L + l;
    double x[kRoleCount];
    for (int p = 0; p < P; ++p) x[p] = d.x[(int64_t)p * U + c];
    if (d.append_at >= 0)
        for (int p = 0; p < P; ++p) d.hist[(size_t)d.append_at * entry + base + (size_t)p * d.L] = x[p];
    if (!d.propose) return;
    const bool de = d.it > 1;
    int64_t e1 = -1, e2 = -1;
    if (de) {            // partners keyed by the walker (as dz_stage)
        uint64_t iz1, iz2;
        demcz_partners(d.key, (uint64_t)(d.chain0 + w), (uint64_t)d.it, iz1, iz2);
        e1 = d.lo + (int64_t)iz1;
        e2 = d.lo + (int64_t)iz2;
    }
    // an entry appended by this launch is the state itself
    const bool c1 = e1 == d.append_at, c2 = e2 == d.append_at;
    const double lamb = d.lamb[c], sc = d.scaling[c];
    const uint64_t ke = rng_mix(d.key + 2);
    for (int p = 0; p < P; ++p) {
        const double z1 = de ? (c1 ? x[p] : d.hist[(size_t)e1 * entry + base + (size_t)p * d.L]) : 0.0;
        const double z2 = de ? (c2 ? x[p] : d.hist[(size_t)e2 * entry + base + (size_t)p * d.L]) : 0.0;
        const double v = dz_value_e(d, de, x[p], z1, z2, lamb, sc, ke, dz_pw_elem(cid, p), (int64_t)p * d.L + l);
        d.prop[(int64_t)p * U + c] = v;
        if (d.prop_x) d.prop_x[(int64_t)p * U + c] = pymc3_backward(d.tr_kind[p], d.tr_a[p], d.tr_b[p], v);
    }
}
NGRTD_KLINK __global__ void __launch_bounds__(256) demcz_propose_pw_kernel(const DemczArgs d) {
    fm_lds_init();                           // fexp (pymc3_backward)
    __syncthreads();
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c < d.W * d.L) demcz_propose_pw_unit(d, c);
}

// Per-well chains, the accept step after the per-unit log-prob (ngrtd_logp_units): one
// thread per unit c = l W + w decides its own chain and copies its P proposal rows.
__device__ __forceinline__ void demc_accept_pw_unit(const DemcAccept& d, const double* __restrict__ ulp, int64_t W,
                                                    int64_t c) {
    const int64_t U = W * d.L;
    const int64_t l = c / W, w = c % W;
    if (demc_decide(d, c, dz_cid(d.well0, l, d.Wg, d.chain0, w), ulp[c], d.key, d.tune_now, 0)) {
        for (int p = 0; p < d.P; ++p) d.x[(int64_t)p * U + c] = d.prop[(int64_t)p * U + c];
        if (d.xu)
            for (int p = 0; p < d.P; ++p) d.xu[(int64_t)p * U + c] = d.prop_u[(int64_t)p * U + c];
    }
}
NGRTD_KLINK __global__ void __launch_bounds__(256) demc_accept_pw_kernel(const DemcAccept d,
                                                                          const double* __restrict__ ulp, int64_t W) {
    fm_lds_init();                           // flog (demc_logu)
    __syncthreads();
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c < W * d.L) demc_accept_pw_unit(d, ulp, W, c);
}
// Step j's accept and step j + 1's append + proposal in one launch (per-well chains): each
// thread decides its unit, then appends and proposes from the state it just wrote -- a chain
// reads only its own history rows -- so the kernel pair's bits with one launch fewer per step
NGRTD_KLINK __global__ void __launch_bounds__(256) demc_accept_propose_pw_kernel(const DemcAccept da,
                                                                                 const double* __restrict__ ulp,
                                                                                 int64_t W, const DemczArgs d) {
    fm_lds_init();                           // flog (demc_logu), fexp (pymc3_backward)
    __syncthreads();
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= W * da.L) return;
    demc_accept_pw_unit(da, ulp, W, c);
    demcz_propose_pw_unit(d, c);
}

// The multi-step launch's LDS copies of its block's chain state (DemcAccept::state_lds):
// rows [P][512] in the chains' space (unit slot i), per-chain lp / lamb / scaling / tuning
// counter [512] (slot: the unit for per-well chains, the block's walker for joint chains).
// on == false: the state lives in global memory (d.zx, d.lp, d.lamb, ...).
// LDS-qualified pointers (address space 3): held in a struct, plain pointers lose the
// address space and every access became a flat load (which waits behind the vector-memory
// queue, here the partner loads).
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) int32_t lds_i32;
struct DzLds {
    bool on = false;
    lds_f64* st = nullptr;
    lds_f64* lp = nullptr;
    lds_f64* lamb = nullptr;
    lds_f64* sc = nullptr;
    lds_i32* nat = nullptr;
};

// Single-launch DEMetropolisZ step (logp_fused_kernel MIX bit 3), unit (walker w, well l)
// of block column i.  Partner entries of chain w (demcz_partners); e = -1 without DE.
__device__ __forceinline__ void dz_partners(const DemcAccept& d, const DzStep& sj, int64_t w, int64_t& e1,
                                            int64_t& e2) {
    e1 = e2 = -1;
    if (sj.it > 1) {
        uint64_t iz1, iz2;
        demcz_partners(sj.key, (uint64_t)(d.chain0 + w), (uint64_t)sj.it, iz1, iz2);
        e1 = sj.lo + (int64_t)iz1;
        e2 = sj.lo + (int64_t)iz2;
    }
}
// Load the unit's state rows and its two partners' rows (chain-major history: entry e of
// chain w at (e W + w) R, row p L + l), append the state at entry h_at, form the proposal
// and write it -- natural space -- to d.dz_prop [P][L][W], the theta rows the rest of the
// launch reads (the block's own lines, behind the barrier); transformed chains keep the
// chains'-space value in LDS row p of th for dz_commit.  (Reading the natural proposals
// back from an LDS copy instead of d.dz_prop was slower: the extra uniform row indices
// spilled SGPRs into the unit body.)
// PW (per-well chains, DemcAccept::per_well): the unit is the chain -- lamb / scaling
// (walker-major scratch copies [W][L] inside the call), proposal noise and accept draw of
// its own (dz_cid); the partner indices are the walker's, so the history layout and its
// loads are the joint chains' ones.
// sl: the chains' LDS state (DzLds; slot = the chain's per-chain slot) or global (sl.on false).
// The unit's partner rows of step sj, rows q0, q0 + STEP, ... (a1 / a2; zeros without a DE
// term or when !valid): loads only.  The multi-step launch issues step j + 1's rows (every
// row, STEP = 1, from the unit's theta lane) at the end of step j's log-prob body, so that
// their HBM latency passes behind the role exchange, the decision and the commit instead of
// opening step j + 1 (dz_stage_all then reads no partner rows itself).  The entry step j + 1
// appends (sj.at: the state after step j's commit) is not in memory when they are issued;
// dz_stage_all substitutes the state for it, as dz_stage does.  Every other entry was appended
// by this same lane in an earlier step or earlier in this one, so its stores precede these
// loads in the lane's own order.  Every element is assigned, so that nothing stays live
// from before the call (the loop-carried registers would otherwise span the log-prob body).
template <int PMAX, int STEP>
__device__ __forceinline__ void dz_partner_rows(const DemcAccept& d, const DzStep& sj, int64_t w, int l, int L,
                                                int64_t W, bool valid, int q0, double* a1, double* a2) {
    constexpr int KMAX = (PMAX + STEP - 1) / STEP;
    int64_t e1, e2;
    dz_partners(d, sj, w, e1, e2);
    if (d.dz_diag & 16) e1 = e2 = -1;
    const bool de = valid && e1 >= 0;
    const int P = d.P;
    const int64_t R = (int64_t)P * L;
    const double* z1 = d.hist + ((size_t)(de ? e1 : 0) * W + w) * R + l;
    const double* z2 = d.hist + ((size_t)(de ? e2 : 0) * W + w) * R + l;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int p = q0 + STEP * k;
        a1[k] = (de && p < P) ? z1[(int64_t)p * L] : 0.0;
        a2[k] = (de && p < P) ? z2[(int64_t)p * L] : 0.0;
    }
}

// dz_stage with the partner rows prefetched (kDzPrefetch): the lane stages its unit's rows
// q0, q0 + STEP, ... (STEP = 2: each role its parity's rows, as dz_stage; STEP = 1: every
// row) from the prefetched partners pf1 / pf2 (dz_partner_rows<PMAX, STEP>, same rows), row
// by row, the same arithmetic as dz_stage (bitwise); every kernel-argument read before the
// first store (as dz_stage).
template <int PMAX, int STEP, bool TR, bool PW>
__device__ __forceinline__ void dz_stage_all(const DemcAccept& d, const DzStep& sj, int64_t U, int64_t u, int i,
                                             int64_t w, int l, int L, int64_t W, bool valid, double* th, double* pl,
                                             const DzLds& sl, int slot, int q0, const double* pf1, const double* pf2) {
    constexpr int KMAX = (PMAX + STEP - 1) / STEP;
    if (!valid || (d.dz_diag & 8)) return;
    const int P = d.P, dg = d.dz_diag;
    if (dg & 1) {   // timing diagnostics: the proposal is the state (no partners, no noise)
        for (int p = q0; p < P; p += STEP)
            d.dz_prop[(int64_t)p * U + u] = sl.on ? sl.st[p * kFusedUnitsDz + i] : d.zx[(int64_t)p * U + u];
        return;
    }
    const double* const S = d.S;
    const double* const zx = d.zx;
    double* const hist = d.hist;
    double* const prop = d.dz_prop;
    const bool skip_g = d.prop_skip != 0;
    const int64_t Wg = d.Wg, ch0 = d.chain0;
    const uint64_t cid = PW ? dz_cid(d.well0, l, Wg, ch0, w) : 0;
    int64_t e1, e2;
    dz_partners(d, sj, w, e1, e2);
    if (dg & 16) e1 = e2 = -1;
    const bool de = e1 >= 0;
    const int64_t R = (int64_t)P * L;
    const int64_t ci = PW ? w * (int64_t)L + l : w;
    const double lamb = sl.on ? sl.lamb[slot] : d.lamb[ci], sc = sl.on ? sl.sc[slot] : d.scaling[ci];
    const bool c1 = e1 == sj.at, c2 = e2 == sj.at;   // an entry appended in this launch is the state
    const uint64_t ke = rng_mix(sj.key + 2);
    NGRTD_PROBE(14);
    double v[KMAX], vu[TR ? KMAX : 1];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int p = q0 + STEP * k;
        if (p < P) {
            const double x = sl.on ? sl.st[p * kFusedUnitsDz + i] : zx[(int64_t)p * U + u];
            const double sr = S ? S[(int64_t)p * L + l] : 1.0;
            const uint64_t el = PW ? dz_pw_elem(cid, p) : (uint64_t)((int64_t)p * L + l) * (uint64_t)Wg +
                                                          (uint64_t)(ch0 + w);
            double vv = dz_value_core(de, x, c1 ? x : pf1[k], c2 ? x : pf2[k], lamb, sc, ke, el, S != nullptr, sr);
            if (TR) {
                vu[TR ? k : 0] = vv;
#if NGRTD_DZ_TR_BRANCH
                // the row's transform kind is wave-uniform (a kernel argument of a compile-time
                // row): branch on it instead of computing every kind and selecting
                vv = pymc3_backward(d.tr_kind[p], d.tr_a[p], d.tr_b[p], vv);
#else
                vv = pymc3_backward_sel(d.tr_kind[p], d.tr_a[p], d.tr_b[p], vv);
#endif
            }
            v[k] = vv;
        }
    }
    NGRTD_PROBE(15);
    const bool app = sj.at >= 0 && !(dg & 2);
    double* hrow = hist + ((size_t)(sj.at < 0 ? 0 : sj.at) * W + w) * R + l;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int p = q0 + STEP * k;
        if (p < P) {
            if (app) hrow[(int64_t)p * L] = sl.on ? sl.st[p * kFusedUnitsDz + i] : zx[(int64_t)p * U + u];
            if (TR) th[p * kFusedUnitsDz + i] = vu[TR ? k : 0];
            if (!skip_g) prop[(int64_t)p * U + u] = v[k];
            if (pl) pl[p * kFusedUnitsDz + i] = v[k];
        }
    }
}

template <int PMAX, bool TR, bool PW = false>
__device__ __forceinline__ void dz_stage(const DemcAccept& d, const DzStep& sj, int64_t U, int64_t u, int i, int64_t w,
                                         int l, int L, int64_t W, bool valid, double* th, int p0, double* pl,
                                         const DzLds& sl, int slot) {
    if (!valid || (d.dz_diag & 8)) return;
    if (d.dz_diag & 1) {   // timing diagnostics: the proposal is the state (no partners, no noise)
        for (int p = p0; p < d.P; p += 2)
            d.dz_prop[(int64_t)p * U + u] = sl.on ? sl.st[p * kFusedUnitsDz + i] : d.zx[(int64_t)p * U + u];
        return;
    }
    // every field of d into a local before the first store: d is read through an opaque
    // kernarg pointer that a store may alias, so a field read after a store is re-loaded and
    // waited for; the role's row parity made wave-uniform so that the per-row kernarg reads
    // (transform kinds and bounds) stay scalar
    const int P = d.P, dg = d.dz_diag;
    const bool skip_g = d.prop_skip != 0;
    const int q0 = __builtin_amdgcn_readfirstlane(p0);
    const double* const S = d.S;
    const double* const zx = d.zx;
    double* const hist = d.hist;
    double* const prop = d.dz_prop;
    const int64_t Wg = d.Wg, ch0 = d.chain0;
    const uint64_t cid = PW ? dz_cid(d.well0, l, Wg, ch0, w) : 0;
    // partner entries: keyed by the walker (chain0 + w) for joint and per-well chains alike --
    // the wells of one walker draw the same history indices (each from its own history), so
    // a wave (one walker's wells) reads two contiguous entries, as the joint chains do
    int64_t e1, e2;
    dz_partners(d, sj, w, e1, e2);
    if (dg & 16) e1 = e2 = -1;   // timing diagnostics: no partner loads (noise only)
    const bool de = e1 >= 0;
    constexpr int KMAX = (PMAX + 1) / 2;
    double x[KMAX], a1[KMAX], a2[KMAX], sr[KMAX], ta[KMAX], tb[KMAX];
    int tk[KMAX];
    // row p of entry e at (e W + w) R + p L + l (R = P L), per-well chains too: a wave (one
    // walker's wells) reads 512-B runs of the walker's two partner entries
    const int64_t R = (int64_t)P * L;
    const double* z1 = hist + ((size_t)(de ? e1 : 0) * W + w) * R + l;
    const double* z2 = hist + ((size_t)(de ? e2 : 0) * W + w) * R + l;
    const int64_t ci = PW ? w * (int64_t)L + l : w;   // per-chain arrays: walker-major [W][L] / [W]
    const double lamb = sl.on ? sl.lamb[slot] : d.lamb[ci], sc = sl.on ? sl.sc[slot] : d.scaling[ci];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {   // every load first
        const int p = q0 + 2 * k;
        if (p < P) {
            x[k] = sl.on ? sl.st[p * kFusedUnitsDz + i] : zx[(int64_t)p * U + u];
            a1[k] = de ? z1[(int64_t)p * L] : 0.0;
            a2[k] = de ? z2[(int64_t)p * L] : 0.0;
            sr[k] = S ? S[(int64_t)p * L + l] : 1.0;
            if (TR) {
                tk[k] = d.tr_kind[p];
                ta[k] = d.tr_a[p];
                tb[k] = d.tr_b[p];
            }
        }
    }
    // an entry appended in this launch is the state itself (as demcz_propose_kernel)
    const bool c1 = e1 == sj.at, c2 = e2 == sj.at;
    double* hrow = hist + ((size_t)(sj.at < 0 ? 0 : sj.at) * W + w) * R + l;
    const uint64_t ke = rng_mix(sj.key + 2);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int p = q0 + 2 * k;
        if (p < P) {
            if (sj.at >= 0 && !(dg & 2)) hrow[(int64_t)p * L] = x[k];
            const uint64_t el = PW ? dz_pw_elem(cid, p) : (uint64_t)((int64_t)p * L + l) * (uint64_t)Wg +
                                                          (uint64_t)(ch0 + w);
            double v = dz_value_core(de, x[k], c1 ? x[k] : a1[k], c2 ? x[k] : a2[k], lamb, sc, ke, el, S != nullptr,
                                     sr[k]);
            // transformed chains: the natural-space value the log-prob reads (and v itself,
            // the chains'-space value, for dz_commit)
            if (TR) {
                th[p * kFusedUnitsDz + i] = v;
                v = pymc3_backward_sel(tk[k], ta[k], tb[k], v);
            }
            if (!skip_g) prop[(int64_t)p * U + u] = v;
            if (pl) pl[p * kFusedUnitsDz + i] = v;
        }
    }
}
// An accepted unit takes the proposal: natural rows from d.dz_prop (written by this lane
// role before the barriers), transformed chains also the chains'-space value that
// dz_stage kept in LDS (row p of th).  LDS state (sl.on): only the chains'-space rows, in LDS
// (the natural rows are re-derived from them when the launch writes its state back).
template <int PMAX, bool TR>
__device__ __forceinline__ void dz_commit(const DemcAccept& d, int64_t U, int64_t u, int i, const double* th,
                                          int p0, const double* pl, const DzLds& sl) {
    constexpr int KMAX = (PMAX + 1) / 2;
    if (sl.on) {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int p = p0 + 2 * k;
            if (p < d.P)
                sl.st[p * kFusedUnitsDz + i] = TR ? th[p * kFusedUnitsDz + i]
                                                  : (pl ? pl[p * kFusedUnitsDz + i] : d.dz_prop[(int64_t)p * U + u]);
        }
        return;
    }
    double pv[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {   // every load first, then every store
        const int p = p0 + 2 * k;
        if (p < d.P) pv[k] = pl ? pl[p * kFusedUnitsDz + i] : d.dz_prop[(int64_t)p * U + u];
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int p = p0 + 2 * k;
        if (p < d.P) {
            const int64_t gi = (int64_t)p * U + u;
            d.x[gi] = pv[k];
            if (TR) d.xu[gi] = th[p * kFusedUnitsDz + i];
        }
    }
}

// STEP: a multi-step DEMetropolisZ launch (the step's schedule sj and log offset), else the
// launch's own DemcAccept fields
// sl.on: the chain's state in the launch's LDS copies at slot (the block's walker w - w0).
template <bool STEP>
__device__ __forceinline__ void walker_out(double* logp, const DemcAccept& d, const DzStep& sj, int64_t log_off,
                                           int64_t w, double tot, int* dec, const DzLds& sl = DzLds{},
                                           int slot = 0) {
    if (logp) logp[w] = tot;
    if (!d.lp) return;
    if (STEP && sl.on)
        *dec = demc_decide_at(d, sl.lp, sl.lamb, sl.sc, sl.nat, nullptr, false, slot, (uint64_t)(d.chain0 + w), tot,
                              sj.key, sj.tune_now, log_off, w, true);
    else
        *dec = STEP ? demc_decide(d, w, tot, sj.key, sj.tune_now, log_off) : demc_decide(d, w, tot);
}

// Exact (matrix-core) channel sums for a wave of logp_fused_kernel with an uncovered tau:
// its 64 units as 4 tiles of 16, then the concentrations and RTD likelihood of the lanes
// that need them (mine = valid and uncovered): a covered lane keeps its surrogate result, so
// no lane's value depends on which units share its wave.
template <int C, bool FULL, bool SEQ, int MIX>
__device__ __forceinline__ void fused_exact(const RtdArgs& a, const UnitArgs& ul, int WB, int64_t w0, int uw,
                                            bool mine, int64_t mu, int ml, double nub, double* conc,
                                            double& like, LwDecay lw = LwDecay{0.0, 0.0}, const WdView* wv = nullptr) {
    constexpr bool LW = (MIX & 32) != 0;
    constexpr int NT = mfma_tiles(C);
    const int col = threadIdx.x & 15;
    const int L = ul.L;
    const int64_t W = ul.W;
    int64_t uoff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int i = (uw * NT + t) * 16 + col;
        if (MIX & 8) {   // DZ: walker-major units and theta (logp_fused_kernel)
            const int wl = i / L, l = i % L;
            uoff[t] = (wl < WB && w0 + wl < W) ? (w0 + wl) * (int64_t)L + l : 0;
        } else {
            const int wl = i % WB, l = i / WB;
            uoff[t] = (l < L && w0 + wl < W) ? (int64_t)l * W + w0 + wl : 0;
        }
    }
    double yy[C], bu;
    if (SEQ) {   // one 16-unit tile per pass: 1/NT of the accumulators live
        const int tq = (threadIdx.x & 63) >> 4;
        bu = 0.0;
#pragma unroll 1
        for (int t = 0; t < NT; ++t) {
            MfmaWave<C, 1> mw;
            mw.init(a, uoff + t);
            mw.steps(a.frag, a.nsteps);
            double y[1][C];
            mw.finish(a, y);
            if (t == tq) {
                bu = mw.beta[0];
#pragma unroll
                for (int c = 0; c < C; ++c) yy[c] = y[0][c];
            }
        }
    } else {
        MfmaWave<C> mw;
        mw.init(a, uoff);
        mw.steps(a.frag, a.nsteps);
        double y[NT][C];
        mw.finish(a, y);
        mfma_pick_tile<C>(y, mw.beta, yy, bu);   // tile tq holds this lane's unit
    }
    // LW: channel 0's exact sum at each unit's tau_eff (a second pass, one tile at a time:
    // lanes 16 t .. 16 t + 15 hold tile t's units)
    double yw = 0.0, bw = 0.0;
    if (LW) {
        const int tq = (threadIdx.x & 63) >> 4;
#pragma unroll 1
        for (int t = 0; t < NT; ++t) {
            const double tv = __shfl(lw.teff, 16 * t + col, 64);
            MfmaWave<C, 1> mw;
            mw.init_tau(&tv);
            mw.steps(a.frag, a.nsteps);
            double y[1][C];
            mw.finish(a, y);
            if (t == tq) {
                yw = y[0][0];
                bw = mw.beta[0];
            }
        }
    }
    if (mine) {
        ThetaPre tp;
        tp.nub = nub;
        double num2[C];
        if (MIX & 1) piston_num<C, LW>(a, mu, num2, lw.lam);
        mfma_unit_conc<C, LW>(a, mu, bu, yy, conc, (MIX & 1) ? num2 : nullptr, lw.lam, yw, bw);
        like = unit_like_rtd<C>(ul, mu, ml, conc, &tp, FULL, nullptr, wv);
    }
}

// The EPM channel table in LDS: blocks of kEpmBlock rows of CP doubles, each block padded by
// 2 doubles.  Every head-loop iteration reads row r of its OWN block in every lane, so with
// unpadded blocks (16 CP doubles = a multiple of 64 banks apart) all lanes hit the same banks;
// the pad rotates consecutive blocks by 4 banks, so the 16 lanes of a ds_read_b128 group
// spread over all 64 banks unless their blocks coincide modulo 16.
__host__ __device__ constexpr int epm_blk_stride(int CP) { return kEpmBlock * CP + 2; }
__host__ __device__ constexpr int epm_lds_doubles(int N, int CP) {
    return (N + kEpmBlock - 1) / kEpmBlock * epm_blk_stride(CP);
}
__device__ __forceinline__ int epm_row(int k, int CP) { return (k / kEpmBlock) * epm_blk_stride(CP) + (k % kEpmBlock) * CP; }
// One table row's C channels: CP / 2 16-B loads (rows are 16-B aligned: CP even, stride even).
template <int C>
__device__ __forceinline__ void epm_row_load(const double* row, double* v) {
    constexpr int CP = cheb_cp(C);
    const double2* r2 = reinterpret_cast<const double2*>(row);
#pragma unroll
    for (int i = 0; i < CP / 2; ++i) {
        const double2 t = r2[i];
        if (2 * i < C) v[2 * i] = t.x;
        if (2 * i + 1 < C) v[2 * i + 1] = t.y;
    }
}

// The block-tail surrogate of one piece: C channels of kChebN coefficients each, channel-major
// (C kChebN doubles, 16-B aligned): channel c's monomial coefficients at [c kChebN, (c + 1) kChebN),
// read as 16-B chunks, each channel's top chunk first as its Horner consumes them.  (Channel-major
// so that the sampled half-life's channel-0 column at its own piece, LW, is one contiguous run of
// kChebN doubles instead of kChebN loads at stride C.)
// The first kEpmTailPre chunks Horner reads, loaded ahead by the caller -- before the head
// loop, so that their L2 latency passes behind it.
#ifndef NGRTD_EPM_TAIL_PRE
#define NGRTD_EPM_TAIL_PRE 5
#endif
constexpr int kEpmTailPre = NGRTD_EPM_TAIL_PRE;
// the DEMetropolisZ instances carry the step's state in registers too: fewer chunks ahead
#ifndef NGRTD_EPM_TAIL_PRE_DZ
#define NGRTD_EPM_TAIL_PRE_DZ 4
#endif
constexpr int kEpmTailPreDz = NGRTD_EPM_TAIL_PRE_DZ;
// the LW instances (the sampled CFC12 half-life): channel 0's own tail column (kChebN doubles)
// is loaded ahead too (kEpmLwPre), in place of some of the shared tail's chunks
#ifndef NGRTD_EPM_TAIL_PRE_LW
#define NGRTD_EPM_TAIL_PRE_LW 4
#endif
constexpr int kEpmTailPreLw = NGRTD_EPM_TAIL_PRE_LW;
#ifndef NGRTD_EPM_LW_PRE
#define NGRTD_EPM_LW_PRE 1
#endif
constexpr bool kEpmLwPre = NGRTD_EPM_LW_PRE != 0;
// Two piece formats, chosen per plan (ngrtd.hip epm_prepare) and per kernel instance (MX):
//  * MX = false (plans without the sampled half-life): C runs of kChebN doubles, channel-major;
//  * MX = true (plans with it, the LW instances): mixed precision -- a channel's monomial
//    coefficients k < kEpmK64 are doubles, the top kEpmK32 = kChebN - kEpmK64 are floats.  Over
//    the pieces [a, 1.25 a] |m_k| <= 2.3e-9 |f| from k = 8 on (checked over the tracer series
//    and blocks), so their float rounding adds < 2e-16 relative -- and every plan's table is
//    validated with this very evaluation (epm_tail_eval1) at kChebTol.  A piece: [C][kEpmK64]
//    doubles, then [C][kEpmK32] floats (one 16-B chunk per channel): 400 B at C = 5 instead of
//    480.  The LW instances read two pieces per unit (the shared tail and channel 0's at
//    tau'_w): 17.6 vs 18.3 us per c4 launch (profiles/r05af_epm_mixed_tail_ab.txt).
constexpr int kEpmK64 = 8, kEpmK32 = kChebN - kEpmK64;
// Every plan -- with or without the sampled half-life -- takes the mixed pieces since the
// prefetch depth of the plain instances went to one channel's chunks (5): 16.4 vs 17.0 us per
// c4 exp_pist_flow launch (profiles/r05aj_epm_mixed_all_ab.txt).  The format is compiled into
// the instances, so a plan whose mixed table fails the kChebTol validation has no all-double
// table to fall back to: it runs without block-tail surrogates (the multi-kernel path), and
// ngrtd_plan_info reports it (info[11] = 0 for an exp_pist_flow plan; epm_prepare logs it with
// NGRTD_VERBOSE=1).  NGRTD_EPM_MIXED_ALL=0 builds the all-double pieces for the plans without
// the sampled half-life (A/B).
#ifndef NGRTD_EPM_MIXED_ALL
#define NGRTD_EPM_MIXED_ALL 1
#endif
constexpr bool kEpmMixedAll = NGRTD_EPM_MIXED_ALL != 0;
static_assert(kEpmK64 % 2 == 0 && kEpmK32 == 4, "per channel: kEpmK64 / 2 double2 chunks + one float4 chunk");
__host__ __device__ constexpr int epm_piece_doubles(int C, bool mx) { return mx ? C * (kEpmK64 + kEpmK32 / 2) : C * kChebN; }
// the 16-B chunks of a channel, in the order Horner consumes them: MX, its float4 (the top
// coefficients) then its double2 chunks top-down; else its double2 chunks top-down
__host__ __device__ constexpr int epm_chunks_per_chan(bool mx) { return mx ? kEpmK64 / 2 + 1 : kChebN / 2; }
__host__ __device__ constexpr int epm_tail_pre_n(int C, int want, bool mx) {
    return want < epm_chunks_per_chan(mx) * C ? want : epm_chunks_per_chan(mx) * C;
}
// double2 index of load position q (channel c = q / chunks-per-channel, s = q % it)
template <int C, bool MX>
__host__ __device__ constexpr int epm_tail_chunk(int q) {
    constexpr int NCH = epm_chunks_per_chan(MX);
    return MX ? ((q % NCH == 0) ? (kEpmK64 / 2) * C + q / NCH : (q / NCH) * (kEpmK64 / 2) + (kEpmK64 / 2 - q % NCH))
              : (q / NCH) * NCH + (NCH - 1 - q % NCH);
}
// channel c's tail at local x, the one evaluation every consumer uses (the device fast path
// below: the same FMAs in the same order; the host validation of every plan's table)
__host__ __device__ __forceinline__ double epm_tail_eval1(const double* pt, int C, int c, double x, bool mx) {
    if (!mx) {
        const double* d = pt + kChebN * c;
        double acc = d[kChebN - 1];
        for (int k = kChebN - 2; k >= 0; --k) acc = fma(acc, x, d[k]);
        return acc;
    }
    const float* f = reinterpret_cast<const float*>(pt + kEpmK64 * C) + kEpmK32 * c;
    const double* d = pt + kEpmK64 * c;
    double acc = (double)f[kEpmK32 - 1];
    for (int k = kEpmK32 - 2; k >= 0; --k) acc = fma(acc, x, (double)f[k]);
    for (int k = kEpmK64 - 1; k >= 0; --k) acc = fma(acc, x, d[k]);
    return acc;
}
template <int C, int NPW, bool MX>
__device__ __forceinline__ void epm_tail_pre(const double* pt, bool on, double2* pre) {
    constexpr int NP = epm_tail_pre_n(C, NPW, MX);
    const double2* p2 = reinterpret_cast<const double2*>(pt);
#pragma unroll
    for (int q = 0; q < NP; ++q) pre[q] = on ? p2[epm_tail_chunk<C, MX>(q)] : double2{0.0, 0.0};
}
// a float4 chunk held in a double2 register pair -> its four floats as doubles
// (register moves only: a memcpy through a local float[4] put it in scratch)
__device__ __forceinline__ void epm_f4(const double2& t, double* v) {
    const unsigned long long a = (unsigned long long)__double_as_longlong(t.x);
    const unsigned long long b = (unsigned long long)__double_as_longlong(t.y);
    v[0] = (double)__uint_as_float((unsigned)a);          // little-endian: floats 0, 1 in t.x
    v[1] = (double)__uint_as_float((unsigned)(a >> 32));
    v[2] = (double)__uint_as_float((unsigned)b);
    v[3] = (double)__uint_as_float((unsigned)(b >> 32));
}
// y_c = sum_k m_{c,k} x^k by Horner from the top coefficient: epm_tail_eval1's FMAs in its order
template <int C, int NPW, bool MX>
__device__ __forceinline__ void epm_tail_sums(const double* pt, double x, double* y, const double2* pre) {
    constexpr int NP = epm_tail_pre_n(C, NPW, MX), NCH = epm_chunks_per_chan(MX);
    const double2* p2 = reinterpret_cast<const double2*>(pt);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        double acc = 0.0;
        if (MX) {
            double hi[kEpmK32];
            epm_f4((c * NCH < NP) ? pre[c * NCH] : p2[epm_tail_chunk<C, MX>(c * NCH)], hi);
            acc = hi[kEpmK32 - 1];
#pragma unroll
            for (int k = kEpmK32 - 2; k >= 0; --k) acc = fma(acc, x, hi[k]);
        }
#pragma unroll
        for (int s = MX ? 1 : 0; s < NCH; ++s) {            // double2 chunks, top-down
            const int q = c * NCH + s;
            const double2 t = (q < NP) ? pre[q] : p2[epm_tail_chunk<C, MX>(q)];
            acc = (!MX && s == 0) ? t.y : fma(acc, x, t.y);
            acc = fma(acc, x, t.x);
        }
        y[c] = acc;
    }
}

// exp_pist_flow channel sums of one unit (numerators num_c and normaliser den = dn / dd, as
// rtd_conc_kernel's EPM finalise: conc = (A + J B) / den):
//   f = first unmasked age (epm_first, the exact mask of :189), m = max(f, 1),
//   Y_c = sum_{k >= m} A_{c,k} q^(k - m), q = exp(-beta), beta = eta / tau
//       = head (ages [m, min(B, N)), Horner over the LDS table, B = (m / S + 1) S)
//         + q^(B - m) T_{B/S}(1 / beta)        (block-tail surrogate, validated per plan)
//   f >= 1: num = Y, den = G = sum_{j < N - m} q^j;  f = 0: num = A_0 + s01 Y, den = 1 + s01 G,
//   den returned as dn / dd (dd = e^(-beta) - 1) for the caller's batched reciprocal.
// Lanes whose tau' = 1 / beta the surrogate does not cover (or NaN) sum their tail exactly;
// the loop is wave-uniform and runs only when some lane needs it.
// LW (the sampled CFC12 half-life, channel 0 undecayed in the table; see lw_decay): channel
// 0's weights are e^(-sigma (k - m)), sigma = beta + lam, so its head runs its own weight
// chain, its tail is the same block-tail function at tau'_w = 1 / sigma (a second piece), and
// its numerator carries e^(-lam tp_m) (m >= 1) or e^(-lam tp_0) (f = 0).  thx: the unit's
// thalf_cfc Beta value; *lam_out: its decay constant (the piston component needs it).
// *nan_out: the reference's normalised weights are NaN as a whole for this unit (epm_sums below).
template <int C, int NPW = kEpmTailPre, bool LW = false>
__device__ __forceinline__ void epm_sums(const RtdArgs& a, const double* tabl, bool mvalid, double tau, double eta,
                                         double* num, double& dn, double& dd, double thx = 0.0,
                                         double* lam_out = nullptr, bool* nan_out = nullptr) {
    constexpr int CP = cheb_cp(C), S = kEpmBlock;
    const int N = a.N;
    const double beta = eta / tau;
    const double ie = 1 / eta;                          // the mask's 1/eta (:189), also tau' = tau / eta
    const int f = epm_first(tau * (1 - ie), a.tp0, a.dtp, N);
    // The reference's weights (eta/tau) e^(-eta tp/tau + eta - 1) over the unmasked ages give NaN
    // concentrations as a whole (0 / 0 or inf / inf after g /= g.sum(), :270) when every age is
    // masked, and when the weights are 0, inf or NaN at both ends of the unmasked range (they are
    // monotone in tp): tau or eta 0, inf or NaN, or the largest weight under- / overflowing.
    // The sums below work relative to the first unmasked weight and stay finite there, so the
    // predicate is evaluated exactly -- in waves holding a lane near those cases only.
    if (nan_out) {
        const double tpf = f == 0 ? a.tp0 : (double)f + a.dtp;
        // (the screen without a division; the check itself in the reference's operation order)
        const bool susp = f >= N || !(beta > 0.0 && beta <= 1.7976931348623157e308) || !(fma(-beta, tpf, eta - 1) > -700.0);
        bool wn = false;
        if (__any(susp) && susp) {
            const double xf = -(eta * tpf / tau) + eta - 1;
            const double tpl = N > 1 ? (double)(N - 1) + a.dtp : a.tp0;
            const double xl = -(eta * tpl / tau) + eta - 1;
            const double ce = eta / tau;
            const double w0 = ce * fexp(xf), w1 = ce * fexp(xl);
            wn = f >= N || !(fabs(w0) <= 1.7976931348623157e308) || !(fabs(w1) <= 1.7976931348623157e308) ||
                 (w0 == 0.0 && w1 == 0.0);
        }
        *nan_out = wn;
    }
    const int m = f > 1 ? f : 1;
    const int blk = m / S + 1, B = blk * S;
    const double q = fexp(-beta);
    // the staged rows [0, Nst); a windowed table (a.ew_on, ngrtd.hip epm_window) holds the rows of
    // every unit inside the priors' support box, and the units outside it (log-prob -inf by their
    // priors; NaN where nan_out says so) read no row past it: no exact tails, zero sums
    const int Nst = a.epm_nw < N ? a.epm_nw : N;
    const bool outw = a.ew_on && !(tau >= a.ew_tau_lo && tau <= a.ew_tau_hi && eta >= a.ew_eta_lo &&
                                   eta <= a.ew_eta_hi && (!LW || (thx >= 0.0 && thx <= 1.0)));
    // the block tail's surrogate piece first: its top chunks are loaded before the head loop
    const bool tail = B < N;
    double ex = 0.0;
    const double taup = tau * ie;
    int pc = (tail && a.epm) ? epm_piece(taup, ex) - a.epm_p0 : -1;
    pc = (unsigned)pc < (unsigned)a.epm_np ? pc : -1;
    double lam = 0.0, qw = 0.0, taupw = 0.0, exw = 0.0;
    int pcw = -1;
    if (LW) {   // t_half -> lam and tau'_w = 1 / (eta / tau + lam) = tau t / (eta t + ln2 tau): one division
        const double th = a.thalf_a * thx + a.thalf_b;
        const double dl[2] = {th, eta * th + kLn2Ref * tau};
        double rl[2];
        batch_recip<2>(dl, rl);
        lam = kLn2Ref * rl[0];
        taupw = (tau * th) * rl[1];
        qw = fexp(-(beta + lam));
        pcw = (tail && a.epm) ? epm_piece(taupw, exw) - a.epm_p0 : -1;
        pcw = (unsigned)pcw < (unsigned)a.epm_np ? pcw : -1;
        if (lam_out) *lam_out = lam;
    }
    const bool tail_on = tail && !(a.epm_diag & 2);
    const int bt = (tail_on ? (blk < a.epm_nb ? blk : a.epm_nb) : 1) - 1;   // (a windowed table's blocks: clamped)
    const double* pt = a.epm + ((size_t)bt * a.epm_np + (pc < 0 ? 0 : pc)) * (size_t)epm_piece_doubles(C, LW || kEpmMixedAll);
    constexpr bool MX = LW || kEpmMixedAll;             // the plan's piece format (epm_prepare)
    double2 tpre[epm_tail_pre_n(C, NPW, MX) > 0 ? epm_tail_pre_n(C, NPW, MX) : 1];
    epm_tail_pre<C, NPW, MX>(pt, tail_on, tpre);
    // LW: channel 0's tail coefficients at tau'_w (column 0 of its own piece, L2), loaded
    // before the head loop as well (kEpmLwPre)
    double twp[LW ? kChebN : 1];
    if (LW && kEpmLwPre) {
        const double* pw = a.epm + ((size_t)bt * a.epm_np + (pcw < 0 ? 0 : pcw)) * (size_t)epm_piece_doubles(C, LW || kEpmMixedAll);
#pragma unroll
        for (int k = 0; k < kEpmK64 / 2; ++k) {   // channel 0: its double run and its float4
            const double2 t = tail_on ? reinterpret_cast<const double2*>(pw)[k] : double2{0.0, 0.0};
            twp[2 * k] = t.x;
            twp[2 * k + 1] = t.y;
        }
        epm_f4(tail_on ? reinterpret_cast<const double2*>(pw)[(kEpmK64 / 2) * C] : double2{0.0, 0.0}, twp + kEpmK64);
    }
    double y[C];
#pragma unroll
    for (int c = 0; c < C; ++c) y[c] = 0.0;
    // head: the S rows of m's block [B - S, B), bottom-up with the weight w = q^(k - m) for
    // k >= m and 0 below (rows past N are zeros in LDS): one select per row instead of one
    // per channel, and the rows at fixed offsets from the block's base (no per-row index
    // arithmetic).  Lanes with q > 1 or NaN (beta < 0: tau or eta outside every prior) take
    // the top-down predicated Horner instead, whose inf / NaN results the reference's
    // overflowing weights give (w = inf times a zero row would be NaN); it runs only in
    // waves holding such a lane and replaces only those lanes' sums, so every lane's result
    // is its own whatever its wave-mates are (the multi-step sampler's walker-major waves
    // and the log-prob kernel's well-major waves give the same bits).
    double qB = -1.0, qBw = -1.0;                       // q^(B - m) from the head's weights (fast path)
    if (!(a.epm_diag & 1)) {
        const bool qok = q <= 1.0 && (!LW || qw <= 1.0);
        // m >= N (every age masked: tau (1 - 1/eta) beyond the series, the reference's g is 0 / 0):
        // m's block is past the staged table, so read the last staged block, where k < m for every
        // row and every weight stays 0 (then y = 0, G = 0: NaN concentrations, as the reference's)
        const int hb0 = B - S < (Nst - 1) / S * S ? B - S : (Nst - 1) / S * S;
        const double* hb = tabl + epm_row(hb0, CP);
        double w = 0.0, w2 = 0.0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const int k = hb0 + i;
            w = k == m ? 1.0 : w * q;
            if (LW) w2 = k == m ? 1.0 : w2 * qw;     // channel 0's own weights (LW)
            double rv[C];
            epm_row_load<C>(hb + i * CP, rv);
#pragma unroll
            for (int c = 0; c < C; ++c) y[c] = fma(rv[c], (LW && c == 0) ? w2 : w, y[c]);
        }
        qB = qok ? w * q : -1.0;                        // w = q^(B - 1 - m) after the last row
        if (LW) qBw = qok ? w2 * qw : -1.0;
        if (__any(!qok)) {
            const int kt = (B < Nst ? B : Nst) - 1;
            double yt[C];
#pragma unroll
            for (int c = 0; c < C; ++c) yt[c] = 0.0;
#pragma unroll 4
            for (int i = 0; i < S; ++i) {
                const int k = kt - i;
                const bool on = !qok && k >= m && !outw;
                double rv[C];
                epm_row_load<C>(tabl + epm_row(on ? k : 0, CP), rv);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const double t = fma(yt[c], (LW && c == 0) ? qw : q, rv[c]);
                    yt[c] = on ? t : yt[c];
                }
            }
#pragma unroll
            for (int c = 0; c < C; ++c) y[c] = qok ? y[c] : yt[c];
        }
    }
    const bool bad = mvalid && tail && !outw && (pc < 0 || (LW && pcw < 0));
    double tl[C];
#pragma unroll
    for (int c = 0; c < C; ++c) tl[c] = 0.0;
    if (tail_on) epm_tail_sums<C, NPW, MX>(pt, ex, tl, tpre);
    if (LW && tail_on) {   // channel 0's tail at tau'_w: column 0 of its own piece (L2)
        const double* pw = a.epm + ((size_t)bt * a.epm_np + (pcw < 0 ? 0 : pcw)) * (size_t)epm_piece_doubles(C, LW || kEpmMixedAll);
        double v;
        if (kEpmLwPre) {   // epm_tail_eval1(pw, C, 0, exw, true) over the prefetched coefficients
            v = twp[kChebN - 1];
#pragma unroll
            for (int k = kChebN - 2; k >= 0; --k) v = fma(v, exw, twp[k]);
        } else {
            v = epm_tail_eval1(pw, C, 0, exw, true);
        }
        tl[0] = v;
    }
    if (__any(bad) && !(a.epm_diag & 4)) {              // exact tails of the uncovered lanes
        // tau' below the table (q < e^-16): the tail's terms fall below 1e-400 of its first
        // after 64 ages, so it is summed over [B, B + 64) only -- 64 iterations over each lane's own
        // LDS rows, whatever the spread of B across the wave; other uncovered tau' (NaN,
        // <= 0, beyond the table) over the whole series, the wave's union of those ranges.
        // Both are the same top-down Horner as before per lane (same bits).  LW: channel 0
        // with its own q (qw); short only when both tau' and tau'_w are below the table.
        constexpr double kEpmTauLo = 1.0 / (double)(1 << -kEpmOct0);
        const bool shortq = taup > 0.0 && taup < kEpmTauLo && (!LW || (taupw > 0.0 && taupw < kEpmTauLo));
        const bool sb = bad && shortq, lb = bad && !shortq;
        double te[C];
#pragma unroll
        for (int c = 0; c < C; ++c) te[c] = 0.0;
        if (__any(sb)) {
#pragma unroll 8
            for (int j = 63; j >= 0; --j) {
                const int k = B + j;
                const bool on = sb && k <= Nst - 1;
                double rv[C];
                epm_row_load<C>(tabl + epm_row(on ? k : 0, CP), rv);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const double t = fma(te[c], (LW && c == 0) ? qw : q, rv[c]);
                    te[c] = on ? t : te[c];
                }
            }
        }
        if (__any(lb)) {
            int bmin = lb ? B : N, kmax = lb ? Nst - 1 : -1;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const int o = __shfl_xor(bmin, off, 64), o2 = __shfl_xor(kmax, off, 64);
                bmin = o < bmin ? o : bmin;
                kmax = o2 > kmax ? o2 : kmax;
            }
#pragma unroll 8
            for (int k = kmax; k >= bmin; --k) {
                const bool on = lb && k >= B;
                double rv[C];
                epm_row_load<C>(tabl + epm_row(k, CP), rv);
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const double t = fma(te[c], (LW && c == 0) ? qw : q, rv[c]);
                    te[c] = on ? t : te[c];
                }
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) tl[c] = bad ? te[c] : tl[c];
    }
    if (tail) {
        if (qB < 0.0) qB = fexp(-beta * (double)(B - m));
        if (LW && qBw < 0.0) qBw = fexp(-(beta + lam) * (double)(B - m));
#pragma unroll
        for (int c = 0; c < C; ++c) y[c] = fma((LW && c == 0) ? qBw : qB, tl[c], y[c]);
    }
    // the normaliser as a fraction den = dn / dd (the caller's one batched reciprocal
    // takes 1 / dn): G = (e^(-beta n) - 1) / (e^(-beta) - 1) over the n = N - m unmasked ages
    const int n = N - m;
    const double e1 = n > 0 ? fexpm1(-beta * (double)n) : 0.0, e2 = n > 0 ? fexpm1(-beta) : 1.0;
    if (f == 0) {
        const double d01 = (1.0 + a.dtp) - a.tp0;
        const double s01 = fexp(-beta * d01);
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = a.tab0[c] + s01 * y[c];
        if (LW) num[0] = fexp(-lam * a.tp0) * (a.tab0[0] + fexp(-(beta + lam) * d01) * y[0]);
        dn = fma(s01, e1, e2);                          // (1 + s01 G) e2
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = y[c];
        if (LW) num[0] = fexp(-lam * ((double)m + a.dtp)) * y[0];   // e^(-lam tp_m) Y_w
        dn = e1;                                        // G e2
    }
    dd = e2;
    if (outw) {                                         // outside the window: finite zeros (see above)
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = 0.0;
        dn = 1.0;
        dd = 1.0;
    }
}

// The piston component's channel-table row ix of an exp_pist_flow plan (BMM exp_pist_flow-piston):
// from the LDS table when staged there, else (a windowed table, ix past its rows) from the global
// table -- the same values.
template <int C>
__device__ __forceinline__ void epm_piston_row(const RtdArgs& a, const double* tabl, int ix, double* v) {
    constexpr int CP = cheb_cp(C);
    if (ix < a.epm_nw) {
        epm_row_load<C>(tabl + epm_row(ix, CP), v);
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = a.tab[(int64_t)ix * a.CP + c];
    }
}

// ------------------------------------------------------ generic components (MIX bit 6)
// The single-launch kernel's generic instances serve every model pair of run_age_mcmc.py:61-70
// that has no specialised instance: first component piston / exponential / exp_pist_flow /
// dispersion, second none or any of the four (convolution_integral_utils.py:178-196 per
// component, the mix of run_age_mcmc_utils.py:96-154).  Per component and lane:
//   piston         the channel-table row at the first argmin |tp - tau| (a lookup);
//   exponential    the surrogate (cheb_sums) when tau (and tau_eff, LW) lie in the staged
//                  window, else gen_exact -- or, with the priors on and tau outside its Uniform
//                  prior's support, no sums at all (the log-prob is -inf) but exp_rtd_nan;
//   exp_pist_flow  epm_sums (head Horner + block-tail surrogate, exact tails where uncovered);
//   dispersion     gen_exact.
//
// Exact channel sums of one component over all N ages, for the lanes with `on` (the age loop is
// wave-uniform: all lanes read the same table row), with the reference's weights
//   exponential    w = (1/tau) e^(-tp/tau)                                         (:184)
//   exp_pist_flow  w = (eta/tau) e^(-eta tp/tau + eta - 1) where tp >= tau (1 - 1/eta), else 0
//   dispersion     w = (1/tau) / sqrt(4 pi D x) (1/x) e^(-(1-x)^2 / (4 D x)),  x = tp/tau
//                    = sqrt(tau / (4 pi D)) tp^(-3/2) e^(-(1-x)^2 (tau/tp) / (4 D))
//                  with 1/tp_k and tp_k^(-3/2) from a.disp_aux (no division, sqrt or power per age)
// num_c = sum_k A_{c,k} w_k (the per-unit decayed channel, LW: w_k e^(-lam tp_k)), den = sum_k w_k,
// so conc = num / den is the normalised g (:270) dotted with the series (:336-340).  Zero, inf and
// NaN weights give the reference's NaN / inf concentrations (0 / 0, inf / inf).
//
// Dispersion plans stage the channel table (epm_row layout) and disp_aux in LDS (tl, dl non-null):
// the dispersion loop then reads its per-age operands from LDS, unrolled by 4 so that four ages'
// reads are in flight at once (the global loads of the generic loop waited once per age: ~530 us
// per c4 launch).  Same expressions in the same order: the same bits as the generic loop.
#ifndef NGRTD_GEN_DISP_UNROLL
#define NGRTD_GEN_DISP_UNROLL 4
#endif
constexpr int kGenDispUnroll = NGRTD_GEN_DISP_UNROLL;
// LW: age groups between two exact decay anchors in the dispersion loop (8 x 4 = 32 ages)
#ifndef NGRTD_DISP_DECAY_GROUPS
#define NGRTD_DISP_DECAY_GROUPS 8
#endif
constexpr int kDispDecayGroups = NGRTD_DISP_DECAY_GROUPS;

// e^(y ln2 / T), T = kDispExpTab, for an argument already scaled by T / ln 2 (the dispersion
// loop forms y with the scale folded into its per-unit coefficients, so the reduction needs no
// product): y = T k' + j + f, |f| <= 1/2, e^(y ln2/T) = 2^k' 2^(j/T) e^r, r = f ln2/T, with
// 2^(j/T) from the plan's table (tab, LDS: the correctly rounded values) and e^r - 1 by its
// Taylor series to r^4/24 (|r| <= ln2/512: truncation < 4e-17 relative).  <= ~1.2 ulp.  y <= 0
// here.  The conversion of k = rint(y) to int is the hardware's v_cvt_i32_f64, written as
// one instruction (fcvt_i32): it saturates out-of-range values and maps NaN to 0, a defined
// result for every input (a C++ cast of an out-of-range double is undefined, and LLVM may
// fold it to poison).  A very negative y then gives k = INT_MIN, k >> 8 far below -1075, and
// ldexp returns 0; NaN propagates through f and the polynomial.
// The polynomial is in f itself, its coefficients (ln2/T)^n / n! (no separate r = f ln2/T).
__device__ __forceinline__ int fcvt_i32(double x) {
    int k;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(k) : "v"(x));
    return k;
}
__device__ __forceinline__ double fexp_tab(double y, const double* tab) {
    constexpr double L1 = 6.93147180559945309417e-01 / kDispExpTab;
    constexpr double L2 = L1 * L1 / 2.0, L3 = L1 * L1 * L1 / 6.0, L4 = L1 * L1 * L1 * L1 / 24.0;
    const double kd = rint(y);
    const double f = y - kd;
    double q = fma_k(L4, f, L3);
    q = fma_k(q, f, L2);
    q = fma_k(q, f, L1);
    const double p = q * f;                              // e^r - 1, r = f ln2/T
    const int k = fcvt_i32(kd);
    const double th = tab[k & (kDispExpTab - 1)];
    return ldexp(fma(th, p, th), k >> 8);
}
static_assert(kDispExpTab == 256, "fexp_tab: k >> 8");

// Wave-uniform global data read through the constant address space: the loads are scalar
// (s_load, the scalar cache) -- no LDS or vector-memory instruction per age.  Read-only.
typedef __attribute__((address_space(4))) const double k_f64;

// LW: the sampled half-life decays channel 0 and only it (ngrtd.hip lw_ok admits no other plan to
// the single-launch instances), a compile-time channel: a runtime a.chan_lamw[c] select cost two
// v_cndmask_b32 per channel per age in the dispersion loop (10 of its ~40 VALU per age).
template <int C, bool LW, bool DSP = false>
__device__ __forceinline__ void gen_exact(const RtdArgs& a, int mod, bool on, double tau, double eta, double D,
                                          double lam, double* num, double& den, const double* etl = nullptr,
                                          int age0 = 0, int age1 = -1) {
    double s[C + 1];
#pragma unroll
    for (int c = 0; c <= C; ++c) s[c] = 0.0;
    if (DSP && mod == MOD_DISP && etl) {
        // The dispersion weight with its exponent expanded (round 5):
        //   w_k = k1 tp_k^(-3/2) e^(x_k),  x_k = -(1 - tp/tau)^2 (tau/tp) / (4D) = -k2 (tau / tp + tp / tau - 2)
        // so x_k T/ln2 = ya / tp_k + yb tp_k + yc is two FMAs over the per-age 1/tp_k
        // (ya, yb, yc per unit: the T/ln2 of the exponential's reduction folded in, fexp_tab on the
        // plan's 256-entry table in LDS, etl: a degree-4 polynomial instead of fexp's degree 6),
        // and the per-unit factor k1 = sqrt(tau / (4 pi D)) multiplies the sums once at the end
        // (the normalised weights do not depend on it; its NaN / inf still reach the sums, so
        // invalid tau and D give the reference's NaN).  tp_k comes with the row (no per-lane add).
        // The sums differ from the reference's per-age expression by rounding only: near the
        // mode the expanded exponent cancels to ~k2 ulp (k2 <= 25 over the D prior): < 2e-14
        // relative, inside the 1e-12 parity bar.  LW: the per-unit decay e^(-lam tp_k) is
        // re-anchored by an fexp at the first age of every unrolled group and advanced by
        // e^(-lam) within it (<= 3 products: a few ulp).
        // The per-age operands (channel row, 1/tp_k, tp_k^(-3/2): a.disp_rows) are the same for
        // every lane: scalar loads, one 64-B row per age, so the loop's only LDS read is the
        // table lookup and nothing of the series is staged (any N).
        if (__any(on)) {
            constexpr double LTE = kDispExpTab / 6.93147180559945309417e-01;   // T / ln 2
            const double rt = 1.0 / tau;
            const double k1 = sqrt(tau / (4. * kPi * D));
            const double k2 = 1.0 / (4. * D);
            const double ya = -(k2 * tau) * LTE, yb = -(k2 * rt) * LTE, yc = (2.0 * k2) * LTE;
            const double rl = LW ? fexp(-lam) : 1.0;         // e^(-lam): one year of decay
            const int N = a.N;
            const k_f64* rows = (const k_f64*)a.disp_rows;
            // row: A_c at [c], tp_k at [kDispRow - 3], 1/tp_k, tp_k^(-3/2) at the last two
            auto age = [&](const double* r, double dec) {
                const double w = r[kDispRow - 1] * fexp_tab(fma(ya, r[kDispRow - 2], fma(yb, r[kDispRow - 3], yc)), etl);
                const double wd = LW ? w * dec : w;
#pragma unroll
                for (int c = 0; c < C; ++c) s[c] = fma(r[c], (LW && c == 0) ? wd : w, s[c]);
                s[C] += w;
            };
            auto load = [&](int k, double* r) {
#pragma unroll
                for (int j = 0; j < kDispRow; ++j) r[j] = rows[(int64_t)k * kDispRow + j];
            };
            constexpr int UA = kGenDispUnroll;
            const int ke = age1 < 0 ? N : age1;             // ages [age0, ke)
            int k = age0;
            if (k == 0 && k < ke) {                          // age 0: tp_0 = 1e-5 + dtp (off the unit grid: its own decay)
                double r[kDispRow];
                load(0, r);
                age(r, LW ? fexp(-lam * a.tp0) : 1.0);
                k = 1;
            }
            // LW: the decay e^(-lam tp_k) re-anchored by an fexp at the first age of every
            // kDispDecayGroups-th group (a wave-uniform branch: k is the same in every lane) and
            // advanced by e^(-lam) in between (< kDispDecayGroups UA products: a few ulp)
            double dec = 1.0;
            for (int g = 0; k + UA <= ke; k += UA, ++g) {   // UA ages' rows first, then their sums
                double r[UA][kDispRow];
#pragma unroll
                for (int j = 0; j < UA; ++j) load(k + j, r[j]);
                if (LW && g % kDispDecayGroups == 0) dec = fexp(-lam * r[0][kDispRow - 3]);
#pragma unroll
                for (int j = 0; j < UA; ++j) {
                    age(r[j], dec);
                    if (LW) dec *= rl;
                }
            }
            for (; k < ke; ++k) {
                double r[kDispRow];
                load(k, r);
                age(r, LW ? fexp(-lam * r[kDispRow - 3]) : 1.0);
            }
#pragma unroll
            for (int c = 0; c <= C; ++c) s[c] *= k1;
        }
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = s[c];
        den = s[C];
        return;
    }
    if (__any(on)) {
        const double rt = 1.0 / tau;
        double k1, k2 = 0.0, thr = 0.0;
        if (mod == MOD_EXP) {
            k1 = rt;
        } else if (mod == MOD_EPM) {
            k1 = eta / tau;
            k2 = eta - 1;
            thr = tau * (1 - (1 / eta));
        } else {
            k1 = sqrt(tau / (4. * kPi * D));
            k2 = 1.0 / (4. * D);
        }
        const int N = a.N;
        for (int k = 0; k < N; ++k) {
            const double tp = (k == 0) ? a.tp0 : ((double)k + a.dtp);
            double w;
            if (mod == MOD_EXP) {
                w = k1 * fexp(-tp * k1);
            } else if (mod == MOD_EPM) {
                w = (tp >= thr) ? k1 * fexp(fma(-k1, tp, k2)) : 0.0;
            } else {
                const double d = 1.0 - tp * rt;
                w = (k1 * a.disp_aux[N + k]) * fexp(-((d * d) * (tau * a.disp_aux[k])) * k2);
            }
            const double wd = LW ? w * fexp(-lam * tp) : w;
            const double* row = a.tab + (int64_t)k * a.CP;
#pragma unroll
            for (int c = 0; c < C; ++c) s[c] = fma(row[c], (LW && c == 0) ? wd : w, s[c]);
            s[C] += w;
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) num[c] = s[c];
    den = s[C];
}

// ------------------------------------------------------ dispersion, small ensembles
// The lane-per-unit loop above gives each unit ONE lane that walks all N ages: at the
// reference's own shape (one well, 3 chains, N = 25 256: run_age_mcmc.py:209,
// run_age_mcmc_utils.py:412-417) three lanes of the whole chip run 25 256 dependent
// iterations each, ~1 ms per log-prob.  For plans with few units (ngrtd.hip disp_wide_plan)
// the channel sums of the dispersion component come from this kernel instead, with the ages
// across the lanes: block (g, u) sums unit u's ages [g S, (g + 1) S), S = ceil(N / G), lane t
// every kDispWideThreads-th age of it, each lane reading its own 64-B row of a.disp_rows
// (a wave reads 4 KiB contiguous per iteration).  The per-lane partial sums meet in a fixed
// order -- a butterfly within the wave (__shfl_xor, the same tree every launch), then the
// waves in index order -- so the result is deterministic; it is scaled by
// k1 = sqrt(tau / (4 pi D)) and stored as partial g of unit u, out[(g (C + 1) + c) U + u]
// (c = C: the normaliser).  gen_component adds the G partials in order g = 0..G-1.
// Per age: the weight of gen_exact's loop (same expansion of the exponent, fexp_tab on the
// plan's 2^(j/256) table staged in LDS), LW: its own decay fexp(-lam tp_k) (no re-anchoring).
// The sums differ from the lane-per-unit loop's by summation order only (<= a few ulp of the
// sums; parity vs the oracle at rtol 1e-12 either way).
constexpr int kDispWideThreads = 256;
template <int C, bool LW>
NGRTD_KLINK __global__ void __launch_bounds__(kDispWideThreads) disp_wide_kernel(const RtdArgs a, int32_t comp,
                                                                               int32_t G, double* __restrict__ out) {
    constexpr int NW = kDispWideThreads / 64;
    __shared__ double etl[kDispExpTab];
    __shared__ double red[NW][C + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = blockIdx.x;
    const int64_t u = blockIdx.y;
    for (int i = tid; i < kDispExpTab; i += kDispWideThreads) etl[i] = a.disp_aux[2 * a.N + i];
    if (LW) fm_lds_init();
    const double tau = a.theta[(int64_t)a.row_tau[comp] * a.U + u];
    const double D = a.theta[(int64_t)a.row_D[comp] * a.U + u];
    const double lam = LW ? lw_decay(a, tau, a.theta[(int64_t)a.row_thalf * a.U + u]).lam : 0.0;
    constexpr double LTE = kDispExpTab / 6.93147180559945309417e-01;   // T / ln 2
    const double rt = 1.0 / tau;
    const double k1 = sqrt(tau / (4. * kPi * D));
    const double k2 = 1.0 / (4. * D);
    const double ya = -(k2 * tau) * LTE, yb = -(k2 * rt) * LTE, yc = (2.0 * k2) * LTE;
    const int S = (a.N + G - 1) / G;
    const int k0 = g * S, ke = min(a.N, k0 + S);
    __syncthreads();
    double s[C + 1];
#pragma unroll
    for (int c = 0; c <= C; ++c) s[c] = 0.0;
    const double4* rows = reinterpret_cast<const double4*>(a.disp_rows);
    for (int k = k0 + tid; k < ke; k += kDispWideThreads) {
        const double4 r0 = rows[2 * (int64_t)k], r1 = rows[2 * (int64_t)k + 1];
        const double r[kDispRow] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        const double w = r[kDispRow - 1] * fexp_tab(fma(ya, r[kDispRow - 2], fma(yb, r[kDispRow - 3], yc)), etl);
        const double wd = LW ? w * fexp(-lam * r[kDispRow - 3]) : w;
#pragma unroll
        for (int c = 0; c < C; ++c) s[c] = fma(r[c], (LW && c == 0) ? wd : w, s[c]);
        s[C] += w;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int c = 0; c <= C; ++c) s[c] += __shfl_xor(s[c], o);
    if (lane == 0)
#pragma unroll
        for (int c = 0; c <= C; ++c) red[wave][c] = s[c];
    __syncthreads();
    if (tid <= C) {
        double t = red[0][tid];
#pragma unroll
        for (int w = 1; w < NW; ++w) t += red[w][tid];
        out[((int64_t)g * (C + 1) + tid) * a.U + u] = t * k1;
    }
}

// One component (comp 0: tau1 / eta1 / D1, comp 1: tau2 / eta2 / D2) of a unit: its numerators
// num[c] and reciprocal normaliser rden (conc = (A + J B) rden, unit_conc), and *nanc when the
// concentrations are NaN without being summed (the skip lanes above).  tau: the component's tau
// (loaded by the caller); thx: the unit's thalf_cfc Beta value (LW).
template <int C, bool ROLES2, bool LW, bool DSP = false>
__device__ __forceinline__ void gen_component(const RtdArgs& a, const UnitArgs& uk, const double* cheb,
                                              const double* tabl, int comp, bool mvalid, int64_t mu, bool prior_on,
                                              double tau, double thx, double* num, double& rden, bool& nanc,
                                              const double* daux = nullptr, int split = 0) {
    constexpr int CP = cheb_cp(C), PST = kChebN * CP + 2;   // = cheb_lds_stride(C)
    const int mod = a.mod[comp];
    const double eta = (mod == MOD_EPM && mvalid) ? a.theta[(int64_t)a.row_eta[comp] * a.U + mu] : 1.0;
    const double D = (mod == MOD_DISP && mvalid) ? a.theta[(int64_t)a.row_D[comp] * a.U + mu] : 1.0;
    LwDecay lw{0.0, 0.0};
    if (LW) lw = lw_decay(a, tau, thx);
    nanc = false;
    bool ex = false;                                      // this lane's sums by gen_exact
    if (mod == MOD_PISTON) {
        const int ix = piston_index(tau, a.tp0, a.dtp, a.N);
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = a.tab[(int64_t)ix * a.CP + c];
        if (LW) num[0] *= fexp(-lw.lam * (ix == 0 ? a.tp0 : (double)ix + a.dtp));
        rden = 1.0;
    } else if (mod == MOD_EXP) {
        double cx = 0.0, cxw = 0.0;
        int pc = a.cheb ? cheb_piece(tau, cx) - a.cheb_p0 : -1;
        pc = (unsigned)pc < (unsigned)a.cheb_np ? pc : -1;
        int pcw = 0;
        if (LW) {
            pcw = a.cheb ? cheb_piece(lw.teff, cxw) - a.cheb_p0 : -1;
            pcw = (unsigned)pcw < (unsigned)a.cheb_np ? pcw : -1;
        }
        const bool unc = pc < 0 || (LW && pcw < 0);
        // the log-prob is -inf whatever the sums when tau is outside its Uniform prior (or,
        // LW, thalf_cfc outside [0, 1]); the concentrations matter only through their NaN-ness
        bool skip = false;
        if (unc && prior_on) {
            const int rt = a.row_tau[comp];
            const bool t1 = rt == uk.row_tau1, t2 = rt == uk.row_tau2;
            const double lo = t1 ? uk.tau1_lo : uk.tau2_lo, hi = t1 ? uk.tau1_hi : uk.tau2_hi;
            if ((t1 || t2) && !(tau >= lo && tau <= hi)) {
                skip = true;
                nanc = exp_rtd_nan(a, tau);
            } else if (LW && a.row_thalf == uk.row_thalf && !(thx >= 0.0 && thx <= 1.0)) {
                skip = true;
                nanc = !(thx == thx) || exp_rtd_nan(a, tau);
            }
        }
        ex = mvalid && unc && !skip;
        double zz[C + 1];
        cheb_sums<C + 1, ROLES2>(cheb + (pc < 0 ? 0 : pc) * PST, CP, cx, zz);   // s01 Y_c (c < C), s01 G
        double zw = 0.0;
        if (LW) cheb_sums<1, ROLES2>(cheb + (pcw < 0 ? 0 : pcw) * PST, CP, cxw, &zw);
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = a.tab0[c] + zz[c];
        if (LW) num[0] = fexp(-lw.lam * a.tp0) * (a.tab0[0] + zw);
        rden = 1.0 / (1.0 + zz[C]);
    } else if (mod == MOD_EPM) {
        double dn, dd, lam;
        epm_sums<C, kEpmTailPreDz, LW>(a, tabl, mvalid, tau, eta, num, dn, dd, thx, &lam, &nanc);
        rden = dd / dn;
    } else if (DSP && a.disp_pre) {
        // dispersion sums of disp_wide_kernel (small ensembles): its G partials in order
        double s[C + 1];
#pragma unroll
        for (int c = 0; c <= C; ++c) s[c] = a.disp_pre[(int64_t)c * a.U + mu];
        for (int g = 1; g < a.disp_pre_g; ++g)
#pragma unroll
            for (int c = 0; c <= C; ++c) s[c] += a.disp_pre[((int64_t)g * (C + 1) + c) * a.U + mu];
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = s[c];
        rden = 1.0 / s[C];
    } else {
        ex = mvalid;
    }
    if (__any(ex)) {
        double en[C], den;
        // split (dispersion, staged tables): this wave's ages [split, N); rden holds the raw
        // normaliser sum until the caller adds the theta wave's [0, split)
        if (DSP) {
            gen_exact<C, LW, true>(a, mod, ex, tau, eta, D, lw.lam, en, den, daux, split);
        } else {
            gen_exact<C, LW>(a, mod, ex, tau, eta, D, lw.lam, en, den);
        }
        if (ex) {
#pragma unroll
            for (int c = 0; c < C; ++c) num[c] = en[c];
            rden = (DSP && split) ? den : 1.0 / den;
        }
    }
}

// A kernel argument read through a pointer the compiler cannot see through (an empty asm
// redefines the kernarg segment pointer): loads of its fields stay where they are used --
// a multi-step loop would otherwise hoist every field into registers for the whole loop.
// The pointer is the kernarg segment itself, so the loads stay scalar loads.  (Taking the
// address of the by-value parameter instead makes the compiler copy it to scratch.)
// Explicit kernel arguments sit in order at their natural alignment (the code object's
// .args metadata: RtdArgs at 0, UnitArgs, WB, logp, DemcAccept at kFusedArgD).
__host__ __device__ constexpr size_t ka_align(size_t o, size_t a) { return (o + a - 1) / a * a; }
constexpr size_t kFusedArgU = ka_align(sizeof(RtdArgs), alignof(UnitArgs));
constexpr size_t kFusedArgD =
    ka_align(ka_align(ka_align(kFusedArgU + sizeof(UnitArgs), alignof(int32_t)) + sizeof(int32_t), alignof(double*)) +
                 sizeof(double*),
             alignof(DemcAccept));
template <class T>
__device__ __forceinline__ const T& kernarg_opaque(size_t off) {
    typedef const __attribute__((address_space(4))) char* CP;
    CP p = (CP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const T*)(p + off);
}
template <class T>
__device__ __forceinline__ T opaque_v(T x) {
    asm volatile("" : "+v"(x));
    return x;
}
template <class T>
__device__ __forceinline__ T opaque_s(T x) {
    asm volatile("" : "+s"(x));
    return x;
}

constexpr int kFusedWaves = 8;                 // waves of units per block (512 units)
constexpr int kFusedUnits = 64 * kFusedWaves;
// LDS doubles ahead of the tables: per-unit partial sums [2][512], decisions [512] int, per-
// wave accept counts [16] int (8 doubles, padded to keep the tables 16-B aligned)
constexpr int kFusedHdr = 2 * kFusedUnits + kFusedUnits / 2 + 16;
constexpr int kFusedPrefetch = 6;   // double2 per thread (512 threads): covers kChebPieces*kChebN*6 doubles
// LDS stride of one surrogate piece: kChebN*CP doubles + 2 of padding, so that consecutive
// pieces start 16-B slots an ODD number apart -- lanes gathering different pieces with
// ds_read_b128 then spread over all 16 slots of a bank row instead of 4 (MI355X_MICROARCH.md
// §LDS: a b128 lane group conflicts on equal slots).
__host__ __device__ constexpr int cheb_lds_stride(int C) { return kChebN * cheb_cp(C) + 2; }

// ROLES = 1: one wave per 64 units runs the whole unit (2 waves/SIMD at c4, 228 VGPRs).
// ROLES = 2: the block has 2 x 8 waves; waves 0-7 run the theta-only block (priors, CE model,
// CE likelihood) and waves 8-15 the RTD block (surrogate channel sums, concentrations, RTD
// likelihood, exact fallback) of the SAME 512 units, and their results meet in LDS in the
// reference's addition order (th + like).  Role is wave-uniform (no divergence); each role
// needs fewer registers, so at c4 a SIMD holds 4 waves of two different instruction mixes
// (transcendental-heavy CE, FMA-chain Clenshaw) that hide each other's latency.
// MIX bit 0: BMM with a piston second component (tau2, f1 roles): its concentrations are a
// channel-table lookup, mixed f1 c1 + (1 - f1) c2 (run_age_mcmc_utils.py:126-161).
// MIX bit 2 (FULL only): the plan carries the transform Jacobians (NGRTD_WANT_JACOBIAN).
// MIX bit 1: the first component is exp_pist_flow (eta1 role) instead of exponential: the
// channel table is staged in LDS, every unit sums a head of <= kEpmBlock ages by Horner and
// reads the block-tail surrogate a.epm at tau' = 1 / beta (epm_sums); lanes whose tau' the
// surrogate does not cover sum their tail exactly (Horner over the LDS table).
// MIX bit 3 (FULL, ROLES = 2): one whole DEMetropolisZ step per launch (ngrtd_demcz_run).
// The theta waves load their unit's state rows x and the rows of the chain's two history
// partners (chain-major: a wave's 8 lanes of one walker read 64 contiguous bytes, as they
// do from theta), append x to the history, form the proposal (dz_value) and write it --
// natural space, after the PyMC3 backward transform -- to the theta rows the launch reads
// (a.theta = dacc.dz_prop; each block reads back only its own units' lines, behind the
// barrier).  After the Metropolis decision the accepted units' lanes write the proposal
// into the state (and, transformed, recompute and write the chains'-space value).  Per
// step: 3 reads + 2 writes of the state's size in HBM, against 6 reads + 3 writes (+ the
// accepted copies) for the proposal kernel + log-prob kernel pair.
// MIX bit 4 (with bit 3): per-well chains (one Metropolis decision per unit).
// MIX bit 5: the sampled CFC12 half-life (channel 0's own decay, lw_decay).
// MIX bit 6: the generic components (gen_component: every other model pair, runtime models).
// MIX bit 7 (with bit 6): the plan has a dispersion component (its tables staged in LDS, its
// age sum split over the unit's two waves; csrc/ngrtd_gen_disp.hip).
// the reference's Beta priors compiled into the DEMetropolisZ instances too: 4-16 VGPRs spill
// in their step loop, yet the c4 per-well step runs 20.7 -> 18.7 us transformed and 18.7 ->
// 16.7 us natural (profiles/r04m_dz_refb_ab.jsonl; NGRTD_DZ_REFB=0 builds the runtime loop)
#ifndef NGRTD_DZ_REFB
#define NGRTD_DZ_REFB 1
#endif
constexpr bool kDzRefB = NGRTD_DZ_REFB != 0;
template <int C, bool FULL, int ROLES, int MIX>
__global__ void __launch_bounds__(64 * kFusedWaves * ROLES) logp_fused_kernel(const RtdArgs ak, const UnitArgs ua,
                                                                              int32_t WB, double* __restrict__ logp,
                                                                              const DemcAccept dacc) {
    constexpr bool DZ = (MIX & 8) != 0;
    constexpr bool PW = DZ && (MIX & 16) != 0;   // per-well chains: one Metropolis decision per unit
    constexpr bool LW = (MIX & 32) != 0;         // the sampled CFC12 half-life (channel 0, lw_decay)
    // FULL: the reference's Beta priors as compile-time exponents (kRefBeta: bare / with the
    // Jacobians, without / with thalf_cfc), in the DEMetropolisZ steps too (kDzRefB); the
    // runtime loop gives the same bits
    constexpr int REFB = (FULL && (!DZ || kDzRefB)) ? 1 + ((MIX & 4) ? 1 : 0) + (LW ? 2 : 0) : 0;
    static_assert(!DZ || (FULL && ROLES == 2), "the DEMetropolisZ step runs in the FULL role-split kernel");
    static_assert(kFusedUnitsDz == kFusedUnits, "DZ staging stride");
    const RtdArgs& a = ak;
    constexpr int NT = mfma_tiles(C);
    constexpr int CP = cheb_cp(C);
    constexpr int NTH = 64 * kFusedWaves * ROLES;           // threads per block
    constexpr int NPRE = (kFusedPrefetch * 64 * kFusedWaves + NTH - 1) / NTH;
    constexpr int TAB2MAX = kChebPieces * kChebN * CP / 2;   // double2 entries of the whole table
    const int TAB2 = a.cheb_np * (kChebN * CP / 2);       // ... of the staged window
    constexpr int PST = cheb_lds_stride(C);               // LDS doubles per piece (padded)
    static_assert(NT == 4, "one unit per lane needs 4 tiles per wave");
    static_assert(TAB2MAX <= NPRE * NTH, "prefetch covers the table");
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* part = lds;                                   // [512] per-unit log-prob
    double* part2 = lds + kFusedUnits;                    // [512] RTD likelihood (ROLES = 2)
    int* dec = reinterpret_cast<int*>(lds + 2 * kFusedUnits);   // [512] DE-MC decisions per walker
    int* wcnt = reinterpret_cast<int*>(lds + 2 * kFusedUnits + kFusedUnits / 2);   // [16] per-wave accept counts
    double* cheb = lds + kFusedHdr;                       // [kChebPieces][kChebN][CP]
    if (!DZ) NGRTD_PROBE(0);   // (a stamp here broke the DZ instances' instruction selection)
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int uw = wave % kFusedWaves;                    // unit wave
    const bool do_theta = ROLES == 1 || wave < kFusedWaves;
    const bool do_rtd = ROLES == 1 || wave >= kFusedWaves;
    const int L = ua.L;
    const int64_t W = ua.W;
    // XCD-aware walker blocks: the dispatcher deals block b to XCD b % 8, so consecutive
    // walker blocks (which share the 128-B lines of every theta row when WB * 8 < 128) are
    // renumbered onto the same XCD and its L2 serves the second (profiles: FETCH_SIZE)
    const int nb = gridDim.x;
    const int bl = (nb & 7) == 0 ? ((int)blockIdx.x & 7) * (nb >> 3) + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
    const int64_t w0 = (int64_t)bl * WB;
    // surrogate table -> registers -> LDS (stored after every prologue load is issued)
    double2 pre[NPRE];
    if (a.cheb) {
        const double2* src = reinterpret_cast<const double2*>(a.cheb + (size_t)a.cheb_p0 * kChebN * CP);
#pragma unroll
        for (int r = 0; r < NPRE; ++r) {
            const int i = tid + r * NTH;
            pre[r] = i < TAB2 ? src[i] : double2{0.0, 0.0};
        }
    }
    // this lane's unit
    const int mi = 64 * uw + lane;
    const int mwl = mi % WB, ml = mi / WB;
    const bool mvalid = ml < L && w0 + mwl < W;
    const int64_t mu = mvalid ? (int64_t)ml * W + w0 + mwl : 0;
    // per-well observation data -> LDS (read per lane by the likelihood blocks): all loads
    // issued before any store, so the prologue pays one memory latency
    constexpr bool EPM = (MIX & 2) != 0;
    constexpr bool GEN = (MIX & 64) != 0;        // generic components (gen_component)
    static_assert(!GEN || (MIX & (1 | 2)) == 0, "generic instances: runtime models (plain log-prob or the DZ step)");
    // the channel table staged in LDS: exp_pist_flow components (epm_sums)
    // ... and dispersion components (gen_exact's LDS loop), with their per-age disp_aux: the
    // generic instances with MIX bit 7 (a plan with a dispersion component; the others keep
    // the code without it)
    constexpr bool DSPI = GEN && (MIX & 128) != 0;
    const bool DISPS = DSPI && a.disp_aux && a.disp_rows && (a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP);
    const bool EPMS = EPM || (GEN && (a.mod[0] == MOD_EPM || a.mod[1] == MOD_EPM));
    double* tabl = cheb + a.cheb_np * PST;                // EPM: the channel table (epm_row)
    double* daux = tabl + (EPMS ? epm_lds_doubles(a.epm_nw, CP) : 0);   // DISPS: fexp_tab's table
    double* wd = daux + (DISPS ? kDispExpTab : 0);
    constexpr int kWdRegs = (4 * 64 * kFusedWaves + NTH - 1) / NTH;
    double wv[kWdRegs];
#pragma unroll
    for (int r = 0; r < kWdRegs; ++r) {
        const int i = tid + r * NTH;
        wv[r] = i < ua.wd_n ? ua.wd_src[i] : 0.0;
    }
    fm_lds_init();                                        // fexp/flog tables
    // theta rows of this lane's unit, issued behind the table loads (the LDS stores below
    // wait only for those) so that their HBM latency overlaps the prologue's barrier
    // (A/B against loading them after the barrier: 11.87 vs 11.95 us, tools/gpu_ab_libs.sh)
    ThetaPre tp0{};
    double tau0 = 1.0, eta0 = 1.0, tau20 = 1.0, thx0 = 0.5;
    if (!DZ) {
        if (do_theta) theta_preload(ua, mu, tp0);
        if (do_rtd) {
            tau0 = mvalid ? a.theta[(int64_t)a.row_tau[0] * a.U + mu] : 1.0;
            if (EPM) eta0 = mvalid ? a.theta[(int64_t)a.row_eta[0] * a.U + mu] : 1.0;
            if (MIX & 1) tau20 = mvalid ? a.theta[(int64_t)a.row_tau[1] * a.U + mu] : 1.0;
            if (LW) thx0 = mvalid ? a.theta[(int64_t)a.row_thalf * a.U + mu] : 0.5;
            tp0.nub = (FULL || ua.rtd_on) ? a.theta[(int64_t)ua.row_nu * a.U + mu] : 0.0;
        }
    }
    if (EPMS) {   // channel table -> LDS (rows of CP doubles, CP even: 16-B copies)
        const double2* src = reinterpret_cast<const double2*>(a.tab);
        double2* dst = reinterpret_cast<double2*>(tabl);
        constexpr int RB = kEpmBlock * CP / 2, SB = epm_blk_stride(CP) / 2;   // double2 per block / padded
        // whole blocks: the rows past N of the last block are zeros (epm_sums reads every row
        // of a unit's head block, weighting the ones before its first age by 0); the rows
        // [0, epm_nw) of a windowed table
        const int nr = a.N < a.epm_nw ? a.N : a.epm_nw;
        const int n2 = a.epm_nw / kEpmBlock * RB, nv = nr * CP / 2;
        if (a.CP == CP) {
            for (int i = tid; i < n2; i += NTH) dst[(i / RB) * SB + i % RB] = i < nv ? src[i] : double2{0.0, 0.0};
        } else {   // C = 2, 4: the global table's rows are (C + 1) & ~1 = C doubles, the LDS rows CP = C + 2
            for (int i = tid; i < 2 * n2; i += NTH) {
                const int k = i / CP, c = i % CP;
                tabl[epm_row(k, CP) + c] = (k < nr && c < C) ? a.tab[(int64_t)k * a.CP + c] : 0.0;
            }
        }
    }
    if (DISPS)
        for (int i = tid; i < kDispExpTab; i += NTH) daux[i] = a.disp_aux[2 * a.N + i];
#pragma unroll
    for (int r = 0; r < kWdRegs; ++r) {
        const int i = tid + r * NTH;
        if (i < ua.wd_n) wd[i] = wv[r];
    }
    for (int i = tid + kWdRegs * NTH; i < ua.wd_n; i += NTH) wd[i] = ua.wd_src[i];
    if (a.cheb) {
        double2* dst = reinterpret_cast<double2*>(cheb);
#pragma unroll
        for (int r = 0; r < NPRE; ++r) {
            const int i = tid + r * NTH;
            if (i < TAB2) dst[(i / (kChebN * CP / 2)) * (PST / 2) + i % (kChebN * CP / 2)] = pre[r];
        }
    }
    // DZ: the theta waves form the proposals (a.theta = dacc.dz_prop), after the table stores
    // so that the table registers are free for the 3 P loads
    double* thl = wd + ua.wd_n;                           // DZ, transformed: [P][512] u
    // DZ, LDS state (dacc.state_lds): the block's chains -> LDS, once per launch (each lane the
    // rows of its unit it stages: theta waves the even rows, RTD waves the odd ones)
    bool moved = false;                                   // ... a row of this lane's unit changed
    if (DZ && dacc.state_lds) {
        double* st = thl + ((MIX & 4) ? dacc.P * kFusedUnits : 0) + (dacc.prop_lds ? dacc.P * kFusedUnits : 0);
        const int dwl = mi / L, dml = mi % L;
        const bool dv = dwl < WB && w0 + dwl < W;
        const int64_t du = dv ? (w0 + dwl) * (int64_t)L + dml : 0;
        for (int p = do_theta ? 0 : 1; p < dacc.P; p += 2) st[p * kFusedUnits + mi] = dv ? dacc.zx[(int64_t)p * ua.U + du] : 0.0;
        double* c = st + dacc.P * kFusedUnits;            // lp, lamb, scaling [512] each, tuning counter [512] int
        int32_t* cn = reinterpret_cast<int32_t*>(c + 3 * kFusedUnits);
        // per-chain slots: the unit (per-well chains, walker-major index du) / the walker
        const bool own = PW ? (do_theta && dv) : (tid < WB && w0 + tid < W);
        const int sl = PW ? mi : tid;
        const int64_t gi = PW ? du : w0 + tid;
        if (own) {
            c[sl] = dacc.lp[gi];
            c[kFusedUnits + sl] = dacc.lamb[gi];
            c[2 * kFusedUnits + sl] = dacc.scaling[gi];
            if (dacc.n_acc_tune) cn[sl] = dacc.n_acc_tune[gi];
        }
        __syncthreads();
    }
    // DZ: dacc.n_steps steps of the block's own chains, the tables staged once above
    // (a do-while: without DZ there is no back edge at all -- a one-trip for loop changed the
    // register allocation of the plain log-prob instances)
    const int nst = DZ ? dacc.n_steps : 1;
    int js = 0;
    // DZ: the next step's partner rows, issued at the end of this step's log-prob body
    constexpr int PFS = PW ? kDzPfStepPw : kDzPfStep;    // rows per role of the staging (above)
    double pf1[(kDzMaxP + PFS - 1) / PFS], pf2[(kDzMaxP + PFS - 1) / PFS];
    do {
        ThetaPre tp = tp0;                                // DZ: loaded per step below
        double tau = tau0, eta = eta0, tau2 = tau20, thx = thx0;
        // DZ: the argument structs through an opaque kernarg pointer per step, so that the
        // compiler re-reads their fields where they are used instead of hoisting every field
        // out of the step loop into registers (which spilled to scratch)
        const RtdArgs& a = DZ ? kernarg_opaque<RtdArgs>(0) : ak;
        const UnitArgs& uk = DZ ? kernarg_opaque<UnitArgs>(kFusedArgU) : ua;
        const DemcAccept& dk = DZ ? kernarg_opaque<DemcAccept>(kFusedArgD) : dacc;
        // ... and likewise the lane's unit and the LDS carve-up, re-derived per step from
        // opaque copies (loop-invariant lane addresses hoisted out of the loop spilled too)
        const int tid_s = DZ ? opaque_v(tid) : tid;
        const int64_t w0_s = DZ ? opaque_s(w0) : w0;
        const int tid = tid_s;
        const int64_t w0 = w0_s;
        const int wave = tid >> 6, lane = tid & 63;
        const int uw = wave % kFusedWaves;
        const bool do_theta = ROLES == 1 || wave < kFusedWaves;
        const bool do_rtd = ROLES == 1 || wave >= kFusedWaves;
        const int L = uk.L;
        const int64_t W = uk.W;
        const int mi = 64 * uw + lane;
        // DZ: walker-major units (a wave holds one walker's 64 wells at c4) over the
        // walker-major state / proposal buffers [P][W][L] (ngrtd_demcz_run transposes the
        // caller's [P][L][W] state in and out): every row a lane stages -- state, history
        // append, both partners, proposal -- is then one contiguous 512-B run per wave
        const int mwl = DZ ? mi / L : mi % WB, ml = DZ ? mi % L : mi / WB;
        const bool mvalid = (DZ ? mwl < WB : ml < L) && w0 + mwl < W;
        const int64_t mu = !mvalid ? 0 : DZ ? (w0 + mwl) * (int64_t)L + ml : (int64_t)ml * W + w0 + mwl;
        // the unit's slot in part / part2 ((well, walker) order, as the reduction reads it);
        // DZ lanes past the block's WB L units keep their own slot mi >= WB L, so that their
        // zero partial sums land on no walker's slots
        const int pi = (DZ && mwl >= WB) ? mi : ml * WB + mwl;
        double* tabl = cheb + a.cheb_np * PST;
        double* daux = tabl + (EPMS ? epm_lds_doubles(a.epm_nw, CP) : 0);
        double* wd = daux + (DISPS ? kDispExpTab : 0);
        double* thl = wd + uk.wd_n;
        double* propl = thl + (((MIX & 4) && DZ) ? dk.P * kFusedUnits : 0);   // DZ: [P][512] proposals
        DzLds dl;                                         // DZ: the chains' LDS state (or none)
        if (DZ && dk.state_lds) {
            dl.on = true;
            dl.st = (lds_f64*)(propl + (dk.prop_lds ? dk.P * kFusedUnits : 0));
            dl.lp = dl.st + dk.P * kFusedUnits;
            dl.lamb = dl.lp + kFusedUnits;
            dl.sc = dl.lamb + kFusedUnits;
            dl.nat = (lds_i32*)(dl.sc + kFusedUnits);
        }
        // the per-well data in LDS: the plain instances redirect a copy of the arguments, the DZ
        // instances read the kernarg struct itself beside a view of the LDS pointers (WdView: a
        // redirected copy would live in SGPRs across the step loop -- 238 spilled, ~10% per step)
        UnitArgs ul = uk;
        WdView wv{};
        {
            const int nce = uk.ce_on ? L * uk.G : 0, nrt = uk.rtd_on ? L * uk.K : 0;
            double* q = wd;
            if (uk.ce_on) {
                ul.ce_obs = wv.ce_obs = q; q += nce;
                ul.ce_lam = wv.ce_lam = q; q += nce;
                ul.ce_hll_sum = wv.ce_hll_sum = q; q += L;
                ul.ce_Emin = wv.ce_Emin = q; q += L;
            }
            if (uk.rtd_on) {
                ul.rtd_obs = wv.rtd_obs = q; q += nrt;
                ul.rtd_lam = wv.rtd_lam = q; q += nrt;
                ul.rtd_hll_sum = wv.rtd_hll_sum = q;
            }
            wv.c0_tab = uk.c0_tab ? wd + (uk.c0_tab - uk.wd_src) : nullptr;
            if (uk.c0_tab) ul.c0_tab = wv.c0_tab;
        }
        const UnitArgs& uu = DZ ? uk : ul;
        const WdView* wvp = DZ ? &wv : nullptr;
        DzStep sj{};
        if (DZ) sj = dz_step(dk.sch, js);
        const int64_t log_off = (int64_t)js * W;
        // both roles stage: theta waves the even parameter rows, RTD waves the odd ones
        NGRTD_PROBE(8);
        if (DZ && kDzPrefetch) {
            // each role stages its rows of the unit from partner rows loaded one step ahead
            // (the first step of the launch loads its own here)
            if (js == 0)
                dz_partner_rows<kDzMaxP, PFS>(dk, sj, w0 + mwl, ml, L, W, mvalid && (PFS == 2 || do_theta),
                                                    do_theta ? 0 : 1, pf1, pf2);
            if (PFS == 2 || do_theta)
                dz_stage_all<kDzMaxP, PFS, (MIX & 4) != 0, PW>(dk, sj, uk.U, mu, mi, w0 + mwl, ml, L, W, mvalid,
                                                                     thl, dk.prop_lds ? propl : nullptr, dl,
                                                                     PW ? mi : mwl, do_theta ? 0 : 1, pf1, pf2);
        } else if (DZ) {
            dz_stage<kDzMaxP, (MIX & 4) != 0, PW>(dk, sj, uk.U, mu, mi, w0 + mwl, ml, L, W, mvalid, thl,
                                                  do_theta ? 0 : 1, dk.prop_lds ? propl : nullptr, dl,
                                                  PW ? mi : mwl);
        }
        NGRTD_PROBE(9);
        __syncthreads();
        NGRTD_PROBE(1);
        if (DZ && dk.prop_lds) {                              // the proposal's rows, from LDS
            if (do_theta) {
#pragma unroll
                for (int i = 0; i < 6; ++i) tp.ce[i] = propl[uk.row_ce[i] * kFusedUnits + mi];
                tp.tau1 = propl[uk.row_tau1 * kFusedUnits + mi];
                tp.nub = propl[uk.row_nu * kFusedUnits + mi];
            }
            if (do_rtd) {
                tau = mvalid ? propl[a.row_tau[0] * kFusedUnits + mi] : 1.0;
                if (EPM) eta = mvalid ? propl[a.row_eta[0] * kFusedUnits + mi] : 1.0;
                if (MIX & 1) tau2 = mvalid ? propl[a.row_tau[1] * kFusedUnits + mi] : 1.0;
                if (LW) thx = mvalid ? propl[a.row_thalf * kFusedUnits + mi] : 0.5;
                tp.nub = propl[uk.row_nu * kFusedUnits + mi];
            }
        } else if (DZ) {                                      // the proposal's rows
            if (do_theta) theta_preload(uk, mu, tp);
            if (do_rtd) {
                tau = mvalid ? a.theta[(int64_t)a.row_tau[0] * a.U + mu] : 1.0;
                if (EPM) eta = mvalid ? a.theta[(int64_t)a.row_eta[0] * a.U + mu] : 1.0;
                if (MIX & 1) tau2 = mvalid ? a.theta[(int64_t)a.row_tau[1] * a.U + mu] : 1.0;
                if (LW) thx = mvalid ? a.theta[(int64_t)a.row_thalf * a.U + mu] : 0.5;
                tp.nub = a.theta[(int64_t)uk.row_nu * a.U + mu];
            }
        }
        double th = 0.0, like = 0.0;
        if (do_theta) th = mvalid ? unit_logp_theta<REFB>(uu, mu, ml, &tp, FULL, (MIX & 4) != 0, wvp) : 0.0;
        // RTD waves without a unit (blocks of fewer walkers than kFusedUnits / L: fused_wb) skip
        // their body (wave-uniform)
        const bool rtd_w = do_rtd && (DZ || __any(mvalid));
        if (GEN && !DSPI && rtd_w) {
            // generic components: the first from tau (prologue), the second (BMM) from tau2
            const bool prior_on = FULL || (uk.rtd_on && (uk.flags & NGRTD_WANT_PRIOR));
            double conc[kMaxTracer];
            double n1[C], r1, n2[C], r2 = 1.0;
            bool nan1, nan2 = false;
            gen_component<C, ROLES == 2, LW>(a, uk, cheb, tabl, 0, mvalid, mu, prior_on, tau, thx, n1, r1, nan1);
            const bool two = a.mod[1] != MOD_NONE;
            if (two) {
                const double t2 = mvalid ? a.theta[(int64_t)a.row_tau[1] * a.U + mu] : 1.0;
                gen_component<C, ROLES == 2, LW>(a, uk, cheb, tabl, 1, mvalid, mu, prior_on, t2, thx, n2, r2, nan2);
            }
            // (two calls, not one with a runtime-selected num2 pointer: that put n2 in scratch)
            if (two) unit_conc<C>(a, mu, n1, r1, conc, n2, r2);
            else unit_conc<C>(a, mu, n1, r1, conc);
            if (nan1 || nan2) {
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)
                    if (t < a.K) conc[t] = __builtin_nan("");
            }
            const double rnu = 1.0 / (tp.nub * (uk.rnu_max - uk.rnu_min) + uk.rnu_min);
            like = mvalid ? unit_like_rtd<C>(uu, mu, ml, conc, &tp, FULL, &rnu, wvp) : 0.0;
            if (!FULL && a.conc && mvalid) {                      // forward(): model concentrations
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)   // unrolled: conc stays in registers
                    if (t < a.K) a.conc[(int64_t)t * a.U + mu] = conc[t];
            }
        } else if (DSPI) {
            // generic components: the first from tau (prologue), the second (BMM) from tau2.
            // A dispersion component's exact age sum is split over the unit's two waves
            // (a.disp_split, ROLES = 2): the theta wave, done with its CE block early, sums ages
            // [0, split) into LDS, the RTD wave [split, N), and the RTD wave adds the two after a
            // barrier (block-uniform: every wave reaches it)
            const int dsp = (DISPS && ROLES == 2) ? a.disp_split : 0;
            const int dcomp = a.mod[0] == MOD_DISP ? 0 : 1;
            // [C + 1][kFusedUnits]: after the per-well data, or (DZ) after the step's proposal
            // rows and the chains' LDS state (launch_fused_dz sizes the block's LDS as the sum)
            double* xch = !DZ ? wd + uk.wd_n
                              : propl + (dk.prop_lds ? dk.P * kFusedUnits : 0) +
                                    (dk.state_lds ? dk.P * kFusedUnits + 3 * kFusedUnits + kFusedUnits / 2 : 0);
            if (dsp && do_theta) {
                double pn[C], pd;
                const double tc = mvalid ? a.theta[(int64_t)a.row_tau[dcomp] * a.U + mu] : 1.0;
                const double Dc = mvalid ? a.theta[(int64_t)a.row_D[dcomp] * a.U + mu] : 1.0;
                double lam = 0.0;
                if (LW) lam = lw_decay(a, tc, mvalid ? a.theta[(int64_t)a.row_thalf * a.U + mu] : 0.5).lam;
                gen_exact<C, LW, true>(a, MOD_DISP, mvalid, tc, 1.0, Dc, lam, pn, pd, daux, 0, dsp);
#pragma unroll
                for (int c = 0; c < C; ++c) xch[c * kFusedUnits + mi] = pn[c];
                xch[C * kFusedUnits + mi] = pd;
            }
            const bool prior_on = FULL || (uk.rtd_on && (uk.flags & NGRTD_WANT_PRIOR));
            double n1[C], r1 = 1.0, n2[C], r2 = 1.0;
#pragma unroll
            for (int c = 0; c < C; ++c) n1[c] = n2[c] = 0.0;
            bool nan1 = false, nan2 = false;
            const bool two = a.mod[1] != MOD_NONE;
            const double* dxl = DISPS ? daux : nullptr;
            if (rtd_w) {
                gen_component<C, ROLES == 2, LW, true>(a, uk, cheb, tabl, 0, mvalid, mu, prior_on, tau, thx, n1, r1, nan1, dxl,
                                                 dcomp == 0 ? dsp : 0);
                if (two) {
                    const double t2 = mvalid ? a.theta[(int64_t)a.row_tau[1] * a.U + mu] : 1.0;
                    gen_component<C, ROLES == 2, LW, true>(a, uk, cheb, tabl, 1, mvalid, mu, prior_on, t2, thx, n2, r2, nan2,
                                                     dxl, dcomp == 1 ? dsp : 0);
                }
            }
            if (dsp) {
                __syncthreads();
                if (rtd_w) {   // the split component: theta's ages [0, split) + this wave's [split, N)
                    const double pd = xch[C * kFusedUnits + mi];
                    if (dcomp == 0) {
#pragma unroll
                        for (int c = 0; c < C; ++c) n1[c] = xch[c * kFusedUnits + mi] + n1[c];
                        r1 = 1.0 / (pd + r1);
                    } else {
#pragma unroll
                        for (int c = 0; c < C; ++c) n2[c] = xch[c * kFusedUnits + mi] + n2[c];
                        r2 = 1.0 / (pd + r2);
                    }
                }
            }
          if (rtd_w) {
            double conc[kMaxTracer];
            if (two) unit_conc<C>(a, mu, n1, r1, conc, n2, r2);
            else unit_conc<C>(a, mu, n1, r1, conc);
            if (nan1 || nan2) {
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)
                    if (t < a.K) conc[t] = __builtin_nan("");
            }
            const double rnu = 1.0 / (tp.nub * (uk.rnu_max - uk.rnu_min) + uk.rnu_min);
            like = mvalid ? unit_like_rtd<C>(uu, mu, ml, conc, &tp, FULL, &rnu, wvp) : 0.0;
            if (!FULL && a.conc && mvalid) {                      // forward(): model concentrations
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)   // unrolled: conc stays in registers
                    if (t < a.K) a.conc[(int64_t)t * a.U + mu] = conc[t];
            }
          }
        } else if (EPM && rtd_w) {
            double conc[kMaxTracer];
            {
                double num[C], dn, dd, lam = 0.0;
                bool wnan;
                epm_sums<C, DZ ? kEpmTailPreDz : LW ? kEpmTailPreLw : kEpmTailPre, LW>(a, tabl, mvalid, tau, eta, num, dn,
                                                                                     dd, thx, &lam, &wnan);
                const double dr[2] = {dn, tp.nub * (uk.rnu_max - uk.rnu_min) + uk.rnu_min};
                double rr[2];
                batch_recip<2>(dr, rr);
                double num2[C];
                if (MIX & 1) {                  // the piston row from the channel table (LDS)
                    const int ix = piston_index(tau2, a.tp0, a.dtp, a.N);
                    epm_piston_row<C>(a, tabl, ix, num2);
                    if (LW) num2[0] *= fexp(-lam * (ix == 0 ? a.tp0 : (double)ix + a.dtp));
                }
                unit_conc<C>(a, mu, num, dd * rr[0], conc, (MIX & 1) ? num2 : nullptr);
                if (wnan) {
#pragma unroll
                    for (int t = 0; t < kMaxTracer; ++t)
                        if (t < a.K) conc[t] = __builtin_nan("");
                }
                like = mvalid ? unit_like_rtd<C>(uu, mu, ml, conc, &tp, FULL, &rr[1], wvp) : 0.0;
            }
            if (!FULL && a.conc && mvalid) {                      // forward(): model concentrations
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)   // unrolled: conc stays in registers
                    if (t < a.K) a.conc[(int64_t)t * a.U + mu] = conc[t];
            }
        } else if (!GEN && rtd_w) {
            // The surrogate channel sums, the concentrations and the RTD likelihood.  Lanes
            // whose tau the surrogate does not cover evaluate piece 0 here and are redone
            // exactly below.
            double cx = 0.0;
            int cpc = a.cheb ? cheb_piece(tau, cx) - a.cheb_p0 : -1;
            cpc = (unsigned)cpc < (unsigned)a.cheb_np ? cpc : -1;   // outside the staged window
            // LW: channel 0 from the surrogate at tau_eff (its own piece of the staged window)
            LwDecay lw{0.0, 0.0};
            double cxw = 0.0;
            int cpw = 0;
            if (LW) {
                lw = lw_decay(a, tau, thx);
                cpw = a.cheb ? cheb_piece(lw.teff, cxw) - a.cheb_p0 : -1;
                cpw = (unsigned)cpw < (unsigned)a.cheb_np ? cpw : -1;
            }
            const bool unc = cpc < 0 || (LW && cpw < 0);
            // An uncovered tau (< 1/2, NaN) outside the support of the tau1 Uniform prior makes the
            // unit's log-prob -inf whatever the concentrations are -- unless they are NaN, which
            // the reference's weights produce exactly when (1/tau) exp(-tp/tau) overflows or
            // divides by 0 (convolution_integral_utils.py:184, then g / g.sum(), :270): such a
            // lane needs no channel sums, only that NaN predicate.  DE-MC proposals below the
            // prior bound are common; they would otherwise send whole waves to the exact path.
            bool skip = false, cnan = false;
            const bool prior_on = FULL || (uk.rtd_on && (uk.flags & NGRTD_WANT_PRIOR));
            if (unc && a.cheb && prior_on && a.row_tau[0] == uk.row_tau1 && !(tau >= uk.tau1_lo && tau <= uk.tau1_hi) &&
                !(uk.tau1_lo < kChebTauLo && tau >= uk.tau1_lo)) {
                skip = true;
                cnan = exp_rtd_nan(a, tau);
            }
            // LW: a thalf_cfc Beta value outside [0, 1] makes the log-prob -inf as well; NaN
            // gives a NaN decay (and concentration), as the reference's
            if (LW && unc && !skip && a.cheb && prior_on && a.row_thalf == uk.row_thalf && !(thx >= 0.0 && thx <= 1.0)) {
                skip = true;
                cnan = !(thx == thx) || exp_rtd_nan(a, tau);
            }
            const bool bad = unc && !skip;
            cpc = cpc < 0 ? 0 : cpc;
            cpw = cpw < 0 ? 0 : cpw;
            double zz[C + 1];
            NGRTD_PROBE(4);
            cheb_sums<C + 1, ROLES == 2>(cheb + cpc * PST, CP, cx, zz);   // s01 Y_c (c < C), s01 G
            double zw = 0.0;
            if (LW) cheb_sums<1, ROLES == 2>(cheb + cpw * PST, CP, cxw, &zw);   // channel 0 at tau_eff
            NGRTD_PROBE(5);
            double conc[kMaxTracer];
            {
                double num[C];
#pragma unroll
                for (int c = 0; c < C; ++c) num[c] = a.tab0[c] + zz[c];
                if (LW) num[0] = fexp(-lw.lam * a.tp0) * (a.tab0[0] + zw);
                // the normaliser's reciprocal and the Student-t 1/nu: one division
                const double dr[2] = {1.0 + zz[C], tp.nub * (uk.rnu_max - uk.rnu_min) + uk.rnu_min};
                double rr[2];
                batch_recip<2>(dr, rr);
                double num2[C];
                if (MIX & 1) piston_num_tau<C, LW>(a, tau2, num2, lw.lam);
                unit_conc<C>(a, mu, num, rr[0], conc, (MIX & 1) ? num2 : nullptr);
                if (cnan) {
#pragma unroll
                    for (int t = 0; t < kMaxTracer; ++t)
                        if (t < a.K) conc[t] = __builtin_nan("");
                }
                like = mvalid ? unit_like_rtd<C>(uu, mu, ml, conc, &tp, FULL, &rr[1], wvp) : 0.0;
            }
            NGRTD_PROBE(2);
            if (__any(bad)) {                                     // wave-uniform: exact channel sums
                if (DZ && dk.prop_skip) {
                    // the step wrote no global proposal rows: the exact path reads its 64 units'
                    // tau (all of them this wave's lanes) from a.theta = dz_prop, so the lanes put
                    // them there first
                    if (mvalid) const_cast<double*>(a.theta)[(int64_t)a.row_tau[0] * a.U + mu] = tau;
                    __threadfence_block();
                }
                // ROLES = 2: one tile per pass keeps the exact path inside the 128-VGPR budget
                fused_exact<C, FULL, ROLES == 2, MIX>(a, uu, WB, w0, uw, mvalid && bad, mu, ml, tp.nub, conc, like, lw, wvp);
            }
            if (!FULL && a.conc && mvalid) {                      // forward(): model concentrations
#pragma unroll
                for (int t = 0; t < kMaxTracer; ++t)   // unrolled: conc stays in registers
                    if (t < a.K) a.conc[(int64_t)t * a.U + mu] = conc[t];
            }
        }
        NGRTD_PROBE(3);
        if (DZ && kDzPrefetch)   // the next step's partner rows, theta lanes (loads only; zeros elsewhere and
                                 // after the last step: unconditional, so no earlier value stays live)
            dz_partner_rows<kDzMaxP, PFS>(dk, dz_step(dk.sch, js + 1), w0 + mwl, ml, L, W,
                                          mvalid && (PFS == 2 || do_theta) && js + 1 < nst,
                                                do_theta ? 0 : 1, pf1, pf2);
        if (DZ) NGRTD_PROBE(13);
        if (!logp && !dk.lp) return;                        // forward() launch: no log-prob
        if (ROLES == 1) {
            part[pi] = th + like;
        } else {
            if (do_rtd) part2[pi] = like;
            __syncthreads();
            if (do_theta) part[pi] = th + part2[pi];          // th + like, as ROLES = 1
        }
        if (!DZ && uk.unit_out) {   // ngrtd_logp_units: each unit's log-prob, no per-walker sum
            if (do_theta && mvalid) uk.unit_out[mu] = part[pi];
            return;
        }
        NGRTD_PROBE(6);
        // per-well chains decide on their own unit's sum (the theta lane's own part[pi]): no
        // cross-lane read before the decision, so no barrier (the commit barrier follows it)
        if (!PW) __syncthreads();
        if (PW) {   // per-well chains: the unit's own Metropolis decision (its theta lane)
            int a = 0;
            if (dk.dz_diag & 32) {              // timing diagnostics: no decision (all rejected)
                if (do_theta) dec[mi] = 0;
            } else if (do_theta && mvalid) {
                const int64_t wq = w0 + mwl;
                const uint64_t cid = dz_cid(dk.well0, ml, dk.Wg, dk.chain0, wq);
                a = dl.on ? demc_decide_at(dk, dl.lp, dl.lamb, dl.sc, dl.nat, nullptr, false, mi, cid, part[pi],
                                           sj.key, sj.tune_now, (int64_t)js * uk.U, (int64_t)ml * W + wq, false)
                          : demc_decide(dk, wq * (int64_t)L + ml, cid, part[pi], sj.key, sj.tune_now,
                                        (int64_t)js * uk.U, (int64_t)ml * W + wq, false);
                dec[mi] = a;
            }
            if (do_theta && dk.n_acc) {        // the wave's accept count -> LDS (summed after the barrier)
                const unsigned long long m = __ballot(a != 0);
                if (lane == 0) wcnt[uw] = __popcll(m);
            }
        } else if (const int WBc = kFusedUnits / L; WBc <= 64 && (WBc & (WBc - 1)) == 0) {
            // the addition order is the one of WBc = kFusedUnits / L walkers per block whatever
            // WB (<= WBc, a power of two: fused_wb halves WBc), so a walker's log-prob does not
            // depend on the ensemble size (a c5 shard's walkers give the single-GPU run's bits)
            if (wave == 0) {
                const int G = 64 / WBc;                       // well groups (power of two)
                const int wl = lane % WB, g = lane / WB;
                double tot = 0.0;
                if (g < G)
                    for (int l = g; l < L; l += G) tot += part[l * WB + wl];
                for (int off = WB; off < WB * G; off <<= 1) tot += __shfl_xor(tot, off);
                if (g == 0 && w0 + wl < W) walker_out<DZ>(logp, dk, sj, log_off, w0 + wl, tot, dec + wl, dl, wl);
            }
        } else if (tid < WB && w0 + tid < W) {
            double tot = part[tid];
            for (int l = 1; l < L; ++l) tot += part[l * WB + tid];
            walker_out<DZ>(logp, dk, sj, log_off, w0 + tid, tot, dec + tid, dl, tid);
        }
        if (DZ) {
            NGRTD_PROBE(10);
            __syncthreads();
            NGRTD_PROBE(11);
            if (PW && dk.n_acc && tid == 0) {  // one accept-count atomic per block and step
                int n = 0;
#pragma unroll
                for (int i = 0; i < kFusedWaves; ++i) n += wcnt[i];
                if (n) atomicAdd(dk.n_acc, (unsigned long long)n);
            }
            if (mvalid && dec[PW ? mi : mwl] && !(dk.dz_diag & 4)) {
                dz_commit<kDzMaxP, (MIX & 4) != 0>(dk, uk.U, mu, mi, thl, do_theta ? 0 : 1,
                                                   dk.prop_lds ? propl : nullptr, dl);
                moved = true;
            }
            NGRTD_PROBE(12);
        } else if (dk.lp) {   // DE-MC: accepted walkers take the proposal's theta rows of this unit
            __syncthreads();
            if (do_theta && mvalid && dec[mwl]) {
                for (int p = 0; p < dk.P; ++p) dk.x[(int64_t)p * a.U + mu] = dk.prop[(int64_t)p * a.U + mu];
                if (dk.xu)
                    for (int p = 0; p < dk.P; ++p) dk.xu[(int64_t)p * a.U + mu] = dk.prop_u[(int64_t)p * a.U + mu];
            }
        }
    } while (DZ && ++js < nst);   // steps
    if (DZ && dacc.state_lds) {   // the LDS state back: the rows of the units that moved, every chain's scalars
        __syncthreads();
        const double* st = thl + ((MIX & 4) ? dacc.P * kFusedUnits : 0) + (dacc.prop_lds ? dacc.P * kFusedUnits : 0);
        const int dwl = mi / L, dml = mi % L;
        const bool dv = dwl < WB && w0 + dwl < W;
        const int64_t du = dv ? (w0 + dwl) * (int64_t)L + dml : 0;
        if (moved && dv)
            for (int p = do_theta ? 0 : 1; p < dacc.P; p += 2) {
                const double v = st[p * kFusedUnits + mi];
                const int64_t gi = (int64_t)p * ua.U + du;
                if (MIX & 4) {   // transformed chains: u, and the natural value dz_stage derived from it
                    dacc.xu[gi] = v;
                    dacc.x[gi] = pymc3_backward_sel(dacc.tr_kind[p], dacc.tr_a[p], dacc.tr_b[p], v);
                } else {
                    dacc.x[gi] = v;
                }
            }
        const double* c = st + dacc.P * kFusedUnits;
        const int32_t* cn = reinterpret_cast<const int32_t*>(c + 3 * kFusedUnits);
        const bool own = PW ? (do_theta && dv) : (tid < WB && w0 + tid < W);
        const int sl = PW ? mi : tid;
        const int64_t gi = PW ? du : w0 + tid;
        if (own) {
            dacc.lp[gi] = c[sl];
            dacc.lamb[gi] = c[kFusedUnits + sl];
            dacc.scaling[gi] = c[2 * kFusedUnits + sl];
            if (dacc.n_acc_tune) dacc.n_acc_tune[gi] = cn[sl];
        }
    }
    NGRTD_PROBE(7);
}

// logp[w] = sum over wells of ulogp[l*W + w]: 16 fixed well groups per walker summed
// in registers, then combined in a fixed order through LDS (deterministic, no atomics).
NGRTD_KLINK __global__ void __launch_bounds__(1024) walker_reduce_kernel(const double* __restrict__ ulogp, int64_t W,
                                                             int32_t L, double* __restrict__ logp) {
    __shared__ double sh[16][64];
    const int wl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t w = (int64_t)blockIdx.x * 64 + wl;
    double s = 0.0;
    if (w < W)
        for (int l = g; l < L; l += 16) s += ulogp[(int64_t)l * W + w];
    sh[g][wl] = s;
    __syncthreads();
    if (g == 0 && w < W) {
        double t = sh[0][wl];
        for (int i = 1; i < 16; ++i) t += sh[i][wl];
        logp[w] = t;
    }
}

// ------------------------------------------ gen_g_tp() materialised weights
// One block computes the unnormalised weights, a fixed-order block sum, then g /= sum.
NGRTD_KLINK __global__ void __launch_bounds__(1024) rtd_weights_kernel(int32_t mod, double tau, double eta, double D,
                                                           double tp0, double dtp, int32_t N, double* g) {
    __shared__ double red[1024];
    double s = 0.0;
    int ixp = 0;
    if (mod == MOD_PISTON) ixp = piston_index(tau, tp0, dtp, N);
    const double thr = tau * (1 - (1 / eta));
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const double tp = (k == 0) ? tp0 : ((double)k + dtp);
        double w;
        if (mod == MOD_PISTON) {
            w = (k == ixp) ? 1. : 0.;
        } else if (mod == MOD_EXP) {
            w = (1. / tau) * exp(-tp / tau);
        } else if (mod == MOD_EPM) {
            w = (tp >= thr) ? (eta / tau) * exp(-(eta * tp / tau) + eta - 1.) : 0.0;
        } else {
            const double x = tp / tau;
            const double f1 = (1. / tau) / (sqrt(4. * kPi * D * x));
            const double f2 = (1. / x) * exp(-1. * (((1. - x) * (1. - x)) / (4. * D * x)));
            w = f1 * f2;
        }
        g[k] = w;
        s += w;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    const double tot = red[0];
    for (int k = threadIdx.x; k < N; k += blockDim.x) g[k] = g[k] / tot;
}

// convolve(g_tau=g), :298-340: dot(flip(C'), g * decay) with a fixed-order block sum
NGRTD_KLINK __global__ void __launch_bounds__(1024) conv_dot_kernel(const double* c, const double* idx, const double* g,
                                                        double lam, int32_t accum, double J, double tp0,
                                                        double dtp, int32_t N, double* out) {
    __shared__ double red[1024];
    double s = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const double tp = (k == 0) ? tp0 : ((double)k + dtp);
        const double gd = (accum == NGRTD_ACC_HE3) ? g[k] * (1 - exp(-lam * tp)) : g[k] * exp(-lam * tp);
        const double cv = (accum == NGRTD_ACC_HE4 || accum == NGRTD_ACC_SF6) ? c[k] + idx[k] * J : c[k];
        s = fma(cv, gd, s);
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

}  // namespace ngrtd
