// ngrtd_frac.hpp -- gfx950 kernels of the fracture / matrix-diffusion RTD 'frac_inf_diff'
// (utils/convolution_integral_utils.py:238-266).
//
// For every age tp_i the reference integrates over a 1000-point log-spaced advective-time
// grid (frac_rtd_numba_disp :36-65, or frac_rtd_numba :67-97 with an external advective
// RTD):
//
//   tadv_j  = logspace(-6, log10(tp_i - 1e-6), 1000)_j
//   f_ret_j = kappa beta_j / (2 sqrt(pi) t_ret_j^1.5) exp(-kappa^2 beta_j^2 / (4 t_ret_j)),
//             t_ret_j = tp_i - tadv_j,  beta_j = tadv_j / bbar
//   f(tp_i) = trapz(f_ret f_tadv, tadv) / trapz(f_ret[::-1], t_ret[::-1])
//
// i.e. N x 1000 points per parameter set with 3 transcendentals, 2 square roots and ~6
// divisions each -- the only compute-heavy RTD of the reference (numba there).
//
//   frac_inner_kernel  one wavefront per (set, age): lane l owns grid points j = 64 k + l,
//                      the trapezoid pairs (j-1, j) take their left neighbour from lane
//                      l-1 (a shuffle) or, for lane 0, from lane 63 of the previous k; both
//                      sums are wave-reduced in a fixed order.  FP64 VALU-bound.
//   frac_finish_kernel one block per set: f[0] = 0, trapz normalisation over tp_ (tp_[0] =
//                      0), the mean travel time FM_mu, g /= g.sum() (:257-270), then the
//                      convolve() dot product with decay / accumulation (:305-340).
#pragma once
#include <hip/hip_runtime.h>
#include "ngrtd_math.hpp"
#include "../../include/ngrtd.h"

namespace ngrtd {

constexpr int kFracPts = 1000;          // logspace(..., 1000), :48 / :83
constexpr int kFracWaves = 4;           // waves (ages) per block of frac_inner_kernel

struct FracArgs {
    const double *tau, *D, *bbar, *Phi;   // per set (tau / D unused with ext)
    const double* ext;                    // f_tadv_ext rows (age order), or nullptr
    int64_t ext_stride;                   // 0: one row shared by every set
    double tp0, dtp;
    int32_t N;
    int64_t n;                            // sets; this launch covers p0 .. p0 + (waves / N) - 1
    int64_t p0, waves;
    double* f;                            // [n][N] inner integrals f_t_tran
};

// lane l <- lane l-1 of v, lane 0 <- c: DPP wave_shr:1 (a VALU operand modifier on gfx9-family
// gfx950, no LDS crossbar), per 32-bit half
__device__ __forceinline__ double shr1_or(double v, double c) {
    const unsigned long long vb = __double_as_longlong(v), cb = __double_as_longlong(c);
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)cb, (int)(unsigned)vb, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(cb >> 32), (int)(unsigned)(vb >> 32), 0x138, 0xf, 0xf,
                                               false);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// lane 63's value in every lane (v_readlane: VALU -> SGPR, no LDS)
__device__ __forceinline__ double bcast63(double v) {
    const unsigned long long vb = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)vb, 63);
    const int hi = __builtin_amdgcn_readlane((int)(unsigned)(vb >> 32), 63);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// np.interp(x, tp[:i+1], fp[:i+1]) on the uniform age grid tp_k = k + dtp (tp_0 = tp0):
// numpy's linear interpolation with its exact-knot and NaN-retry rules.
__device__ __forceinline__ double interp_age(double x, const double* fp, int i, double tp0, double dtp) {
    if (!(x >= tp0)) return (x == x) ? fp[0] : x;   // left of the grid: fp[0]; NaN x -> NaN
    double kf = floor(x - dtp);
    int j = (kf < 0.0) ? 0 : (kf > (double)i ? i : (int)kf);
    auto tpk = [&](int k) { return k == 0 ? tp0 : (double)k + dtp; };
    while (j < i && tpk(j + 1) <= x) ++j;
    while (j > 0 && tpk(j) > x) --j;
    if (j >= i) return fp[i];                        // x >= tp_i: right value
    const double xj = tpk(j);
    if (xj == x) return fp[j];
    const double slope = (fp[j + 1] - fp[j]) / (tpk(j + 1) - xj);
    double r = slope * (x - xj) + fp[j];
    if (r != r) {
        r = slope * (x - tpk(j + 1)) + fp[j + 1];
        if (r != r && fp[j] == fp[j + 1]) r = fp[j];
    }
    return r;
}

__global__ void __launch_bounds__(64 * kFracWaves) frac_inner_kernel(const FracArgs a) {
    fm_lds_init();                                 // fexp / fexp10 tables (before any exit)
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * kFracWaves + (threadIdx.x >> 6);
    const int64_t pl = gw / a.N;
    const int i = (int)(gw - pl * a.N);
    const int64_t p = a.p0 + pl;
    if (gw >= a.waves || p >= a.n) return;         // whole wave exits together
    const double tp_i = (i == 0) ? a.tp0 : (double)i + a.dtp;
    const double bbar = a.bbar[p];
    const double Phi_im = a.Phi[p];
    // :245-248 -- D_o = (2.3e-9)*60*60*24*365 (left to right), R_im = 1
    const double D_o = 2.3e-9 * 60 * 60 * 24 * 365;
    const double kappa = Phi_im * sqrt((D_o * (Phi_im * Phi_im)) * 1);
    const double k2 = -1 * (kappa * kappa);
    const double* ext = a.ext ? a.ext + p * a.ext_stride : nullptr;
    const double tau = ext ? 1.0 : a.tau[p];
    const double D = ext ? 1.0 : a.D[p];
    const double inv_tau = 1. / tau;
    const double c4piD = 4. * kPi * D;
    const double c4D = 4. * D;
    const double c2spi = 2 * 1.7724538509055159;   // 2*np.sqrt(np.pi)
    const double kc = kappa / c2spi;
    const double inv_bbar = 1.0 / bbar;
    // numpy logspace(-6, stop, 1000) = 10 ** linspace(-6, stop, 1000):
    // y_j = j * step + start, y_999 = stop (step = (stop - start) / 999; step == 0 -> j/999*delta)
    const double start = -6.0;
    const double stop = log10(tp_i - 1.e-6);
    const double delta = stop - start;
    const double step = delta / (kFracPts - 1);
    double s_norm = 0.0, s_int = 0.0;
    double c_t = 0.0, c_fr = 0.0, c_ta = 0.0, c_fi = 0.0;   // lane-63 values of the previous k
#pragma unroll 1
    for (int k = 0; k < (kFracPts + 63) / 64; ++k) {
        const int j = k * 64 + lane;
        const double jd = (double)j;
        double y = (step == 0.0) ? (jd / (kFracPts - 1)) * delta + start : jd * step + start;
        if (j == kFracPts - 1) y = stop;
        // np.power(10.0, y): fexp10 is < 0.51 ulp (t_ret below cancels against tadv)
        const double tadv = fexp10(y);
        double f_tadv;
        if (ext) {
            f_tadv = interp_age(tadv, ext, i, a.tp0, a.dtp);
        } else {
            // ((1/tau)/sqrt(4 pi D x)) (1/x) exp(-(1-x)^2/(4 D x)), x = tadv/tau: the two
            // prefactor divisions merged and x by the hoisted 1/tau (a few ulp; 2 divisions)
            const double x = tadv * inv_tau;
            f_tadv = (inv_tau / (sqrt(c4piD * x) * x)) * fexp(-1. * (((1. - x) * (1. - x)) / (c4D * x)));
        }
        // kappa beta / (2 sqrt(pi) t^1.5) exp(-kappa^2 beta^2 / (4 t)), beta = tadv/bbar:
        // ONE division 1/(t sqrt t) gives both t^-1.5 and 1/t = sqrt(t) / (t sqrt t)
        const double t_ret = tp_i - tadv;
        const double beta = tadv * inv_bbar;
        const double st = sqrt(t_ret);
        const double it15 = 1.0 / (t_ret * st);
        const double f_ret = (kc * beta) * it15 * fexp((k2 * (beta * beta)) * (0.25 * (st * it15)));
        const double fi = f_ret * f_tadv;
        // left neighbour (j - 1): lane - 1 of this k, or lane 63 of the previous k
        const double l_t = shr1_or(t_ret, c_t), l_fr = shr1_or(f_ret, c_fr);
        const double l_ta = shr1_or(tadv, c_ta), l_fi = shr1_or(fi, c_fi);
        if (j >= 1 && j < kFracPts) {
            s_norm += (l_t - t_ret) * (l_fr + f_ret);      // trapz(f_ret[::-1], t_ret[::-1])
            s_int += (tadv - l_ta) * (fi + l_fi);          // trapz(f_ret * f_tadv, tadv)
        }
        c_t = bcast63(t_ret); c_fr = bcast63(f_ret); c_ta = bcast63(tadv); c_fi = bcast63(fi);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        s_norm += __shfl_xor(s_norm, off, 64);
        s_int += __shfl_xor(s_int, off, 64);
    }
    // f_ret / trapz_norm then trapz(f_i): (0.5 s_int) / (0.5 s_norm)
    if (lane == 0) a.f[p * a.N + i] = (0.5 * s_int) / (0.5 * s_norm);
}

struct FracFinish {
    const double* c;         // series by age
    const double* idx;       // series index by age (4He / SF6 accumulation)
    const double* t_half;    // per set or nullptr
    double t_half_c;
    const double* J;         // per set or nullptr
    double J_c;
    int32_t accum;
    double tp0, dtp;
    int32_t N;
    int64_t n;
    double* f;               // [n][N] in: f_t_tran, out: g (normalised weights)
    double* conc;            // [n] or nullptr
    double* fm;              // [n] or nullptr
};

// fixed-order block sum (256 threads)
__device__ __forceinline__ double block_sum256(double v, double* red) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) frac_finish_kernel(const FracFinish a) {
    __shared__ double red[4];
    const int64_t p = blockIdx.x;
    if (p >= a.n) return;
    double* f = a.f + p * a.N;
    const int N = a.N;
    auto tpu = [&](int k) { return k == 0 ? 0.0 : (double)k + a.dtp; };   // tp_ (tp_[0] = 0), :259-260
    // :261 -- f_t_tran[0] = 0; f /= np.trapz(f, tp_)  (d * (y1 + y0) / 2.0)
    double s = 0.0;
    for (int k = threadIdx.x; k < N - 1; k += 256) {
        const double y0 = (k == 0) ? 0.0 : f[k];
        s += ((tpu(k + 1) - tpu(k)) * (f[k + 1] + y0)) / 2.0;
    }
    const double T = block_sum256(s, red);
    // :262-263 -- FM_mu = trapz(g tp_, tp_) / trapz(g, tp_) on the normalised f;  :270 g.sum()
    double s_num = 0.0, s_den = 0.0, s_sum = 0.0;
    for (int k = threadIdx.x; k < N; k += 256) {
        const double gk = ((k == 0) ? 0.0 : f[k]) / T;
        s_sum += gk;
        if (k < N - 1) {
            const double g1 = f[k + 1] / T;
            const double d = tpu(k + 1) - tpu(k);
            s_num += (d * (g1 * tpu(k + 1) + gk * tpu(k))) / 2.0;
            s_den += (d * (g1 + gk)) / 2.0;
        }
    }
    const double S = block_sum256(s_sum, red);
    const double num = block_sum256(s_num, red);
    const double den = block_sum256(s_den, red);
    // g = (f / T) / S, then convolve(): decay / accumulation and the flipped dot (:305-340)
    const double th = a.t_half ? a.t_half[p] : a.t_half_c;
    const double lam = (th != 0.0) ? -1 * log(0.5) / th : 0.0;
    const double J = a.J ? a.J[p] : a.J_c;
    double dot = 0.0;
    for (int k = threadIdx.x; k < N; k += 256) {
        const double g = (((k == 0) ? 0.0 : f[k]) / T) / S;
        f[k] = g;                                  // each thread reads and writes only its own k
        const double tp = (k == 0) ? a.tp0 : (double)k + a.dtp;
        const double gd = (a.accum == NGRTD_ACC_HE3) ? g * (1 - exp(-lam * tp)) : g * exp(-lam * tp);
        const double cv = (a.accum == NGRTD_ACC_HE4 || a.accum == NGRTD_ACC_SF6) ? a.c[k] + a.idx[k] * J : a.c[k];
        dot = fma(cv, gd, dot);
    }
    const double conc = block_sum256(dot, red);
    if (threadIdx.x == 0) {
        if (a.conc) a.conc[p] = conc;
        if (a.fm) a.fm[p] = num / den;
    }
}

}  // namespace ngrtd
