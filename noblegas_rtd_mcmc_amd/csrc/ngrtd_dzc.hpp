// ngrtd_dzc.hpp -- DEMetropolisZ for the reference's own model shapes in ONE launch per
// <= 256 steps: the RTD-only model (run_age_mcmc_utils.py:275-397: 1 or 4 tracers, the
// published exponential / exp_pist_flow (+ piston) RTDs, savenum 0 or 123) and the CE-only
// model (ng_interp/noble_gas_mcmc.py:216-267), each well its own chain (per-well chains,
// DemcAccept::per_well), natural or PyMC3's transformed space.
//
// logp_fused_kernel's DEMetropolisZ step splits a unit over a theta wave and an RTD wave of
// the joint model (the CE block and the RTD block are both heavy there) and exchanges through
// LDS behind barriers.  In these models one block is light (the RTD model's priors; the CE
// model has no RTD block), so here ONE lane runs one chain for the whole launch: its state,
// lamb, scaling, tuning counter and log-prob stay in registers, it loads its two partner
// rows, appends its state to the history, forms the proposal, evaluates the proposal's
// log-prob (the same functions and arithmetic as the log-prob kernels -- so the chains
// equal the torch restatement on ngrtd_logp_units bit for bit), decides and tunes, with no
// barrier inside the step loop at all (chains exchange nothing).  The tables (surrogate
// window, EPM channel table, per-well data, fexp/flog) are staged in LDS once per launch.
//
// The log-prob functions read theta rows through a pointer: the lane writes its proposal's
// natural values to its own LDS slot of a [P][NT] block (a.theta / ua.theta point there,
// U = NT, unit index = slot) and reads them back in the same lane (program order).  The one
// exception is the exact matrix-core fallback (dzc_exact): its MFMA tiles read the tau rows
// of all 64 lanes of the wave.  A wave's LDS accesses complete in issue order, so those rows
// are the ones the lanes just wrote; a wave barrier before the fallback keeps the compiler
// from moving its loads above the other lanes' stores.
#pragma once
#include "ngrtd_kernels.hpp"

namespace ngrtd {

constexpr int kDzcMaxP = 8;        // parameter rows of a lane-chain step
// threads per block: 512, so that the c4 shape's 2048 x 64 chains fill all 256 CUs with one
// block each (2 waves per SIMD; 1024-lane EPM blocks left half the CUs idle: 32.0 us per step,
// profiles/r04i_bench.json) -- and each lane may hold up to 256 VGPRs (the chain's state, the
// next step's partner rows and the log-prob body without spills; 128 spilled up to 46)
__host__ __device__ constexpr int dzc_threads(int) { return 512; }
// LDS doubles: the surrogate window, the EPM table, the per-well data, the proposal rows
// (epm_nw: the EPM table rows staged, RtdArgs::epm_nw)
__host__ __device__ constexpr size_t dzc_lds_doubles(int C, int mix, int cheb_np, int epm_nw, int wd_n, int P) {
    return (size_t)cheb_np * cheb_lds_stride(C) + ((mix & 2) ? (size_t)epm_lds_doubles(epm_nw, cheb_cp(C)) : 0) +
           (size_t)((wd_n + 1) & ~1) + (size_t)P * dzc_threads(mix) + 64;   // (+ the theta parts [64])
}

// Exact (matrix-core) channel sums of the wave's 64 lanes (slots slot0 + 0..63) as 4 tiles
// of 16, then the concentrations and RTD likelihood of the lanes that need them (fused_exact's
// arithmetic; a.theta holds the slots' rows).
template <int C, int MIX>
__device__ __forceinline__ void dzc_exact(const RtdArgs& a, const UnitArgs& ul, int slot0, bool mine, int slot, int ml,
                                          double nub, double* conc, double& like, LwDecay lw) {
    constexpr bool LW = (MIX & 32) != 0;
    constexpr int NT = mfma_tiles(C);
    const int col = threadIdx.x & 15, tq = (threadIdx.x & 63) >> 4;
    double yy[C], bu = 0.0, yw = 0.0, bw = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c) yy[c] = 0.0;
#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
        const int64_t uo = slot0 + 16 * t + col;
        MfmaWave<C, 1> mw;
        mw.init(a, &uo);
        mw.steps(a.frag, a.nsteps);
        double y[1][C];
        mw.finish(a, y);
        if (t == tq) {
            bu = mw.beta[0];
#pragma unroll
            for (int c = 0; c < C; ++c) yy[c] = y[0][c];
        }
        if (LW) {
            const double tv = __shfl(lw.teff, 16 * t + col, 64);
            MfmaWave<C, 1> mv;
            mv.init_tau(&tv);
            mv.steps(a.frag, a.nsteps);
            double y2[1][C];
            mv.finish(a, y2);
            if (t == tq) {
                yw = y2[0][0];
                bw = mv.beta[0];
            }
        }
    }
    if (mine) {
        ThetaPre tp;
        tp.nub = nub;
        double num2[C];
        if (MIX & 1) piston_num<C, LW>(a, slot, num2, lw.lam);
        mfma_unit_conc<C, LW, true>(a, slot, bu, yy, conc, (MIX & 1) ? num2 : nullptr, lw.lam, yw, bw);
        like = unit_like_rtd<C>(ul, slot, ml, conc, &tp, false);
    }
}

// The RTD block's likelihood of the lane's proposal (logp_fused_kernel's RTD role, non-FULL):
// exponential (surrogate, exact matrix-core fallback for uncovered lanes) or exp_pist_flow
// (epm_sums), optionally with a piston second component and the sampled CFC12 half-life.
template <int C, int MIX>
__device__ __forceinline__ double dzc_rtd_like(const RtdArgs& a, const UnitArgs& ul, const double* cheb,
                                               const double* tabl, bool valid, int slot, int slot0, int ml, double tau,
                                               double eta, double tau2, double thx, double nub) {
    constexpr bool EPM = (MIX & 2) != 0, LW = (MIX & 32) != 0;
    constexpr int CP = cheb_cp(C), PST = cheb_lds_stride(C);
    ThetaPre tp;
    tp.nub = nub;
    double conc[kMaxTracer];
    double like = 0.0;
    if (EPM) {
        double num[C], dn, dd, lam = 0.0;
        bool wnan;
        epm_sums<C, kEpmTailPreDz, LW>(a, tabl, valid, tau, eta, num, dn, dd, thx, &lam, &wnan);
        const double dr[2] = {dn, nub * (ul.rnu_max - ul.rnu_min) + ul.rnu_min};
        double rr[2];
        batch_recip<2>(dr, rr);
        double num2[C];
        if (MIX & 1) {
            const int ix = piston_index(tau2, a.tp0, a.dtp, a.N);
            epm_piston_row<C>(a, tabl, ix, num2);
            if (LW) num2[0] *= fexp(-lam * (ix == 0 ? a.tp0 : (double)ix + a.dtp));
        }
        unit_conc<C, true>(a, slot, num, dd * rr[0], conc, (MIX & 1) ? num2 : nullptr);
        if (wnan)
            for (int t = 0; t < C; ++t)
                if (t < a.K) conc[t] = __builtin_nan("");
        like = valid ? unit_like_rtd<C>(ul, slot, ml, conc, &tp, false, &rr[1]) : 0.0;
        return like;
    }
    double cx = 0.0;
    int cpc = a.cheb ? cheb_piece(tau, cx) - a.cheb_p0 : -1;
    cpc = (unsigned)cpc < (unsigned)a.cheb_np ? cpc : -1;
    LwDecay lw{0.0, 0.0};
    double cxw = 0.0;
    int cpw = 0;
    if (LW) {
        lw = lw_decay(a, tau, thx);
        cpw = a.cheb ? cheb_piece(lw.teff, cxw) - a.cheb_p0 : -1;
        cpw = (unsigned)cpw < (unsigned)a.cheb_np ? cpw : -1;
    }
    const bool unc = cpc < 0 || (LW && cpw < 0);
    bool skip = false, cnan = false;
    const bool prior_on = ul.rtd_on && (ul.flags & NGRTD_WANT_PRIOR);
    if (unc && a.cheb && prior_on && a.row_tau[0] == ul.row_tau1 && !(tau >= ul.tau1_lo && tau <= ul.tau1_hi) &&
        !(ul.tau1_lo < kChebTauLo && tau >= ul.tau1_lo)) {
        skip = true;
        cnan = exp_rtd_nan(a, tau);
    }
    if (LW && unc && !skip && a.cheb && prior_on && a.row_thalf == ul.row_thalf && !(thx >= 0.0 && thx <= 1.0)) {
        skip = true;
        cnan = !(thx == thx) || exp_rtd_nan(a, tau);
    }
    const bool bad = unc && !skip;
    cpc = cpc < 0 ? 0 : cpc;
    cpw = cpw < 0 ? 0 : cpw;
    double zz[C + 1];
    cheb_sums<C + 1, true>(cheb + cpc * PST, CP, cx, zz);
    double zw = 0.0;
    if (LW) cheb_sums<1, true>(cheb + cpw * PST, CP, cxw, &zw);
    {
        double num[C];
#pragma unroll
        for (int c = 0; c < C; ++c) num[c] = a.tab0[c] + zz[c];
        if (LW) num[0] = fexp(-lw.lam * a.tp0) * (a.tab0[0] + zw);
        const double dr[2] = {1.0 + zz[C], nub * (ul.rnu_max - ul.rnu_min) + ul.rnu_min};
        double rr[2];
        batch_recip<2>(dr, rr);
        double num2[C];
        if (MIX & 1) piston_num_tau<C, LW>(a, tau2, num2, lw.lam);
        unit_conc<C, true>(a, slot, num, rr[0], conc, (MIX & 1) ? num2 : nullptr);
        if (cnan)
            for (int t = 0; t < a.K; ++t) conc[t] = __builtin_nan("");
        like = valid ? unit_like_rtd<C>(ul, slot, ml, conc, &tp, false, &rr[1]) : 0.0;
    }
    if (__any(bad)) {
        __builtin_amdgcn_wave_barrier();                  // the wave's proposal rows (see the header)
        dzc_exact<C, MIX>(a, ul, slot0, valid && bad, slot, ml, nub, conc, like, lw);
    }
    return like;
}

// Kernel arguments at their natural alignment (RtdArgs at 0, UnitArgs, DemcAccept), read in
// the step loop through the opaque kernarg pointer (kernarg_opaque: otherwise every field is
// hoisted out of the loop into registers)
constexpr size_t kDzcArgU = ka_align(sizeof(RtdArgs), alignof(UnitArgs));
// Probe build (tools/dzc_probe.py --sections): shader-clock cycles per section of the step,
// summed over the launch's steps, lane 0 of each wave -> g_probe[wave][0..5], steps at [6]
#ifdef NGRTD_SECTION_PROBE
#define DZC_MARK(k)                                                                           \
    do {                                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
        pacc[k] += t_ - pt_;                                                                 \
        pt_ = t_;                                                                            \
    } while (0)
#else
#define DZC_MARK(k) do {} while (0)
#endif
constexpr size_t kDzcArgD = ka_align(kDzcArgU + sizeof(UnitArgs), alignof(DemcAccept));

// One lane = one per-well chain (unit (w, l), walker-major: slot i of block b is unit
// b nth + i = w L + l, nth = blockDim.x <= NT threads).  C: RTD channels (0 for the CE-only model); MIX: 1 piston second
// component, 2 exp_pist_flow first component, 4 PyMC3's transformed space (the plan carries
// the Jacobians), 32 the sampled CFC12 half-life, 64 the CE-only model (no RTD block).
// State arrays as logp_fused_kernel's DZ instances: dacc.zx the chains'-space rows and
// dacc.x / dacc.xu the natural / transformed rows ([P][W][L], walker-major), the per-chain
// lp / lamb / scaling / tuning counters [W][L]; logs [n_steps][L][W].
template <int C, int MIX, bool TW = false>
__global__ void __launch_bounds__(dzc_threads(MIX), 2)
    dz_chain_kernel(const RtdArgs ak, const UnitArgs ua, const DemcAccept dacc) {
    constexpr int NT = dzc_threads(MIX);
    constexpr bool EPM = (MIX & 2) != 0, TR = (MIX & 4) != 0, LW = (MIX & 32) != 0, CEO = (MIX & 64) != 0;
    constexpr int CC = CEO ? 1 : C;                       // (table geometry of the CE-only model: unused)
    constexpr int CP = cheb_cp(CC), PST = cheb_lds_stride(CC);
    static_assert(CEO || (C >= 1 && C <= 5), "RTD channels");
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int tid = threadIdx.x;
    const int nth = blockDim.x;                           // <= NT: small ensembles launch fewer waves
    const RtdArgs& a0 = ak;
    // ---- prologue: tables -> LDS, once per launch
    double* cheb = lds;
    double* tabl = cheb + (CEO ? 0 : a0.cheb_np * PST);
    double* wd = tabl + ((!CEO && EPM) ? epm_lds_doubles(a0.epm_nw, CP) : 0);
    double* props = wd + ((ua.wd_n + 1) & ~1);            // [P][NT] the lanes' proposals (natural)
    double* thl = props + (size_t)dacc.P * NT;            // [64] theta parts (dacc.theta_wave)
    if constexpr (!CEO) {
        if (a0.cheb) {
        const int n = a0.cheb_np * (kChebN * CP / 2);
        const double2* src = reinterpret_cast<const double2*>(a0.cheb + (size_t)a0.cheb_p0 * kChebN * CP);
        double2* dst = reinterpret_cast<double2*>(cheb);
#pragma unroll 8
        for (int i = tid; i < n; i += nth) dst[(i / (kChebN * CP / 2)) * (PST / 2) + i % (kChebN * CP / 2)] = src[i];
        }
    }
    if constexpr (!CEO && EPM) {
        const int nrow = a0.epm_nw;                      // (a windowed table: its rows only)
#pragma unroll 8   // (loads batched ahead of the stores: one wave stages alone for small ensembles)
        for (int i = tid; i < nrow * CP; i += nth) {
            const int k = i / CP, c = i % CP;
            tabl[epm_row(k, CP) + c] = (k < a0.N && c < C) ? a0.tab[(int64_t)k * a0.CP + c] : 0.0;
        }
    }
#pragma unroll 8
    for (int i = tid; i < ua.wd_n; i += nth) wd[i] = ua.wd_src[i];
    fm_lds_init();
    __syncthreads();
    // ---- the lane's chain.  TW (dacc.theta_wave: <= 64 chains, 128 threads): wave 0 runs the
    // chains, wave 1 lane i evaluates the theta part of lane i's proposal each step (between two
    // block barriers) while wave 0 evaluates the RTD likelihood -- the two halves of a step's
    // log-prob depend only on the proposal, and one lane ran them one after the other.  Its own
    // instances: the extra paths cost the plain ones registers (spills, 2-5 % per c4 step)
    constexpr bool thw = TW;
    const bool helper = thw && tid >= 64;                 // (wave-uniform)
    const int cl = helper ? tid - 64 : tid;               // the chain lane this lane serves
    const int cpb = thw ? 64 : nth;                       // chains per block
    const int L = ua.L;
    const int64_t W = ua.W, U = (int64_t)L * W;
    const int64_t g = (int64_t)blockIdx.x * cpb + cl;
    const bool valid = g < U;
    const int64_t gv = valid ? g : U - 1;                 // a lane past the end shadows the last unit, stores nothing
    const int64_t w = gv / L;
    const int l = (int)(gv % L);
    const int P = dacc.P;
    const int slot0 = cl & ~63;
    const uint64_t cid = dz_cid(dacc.well0, l, dacc.Wg, dacc.chain0, w);
    double x[kDzcMaxP];                                   // the chain's state (its own space)
#pragma unroll
    for (int p = 0; p < kDzcMaxP; ++p) x[p] = p < P ? dacc.zx[(int64_t)p * U + gv] : 0.0;
    double lp = dacc.lp[gv], lamb = dacc.lamb[gv], sc = dacc.scaling[gv];
    int32_t nat = dacc.n_acc_tune ? dacc.n_acc_tune[gv] : 0;
    unsigned long long nacc = 0;
    const int nst = dacc.n_steps;
    // Step j's partner entries (keyed by the walker, each well reading its own history rows) and
    // their rows, loaded one step ahead: step j + 1's loads are issued right after step j's
    // proposal, so they land during its log-prob.  Every entry they read was appended by this
    // lane earlier in program order, except step j + 1's own append (the state after step j's
    // decision), which the c1 / c2 substitution below takes from the registers.
    int64_t e1 = -1, e2 = -1;
    double a1[kDzcMaxP], a2[kDzcMaxP];
    auto partner_rows = [&](const DemcAccept& d, int j) {
        const bool on = j < nst;
        const DzStep sp = dz_step(d.sch, on ? j : 0);
        dz_partners(d, sp, w, e1, e2);
        const bool de = on && e1 >= 0;
        const int64_t R = (int64_t)P * L;
        const double* z1 = d.hist + ((size_t)(de ? e1 : 0) * W + w) * R + l;
        const double* z2 = d.hist + ((size_t)(de ? e2 : 0) * W + w) * R + l;
#pragma unroll
        for (int p = 0; p < kDzcMaxP; ++p) {
            a1[p] = (de && p < P) ? z1[(int64_t)p * L] : 0.0;
            a2[p] = (de && p < P) ? z2[(int64_t)p * L] : 0.0;
        }
    };
    partner_rows(dacc, 0);
#ifdef NGRTD_SECTION_PROBE
    unsigned long long pacc[6] = {0, 0, 0, 0, 0, 0}, pt_ = __builtin_amdgcn_s_memtime();
#endif
    for (int js = 0; js < nst; ++js) {
        const RtdArgs& a = kernarg_opaque<RtdArgs>(0);
        const UnitArgs& uk = kernarg_opaque<UnitArgs>(kDzcArgU);
        const DemcAccept& d = kernarg_opaque<DemcAccept>(kDzcArgD);
        const DzStep sj = dz_step(d.sch, js);
        // timing diagnostics (NGRTD_DZ_DIAG, tools/dzc_probe.py; wrong results): bit 6 no RTD
        // likelihood, 7 no theta part, 8 no logs, 9 no history append, 10 no partner rows, 11 no
        // backward transform of the proposal, 12 no proposal (the state), 13 no tuning, 14 no
        // Metropolis draw (logu = 0)
        const int dg = d.dz_diag;
        const bool de = e1 >= 0 && !(dg & 1024);
        const int64_t R = (int64_t)P * L;
        // the state becomes history entry sj.at (chains' space)
        if (!helper && valid && sj.at >= 0 && !(dg & 512)) {
            double* hrow = d.hist + ((size_t)sj.at * W + w) * R + l;
#pragma unroll
            for (int p = 0; p < kDzcMaxP; ++p)
                if (p < P) hrow[(int64_t)p * L] = x[p];
        }
        DZC_MARK(0);                                      // schedule + history append
        const bool c1 = e1 == sj.at, c2 = e2 == sj.at;    // an entry appended in this launch is the state
        const uint64_t ke = rng_mix(sj.key + 2);
        double v[kDzcMaxP];
#pragma unroll
        for (int p = 0; p < kDzcMaxP; ++p) {
            if (p < P && !helper) {
                const double sr = d.S ? d.S[(int64_t)p * L + l] : 1.0;
                v[p] = (dg & 4096) ? x[p]
                                   : dz_value_core(de, x[p], c1 ? x[p] : a1[p], c2 ? x[p] : a2[p], lamb, sc, ke,
                                                   dz_pw_elem(cid, p), d.S != nullptr, sr);
                props[p * NT + tid] = (TR && !(dg & 2048)) ? pymc3_backward(d.tr_kind[p], d.tr_a[p], d.tr_b[p], v[p]) : v[p];
            } else {
                v[p] = 0.0;
            }
        }
        DZC_MARK(1);                                      // proposal values, natural rows -> LDS
        if (!helper) partner_rows(d, js + 1);             // the next step's partners (in flight from here)
        if (thw) __syncthreads();                         // the proposal rows -> the theta wave
        DZC_MARK(2);
        // the proposal's log-prob: the log-prob kernels' functions over the LDS rows
        RtdArgs ar = a;   // (from the by-value parameter: no gain, profiles/r06w_dzc_rtdargs_ab.txt)
        ar.theta = props;
        ar.U = NT;
        ar.conc = nullptr;
        // the unit view from the by-value parameter, not the opaque kernarg reference: the fields
        // the theta part and the likelihood read stay in registers (SGPRs, spilled to VGPR lanes)
        // across the loop instead of a scalar load and wait per field and step -- 12.1 -> 11.0 us
        // per 4-tracer c4 step, 9.3 -> 8.3 us at the reference's 3 chains
        // (profiles/r06v_dzc_unitargs_ab.txt)
#ifdef NGRTD_DZC_UA_OPAQUE   // (A/B: the opaque reference)
        UnitArgs ul = uk;
#else
        UnitArgs ul = ua;
#endif
        ul.theta = props;
        ul.U = NT;
        ul.W = W;
        {
            const int nce = uk.ce_on ? L * uk.G : 0, nrt = uk.rtd_on ? L * uk.K : 0;
            double* q = wd;
            if (uk.ce_on) {
                ul.ce_obs = q; q += nce;
                ul.ce_lam = q; q += nce;
                ul.ce_hll_sum = q; q += L;
                ul.ce_Emin = q; q += L;
            }
            if (uk.rtd_on) {
                ul.rtd_obs = q; q += nrt;
                ul.rtd_lam = q; q += nrt;
                ul.rtd_hll_sum = q;
            }
            if (uk.c0_tab) ul.c0_tab = wd + (uk.c0_tab - uk.wd_src);
        }
        ul.ce_out = nullptr;
        ul.unit_out = nullptr;
        ThetaPre tp{};
        if constexpr (CEO) {
#pragma unroll
            for (int i = 0; i < 6; ++i) tp.ce[i] = props[uk.row_ce[i] * NT + cl];
        } else {
            tp.tau1 = props[uk.row_tau1 * NT + cl];
            tp.nub = props[uk.row_nu * NT + cl];
        }
        double th = 0.0;
        if (!(dg & 128) && (!thw || helper)) th = unit_logp_theta(ul, cl, l, &tp, false, false);
        DZC_MARK(3);                                      // argument views, theta part
        double like = 0.0;
        if constexpr (!CEO) {
            if (!(dg & 64) && !helper) {
                const double tau = props[a.row_tau[0] * NT + tid];
                const double eta = EPM ? props[a.row_eta[0] * NT + tid] : 1.0;
                const double tau2 = (MIX & 1) ? props[a.row_tau[1] * NT + tid] : 1.0;
                const double thx = LW ? props[a.row_thalf * NT + tid] : 0.5;
                like = dzc_rtd_like<C, MIX>(ar, ul, cheb, tabl, valid, tid, slot0, l, tau, eta, tau2, thx, tp.nub);
            }
        }
        if (thw) {                                        // the theta parts -> the chain lanes
            if (helper) thl[cl] = th;
            __syncthreads();
            if (!helper) th = thl[cl];
        }
        const double lpp = th + like;
        DZC_MARK(4);                                      // RTD likelihood
        // metrop_select + tune (demc_decide_at_u's arithmetic, on the registers)
        const double logu = (dg & 16384) ? 0.0 : demc_logu(sj.key, cid);
        const double mr = lpp - lp;
        const bool acc = __builtin_isfinite(mr) && logu < mr;
        const double cur = acc ? lpp : lp;
        if (d.n_acc_tune && !(dg & 8192)) {
            int32_t na = nat + (acc ? 1 : 0);
            if (sj.tune_now) {
                const double rate = (double)na / (double)d.tune_interval;
                if (d.tune_target == 2) lamb = pymc3_tune(lamb, rate);
                else if (d.tune_target == 1) sc = pymc3_tune(sc, rate);
                na = 0;
            }
            nat = na;
        }
        if (valid && !helper && !(dg & 256)) {
            const int64_t li = (int64_t)js * U + (int64_t)l * W + w;
            if (d.acc_log) d.acc_log[li] = (uint8_t)acc;
            if (d.lp_log) d.lp_log[li] = cur;
            if (d.ar_log) d.ar_log[li] = exp(mr);
        }
        nacc += (valid && !helper && acc) ? 1 : 0;
        lp = cur;
#pragma unroll
        for (int p = 0; p < kDzcMaxP; ++p) x[p] = acc ? v[p] : x[p];
        DZC_MARK(5);                                      // decision, tuning, logs
    }
#ifdef NGRTD_SECTION_PROBE
    if ((tid & 63) == 0) {
        unsigned long long* o = g_probe + ((size_t)blockIdx.x * (nth >> 6) + (tid >> 6)) * kProbeSlots;
        for (int k = 0; k < 6; ++k) o[k] = pacc[k];
        o[6] = (unsigned long long)nst;
    }
#endif
    // ---- the chain back: state (natural, and transformed), per-chain scalars, accept count
    if (valid && !helper) {
#pragma unroll
        for (int p = 0; p < kDzcMaxP; ++p) {
            if (p < P) {
                const int64_t gi = (int64_t)p * U + g;
                if (TR) {
                    dacc.xu[gi] = x[p];
                    dacc.x[gi] = pymc3_backward(dacc.tr_kind[p], dacc.tr_a[p], dacc.tr_b[p], x[p]);
                } else {
                    dacc.x[gi] = x[p];
                }
            }
        }
        dacc.lp[g] = lp;
        dacc.lamb[g] = lamb;
        dacc.scaling[g] = sc;
        if (dacc.n_acc_tune) dacc.n_acc_tune[g] = nat;
    }
    if (dacc.n_acc) {   // one atomic per wave and launch
        unsigned long long s = nacc;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((tid & 63) == 0 && s) atomicAdd(dacc.n_acc, s);
    }
}

}  // namespace ngrtd
