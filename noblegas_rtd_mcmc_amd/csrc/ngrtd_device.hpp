// ngrtd_device.hpp -- kernel argument blocks shared by the host launcher and the kernels.
#pragma once
#include <stdint.h>

namespace ngrtd {

constexpr int kMaxChan = 8;     // RTD channels (tracer A/B tables) per launch
constexpr int kMaxTracer = 8;
constexpr int kMaxGas = 5;
constexpr int kMaxBeta = 7;     // Beta-prior slots per unit (5 CE + RTD nu + thalf_cfc)

enum Mod { MOD_NONE = -1, MOD_PISTON = 0, MOD_EXP = 1, MOD_EPM = 2, MOD_DISP = 3 };

// RTD convolution launch (one thread = R units x one age sub-range; see rtd_conc_kernel)
struct RtdArgs {
    const double* theta;    // parameter rows, row r of unit u at theta[r * U + u]
    int64_t U;              // units (walker x well)
    int32_t row_tau[2], row_eta[2], row_D[2];
    int32_t row_f1, row_J, row_thalf, row_lamsf6;
    int32_t J_is_log10;     // 1: J = 10**theta[row_J] (ForwardMod :101); 0: J = theta[row_J]
    double thalf_a, thalf_b;// t_half = thalf_a * theta[row_thalf] + thalf_b
    const double* tab;      // channel table [N][CP]
    double tab0[kMaxChan];  // its row 0 (age 0), as kernel arguments
    int32_t N, C, CP;
    double tp0, dtp;        // age grid: tp_0 = tp0, tp_k = k + dtp (k >= 1)
    int32_t mod[2];         // component models; mod[1] = MOD_NONE for a single RTD
    int32_t LW;             // ages per wave per LDS slice
    int32_t K;              // tracers
    int32_t chan_tracer[kMaxChan];
    int32_t chan_isB[kMaxChan];     // 1: accumulation table (multiplied by J)
    int32_t chan_lamw[kMaxChan];    // 1: per-unit decay from row_thalf (not folded)
    int32_t tr_sf6[kMaxTracer];     // apply (1 + lamsf6)
    double tr_J[kMaxTracer];        // fixed J per tracer when row_J < 0
    double* conc;           // out [K][U]
    // MFMA fragments (rtd_exp_mfma_kernel): GEMM rows = (channel, age segment)
    const double* frag;     // [nsteps][R][64] A-operand fragments of v_mfma_f64_16x16x4f64
    int32_t nsteps, S_seg, Lseg;
    // Chebyshev surrogate of the exponential channel sums (logp_fused_kernel), or null
    const double* cheb;     // [kChebPieces][kChebN][CP]
    // pieces [cheb_p0, cheb_p0 + cheb_np) of it that logp_fused_kernel stages in LDS (the
    // window covering the tau1 prior's support; launch_fused)
    int32_t cheb_p0, cheb_np;
    // exp_pist_flow block tails (logp_fused_kernel EPM mode, ngrtd.hip epm_prepare): table
    // b = 1..epm_nb holds pieces [epm_p0, epm_p0 + epm_np) of the surrogate of
    //   T_b(tau') = sum_{k >= b S} A_{c,k} exp(-(k - b S) / tau'),  S = kEpmBlock,
    // laid out [b - 1][piece - epm_p0] x (C kEpmK64 doubles, then C kEpmK32 floats: the mixed
    // pieces every plan takes, ngrtd_kernels.hpp kEpmMixedAll / epm_tail_eval1; [C][kChebN]
    // doubles, channel-major, in a build with NGRTD_EPM_MIXED_ALL=0 for the plans without the
    // sampled half-life); null when the plan has none
    const double* epm;
    int32_t epm_nb, epm_p0, epm_np;
    // rows [0, epm_nw) of the channel table staged in LDS for the exp_pist_flow sums (a multiple
    // of kEpmBlock).  The whole table, padded, unless the plan's priors bound every in-support
    // unit's first unmasked age (ngrtd.hip epm_window: ew_on = 1; the reference's series length
    // N = 25 256 does not fit LDS): then only the rows those units read, and units outside the
    // support box [ew_tau_lo, ew_tau_hi] x [ew_eta_lo, ew_eta_hi] (x thalf_cfc's Beta [0, 1])
    // -- whose log-prob is -inf by their priors -- read no table row past it (epm_sums)
    int32_t epm_nw, ew_on;
    double ew_tau_lo, ew_tau_hi, ew_eta_lo, ew_eta_hi;
    int32_t epm_diag;       // timing diagnostics only (NGRTD_EPM_DIAG, tools/epm_probe.py): bit 0 skips
                            // the head, bit 1 the tail surrogate, bit 2 the exact tails (wrong results)
    // dispersion components of the generic single-launch instances (gen_exact): per age k,
    // 1 / tp_k at [k] and tp_k^(-3/2) at [N + k], then the kDispExpTab values 2^(j / kDispExpTab)
    // of the dispersion loop's exponential (fexp_tab) at [2N + j]; null when the plan has no
    // dispersion component
    const double* disp_aux;
    // ... and the dispersion loop's per-age operands interleaved, one 64-B row per age k
    // (read with scalar loads: the rows are wave-uniform): A_{c,k} at [k][c] (c < C <= 5),
    // tp_k at [k][5], 1 / tp_k at [k][6], tp_k^(-3/2) at [k][7]
    const double* disp_rows;
    // 1: K = C and tracer t owns exactly channel t (unit_conc's direct path)
    int32_t conc_ident;
    // generic instances with a dispersion component (ngrtd.hip gen_disp_split): its ages
    // [0, disp_split) are summed by the unit's theta wave, [disp_split, N) by its RTD wave; 0: not split
    int32_t disp_split;
    // small ensembles (ngrtd.hip disp_wide_plan): the dispersion component's channel sums come
    // from disp_wide_kernel, disp_pre_g partials per unit at disp_pre[(g (C + 1) + c) U + u]
    // (c = C: the normaliser), added in order by gen_component; null: gen_exact's loop
    const double* disp_pre;
    int32_t disp_pre_g;
};

// exp_pist_flow (convolution_integral_utils.py:186-190) on the yearly grid: the unmasked
// weights are exp(-beta tp_k), beta = eta / tau, from the first index m with
// tp_m >= tau (1 - 1/eta); the channel sums Y = sum_{k >= m} A_k q^(k - m), q = exp(-beta),
// split at the block boundary B = (m / S + 1) S into a head of < S + 1 ages (Horner over the
// LDS-staged channel table) and q^(B - m) T_{B/S}(1 / beta) from the block-tail surrogates.
constexpr int kEpmBlock = 16;
// entries of the dispersion loop's exponential table (RtdArgs::disp_aux; ngrtd_kernels.hpp fexp_tab)
constexpr int kDispExpTab = 256;
// doubles per age of RtdArgs::disp_rows (one s_load_dwordx16)
constexpr int kDispRow = 8;

// Chebyshev surrogate of Z_c(tau) = s01(tau) sum_{j>=0} A_{c,1+j} exp(-j / tau) (the
// exponential RTD channel sums times s01 = exp(-(tp_1 - tp_0) / tau)) for every channel c,
// and of Z_G(tau) = s01(tau) sum_{j=0}^{N-2} exp(-j / tau) (the normaliser), so that
// conc = (A_{c,0} + Z_c) / (1 + Z_G) with no exp/expm1/division per unit.  Pieces follow
// tau's binary representation: kChebSub per octave over the kChebOcts octaves
// [2^kChebOct0, 2^(kChebOct0 + kChebOcts)); piece (e - kChebOct0) kChebSub + j holds
// tau = 2^e m whose significand m in [1, 2) has top bits j, in the local x = 8 (m - c_j),
// c_j = 1 + (2j + 1)/8 (exact in binary: the piece index and x need no log).  Then one
// piece in s = 1/tau over [0, kChebSHi] for the tail up to tau = inf.  kChebN
// coefficients per piece and channel.  Built and validated per plan on the host
// (ngrtd.hip cheb_build); tau < 1/2, NaN take the exact matrix-core path.
constexpr int kChebN = 12;
constexpr int kChebSub = 4;
constexpr int kChebOct0 = -1;                      // tau >= 1/2
constexpr int kChebOcts = 19;                      // up to 2^18 = 262 144
constexpr int kChebBinPieces = kChebSub * kChebOcts;
constexpr int kChebPieces = kChebBinPieces + 1;
constexpr double kChebTauLo = 0.5;
constexpr double kChebSHi = 0x1p-18;               // the tail: s = 1/tau in [0, 2^-18]
// The exp_pist_flow block-tail surrogates (ngrtd.hip epm_prepare) use the same pieces over
// a wider range, tau' = tau / eta down to 2^kEpmOct0 (the priors reach tau' = 1 / 5): a
// Chebyshev piece [a, 1.25 a] converges as fast at any scale (each term e^(-j / tau') is
// analytic in log tau' over |Im| < pi/2), so no lane of the priors' support sums its tail
// exactly.  Same tail piece (s = 1/tau' in [0, kChebSHi]).
constexpr int kEpmOct0 = -4;
constexpr int kEpmOcts = kChebOct0 + kChebOcts - kEpmOct0;   // up to 2^18 as well
constexpr int kEpmBinPieces = kChebSub * kEpmOcts;
constexpr int kEpmPieces = kEpmBinPieces + 1;
// surrogate table row length for C channels: C numerator sums + the normaliser, even
__host__ __device__ constexpr int cheb_cp(int C) { return (C + 2) & ~1; }

// Row tiles of the exponential-RTD GEMM for C channels: R tiles of 16 rows hold 4R row
// groups; group g = c + C*m (m < 4R/C) of channel c carries the 4 age segments 4m..4m+3.
// R = C (C >= 3) keeps every row busy; C = 1, 2 use 4 tiles so that each B operand (one
// VALU multiply per lane per step) feeds at least 4 MFMAs.
__host__ __device__ constexpr int mfma_rows(int C) { return C >= 3 ? C : 4; }
__host__ __device__ constexpr int mfma_groups_per_chan(int C) { return 4 * mfma_rows(C) / C; }

// Per-unit CE + likelihood + prior launch (unit_logp_kernel)
struct UnitArgs {
    const double* theta;
    int64_t U;              // L * W
    int64_t W;
    int32_t L;
    int32_t flags;          // NGRTD_WANT_*
    int32_t ce_on, G;
    int32_t gas[kMaxGas];
    // per likelihood slot j < kMaxGas: coefficients of gas[j] (slots >= G repeat slot 0), so
    // the per-unit CE loop is unrolled over constant slots with uniform (SGPR) coefficients
    double gz[kMaxGas], gA0[kMaxGas], gA1[kMaxGas], gA2[kMaxGas], gA3[kMaxGas];
    int32_t g_he[kMaxGas];
    int32_t row_ce[6];      // Ae_beta, F_beta, E_beta, m, b_beta, nu_ce_beta
    const double* ce_obs;   // [L][G]
    const double* ce_sd;
    const double* ce_lam;   // [L][G] sd^-2 (<= 0 when sd <= 0: StudentT bound -> -inf)
    const double* ce_hll;   // [L][G] 0.5 * log(sd^-2)
    const double* ce_hll_sum;   // [L] sum over gases of ce_hll
    int32_t ce_bia[5], ce_bib[5];   // integer Beta exponents a-1, b-1 (or -1): beta_logp_fast
    const double* ce_Emin;  // [L]
    double E_max, logA_min, logA_max, logF_min, logF_max, b_min, b_max, nu_min, nu_max;
    double m_mu, m_tau, m_log_tau_2pi;
    double ce_ba[5], ce_bb[5], ce_betaln[5];
    int32_t rtd_on, K;
    const double* conc;     // [K][U] model concentrations from rtd_conc_kernel
    const double* rtd_obs;  // [L][K]
    const double* rtd_sd;
    const double* rtd_lam;  // [L][K]
    const double* rtd_hll;
    const double* rtd_hll_sum;  // [L]
    int32_t rnu_ia, rnu_ib, th_ia, th_ib;
    int32_t row_tau1, row_nu, row_tau2, row_f1, row_eta1, row_eta2, row_D1, row_D2, row_J, row_thalf, row_lamsf6;
    double tau1_lo, tau1_hi, tau1_nlw, tau2_lo, tau2_hi, tau2_nlw, f1_lo, f1_hi, f1_nlw;
    double eta1_lo, eta1_hi, eta1_nlw, eta2_lo, eta2_hi, eta2_nlw;
    double D1_lo, D1_hi, D1_nlw, D2_lo, D2_hi, D2_nlw;
    double J_mu, J_tau, J_log_tau_2pi;
    double th_a, th_b, th_betaln;
    double ls_tau, ls_half_log;
    double rnu_min, rnu_max, rnu_a, rnu_b, rnu_betaln;
    double* ulogp;          // out [U]
    double* ce_out;         // optional out [G][U] (forward)
    // All Beta priors of a unit (CE: Ae, F, E, b, nu; RTD: nu, thalf_cfc), with their
    // logodds Jacobians folded in (beta_block): slot i reads theta row bt_row[i] = x and
    // contributes x^bt_ia (1-x)^bt_ib to ONE product (integer exponents 0..7) plus
    // bt_fa log x + bt_fb log(1-x) for non-integer exponents; bt_betaln = sum of betaln.
    // per-well observation data packed for one contiguous LDS copy (logp_fused_kernel):
    // [ce_obs L*G | ce_lam L*G | ce_hll_sum L | ce_Emin L | rtd_obs L*K | rtd_lam L*K |
    //  rtd_hll_sum L | pad to even | c0 table c0_np*kC0N] (blocks present only when that
    // model block is on)
    const double* wd_src;
    int32_t wd_n;
    // Student-t normaliser table (ngrtd_math.hpp c0_piece; null: exact c0 everywhere)
    const double* c0_tab;
    int32_t c0_e0, c0_np;
    int32_t bt_n;
    int32_t bt_row[kMaxBeta], bt_ia[kMaxBeta], bt_ib[kMaxBeta];
    double bt_fa[kMaxBeta], bt_fb[kMaxBeta];
    double bt_betaln;
    // out [L][W]: logp_fused_kernel writes each unit's log-prob here and returns before the
    // per-walker sum (ngrtd_logp_units; null: the per-walker log-prob)
    double* unit_out;
};

// Metropolis accept of a device DEMetropolisZ step, done where the proposal's log-prob is
// formed (the per-walker reduction of logp_fused_kernel, or demc_accept_kernel): the
// chain's current log-prob lp[w] is replaced by the proposal's when accepted and its theta
// rows are copied from the proposal; n_acc counts acceptances; the per-chain tuning
// counters and, at the end of a tune interval, the tuned lamb / scaling are updated here
// (one thread per chain, so no other thread reads them during the launch).
struct DemcAccept {
    double* lp;             // [W] current log-prob (in/out); null: plain log-prob launch
    int32_t* acc;           // [W] out: this step's decisions
    unsigned long long* n_acc;
    double* x;              // [P][L][W] current state, updated for accepted chains
    const double* prop;     // [P][L][W] the proposal being evaluated
    int32_t P;              // parameter rows per (walker, well)
    uint64_t key;           // per-step random key (demc_key)
    int32_t* n_acc_tune;    // [W] accepted since the last tune (null: no tuning state)
    double* lamb;           // [W] per-chain lambda
    double* scaling;        // [W] per-chain scaling
    int32_t tune_now;       // apply PyMC3 tune() after this step's decision
    int32_t tune_target;    // 1 = scaling, 2 = lambda
    int32_t tune_interval;
    uint8_t* acc_log;       // [W] this step's decisions (null: not logged)
    double* lp_log;         // [W] each chain's log-prob after this step (null: not logged)
    int64_t chain0;         // global index of chain 0 in the random stream
    double* xu;             // [P][L][W] transformed state (null: natural-space chains)
    const double* prop_u;   // [P][L][W] the transformed proposal, copied to xu on accept
    // Single-launch DEMetropolisZ step (logp_fused_kernel MIX bit 3): the kernel forms the
    // proposal itself from the state and two history entries (demcz_propose_kernel's
    // arithmetic) into dz_prop, appends the state to the history and evaluates the
    // proposal; prop and prop_u are unused.  Other fields as DemczArgs.
    const double* zx;       // [P][L][W] state in the chains' space (x, or xu when transformed)
    double* dz_prop;        // [P][L][W] out: the proposal, natural space (the launch's theta)
    double* hist;           // [cap][W][R] chain-major histories
    int64_t h_lo, h_it, h_at;   // partners from entries h_lo + [0, h_it); append x at h_at (-1: none)
    int64_t Wg;             // chains of the whole ensemble (the noise stream's row stride)
    const double* S;        // [R] proposal scale per row (null: ones)
    int32_t L;
    int32_t dz_diag;        // timing diagnostics only (NGRTD_DZ_DIAG, tools/dz_probe.py): bit 0: proposal =
                            // state, 1: no history store, 2: no commit, 3: no staging, 4: no partner
                            // loads (noise-only proposals), 5: no per-well decision (wrong results)
    int32_t tr_kind[NGRTD_ROLE_COUNT];
    double tr_a[NGRTD_ROLE_COUNT], tr_b[NGRTD_ROLE_COUNT];
    // Multi-step launch (MIX bit 3): the block runs n_steps consecutive steps of its own
    // chains (chains exchange nothing, so no grid-wide sync); step j's key / partner range /
    // append entry / tune flag come from dz_step(sch, j), the host loop's own schedule, and
    // its logs from acc_log / lp_log + j W.  n_steps = 1 with the fields above otherwise.
    int32_t n_steps;
    // 1: the block's LDS also holds the natural-space proposal rows [P][512] (after the
    // transformed rows): dz_stage writes them there as well as to dz_prop, and the step's
    // own theta loads and commit read them from LDS instead of back from L2
    int32_t prop_lds;
    // 1: the block keeps its chains' state in LDS for the whole launch -- the state rows in
    // the chains' space [P][512] and the per-chain lp / lamb / scaling / tuning counter [512]
    // (per-well chains: slot = unit; joint chains: slot = walker) -- loaded once before the
    // first step and written back (x, xu for the chains that moved; the per-chain arrays)
    // after the last: per step no state loads, no commit stores, no per-chain round trips
    int32_t state_lds;
    // 1 (with prop_lds): every theta row the launch reads is one of the LDS proposal rows
    // (the joint exponential plan: 6 CE rows, tau1, nu_rtd), so dz_stage does not write the
    // proposals to dz_prop (a state-sized store stream per step) and the exact fallback reads
    // tau from LDS too
    int32_t prop_skip;
    struct Sched {
        uint64_t seed;
        int64_t s0;         // steps_done at the launch's first step
        int64_t h_len0, h_lo0;   // history length / first usable entry before it
        int32_t append0;    // the first step appends its state (not the call's first step)
        int64_t n_tune;
        double drop;        // stop_tuning's drop fraction, applied at step n_tune
        int32_t tune_target, tune_interval;
    } sch;
    // Per-well chains (ngrtd_demcz_state.per_well): every (walker w, well l) unit is its own
    // chain -- the reference runs one PyMC3 model per well (run_age_mcmc.py:122-231,
    // noble_gas_mcmc.py:95-104).  Chain c = l W + w: lp / acc / n_acc_tune / lamb / scaling
    // and the logs are [L][W]; proposal noise and accept draws are keyed by cid = (well0 + l)
    // Wg + chain0 + w, the partner indices by the walker; the history layout is the joint one.
    int32_t per_well;
    int64_t well0;
    double* ar_log;         // [chains] this step's PyMC3 `accept` stat exp(mr) (null: not logged)
    // lane-chain step (ngrtd_dzc.hpp dz_chain_kernel) of <= 64 chains: 1 = the block's second
    // wave evaluates the chains' theta parts while the first evaluates their RTD likelihoods
    int32_t theta_wave;
};

// One DEMetropolisZ step's schedule (ngrtd_demcz_run's host loop, restated so that a
// multi-step launch derives it on the device): random key, partner range [lo, lo + it),
// append entry at (-1: none), tune flag, and the history length after the append.
struct DzStep {
    uint64_t key;
    int64_t lo, it, at, len;
    int32_t tune_now;
};

// DEMetropolisZ proposal / history append over theta rows [R][W] (demcz_propose_kernel)
constexpr int kRoleCount = NGRTD_ROLE_COUNT;
struct DemczArgs {
    const double* x;        // [R][W] current state
    double* prop;           // [R][W] new proposal
    double* hist;           // [cap][W][R] chain histories (chain-major)
    const double* lamb;     // [W]
    const double* scaling;  // [W]
    int64_t W, R;
    int32_t propose;        // 0: append only (no proposal)
    int64_t append_at;      // history entry that receives x (-1: none)
    int64_t lo, it;         // partners come from entries lo + [0, it)
    uint64_t key;           // per-step random key (demc_key)
    int64_t chain0;         // global index of chain 0 in the random stream
    int64_t Wg;             // chains of the whole ensemble (the element stream's row stride)
    const double* S;        // [R] proposal scale per row (null: ones)
    double* prop_x;         // [R][W] backward(prop) for transformed chains (null: natural space)
    int32_t L;              // wells: row r belongs to parameter r / L
    int32_t tr_kind[kRoleCount];
    double tr_a[kRoleCount], tr_b[kRoleCount];
    int32_t per_well;       // per-well chains (demcz_propose_pw_kernel; DemcAccept::per_well)
    int64_t well0;
    int32_t P;
};

}  // namespace ngrtd
