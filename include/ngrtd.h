/*
 * ngrtd.h -- C ABI of libngrtd.so, the MI355X (gfx950) engine for the two
 * log-likelihood hot paths of uz226/NobleGas_RTD_MCMC:
 *
 *   CE  : closed-equilibrium noble-gas forward model  (utils/noble_gas_utils.py)
 *   RTD : residence-time-distribution convolution     (utils/convolution_integral_utils.py)
 *
 * and the per-walker log-probabilities built on them by the reference's PyMC3 models
 * (ng_interp/noble_gas_mcmc.py:184-267, age_ens_runs_mcmc/run_age_mcmc_utils.py:275-397).
 *
 * Plain C: pointers + sizes, no framework types.  Every entry returns an int status
 * (NGRTD_OK == 0, < 0 on API/device error; the message is ngrtd_last_error(ctx)).
 * Invalid parameter VALUES are not errors: like the reference they propagate as
 * NaN / -9999 sentinels / -inf log densities with status 0.
 *
 * Memory: every compute entry takes `mem` = NGRTD_MEM_HOST (pointers are host memory;
 * the call stages through ctx-owned device buffers and returns after the results are
 * back) or NGRTD_MEM_DEVICE (pointers are device memory; the call is enqueued on the
 * ctx stream and returns immediately).  Float data is IEEE float64 throughout.
 *
 * Threading: a ctx is bound to one device and one stream; it is not re-entrant.  Create
 * it after any fork() (the reference forks PyMC3 chains, run_age_mcmc_utils.py:416).
 */
#ifndef NGRTD_H
#define NGRTD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGRTD_ABI_VERSION 1

enum ngrtd_status {
    NGRTD_OK = 0,
    NGRTD_EINVAL = -1,   /* bad argument / unsupported configuration */
    NGRTD_EDEVICE = -2,  /* HIP runtime error */
    NGRTD_ENOMEM = -3,   /* allocation failed */
    NGRTD_ESTATE = -4    /* unknown handle / destroyed object */
};

enum ngrtd_mem { NGRTD_MEM_HOST = 0, NGRTD_MEM_DEVICE = 1 };

/* noble gases, utils/noble_gas_utils.py:38-73,138-149 */
enum ngrtd_gas { NGRTD_HE = 0, NGRTD_NE = 1, NGRTD_AR = 2, NGRTD_KR = 3, NGRTD_XE = 4 };

/* lumped-parameter RTD models, utils/convolution_integral_utils.py:178-196 */
enum ngrtd_rtd_model {
    NGRTD_MOD_NONE = -1,
    NGRTD_MOD_PISTON = 0,
    NGRTD_MOD_EXPONENTIAL = 1,
    NGRTD_MOD_EXP_PIST_FLOW = 2,
    NGRTD_MOD_DISPERSION = 3
};

/* rad_accum, convolution_integral_utils.py:313-333 */
enum ngrtd_accum { NGRTD_ACC_NONE = 0, NGRTD_ACC_HE3 = 1, NGRTD_ACC_HE4 = 2, NGRTD_ACC_SF6 = 3 };

typedef struct ngrtd_ctx ngrtd_ctx;
typedef struct ngrtd_plan ngrtd_plan;

/* ------------------------------------------------------------------ context */
int ngrtd_abi_version(void);
int ngrtd_create(ngrtd_ctx** out, int device);
int ngrtd_destroy(ngrtd_ctx* ctx);
const char* ngrtd_last_error(const ngrtd_ctx* ctx);
/* Enqueue on an external hipStream_t from now on (e.g. torch.cuda.current_stream()
 * .cuda_stream); NULL selects HIP's null (default) stream.  Until the first call the ctx
 * uses a non-blocking stream of its own. */
int ngrtd_set_stream(ngrtd_ctx* ctx, void* hip_stream);
int ngrtd_synchronize(ngrtd_ctx* ctx);
/* When on, every plan launch brackets each kernel with hipEvents on the ctx stream;
 * ngrtd_plan_kernel_stats() then reports the accumulated device time per kernel. */
int ngrtd_set_profiling(ngrtd_ctx* ctx, int on);

/* ------------------------------------------------------- CE forward model
 * Replaces noble_gas_fun(gases, E, T, Ae, F, P, S).<method>() of
 * utils/noble_gas_utils.py:75-261, vectorised over n independent parameter sets.
 *   what = NGRTD_CE_*:   out is [n][n_gases] (LAPSE_RATE / VAPOR_PRESSURE: [n])
 *   p_mode:              pressure as parse_P (:91-100): lapse_rate(E), '1atm', or P[i]
 *   S may be NULL (salinity 0.0, the reference default).                            */
enum ngrtd_ce_what {
    NGRTD_CE_EXC_TOTAL = 0,     /* ce_exc(add_eq_conc=True)       :235-253 */
    NGRTD_CE_EXC_EXCESS = 1,    /* ce_exc(add_eq_conc=False)      :235-253 */
    NGRTD_CE_EQUIL_DRY = 2,     /* equil_conc_dry()               :216-232 */
    NGRTD_CE_EQUIL = 3,         /* equil_conc()                   :202-213 */
    NGRTD_CE_SOLUBILITY = 4,    /* solubility(gas)                :117-180 */
    NGRTD_CE_VAPOR_PRESSURE = 5,/* vapor_pressure()               :184-199 */
    NGRTD_CE_PRESSURE = 6       /* self.P after parse_P           :91-113  */
};
enum ngrtd_p_mode { NGRTD_P_LAPSE_RATE = 0, NGRTD_P_1ATM = 1, NGRTD_P_GIVEN = 2 };

int ngrtd_ce_forward(ngrtd_ctx* ctx, int32_t what, int32_t p_mode,
                     const double* E, const double* T, const double* Ae, const double* F,
                     const double* P, const double* S, int64_t n,
                     const int32_t* gas_ids, int32_t n_gases, double* out, int32_t mem);

/* -------------------------------------- prep ensemble propagation (He, CFC, SF6)
 * The CE posterior ensemble pushed through to tracer observations
 * (age_modeling_mcmc.prep.py:247-397), one element per ensemble member.  Inputs are
 * per-member arrays [n]; outputs are structure-of-arrays.
 *
 * ngrtd_he_comps replaces ng_parse(obs_dict, Ae, F, E, T).He_comps(Rterr)
 * (utils/noble_gas_utils.py:380-422): out[k][n] for k = enum ngrtd_he_out, the
 * obs_dict_ entries He4_eq, He4_atm, He4_ter, He4_del, He3_tu.  Rterr may be NULL to use
 * Rterr_const for every member (prep.py:341 passes a constant list).                 */
enum ngrtd_he_out { NGRTD_HE_EQ = 0, NGRTD_HE_ATM = 1, NGRTD_HE_TER = 2, NGRTD_HE_DEL = 3, NGRTD_HE_TU = 4,
                    NGRTD_HE_NOUT = 5 };
int ngrtd_he_comps(ngrtd_ctx* ctx, const double* He4_obs, const double* He3_obs, const double* Ae,
                   const double* F, const double* E, const double* T, const double* Rterr,
                   double Rterr_const, int64_t n, double* out, int32_t mem);

/* ngrtd_cfc_corr replaces the methods of cfc_ce_corr(cfc_num, E, T, Ae, F, S) and
 * sf6_ce_corr(E, T, Ae, F, S) (utils/cfc_utils.py:25-306) for n members and n_species
 * species (enum ngrtd_cfc_species; NGRTD_SF6 selects the sf6_ce_corr unit factors).
 *   what = NGRTD_CFC_EQUIL_AIR  equil_air_conc_*(x = C_meas)  :86-106, :229-249
 *          NGRTD_CFC_EQUIL_AQ   equil_aq_conc_*(x = z_i)      :108-124, :264-278
 *          NGRTD_CFC_CE_EXC     ce_exc_conc_*(x = z_i), with P = self.P [atm]  :126-142, :280-296
 *          NGRTD_CFC_SOLUBILITY solubility_cfc / _sf6          :64-84, :208-221
 *          NGRTD_CFC_VAPOR_PRESSURE_ATM, NGRTD_CFC_LAPSE_RATE_ATM  ([n] outputs)
 * x and out are [n_species][n].  Ae is self.Ae: the constructor's Ae*1000. [ccSTP/kg] (:30).
 * S, P, x may be NULL when the entry does not read them (S NULL = 0.0).             */
#define NGRTD_MAX_CFC 4
enum ngrtd_cfc_species { NGRTD_CFC11 = 0, NGRTD_CFC12 = 1, NGRTD_CFC113 = 2, NGRTD_SF6 = 3 };
enum ngrtd_cfc_what {
    NGRTD_CFC_EQUIL_AIR = 0,
    NGRTD_CFC_EQUIL_AQ = 1,
    NGRTD_CFC_CE_EXC = 2,
    NGRTD_CFC_SOLUBILITY = 3,
    NGRTD_CFC_VAPOR_PRESSURE_ATM = 4,
    NGRTD_CFC_LAPSE_RATE_ATM = 5
};
int ngrtd_cfc_corr(ngrtd_ctx* ctx, int32_t what, const int32_t* species, int32_t n_species,
                   const double* E, const double* T, const double* Ae, const double* F,
                   const double* S, const double* P, const double* x, int64_t n, double* out,
                   int32_t mem);

/* ----------------------------------------------------------- RTD series
 * The C_t input of tracer_conv_integral(C_t, t_samp) (convolution_integral_utils.py:106):
 *   c_by_age[k]   = np.flip(C_t.to_numpy().ravel())[k]  (age k, :336)
 *   idx_by_age[k] = np.flip(C_t.index)[k]  (4He/SF6 accumulation, :323/:331); NULL => k
 *   dtp           = floor(t_samp - C_t.index[-1])  (:172)
 * Host memory; copied.  Returns a handle >= 0 in *series_id.                        */
int ngrtd_series_create(ngrtd_ctx* ctx, const double* c_by_age, const double* idx_by_age,
                        int64_t n, double dtp, int32_t* series_id);
int ngrtd_series_destroy(ngrtd_ctx* ctx, int32_t series_id);

/* -------------------------------------------- single-tracer convolution
 * tracer_conv_integral.update_pars(...) + .convolve() (:111-142, :284-340) for n
 * independent parameter sets (one call = n convolutions of one series).  Per-set
 * arrays may be NULL when the model does not read them (eta: exp_pist_flow only,
 * D: dispersion only).  t_half: per-set half-life array, or NULL to use t_half_const
 * (<= 0 or NaN => lamba = 0, :117-121).  J: per-set accumulation rate (the J / J_sf6
 * kwarg, already 10**log10J), or NULL to use J_const.                                */
int ngrtd_conv(ngrtd_ctx* ctx, int32_t series_id, int32_t mod_type, int32_t accum,
               const double* tau, const double* eta, const double* D,
               const double* t_half, double t_half_const,
               const double* J, double J_const,
               int64_t n, double* out, int32_t mem);

/* gen_g_tp() (:155-281): the normalised weight vector g[N] of one parameter set. */
int ngrtd_rtd_weights(ngrtd_ctx* ctx, int32_t series_id, int32_t mod_type,
                      double tau, double eta, double D, double* g_out, int32_t mem);

/* Fracture / matrix-diffusion RTD 'frac_inf_diff' (:238-266) for n parameter sets on the
 * age grid of series_id: the inner integral over 1000 log-spaced advective times per age
 * (frac_rtd_numba_disp :36-65 with the dispersion advective RTD of tau, D; or
 * frac_rtd_numba :67-97 when f_tadv_ext != NULL: rows of N values in age order, row
 * stride ext_stride doubles, 0 = one row shared by every set), then f[0] = 0, the trapz
 * normalisation, FM_mu and g /= g.sum() (:257-270), then convolve() (:305-340) with
 * decay / accumulation as ngrtd_conv.  Outputs (each may be NULL, at least one not):
 *   conc [n]      convolve()
 *   g_out [n][N]  gen_g_tp()
 *   fm_mu [n]     the FM_mu attribute (mean travel time, :262-263)
 * Per-set arrays: tau, D (NULL allowed with f_tadv_ext), bbar, Phi_im (required); t_half
 * and J as in ngrtd_conv.                                                            */
int ngrtd_frac_conv(ngrtd_ctx* ctx, int32_t series_id, int32_t accum,
                    const double* tau, const double* D, const double* bbar, const double* Phi_im,
                    const double* f_tadv_ext, int64_t ext_stride,
                    const double* t_half, double t_half_const, const double* J, double J_const,
                    int64_t n, double* conc, double* g_out, double* fm_mu, int32_t mem);

/* convolve(g_tau=g) (:298-302): dot product with an externally supplied weight vector. */
int ngrtd_conv_dot(ngrtd_ctx* ctx, int32_t series_id, const double* g, double t_half,
                   int32_t accum, double J, double* out, int32_t mem);

/* ------------------------------------------------- batched log-probability
 * Parameter roles of one (walker, well) -- the PyMC3 free RVs in natural space.   */
enum ngrtd_role {
    NGRTD_ROLE_AE_BETA = 0,      /* noble_gas_mcmc.py:224 */
    NGRTD_ROLE_F_BETA = 1,       /* :225 */
    NGRTD_ROLE_E_BETA = 2,       /* :226 */
    NGRTD_ROLE_M = 3,            /* :234 */
    NGRTD_ROLE_B_BETA = 4,       /* :237 */
    NGRTD_ROLE_NU_CE_BETA = 5,   /* :249 */
    NGRTD_ROLE_TAU1 = 6,         /* run_age_mcmc_utils.py:286 */
    NGRTD_ROLE_TAU2 = 7,         /* :302 */
    NGRTD_ROLE_F1 = 8,           /* :303 */
    NGRTD_ROLE_ETA1 = 9,         /* :312 */
    NGRTD_ROLE_ETA2 = 10,        /* :316 */
    NGRTD_ROLE_D1 = 11,          /* :320 */
    NGRTD_ROLE_D2 = 12,          /* :324 */
    NGRTD_ROLE_J = 13,           /* log10 J, :298 */
    NGRTD_ROLE_THALF_BETA = 14,  /* :334 */
    NGRTD_ROLE_LAMSF6 = 15,      /* :343 */
    NGRTD_ROLE_NU_RTD_BETA = 16, /* :291 */
    NGRTD_ROLE_COUNT = 17
};

#define NGRTD_MAX_GASES 5
#define NGRTD_MAX_TRACERS 8

typedef struct {
    int32_t series_id;
    int32_t accum;          /* enum ngrtd_accum */
    double t_half;          /* decay half-life (H3/He3: 12.34); <= 0 => none */
    double J;               /* fixed accumulation rate (10**log10J or J_sf6) if not sampled */
    int32_t is_cfc12;       /* per-walker decay from the thalf_cfc role (:107-109) */
    int32_t is_sf6;         /* cout *= (1 + lamsf6) when the lamsf6 role is present (:160-161) */
} ngrtd_tracer_desc;

/* NGRTD_EXACT_RTD: never use the plan-time surrogate of the exponential channel sums;
 * every unit evaluates them exactly (matrix-core Horner over all N ages).  For A/B and
 * for the exact-path rate bench.py reports beside the headline. */
/* NGRTD_DISP_WIDE / NGRTD_DISP_LANE: the geometry of a dispersion component's age sum.  By
 * default a plan of at most 256 units (n_wells x max_walkers) sums each unit's ages across the
 * lanes of a separate kernel (the reference's own runs: 1 well x 3 chains, N = 25 256) and a
 * larger plan gives each unit one lane; the flags force either (A/B and tests). */
enum ngrtd_flags { NGRTD_WANT_LIKE = 1, NGRTD_WANT_PRIOR = 2, NGRTD_WANT_JACOBIAN = 4, NGRTD_EXACT_RTD = 8,
                   NGRTD_DISP_WIDE = 16, NGRTD_DISP_LANE = 32 };

typedef struct {
    int32_t n_wells;                        /* L */
    int32_t n_params;                       /* P (rows of theta per well) */
    int32_t role_index[NGRTD_ROLE_COUNT];   /* row of each role within P, -1 = absent */
    int32_t flags;                          /* enum ngrtd_flags */
    /* CE block (ng_interp/noble_gas_mcmc.py:184-267) */
    int32_t ce_enabled;
    int32_t ce_n_gases;
    int32_t ce_gas_ids[NGRTD_MAX_GASES];
    const double* ce_obs;                   /* [L][G] */
    const double* ce_sd;                    /* [L][G] */
    const double* ce_E_min;                 /* [L] */
    double ce_E_max, ce_logA_min, ce_logA_max, ce_logF_min, ce_logF_max;
    double ce_b_min, ce_b_max, ce_m_mu, ce_m_sd, ce_nu_min, ce_nu_max;
    double ce_beta_a[5], ce_beta_b[5];      /* Beta priors: Ae, F, E, b, nu */
    /* RTD block (run_age_mcmc_utils.py:275-397) */
    int32_t rtd_enabled;
    int32_t n_tracers;                      /* K */
    int32_t mod_type1, mod_type2;           /* enum ngrtd_rtd_model; mod_type2 = NONE if single */
    ngrtd_tracer_desc tracers[NGRTD_MAX_TRACERS];
    const double* rtd_obs;                  /* [L][K] */
    const double* rtd_sd;                   /* [L][K] */
    double tau1_lo, tau1_hi, tau2_lo, tau2_hi, f1_lo, f1_hi;
    double eta1_lo, eta1_hi, eta2_lo, eta2_hi, D1_lo, D1_hi, D2_lo, D2_hi;
    double J_mu, J_sd, thalf_lo, thalf_hi, thalf_a, thalf_b, lamsf6_sd;
    double rtd_nu_min, rtd_nu_max, rtd_nu_a, rtd_nu_b;
} ngrtd_model_desc;

int ngrtd_plan_create(ngrtd_ctx* ctx, const ngrtd_model_desc* desc, int64_t max_walkers,
                      ngrtd_plan** out);
int ngrtd_plan_destroy(ngrtd_plan* plan);

/* logp[w] = sum over wells of (log-likelihood + log-prior [+ log|Jacobian|]) for theta
 * laid out structure-of-arrays [P][L][W] (float64).  W <= max_walkers.               */
int ngrtd_logp(ngrtd_plan* plan, const double* theta, int64_t W, double* logp, int32_t mem);

/* n back-to-back log-probs of the same device buffers, enqueued by one call (device
 * memory only): the shape of the reference's sampling loop -- one model log-prob per
 * step, pm.sample in run_age_mcmc_utils.py:416 / noble_gas_mcmc.py:410-415 -- without
 * the host round trip per step.  Every step is one full launch over all W walkers; logp
 * holds the last one.  Used by bench.py (N = 1) via distributed.LogpStepLoop.run. */
int ngrtd_logp_n(ngrtd_plan* plan, const double* theta, int64_t W, double* logp, int64_t n);

/* Device time (ms) between two events the last ngrtd_logp_n call recorded on the plan's
 * stream before its first and after its last launch (waits for the second).  bench.py's
 * kernel time for the roofline: the n launches back to back, as rocprofv3 sees them. */
int ngrtd_plan_region_ms(ngrtd_plan* plan, float* ms);

/* Multi-GPU walker blocks (BASELINE c5; the reference itself runs one process per PyMC3 chain,
 * run_age_mcmc_utils.py:416, and has no multi-GPU counterpart): an RCCL communicator over the
 * job's ranks (one process per GPU) and the bench step loop with its all-gather in native code.
 * rccl_path: the RCCL library to dlopen (the one torch loaded, so that both share it; NULL:
 * "librccl.so.1").  ngrtd_comm_unique_id runs on rank 0; the caller broadcasts the 128 bytes. */
typedef struct ngrtd_comm ngrtd_comm;
int ngrtd_comm_unique_id(const char* rccl_path, uint8_t* id128);
int ngrtd_comm_create(ngrtd_ctx* ctx, const char* rccl_path, const uint8_t* id128, int32_t nranks, int32_t rank,
                      ngrtd_comm** out);
int ngrtd_comm_destroy(ngrtd_comm* comm);

/* n steps of distributed.LogpStepLoop on device buffers: step i writes this rank's block log-probs
 * (W walkers) into bufs + (i % 2) per and all-gathers the per-entry blocks of every rank into
 * gathered + (i % 2) per nranks (ncclAllGather on the communicator's own stream), two steps in
 * flight: step i's gather overlaps step i + 1's launch, step i + 2's launch waits for it (it
 * reuses the buffer) -- stream events, no host synchronisation, no per-step host round trip.
 * bufs: [2][per] (entries W..per-1 untouched: the caller pads them), gathered: [2][nranks per].
 * The plan's stream waits for the last gathers before returning, so a sync on it covers them;
 * ngrtd_plan_region_ms then gives the n steps' device time (launches + gathers). */
int ngrtd_logp_gather_n(ngrtd_plan* plan, ngrtd_comm* comm, const double* theta, int64_t W, int64_t per,
                        double* bufs, double* gathered, int64_t n);

/* Forward model outputs of the plan (posterior predictive, run_age_mcmc.py:251-319,
 * noble_gas_mcmc.py:645-653): ce_out [G][L][W] (may be NULL), rtd_out [K][L][W]
 * (may be NULL).                                                                     */
int ngrtd_forward(ngrtd_plan* plan, const double* theta, int64_t W, double* ce_out,
                  double* rtd_out, int32_t mem);

/* Accumulated device time (ms) and launch count of each kernel the plan launched while
 * profiling was on: index 0 = RTD convolution kernel, 1 = per-unit CE/likelihood kernel,
 * 2 = per-walker reduction, 3 = single-launch log-prob kernel (RTD + CE + likelihood +
 * per-walker sum).  times_ms/counts have room for n entries; resets if reset. */
int ngrtd_plan_kernel_stats(ngrtd_plan* plan, double* times_ms, int64_t* counts, int32_t n,
                            int32_t reset);

/* Launch geometry the plan chose for its RTD kernel: info[0..12] = units per lane (VALU
 * path) or 16-unit tiles per wave (MFMA path), waves per block, blocks, ages per LDS slice
 * (VALU) or per segment (MFMA), channels, N, LDS bytes, units, MFMA row tiles (0 = VALU
 * path), age segments, 4-age MFMA steps, Chebyshev surrogate in use (0 none, 1 exponential channel sums, 2 exp_pist_flow block tails), the
 * surrogate's validated max relative error in units of 1e-18 (-1: not built), and
 * info[13] = pieces of the Student-t normaliser table (0: exact c0), info[14] = partial
 * sums per unit of a small-ensemble dispersion plan's wide kernel (0: one lane per unit;
 * NGRTD_DISP_WIDE), info[15] reserved.  For the roofline accounting in bench.py. */
int ngrtd_plan_info(ngrtd_plan* plan, int64_t W, int64_t* info, int32_t n);

/* Device-resident DEMetropolisZ: the sampler of the reference, PyMC3 3.11.2
 * DEMetropolisZ (pymc3/step_methods/metropolis.py; called at run_age_mcmc_utils.py:412-417
 * and noble_gas_mcmc.py:410-415), for W independent chains at once -- one chain per walker
 * (the reference runs 3-4 chains in separate processes).  Per chain w and step s:
 *   tuning (s < n_tune): at the start of every step s = k tune_interval (k >= 1),
 *     lamb_w (tune_target LAMBDA, PyMC3's default) or scaling_w (SCALING) *= pymc3 tune()
 *     of the acceptance rate over the last interval, and the counter restarts;
 *   before step s = n_tune (stop_tuning): the first floor(drop_fraction * it) history
 *     entries are dropped (hist_lo advances), it = entries in the history;
 *   eps = U(-1, 1) S_r scaling_w per parameter row r (UniformProposal(S) * scaling; S NULL =
 *     ones, PyMC3's default);
 *   space: PyMC3 proposes in the TRANSFORMED space of its free variables (Beta: logodds,
 *     Uniform: interval, HalfNormal: log; pymc3/distributions/transforms.py).  With theta_u
 *     set, the chains, their histories and the proposals live in that space: the proposal
 *     kernel maps every proposed row back, x = backward(u) (logodds 1/(1+exp(-u)), interval
 *     s b + (1-s) a with s = 1/(1+exp(-u)), log exp(u)), and the plan must carry
 *     NGRTD_WANT_JACOBIAN so that logp is the density of u.  theta holds backward(theta_u).
 *     theta_u NULL: the chains move in the natural space of theta (no Jacobian).
 *   it = hist_len - hist_lo;  it > 1: iz1 != iz2 uniform in [0, it),
 *     x* = x + lamb_w (Z_w[hist_lo + iz1] - Z_w[hist_lo + iz2]) + eps;  else x* = x + eps;
 *   mr = logp(x*) - logp(x): accept iff mr is finite and log(u) < mr (metrop_select);
 *   the chain's new state is appended to its history Z_w.
 * Random numbers come from a counter-based generator keyed by (seed, s, chain0 + w), so a
 * run split over several calls, or over walker-block shards, equals one call.  theta [P][L][W] and logp [W] are DEVICE
 * pointers updated in place on the ctx stream; logp must hold logp(theta) on entry.
 * Every array in the state is device memory owned by the caller.  History layout:
 * [hist_cap][W][P*L] float64 (chain-major): entry e, theta row r of chain w at
 * (e*W + w)*P*L + r -- a chain's state is one contiguous run.  Entry e is the state after
 * step e (hist_len == steps_done after every call).
 * accepted_log [n_steps][W] (uint8) and logp_log [n_steps][W] (each chain's log-prob after
 * the step; per-well chains: [n_steps][L][W], and logp is [L][W]) may be NULL.  n_accepted (device uint64, may be NULL) counts acceptances.
 * Joint plans with a single-launch instance (C = 5 channels: c3, c4, the published models):
 * one launch per chunk of up to NGRTD_DZ_CHUNK (default 256) steps, each block stepping its
 * own chains (proposal, history append, log-prob, decision, tuning, commit per step).
 * Other plans (or NGRTD_DZ_MODE=pair): 2 launches per step, the proposal kernel (which also
 * appends the previous state) and the log-prob kernel with the accept in its per-walker
 * reduction.  One append at the end. */
enum ngrtd_tune_target { NGRTD_TUNE_NONE = 0, NGRTD_TUNE_SCALING = 1, NGRTD_TUNE_LAMBDA = 2 };
enum ngrtd_transform { NGRTD_TR_NONE = 0, NGRTD_TR_LOGODDS = 1, NGRTD_TR_INTERVAL = 2, NGRTD_TR_LOG = 3 };
typedef struct {
    double* lamb;            /* [W] per-chain lambda (PyMC3 default 2.38 / sqrt(2 ndim)) */
    double* scaling;         /* [W] per-chain scaling (PyMC3 default 0.001) */
    int32_t* n_acc_tune;     /* [W] acceptances since the last tune (start at 0) */
    double* hist;            /* [hist_cap][W][P*L] */
    int64_t hist_cap;
    int64_t hist_len;        /* in/out: entries written */
    int64_t hist_lo;         /* in/out: first entry proposals draw from */
    int64_t steps_done;      /* in/out: steps taken so far (tune schedule, random stream) */
    int64_t n_tune;          /* tuning steps of the run (PyMC3 tune=) */
    int32_t tune_interval;   /* PyMC3 tune_interval (default 100; the reference: 1000 / 5000) */
    int32_t tune_target;     /* enum ngrtd_tune_target */
    double drop_fraction;    /* PyMC3 tune_drop_fraction (default 0.9) */
    uint64_t seed;
    int64_t chain0;          /* global index of chain 0 in the random stream (walker-block
                                shards of one ensemble draw the numbers of their own chains) */
    int64_t n_chains_total;  /* chains of the whole ensemble (0: W, unsharded) */
    const double* S;         /* [P*L] proposal scale per theta row (PyMC3 S), device; NULL = ones */
    double* theta_u;         /* [P][L][W] transformed state (device), NULL = natural space */
    int32_t tr_kind[NGRTD_ROLE_COUNT];  /* per parameter row p < P: enum ngrtd_transform */
    double tr_a[NGRTD_ROLE_COUNT], tr_b[NGRTD_ROLE_COUNT];   /* interval bounds */
    /* Per-well chains (1) -- the reference's structure: one PyMC3 model, hence one chain,
     * per well (age_ens_runs_mcmc/run_age_mcmc.py:122-231 loops `for ww in wells`;
     * ng_interp/noble_gas_mcmc.py:95-104 runs one well) -- or one chain per walker over all
     * its wells (0).  Per-well: every (walker w, well l) is a P-dimensional chain c = l W + w
     * with its own Metropolis decision, lamb / scaling / n_acc_tune (PyMC3 default lamb
     * 2.38 / sqrt(2 P)); logp, lamb, scaling, n_acc_tune and the logs are [L][W] (the order
     * of theta's rows).  The proposal noise and the accept draw of a unit are keyed by
     * cid = (well0 + l) n_chains_total + chain0 + w; the history partner indices by the
     * walker chain0 + w (the wells of a walker draw the same indices, each into its own
     * history, which keeps the joint chains' history layout and its 512-B loads; every
     * well's chain is still exactly a DEMetropolisZ chain).  So a run of all L wells equals
     * L runs of one well each (well0 = l) chain for chain. */
    int32_t per_well;
    /* Wells of the whole run whose streams this call's wells [well0, well0 + L) are part of:
     * ngrtd_demcz_run rejects well0 + L > n_wells_total, so that two calls never share a
     * well's random streams by accident.  0: unchecked (the caller keeps well0 ranges
     * disjoint). */
    int32_t n_wells_total;
    int64_t well0;           /* global index of well 0 (per-well streams) */
    /* Per call, like accepted_log: [n_steps][chains] PyMC3's `accept` sample stat,
     * exp(logp(x*) - logp(x)) (DEMetropolisZ.astep), device memory; NULL = not logged. */
    double* accept_log;
} ngrtd_demcz_state;
int ngrtd_demcz_run(ngrtd_plan* plan, double* theta, double* logp, int64_t W, int64_t n_steps,
                    ngrtd_demcz_state* state, uint8_t* accepted_log, double* logp_log,
                    uint64_t* n_accepted);

/* Per-unit log-probabilities: out[l][w] = log-likelihood + log-prior [+ log|Jacobian|] of
 * (walker w, well l) alone -- the log-prob of one well's PyMC3 model (the reference builds
 * one model per well, run_age_mcmc.py:122-231 / noble_gas_mcmc.py:216-267); ngrtd_logp is
 * its sum over wells.  The per-well sampler's initial log-probs. */
int ngrtd_logp_units(ngrtd_plan* plan, const double* theta, int64_t W, double* out, int32_t mem);

/* The elementwise math of the device DEMetropolisZ step, for samplers that restate its
 * arithmetic (sampler.DEMetropolisZ on torch ops) and must agree with it bit for bit.
 * Device pointers, enqueued on the context stream.
 * ngrtd_pymc3_backward: x = backward(u) of PyMC3 3.11's default transforms
 * (pymc3/distributions/transforms.py; the Beta / Uniform / HalfNormal free variables of
 * run_age_mcmc_utils.py:286-344 and noble_gas_mcmc.py:224-250): u, x [lead][P][inner], row p
 * with transform kind[p] (enum ngrtd_transform) and interval bounds a[p], b[p] (P <=
 * NGRTD_ROLE_COUNT); exp is the table-driven one the kernels use (<= 1 ulp).
 * ngrtd_fm_log: out = log(in), the kernels' table-driven log (<= 1 ulp): the accept draw's
 * log(u) of metrop_select (pymc3 step_methods/arraystep.py). */
int ngrtd_pymc3_backward(ngrtd_ctx* ctx, const double* u, double* x, int64_t lead, int32_t P, int64_t inner,
                         const int32_t* kind, const double* a, const double* b);
int ngrtd_fm_log(ngrtd_ctx* ctx, const double* in, double* out, int64_t n);

/* Host-only (no device needed): build the piecewise-Chebyshev surrogate the exponential
 * log-prob kernel uses for its channel sums and validate it against a long-double
 * evaluation of the same sums.  With s = 1/tau and s01 = exp(-(tp_1 - tp_0) s) (tp as in
 * gen_g_tp, convolution_integral_utils.py:168-174, for dtp = floor(t_samp - C_t.index[-1])):
 *   Z_c(tau) = s01 sum_{j>=0} A_c[1+j] exp(-j s)      c < C  (exponential g(tp), :184, times
 *                                                             the decay-folded series, :305-340)
 *   Z_C(tau) = s01 sum_{j=0}^{N-2} exp(-j s)                  (the normaliser g.sum(), :270)
 * cols: [C][N] channel columns (age order); coef (may be NULL): receives
 * [NGRTD_CHEB_PIECES][NGRTD_CHEB_N][(C+2)&~1], per piece the Chebyshev interpolant in
 * monomial form (coefficient k of x^k, x the piece's local coordinate in [-1, 1], as the
 * kernel evaluates it by Horner).  Pieces 0..75 split the octaves [2^-1, 2^18) of tau in
 * four: piece 4 (e + 1) + j holds tau = 2^e m (m in [1, 2)) with floor(4 (m - 1)) = j, and
 * x = 8 (m - 1.125 - j/4); piece 76 is the tail tau >= 2^18 in s = 1/tau, x = 2^19 s - 1; *max_rel_err: max |surrogate - exact| / exact over the
 * validation points.  Plans use the surrogate only when this is <= 5e-14. */
#define NGRTD_CHEB_N 12
#define NGRTD_CHEB_PIECES 77
int ngrtd_surrogate_check(const double* cols, int32_t C, int64_t N, double dtp, double* coef,
                          double* max_rel_err);

/* Host-only (no device needed): build the piecewise polynomial of the Student-t normaliser
 *   c0(nu) = lgamma((nu+1)/2) - lgamma(nu/2) - log(pi nu)/2
 * (PyMC3 3.11.2 StudentT.logp, the likelihoods of run_age_mcmc_utils.py:390/396 and
 * noble_gas_mcmc.py:266) that a plan evaluates instead of the lgamma difference, over
 * the binary octaves spanning [nu_lo, nu_hi] (the nu priors' supports): NGRTD_C0_SUB
 * pieces per octave, from octave *e0 (nu in [2^e0, 2^(e0+1))), piece p covering
 * nu = 2^(e0 + p/4) (1 + (p%4)/4 + [0, 1/4)); coef (may be NULL, room for
 * NGRTD_C0_MAX_PIECES * NGRTD_C0_N) receives [n_pieces][NGRTD_C0_N] monomial coefficients
 * (coefficient k of x^k, x = 8 (m - 1 - (2 (p%4) + 1)/8), m = nu / 2^(e0 + p/4)).
 * *max_abs_err: max |table - lgammal| over 41 points per piece (HUGE_VAL: no table, e.g.
 * nu_lo <= 0, non-finite, or more than NGRTD_C0_MAX_PIECES pieces).  Plans use the table
 * when this is <= 2e-14, else the exact expression. */
#define NGRTD_C0_N 12
#define NGRTD_C0_SUB 4
#define NGRTD_C0_MAX_PIECES 64
int ngrtd_c0_check(double nu_lo, double nu_hi, double* coef, int32_t* e0, int32_t* n_pieces,
                   double* max_abs_err);

/* Host-only (no GPU): the exp_pist_flow channel-table rows a plan with tau1 ~ U(., tau_hi),
 * eta1 ~ U(., eta_hi) stages in LDS at series length N, age grid tp_k = k + dtp (k >= 1)
 * (ngrtd.hip epm_window: the head block of every in-support unit's first unmasked age of
 * convolution_integral_utils.py:189's mask, plus 64 rows); *rows = -1 when the priors bound no
 * window smaller than the series.  Exposed so that tests check the bound against the mask. */
int ngrtd_epm_window_check(double tau_hi, double eta_hi, double dtp, int32_t N, int32_t* rows);

#ifdef __cplusplus
}
#endif
#endif /* NGRTD_H */
