// ngrtd.hip -- host side of libngrtd.so: the C ABI of include/ngrtd.h.
//
// Owns device state (series, channel tables, plan workspaces), builds the RTD channel
// tables (fixed-half-life decay and 4He/SF6 accumulation folded per tracer, as
// convolution_integral_utils.py:305-333 applies them), chooses the launch geometry and
// enqueues the kernels of ngrtd_kernels.hpp on the context stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>
#include <thread>

#include "../../include/ngrtd.h"
#include "ngrtd_kernels.hpp"
#include "ngrtd_prep.hpp"
#include "ngrtd_frac.hpp"
#include "ngrtd_dzc.hpp"

using namespace ngrtd;

namespace ngrtd {
// ngrtd_dz.hip: the single-launch DEMetropolisZ instances (compiled without machine LICM)
hipError_t launch_fused_dz_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                    const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st);
bool fused_dz_instance_exists(int mix);
// ngrtd_dzc.hip: the lane-chain DEMetropolisZ instances (RTD-only / CE-only models, per-well chains)
bool dz_chain_instance_exists(int C, int mix);
hipError_t launch_dz_chain(int C, int mix, const RtdArgs& a, const UnitArgs& u, const DemcAccept& da, int64_t U,
                           size_t lds, size_t max_lds, hipStream_t st);
// ngrtd_gen.hip: the generic-component log-prob instances (MIX bit 6, gen_component)
bool gen_instance_exists(int C, bool full, int mix);
hipError_t launch_fused_gen_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W,
                                     double* logp, const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st);
// ngrtd_lw.hip: the log-prob instances with the sampled CFC12 half-life (MIX bit 5)
hipError_t launch_fused_lw_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W,
                                    double* logp, const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st);
}

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    double* d() const { return static_cast<double*>(p); }
};

struct SeriesHost {
    std::vector<double> c, idx;
    double dtp = 0.0;
    int64_t n = 0;
};

struct TableDev {
    DevBuf buf;
    DevBuf frag;            // MFMA A-operand fragments (rtd_exp_mfma_kernel)
    DevBuf cheb;            // Chebyshev surrogate of the exponential channel sums (cheb_build)
    bool cheb_ok = false;
    double cheb_err = -1.0; // max relative error measured by the validation (-1: not built)
    DevBuf epm;             // exp_pist_flow block-tail surrogates (epm_prepare)
    DevBuf disp;            // dispersion components: 1 / tp_k, tp_k^(-3/2) (RtdArgs::disp_aux)
    DevBuf disp_rows;       // ... with the channel rows, one 64-B row per age (RtdArgs::disp_rows)
    bool epm_ok = false;
    double epm_err = -1.0;
    int epm_nb = 0, epm_p0 = 0, epm_np = 0;
    std::vector<std::vector<double>> cols_host;   // channel columns (kept for cheb_build)
    int S_seg = 1, Lseg = 0, nsteps = 0;
    int C = 0, CP = 0;
    int chan_tracer[kMaxChan] = {}, chan_isB[kMaxChan] = {}, chan_lamw[kMaxChan] = {};
};

struct LaunchStats {
    double ms[4] = {0, 0, 0, 0};
    int64_t n[4] = {0, 0, 0, 0};
};

}  // namespace

struct ngrtd_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    bool profiling = false;
    int next_series = 0;
    std::map<int, SeriesHost> series;
    // conv-API channel tables keyed by (series, lambda bits, accum, per-set decay)
    std::map<std::tuple<int, uint64_t, int, int>, std::unique_ptr<TableDev>> tables;
    DevBuf stage[16];
    std::vector<hipEvent_t> event_pool;   // recycled profiling events
    hipEvent_t take_event() {
        if (!event_pool.empty()) { hipEvent_t e = event_pool.back(); event_pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
};

namespace {
struct PendingTiming { int kind; hipEvent_t a, b; };
}

struct ngrtd_plan {
    ngrtd_ctx* ctx = nullptr;
    ngrtd_model_desc desc{};
    int64_t max_w = 0;
    // device copies of the model data
    DevBuf ce_obs, ce_sd, ce_emin, rtd_obs, rtd_sd, ce_lam, rtd_lam, welldata;
    TableDev table;
    int N = 0;
    double tp0 = 1e-5, dtp = 0.0;
    // workspaces
    DevBuf conc, ulogp, theta_stage, out_stage, ce_stage;
    DevBuf demc_prop[2], demc_lp, demc_acc;   // ngrtd_demcz_run scratch
    DevBuf demc_xw[2];      // the multi-step launch's walker-major state [P][W][L] (natural, transformed)
    DevBuf demc_pw;         // ... and per-well chains' lp, lamb, scaling [W][L] f64 + n_acc_tune [W][L] i32
    DevBuf disp_pre;        // disp_wide_kernel's partial sums [G][C + 1][U] (RtdArgs::disp_pre)

    RtdArgs rtd{};
    UnitArgs unit{};
    LaunchStats stats;
    std::vector<PendingTiming> pending;   // event pairs not yet read back (no host sync per launch)
    hipEvent_t region[2] = {nullptr, nullptr};   // around the last ngrtd_logp_n call's launches
    bool region_set = false;
};

static int drain_timings(ngrtd_plan* p);

// ------------------------------------------------------------------ helpers
static int set_err(ngrtd_ctx* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
static int set_err(ngrtd_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

#define HIP_TRY(ctx, expr)                                                                        \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return set_err((ctx), NGRTD_EDEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                           __FILE__, __LINE__);                                                   \
    } while (0)

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

static double lam_of(double t_half) {
    // update_pars / thalf_2_lambda (:117-121, :150): a falsy t_half means no decay
    return (t_half != 0.0) ? -1 * std::log(0.5) / t_half : 0.0;
}

static double host_betaln(double a, double b) { return std::lgamma(a) + std::lgamma(b) - std::lgamma(a + b); }

// Build the channel table [N][CP] of a set of tracers.  Per tracer: A_k = c_k d_k and,
// for 4He/SF6 accumulation, B_k = idx_k d_k (conc = (sum A w + J sum B w) / sum w);
// d_k = exp(-lam tp_k) (3He: 1 - exp(-lam tp_k)) unless the decay is per-unit (lamw).
// An identically-zero A (He4_ter: C_t * 0.0, run_age_mcmc.py:212) is dropped.
struct TracerBuild {
    const SeriesHost* s;
    int accum;
    double lam;
    bool lamw;
};

// Channels of per-unit-decay tracers (lamw: the sampled CFC12 half-life) come first, so that
// the single-launch kernel's LW instances find it at channel 0 (a compile-time index).
static int build_table(ngrtd_ctx* ctx, const std::vector<TracerBuild>& trs, TableDev& tab) {
    const int64_t N = trs[0].s->n;
    std::vector<std::vector<double>> cols;
    int C = 0;
    std::vector<size_t> order;
    for (int pass = 0; pass < 2; ++pass)
        for (size_t t = 0; t < trs.size(); ++t)
            if (trs[t].lamw == (pass == 0)) order.push_back(t);
    for (size_t t : order) {
        const TracerBuild& tb = trs[t];
        if (tb.s->n != N) return set_err(ctx, NGRTD_EINVAL, "tracers must share the series length");
        std::vector<double> d(N, 1.0);
        if (!tb.lamw) {
            for (int64_t k = 0; k < N; ++k) {
                const double tp = (k == 0) ? (0.0 + 1e-5) + tb.s->dtp : (double)k + tb.s->dtp;
                const double e = std::exp(-tb.lam * tp);
                d[k] = (tb.accum == NGRTD_ACC_HE3) ? (1 - e) : e;
            }
        } else if (tb.accum == NGRTD_ACC_HE3) {
            return set_err(ctx, NGRTD_EINVAL, "per-unit decay with 3He accumulation is not supported");
        }
        bool anyA = false;
        std::vector<double> A(N), B;
        for (int64_t k = 0; k < N; ++k) {
            A[k] = tb.s->c[k] * d[k];
            anyA |= (tb.s->c[k] != 0.0);
        }
        const bool hasB = (tb.accum == NGRTD_ACC_HE4 || tb.accum == NGRTD_ACC_SF6);
        if (anyA || !hasB) {
            if (C >= kMaxChan) return set_err(ctx, NGRTD_EINVAL, "more than %d RTD channels", kMaxChan);
            tab.chan_tracer[C] = (int)t; tab.chan_isB[C] = 0; tab.chan_lamw[C] = tb.lamw;
            cols.push_back(std::move(A));
            ++C;
        }
        if (hasB) {
            if (C >= kMaxChan) return set_err(ctx, NGRTD_EINVAL, "more than %d RTD channels", kMaxChan);
            B.resize(N);
            for (int64_t k = 0; k < N; ++k) B[k] = tb.s->idx[k] * d[k];
            tab.chan_tracer[C] = (int)t; tab.chan_isB[C] = 1; tab.chan_lamw[C] = tb.lamw;
            cols.push_back(std::move(B));
            ++C;
        }
    }
    tab.C = C;
    tab.CP = (C + 1) & ~1;
    tab.cols_host = cols;
    std::vector<double> h((size_t)N * tab.CP, 0.0);
    for (int c = 0; c < C; ++c)
        for (int64_t k = 0; k < N; ++k) h[(size_t)k * tab.CP + c] = cols[c][k];
    HIP_TRY(ctx, tab.buf.ensure(h.size() * sizeof(double) + 16));
    HIP_TRY(ctx, hipMemcpy(tab.buf.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    // MFMA fragment table (rtd_exp_mfma_kernel): S = 4*SG segments of Lseg ages; entry
    // [step][rt][lane] is the A operand of lane (row i = lane&15, k-slot kq = lane>>4) of row
    // tile rt: group g = 4*rt + (i>>2) -> channel g % C, segment s = 4*(g / C) + (i&3),
    // age index j = s*Lseg + 4*step + kq (table row 1 + j).
    if (C >= 1 && C <= kMaxChan) {
        const int R = mfma_rows(C), SG = mfma_groups_per_chan(C), S = 4 * SG;
        const int64_t n = std::max<int64_t>(N - 1, 0);
        const int64_t Lseg = cdiv(cdiv(n, S), 4) * 4;
        tab.S_seg = S;
        tab.Lseg = (int)Lseg;
        tab.nsteps = (int)(Lseg / 4);
        std::vector<double> fr((size_t)tab.nsteps * R * 64, 0.0);
        for (int step = 0; step < tab.nsteps; ++step)
            for (int rt = 0; rt < R; ++rt)
                for (int lane = 0; lane < 64; ++lane) {
                    const int i = lane & 15, kq = lane >> 4;
                    const int g = 4 * rt + (i >> 2);
                    if (g >= C * SG) continue;
                    const int c = g % C, sg = 4 * (g / C) + (i & 3);
                    const int64_t j = sg * Lseg + 4 * step + kq;
                    if (j < n) fr[((size_t)step * R + rt) * 64 + lane] = cols[c][1 + j];
                }
        HIP_TRY(ctx, tab.frag.ensure(fr.size() * sizeof(double) + 16));
        if (!fr.empty())
            HIP_TRY(ctx, hipMemcpy(tab.frag.p, fr.data(), fr.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return NGRTD_OK;
}

// ------------------------------------------------- Chebyshev surrogate tables
static_assert(kChebN == NGRTD_CHEB_N && kChebPieces == NGRTD_CHEB_PIECES, "surrogate geometry vs ngrtd.h");

// s01(s) * sum_{j=0}^{N-2} A_{1+j} e^{-j s} (s = 1/tau, s01 = e^{-d01 s}) in long double:
// the function the surrogate is fitted to and validated against.  `ones` sums 1 instead
// of A (the normaliser Z_G).
static long double cheb_exact(const std::vector<double>& A, long double s, long double d01, bool ones) {
    const long double q = expl(-s);
    long double y = 0.0L;
    for (size_t j = A.size(); j-- > 1;) y = y * q + (ones ? 1.0L : (long double)A[j]);
    return y * expl(-d01 * s);
}

// Fit kChebN Chebyshev coefficients per piece for the C channel functions and the
// normaliser (interpolation at the Chebyshev nodes of each piece), then validate every
// piece at 26 points per piece through the same cheb_piece/cheb_sums code the kernel runs.
// Returns the max relative error.  Channels with negative or non-finite entries are not
// expanded (HUGE_VAL): for non-negative columns the error is relative to |value|.
// d01 = tp_1 - tp_0 as the kernel forms it: (1 + dtp) - (1e-5 + dtp).
static double cheb_build(const std::vector<std::vector<double>>& cols, int C, double d01, std::vector<double>& coef,
                         int p_lo = 0, int p_hi = kChebPieces) {
    const int n = kChebN, CP = cheb_cp(C);
    coef.assign((size_t)kChebPieces * n * CP, 0.0);
    for (int c = 0; c < C; ++c)
        for (double v : cols[c])
            if (!(v >= 0.0) || !std::isfinite(v)) return HUGE_VAL;
    const long double PI = 3.14159265358979323846264338327950288L;
    const long double dd = d01;
    // power-basis coefficients of T_j: T_0 = 1, T_1 = x, T_{j+1} = 2x T_j - T_{j-1} (exact)
    std::vector<std::vector<long double>> Tm(n, std::vector<long double>(n, 0.0L));
    Tm[0][0] = 1.0L;
    if (n > 1) Tm[1][1] = 1.0L;
    for (int j = 2; j < n; ++j)
        for (int k = 0; k < n; ++k)
            Tm[j][k] = (k > 0 ? 2.0L * Tm[j - 1][k - 1] : 0.0L) - Tm[j - 2][k];
    long double cs[kChebN][kChebN], xn[kChebN];   // cos(pi j (k + 1/2) / n), the nodes
    for (int k = 0; k < n; ++k) {
        xn[k] = cosl(PI * (k + 0.5L) / n);
        for (int j = 0; j < n; ++j) cs[j][k] = cosl(PI * j * (k + 0.5L) / n);
    }
    // pieces split over host threads: fit, then validate (each piece's own coefficients)
    std::vector<double> worst_t(64, 0.0);
    auto work = [&](int t, int nt) {
        std::vector<long double> f(n), ch(n);
        double worst = 0.0;
        for (int p = p_lo + t; p < p_hi; p += nt) {
            for (int c = 0; c <= C; ++c) {
                const std::vector<double>& col = cols[c < C ? c : 0];
                for (int k = 0; k < n; ++k) {
                    long double sv;
                    if (p < kChebBinPieces) {
                        const int e = kChebOct0 + p / kChebSub, j = p % kChebSub;
                        sv = 1.0L / ldexpl(1.125L + 0.25L * j + xn[k] / 8.0L, e);
                    } else {
                        sv = 0.5L * (long double)kChebSHi * (1.0L + xn[k]);
                    }
                    f[k] = cheb_exact(col, sv, dd, c == C);
                }
                for (int j = 0; j < n; ++j) {
                    long double acc = 0.0L;
                    for (int k = 0; k < n; ++k) acc += f[k] * cs[j][k];
                    ch[j] = acc * (j == 0 ? 1.0L : 2.0L) / n;
                }
                // Chebyshev -> monomial coefficients in the piece's local x (long double): the
                // kernel evaluates one FMA per coefficient by Horner.  The coefficients decay
                // like rho^-j with rho ~ 25 (the strip |Im log tau| < pi/2 over half-width 1/8),
                // far above 1 + sqrt 2, so the monomial form amplifies rounding by ~1.1 only.
                for (int k = 0; k < n; ++k) {
                    long double m = 0.0L;
                    for (int j = k; j < n; ++j) m += ch[j] * Tm[j][k];
                    coef[((size_t)p * n + k) * CP + c] = (double)m;
                }
            }
            const int M = 24;
            for (int i = 0; i <= M + 1; ++i) {
                double tau;
                if (p < kChebBinPieces) {
                    const int e = kChebOct0 + p / kChebSub, j = p % kChebSub;
                    const long double tt = (i == 0) ? 0.0L : (i == M + 1) ? 1.0L - 1e-12L : (i - 0.5L) / M;
                    tau = (double)ldexpl(1.0L + 0.25L * (j + tt), e);
                } else {
                    const long double sv = (long double)kChebSHi * (i / (long double)(M + 1));
                    tau = (sv == 0.0L) ? HUGE_VAL : (double)(1.0L / sv);
                }
                double x = 0.0;
                const int pp = cheb_piece(tau, x);
                if (pp != p) { worst = HUGE_VAL; continue; }
                const long double sv = 1.0L / (long double)tau;
                for (int c = 0; c <= C; ++c) {
                    double y = 0.0;
                    cheb_sums<1>(coef.data() + (size_t)pp * n * CP + c, CP, x, &y);
                    const long double ex = cheb_exact(cols[c < C ? c : 0], sv, dd, c == C);
                    const double e = (ex > 0) ? (double)(fabsl((long double)y - ex) / ex) : (y == 0.0 ? 0.0 : HUGE_VAL);
                    if (!(e <= worst)) worst = e;   // NaN -> worst = NaN
                }
            }
        }
        worst_t[t] = worst;
    };
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t, nt);
    work(0, nt);
    for (auto& t : th) t.join();
    double worst = 0.0;
    for (int t = 0; t < nt; ++t)
        if (!(worst_t[t] <= worst)) worst = worst_t[t];
    return worst;
}

// Surrogate for a table whose exponential plan runs logp_fused_kernel.  Used only when the
// validation bound holds (kChebTol), else the kernel takes the exact matrix-core path.
constexpr double kChebTol = 5e-14;
static int cheb_prepare(ngrtd_ctx* ctx, TableDev& tab, double d01) {
    static const bool disabled = std::getenv("NGRTD_NO_CHEB") != nullptr;
    tab.cheb_ok = false;
    if (disabled || tab.C < 1 || tab.cols_host.empty() || tab.cols_host[0].size() < 2) return NGRTD_OK;
    std::vector<double> coef;
    tab.cheb_err = cheb_build(tab.cols_host, tab.C, d01, coef);
    if (!(tab.cheb_err <= kChebTol)) return NGRTD_OK;
    HIP_TRY(ctx, tab.cheb.ensure(coef.size() * sizeof(double)));
    HIP_TRY(ctx, hipMemcpy(tab.cheb.p, coef.data(), coef.size() * sizeof(double), hipMemcpyHostToDevice));
    tab.cheb_ok = true;
    return NGRTD_OK;
}

// exp_pist_flow block-tail surrogates: for every block b = 1.. with b S < N, per channel c
//   T_b,c(tau') = sum_{k >= b S} A_{c,k} e^{-(k - b S) / tau'}     (and the normaliser, A = 1)
// over the pieces [p_lo, p_hi) of epm_piece.  At one tau' ALL blocks' values come from one
// backward recursion over the series, R_k = A_k + q R_{k+1} (q = e^{-1/tau'}, long double),
// T_b = R_{b S}: the fit needs kChebN such passes per piece and the validation 26, instead of
// one sum per block and point.  The Chebyshev interpolant of each (block, piece, channel) is
// turned into monomial form (long double) and every piece is validated at 26 points through
// epm_piece + cheb_sums, the kernel's own code, at the plan tolerance kChebTol.  Threads split
// the pieces.  Used only if every table validates (else the plan keeps the multi-kernel path).
// nb_cap > 0: only blocks 1..nb_cap (the blocks a windowed table's units reach, epm_window).
static int epm_prepare(ngrtd_ctx* ctx, TableDev& tab, int N, int p_lo, int p_hi, int nb_cap = 0, bool mx = false) {
    tab.epm_ok = false;
    const int C = tab.C, S = kEpmBlock, n = kChebN;
    if (C < 1 || C > 5 || tab.cols_host.empty() || N <= S + 1 || p_lo < 0 || p_hi > kEpmPieces || p_hi <= p_lo)
        return NGRTD_OK;
    for (int c = 0; c < C; ++c)
        for (double v : tab.cols_host[c])
            if (!(v >= 0.0) || !std::isfinite(v)) return NGRTD_OK;   // the relative bound needs A >= 0
    const int nb = nb_cap > 0 ? std::min((N - 1) / S, nb_cap) : (N - 1) / S;   // b S < N for b = 1..nb
    const int np = p_hi - p_lo;
    // the C channel columns only (the kernel sums the normaliser's tail in closed form),
    // channel-major, read with 16-B loads; mx (plans with the sampled half-life, the LW
    // instances): mixed precision (ngrtd_kernels.hpp epm_tail_eval1), C runs of kEpmK64
    // doubles then C runs of kEpmK32 floats
    const size_t per = (size_t)epm_piece_doubles(C, mx);
    std::vector<double> h((size_t)nb * np * per, 0.0);
    const long double PI = 3.14159265358979323846264338327950288L;
    std::vector<std::vector<long double>> Tm(n, std::vector<long double>(n, 0.0L));
    Tm[0][0] = 1.0L;
    Tm[1][1] = 1.0L;
    for (int j = 2; j < n; ++j)
        for (int k = 0; k < n; ++k)
            Tm[j][k] = (k > 0 ? 2.0L * Tm[j - 1][k - 1] : 0.0L) - Tm[j - 2][k];
    // tail values of every block at s = 1/tau': out[(b - 1) C + c]
    auto tails = [&](long double sv, std::vector<long double>& out) {
        const long double q = expl(-sv);
        out.assign((size_t)nb * C, 0.0L);
        for (int c = 0; c < C; ++c) {
            long double r = 0.0L;
            for (int k = N - 1; k >= S; --k) {
                r = r * q + (long double)tab.cols_host[c][k];
                if (k % S == 0 && k / S <= nb) out[(size_t)(k / S - 1) * C + c] = r;   // (nb_cap: blocks 1..nb)
            }
        }
    };
    auto s_of = [&](int p, long double x) {       // s = 1/tau' at local x of piece p
        if (p < kEpmBinPieces) {
            const int e = kEpmOct0 + p / kChebSub, j = p % kChebSub;
            return 1.0L / ldexpl(1.125L + 0.25L * j + x / 8.0L, e);
        }
        return 0.5L * (long double)kChebSHi * (1.0L + x);
    };
    long double cs[kChebN][kChebN], xn[kChebN];   // cos(pi j (k + 1/2) / n), the nodes
    for (int k = 0; k < n; ++k) {
        xn[k] = cosl(PI * (k + 0.5L) / n);
        for (int j = 0; j < n; ++j) cs[j][k] = cosl(PI * j * (k + 0.5L) / n);
    }
    std::vector<double> worst_t(64, 0.0);
    auto work = [&](int t, int nt) {
        std::vector<long double> f((size_t)n * nb * C), v;
        double worst = 0.0;
        for (int p = p_lo + t; p < p_hi; p += nt) {
            for (int k = 0; k < n; ++k) {          // values at the Chebyshev nodes
                tails(s_of(p, xn[k]), v);
                std::copy(v.begin(), v.end(), f.begin() + (size_t)k * nb * C);
            }
            for (int b = 0; b < nb; ++b)
                for (int c = 0; c < C; ++c) {
                    long double ch[kChebN];
                    for (int j = 0; j < n; ++j) {
                        long double acc = 0.0L;
                        for (int k = 0; k < n; ++k)
                            acc += f[((size_t)k * nb + b) * C + c] * cs[j][k];
                        ch[j] = acc * (j == 0 ? 1.0L : 2.0L) / n;
                    }
                    double* pd = h.data() + ((size_t)b * np + (p - p_lo)) * per;
                    for (int k = 0; k < n; ++k) {
                        long double m = 0.0L;
                        for (int j = k; j < n; ++j) m += ch[j] * Tm[j][k];
                        if (!mx) pd[(size_t)c * n + k] = (double)m;
                        else if (k < kEpmK64) pd[(size_t)c * kEpmK64 + k] = (double)m;
                        else reinterpret_cast<float*>(pd + (size_t)kEpmK64 * C)[(size_t)c * kEpmK32 + (k - kEpmK64)] = (float)m;
                    }
                }
            const int M = 24;                        // validation: 26 points per piece
            for (int i = 0; i <= M + 1; ++i) {
                double taup;
                if (p < kEpmBinPieces) {
                    const int e = kEpmOct0 + p / kChebSub, j = p % kChebSub;
                    const long double tt = (i == 0) ? 0.0L : (i == M + 1) ? 1.0L - 1e-12L : (i - 0.5L) / M;
                    taup = (double)ldexpl(1.0L + 0.25L * (j + tt), e);
                } else {
                    const long double sv = (long double)kChebSHi * (i / (long double)(M + 1));
                    taup = (sv == 0.0L) ? HUGE_VAL : (double)(1.0L / sv);
                }
                double x = 0.0;
                if (epm_piece(taup, x) != p) { worst = HUGE_VAL; continue; }
                tails(1.0L / (long double)taup, v);
                for (int b = 0; b < nb; ++b)
                    for (int c = 0; c < C; ++c) {
                        const double y = epm_tail_eval1(h.data() + ((size_t)b * np + (p - p_lo)) * per, C, c, x, mx);
                        const long double ex = v[(size_t)b * C + c];
                        const double e = (ex > 0) ? (double)(fabsl((long double)y - ex) / ex) : (y == 0.0 ? 0.0 : HUGE_VAL);
                        if (!(e <= worst)) worst = e;   // NaN -> worst = NaN
                    }
            }
        }
        worst_t[t] = worst;
    };
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t, nt);
    work(0, nt);
    for (auto& t : th) t.join();
    double worst = 0.0;
    for (int t = 0; t < nt; ++t)
        if (!(worst_t[t] <= worst)) worst = worst_t[t];
    tab.epm_err = worst;
    if (!(worst <= kChebTol)) {
        // no table: the plan runs the multi-kernel path (ngrtd_plan_info info[11] = 0); the
        // instances compile one piece format, so there is no all-double retry (kEpmMixedAll)
        if (std::getenv("NGRTD_VERBOSE"))
            std::fprintf(stderr, "ngrtd: exp_pist_flow block-tail table (%s pieces) fails validation: max rel err %.3g > %.3g\n",
                         mx ? "mixed" : "double", worst, kChebTol);
        return NGRTD_OK;
    }
    HIP_TRY(ctx, tab.epm.ensure(h.size() * sizeof(double)));
    HIP_TRY(ctx, hipMemcpy(tab.epm.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    tab.epm_ok = true;
    tab.epm_nb = nb;
    tab.epm_p0 = p_lo;
    tab.epm_np = np;
    return NGRTD_OK;
}

// Student-t normaliser table (ngrtd_math.hpp c0_piece / c0_poly) over the octaves of
// [lo, hi]: per piece, the Chebyshev interpolant of c0 at kC0N nodes from lgammal, turned
// into monomial coefficients in long double, then checked at 40 points per piece (ends
// included) through the kernel's own c0_piece + c0_poly against lgammal.  Returns the
// worst absolute error (HUGE_VAL when the range has no table: non-finite, <= 0, or more
// than kC0MaxPieces pieces).
constexpr double kC0Tol = 2e-14;
static long double c0_ref(long double nu) {
    const long double PI = 3.14159265358979323846264338327950288L;
    return lgammal(0.5L * (nu + 1.0L)) - lgammal(0.5L * nu) - 0.5L * logl(PI * nu);
}
static double c0_build(double lo, double hi, std::vector<double>& tab, int& e0, int& np) {
    tab.clear();
    np = 0;
    if (!(lo > 0.0) || !(hi >= lo) || !std::isfinite(hi) || !std::isnormal(lo)) return HUGE_VAL;
    int ea, eb;
    (void)std::frexp(lo, &ea);
    (void)std::frexp(hi, &eb);
    e0 = ea - 1;                          // lo in [2^e0, 2^(e0+1))
    np = (eb - ea + 1) * kC0Sub;
    if (np > kC0MaxPieces) { np = 0; return HUGE_VAL; }
    const int n = kC0N;
    const long double PI = 3.14159265358979323846264338327950288L;
    std::vector<std::vector<long double>> Tm(n, std::vector<long double>(n, 0.0L));
    Tm[0][0] = 1.0L;
    Tm[1][1] = 1.0L;
    for (int j = 2; j < n; ++j)
        for (int k = 0; k < n; ++k)
            Tm[j][k] = (k > 0 ? 2.0L * Tm[j - 1][k - 1] : 0.0L) - Tm[j - 2][k];
    tab.assign((size_t)np * n, 0.0);
    std::vector<long double> f(n), ch(n);
    for (int p = 0; p < np; ++p) {
        const long double sc = ldexpl(1.0L, e0 + p / kC0Sub), c = 1.125L + 0.25L * (p % kC0Sub);
        for (int k = 0; k < n; ++k) f[k] = c0_ref(sc * (c + cosl(PI * (k + 0.5L) / n) / 8.0L));
        for (int j = 0; j < n; ++j) {
            long double acc = 0.0L;
            for (int k = 0; k < n; ++k) acc += f[k] * cosl(PI * j * (k + 0.5L) / n);
            ch[j] = acc * (j == 0 ? 1.0L : 2.0L) / n;
        }
        for (int k = 0; k < n; ++k) {
            long double m = 0.0L;
            for (int j = k; j < n; ++j) m += ch[j] * Tm[j][k];
            tab[(size_t)p * n + k] = (double)m;
        }
    }
    double worst = 0.0;
    const int M = 40;
    for (int p = 0; p < np; ++p) {
        const double base = std::ldexp(1.0 + 0.25 * (p % kC0Sub), e0 + p / kC0Sub);
        const double w = std::ldexp(0.25, e0 + p / kC0Sub);
        for (int i = 0; i <= M; ++i) {
            double nu = (i == M) ? std::nextafter(base + w, 0.0) : base + w * i / M;
            double x = 0.0;
            const int pp = c0_piece(nu, e0, np, x);
            if (pp != p) return HUGE_VAL;
            const double e = (double)fabsl((long double)c0_poly(tab.data() + (size_t)pp * n, x) - c0_ref(nu));
            if (!(e <= worst)) worst = e;   // NaN -> worst = NaN
        }
    }
    return worst;
}

static void set_frag(RtdArgs& a, const TableDev& tab) {
    for (int c = 0; c < kMaxChan; ++c)
        a.tab0[c] = (c < tab.C && !tab.cols_host.empty()) ? tab.cols_host[c][0] : 0.0;
    a.frag = tab.frag.d();
    a.nsteps = tab.nsteps;
    a.S_seg = tab.S_seg;
    a.Lseg = tab.Lseg;
}

// ------------------------------------------------------- RTD kernel dispatch
typedef void (*RtdKernel)(RtdArgs);

template <int R, int C, bool L>
static RtdKernel rtd_k() { return rtd_conc_kernel<R, C, L>; }

static RtdKernel pick_rtd(int R, int C, bool lamw) {
#define NGRTD_CASE_C(RR, LL)                                                                          \
    switch (C) {                                                                                      \
    case 1: return rtd_k<RR, 1, LL>(); case 2: return rtd_k<RR, 2, LL>(); case 3: return rtd_k<RR, 3, LL>(); \
    case 4: return rtd_k<RR, 4, LL>(); case 5: return rtd_k<RR, 5, LL>(); case 6: return rtd_k<RR, 6, LL>(); \
    case 7: return rtd_k<RR, 7, LL>(); case 8: return rtd_k<RR, 8, LL>(); default: return nullptr;      \
    }
    if (lamw) {
        if (R == 1) { NGRTD_CASE_C(1, true) }
        if (R == 2) { NGRTD_CASE_C(2, true) }
        return nullptr;
    }
    if (R == 1) { NGRTD_CASE_C(1, false) }
    if (R == 2) { NGRTD_CASE_C(2, false) }
    if (R == 4) { NGRTD_CASE_C(4, false) }
#undef NGRTD_CASE_C
    return nullptr;
}

struct RtdGeom {
    int R, NW, LW, blocks;
    size_t lds;
};

static RtdGeom rtd_geometry(int64_t U, int N, int C, bool lamw) {
    RtdGeom g{};
    const int CP = (C + 1) & ~1;
    int Rmax = (C <= 5) ? 4 : 2;
    if (lamw) Rmax = std::min(Rmax, 2);
    int R = Rmax;
    while (R > 1 && cdiv(U, 64 * R) < 512) R /= 2;
    g.R = R;
    g.NW = 4;
    const int max_rows = (64 * 1024) / (CP * 8);
    g.LW = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(N, g.NW), max_rows / g.NW));
    g.blocks = (int)cdiv(U, 64 * R);
    const size_t tab_bytes = (size_t)g.NW * g.LW * CP * sizeof(double);
    const size_t comb_bytes = (size_t)g.NW * R * (C + 1) * 64 * sizeof(double);
    g.lds = std::max(tab_bytes, comb_bytes);
    return g;
}

static bool mfma_path(const RtdArgs& a, bool lamw) {
    static const bool disabled = std::getenv("NGRTD_NO_MFMA") != nullptr;
    return !disabled && a.mod[0] == MOD_EXP && a.mod[1] == MOD_NONE && !lamw && a.C >= 1 && a.C <= kMaxChan &&
           a.frag != nullptr;
}

// Dynamic LDS of the MFMA kernel: one fragment chunk, at least 56 KiB so that no more than
// two 256-unit blocks share a CU (an odd third block would double that CU's matrix-core
// time while others idle: tools/mfma_probe.hip).
static size_t mfma_lds(const RtdArgs& a) {
    const size_t chunk = (size_t)std::min(a.nsteps, kMfmaLdsBytes / (mfma_rows(a.C) * 512)) * mfma_rows(a.C) * 512;
    return std::max<size_t>(chunk, 56 * 1024);
}

template <int C>
static void launch_mfma(const RtdArgs& a, const UnitArgs& u, int32_t fuse, hipStream_t st) {
    const unsigned blocks = (unsigned)cdiv(a.U, kMfmaUnitsPerBlock);
    hipLaunchKernelGGL(rtd_exp_mfma_kernel<C>, dim3(blocks), dim3(64 * mfma_waves(C)), mfma_lds(a), st, a, u, fuse);
}

// Single-launch log-prob (logp_fused_kernel): exponential RTD on the MFMA path with 4
// tiles per wave (C <= 5), the whole fragment table in LDS next to the 512 per-unit
// partial sums, and L <= 512 wells.
// LDS: the 512 per-unit partial sums, the surrogate table (the exact path's fragments are
// read from global memory: they are needed only by waves with an uncovered tau) and the
// packed per-well data (ce obs, 1/sd^2, sums of 0.5 log 1/sd^2, E_min; rtd obs, 1/sd^2,
// sums; the Student-t normaliser table).
constexpr size_t kFusedMaxLds = 157 * 1024;   // gfx950: 160 KiB per workgroup, less the static fexp/flog tables
static size_t fused_lds(const RtdArgs& a, const UnitArgs& u, int dz_p = 0) {
    // EPM: the channel table, rows of cheb_cp(C) doubles in LDS (the kernel's layout; the global
    // table's rows are a.CP = (C + 1) & ~1, shorter for C = 2, 4)
    // generic instances with a dispersion component: fexp_tab's table (the per-age operands are
    // read from global memory with scalar loads, any N)
    const bool disp = a.disp_aux && a.disp_rows && (a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP);
    const size_t epm_tab = ((a.mod[0] == MOD_EPM || a.mod[1] == MOD_EPM) ? (size_t)epm_lds_doubles(a.epm_nw, cheb_cp(a.C)) : 0) +
                           (disp ? (size_t)kDispExpTab : 0);
    const size_t dz = (size_t)dz_p * kFusedUnits;                          // DZ step: the proposals
    // generic instances, dispersion split over the unit's two waves: the theta waves' partial sums
    const size_t xch = (disp && a.disp_split > 0) ? (size_t)(a.C + 1) * kFusedUnits : 0;
    return (size_t)(kFusedHdr + a.cheb_np * cheb_lds_stride(a.C) + epm_tab + u.wd_n + dz + xch) *
           sizeof(double);
}
// Surrogate pieces the fused kernel stages: when the unit's log-prob carries the tau1
// Uniform prior and the RTD's tau is tau1, only the pieces over the prior's support
// [tau1_lo, tau1_hi] -- a tau outside it makes the log-prob -inf whatever the channel sums
// (the kernel's `skip` lanes), so no lane reads another piece.  Else the whole table.
// The smallest tau_eff = 1 / (1 / tau + lam) of the sampled CFC12 half-life (LW) over tau >= tau_lo
// and the thalf_cfc prior's support: t_half in [thalf_b, thalf_a + thalf_b], lam = ln2 / t_half
// (0 when there is no such half-life or its range reaches 0: no bound).
static double lw_tau_lo(const RtdArgs& a, double tau_lo) {
    if (a.row_thalf < 0) return tau_lo;
    const double tmin = std::min(a.thalf_b, a.thalf_a + a.thalf_b);
    if (!(tmin > 0.0)) return 0.0;
    return tau_lo * tmin / (tmin + kLn2Ref * tau_lo);
}
// The exp_pist_flow channel-table rows a single-launch EPM plan stages in LDS (RtdArgs::epm_nw;
// the kernel's side: epm_sums).  The whole table fits LDS up to N ~ 1600 (C = 5); the
// reference's own runs convolve N = 25 256 ages (run_age_mcmc.py:46,209), 1.24 MB.  But a unit
// reads only its head block [B - 16, B) of the table, B = (m / 16 + 1) 16 past its first unmasked
// age m (the tail comes from the block-tail surrogate), and m is bounded over the priors'
// support: tp_m >= tau (1 - 1/eta) is first met at m <= ceil(tau1_hi (1 - 1/eta1_hi) - dtp).  So a
// plan whose exp_pist_flow component is tau1 / eta1 under their Uniform priors stages rows
// [0, (m_max / 16 + 1) 16 + 80) (the +64 rows serve the exact short tails, which no unit of the
// support needs: the block-tail table covers its tau'); units outside the support box have
// log-prob -inf by their priors and epm_sums gives them finite zero sums (or NaN where the
// reference's weights are NaN).  NGRTD_EPM_WINDOW: 1 (default) only when the whole table does not
// fit with room for a DEMetropolisZ step's rows beside it (kEpmDzMargin: the single-launch and the
// lane-chain steps add up to kDzMaxP proposal rows per unit slot; windowing the plain log-prob of
// such a plan too keeps one table for every launch of the plan -- in-support units get the same
// sums from either table), 2 whenever the window is smaller (A/B runs), 0 never.
static int epm_window_rows(double tau_hi, double eta_hi, double dtp, int N) {
    if (!(tau_hi >= 0.0 && eta_hi >= 1.0) || !std::isfinite(tau_hi) || !std::isfinite(eta_hi)) return -1;
    const double mm = std::ceil(tau_hi * (1 - 1 / eta_hi) - dtp) + 1.0;
    if (!(mm >= 0.0 && mm < (double)N)) return -1;
    return ((int)mm / kEpmBlock + 1) * kEpmBlock + 64 + kEpmBlock;
}
static void epm_window(RtdArgs& a, const UnitArgs& u) {
    static const int mode = [] {
        const char* e = std::getenv("NGRTD_EPM_WINDOW");
        return e ? std::atoi(e) : 1;
    }();
    a.epm_nw = (int)cdiv(a.N, kEpmBlock) * kEpmBlock;
    a.ew_on = 0;
    if (mode == 0 || a.mod[0] != MOD_EPM || !(a.mod[1] == MOD_NONE || a.mod[1] == MOD_PISTON) || !a.epm) return;
    if (!u.rtd_on || !(u.flags & NGRTD_WANT_PRIOR) || u.row_eta1 < 0 || a.row_tau[0] != u.row_tau1 ||
        a.row_eta[0] != u.row_eta1 || (a.row_thalf >= 0 && a.row_thalf != u.row_thalf))
        return;
    if (!(u.tau1_lo <= u.tau1_hi && u.eta1_lo <= u.eta1_hi && u.eta1_lo > 0.0)) return;
    const int rows = epm_window_rows(u.tau1_hi, u.eta1_hi, a.dtp, a.N);
    if (rows < 0 || rows >= a.epm_nw || rows / kEpmBlock > a.epm_nb) return;
    constexpr size_t kEpmDzMargin = (size_t)kDzMaxP * kFusedUnits * sizeof(double);
    if (mode == 1 && fused_lds(a, u, 0) + kEpmDzMargin <= kFusedMaxLds) return;
    a.epm_nw = rows;
    a.ew_on = 1;
    a.ew_tau_lo = u.tau1_lo; a.ew_tau_hi = u.tau1_hi;
    a.ew_eta_lo = u.eta1_lo; a.ew_eta_hi = u.eta1_hi;
}
static void cheb_window_tau(RtdArgs& a, const UnitArgs& u);
// the staged windows of a single-launch plan: the surrogate pieces and the EPM table rows
static void cheb_window(RtdArgs& a, const UnitArgs& u) {
    cheb_window_tau(a, u);
    epm_window(a, u);
}
static void cheb_window_tau(RtdArgs& a, const UnitArgs& u) {
    a.cheb_p0 = 0;
    a.cheb_np = a.cheb ? kChebPieces : 0;
    if (!a.cheb || !u.rtd_on || !(u.flags & NGRTD_WANT_PRIOR) || a.row_tau[0] != u.row_tau1) return;
    double x;
    // LW plans also read channel 0 at tau_eff <= tau: the window starts at the least tau_eff
    // (a thalf_cfc outside its prior makes the log-prob -inf, like a tau outside tau1's)
    const double lo = (a.row_thalf >= 0 && u.row_thalf >= 0) ? lw_tau_lo(a, u.tau1_lo) : u.tau1_lo;
    if (!(lo > 0.0)) return;
    const int pa = cheb_piece(std::max(lo, kChebTauLo), x), pb = cheb_piece(u.tau1_hi, x);
    if (pa < 0 || pb < pa) return;
    a.cheb_p0 = pa;
    a.cheb_np = pb - pa + 1;
}
// A per-unit CFC12 half-life (row_thalf) runs in the single launch (the LW instances) when it
// decays exactly one channel, channel 0 (build_table puts it first), with the instance
// counts of lw_instance (C = 5 for the joint plans, C = 4 or 5 otherwise).
// The FULL instances' plan: the joint model (CE and RTD blocks, priors and likelihoods) with
// the reference's Beta priors, which they compile in (kRefBeta: the set of the plan's Jacobian
// flag and sampled half-life, compared exactly with add_beta's split).  Other joint plans run
// the runtime-flag instances.  NGRTD_NO_REFB=1 treats every plan as other (A/B runs).
static bool full_plan(const RtdArgs& a, const UnitArgs& u) {
    const bool joint = u.ce_on && u.rtd_on && (u.flags & NGRTD_WANT_LIKE) && (u.flags & NGRTD_WANT_PRIOR);
    if (!joint || std::getenv("NGRTD_NO_REFB")) return false;
    const BetaExp& e = kRefBeta[((u.flags & NGRTD_WANT_JACOBIAN) ? 1 : 0) + (a.row_thalf >= 0 ? 2 : 0)];
    if (u.bt_n != e.n) return false;
    for (int i = 0; i < e.n; ++i)
        if (u.bt_ia[i] != e.ia[i] || u.bt_ib[i] != e.ib[i] || u.bt_fa[i] != e.fa[i] || u.bt_fb[i] != e.fb[i])
            return false;
    return true;
}
static bool lw_instance(const RtdArgs& a, const UnitArgs& u, int C) {
    return full_plan(a, u) ? C == 5 : (C == 4 || C == 5);
}
static bool lw_ok(const RtdArgs& a, const UnitArgs& u) {
    if (a.row_thalf < 0) return true;
    int n = 0;
    for (int c = 0; c < a.C; ++c) n += a.chan_lamw[c] ? 1 : 0;
    return n == 1 && a.chan_lamw[0] && !a.chan_isB[0] && lw_instance(a, u, a.C);
}
static bool fused_path(const RtdArgs& a0, const UnitArgs& u) {
    static const bool disabled = std::getenv("NGRTD_NO_FUSED") != nullptr;
    RtdArgs a = a0;
    cheb_window(a, u);
    // exponential first component on the matrix-core / surrogate path, optionally mixed
    // with a piston second component (BMM exponential-piston, one lookup per unit)
    // or an exp_pist_flow first component with validated block-tail surrogates
    RtdArgs a1 = a;
    a1.mod[1] = MOD_NONE;
    a1.mod[0] = MOD_EXP;
    const bool mod2 = a.mod[1] == MOD_NONE || a.mod[1] == MOD_PISTON;
    const bool mods = mod2 && (a.mod[0] == MOD_EXP || (a.mod[0] == MOD_EPM && a.epm != nullptr));
    return !disabled && mods && mfma_path(a1, false) && lw_ok(a, u) && a.C <= 5 && u.L >= 1 &&
           u.L <= kFusedUnits && fused_lds(a, u) <= kFusedMaxLds;
}
// The generic instances (MIX bit 6, ngrtd_gen.hip) for the model pairs fused_path does not
// take: the staged surrogate window covers the Uniform priors' supports of every exponential
// component's tau (tau1, tau2; down to the least tau_eff with the sampled half-life), or the
// whole table when a component's tau has no prior in the plan.
static bool gen_mods(const RtdArgs& a) {
    auto ok = [](int m) { return m == MOD_PISTON || m == MOD_EXP || m == MOD_EPM || m == MOD_DISP; };
    return ok(a.mod[0]) && (a.mod[1] == MOD_NONE || ok(a.mod[1]));
}
static void gen_cheb_window(RtdArgs& a, const UnitArgs& u) {
    a.cheb_p0 = 0;
    a.cheb_np = a.cheb ? kChebPieces : 0;
    if (!a.cheb) return;
    int pa = kChebPieces, pb = -1;
    for (int c = 0; c < 2; ++c) {
        if (a.mod[c] != MOD_EXP) continue;
        const bool t1 = a.row_tau[c] == u.row_tau1, t2 = a.row_tau[c] == u.row_tau2 && u.row_tau2 >= 0;
        if (!u.rtd_on || !(u.flags & NGRTD_WANT_PRIOR) || !(t1 || t2)) return;   // no bound: every piece
        double lo = t1 ? u.tau1_lo : u.tau2_lo;
        const double hi = t1 ? u.tau1_hi : u.tau2_hi;
        if (a.row_thalf >= 0 && u.row_thalf >= 0) lo = lw_tau_lo(a, lo);
        double x;
        if (!(lo > 0.0)) return;
        const int qa = cheb_piece(std::max(lo, kChebTauLo), x), qb = cheb_piece(hi, x);
        if (qa < 0 || qb < qa) return;
        pa = std::min(pa, qa);
        pb = std::max(pb, qb);
    }
    if (pb < pa) {   // no exponential component: nothing staged
        a.cheb_np = 0;
        return;
    }
    a.cheb_p0 = pa;
    a.cheb_np = pb - pa + 1;
}
// The dispersion component's age split between the unit's theta and RTD waves (the kernel's GEN
// branch): the theta waves sum the first 55 % of the ages (their CE block is shorter than the
// RTD waves' concentrations + likelihood: the log-prob gains up to 0.65-0.7, but the DEMetropolisZ
// step, whose theta waves also stage the proposals, loses from 0.6 on and must use the same split
// for bitwise chains: profiles/r05ab_dispersion_split_ab.txt, r05ad_dispersion_split_dz_ab.txt),
// when the theta waves' partial sums fit the LDS budget (else the RTD wave sums all ages).
// NGRTD_NO_DISP_SPLIT=1 disables it, NGRTD_DISP_SPLIT_FRAC sets the share (A/B runs).
static void gen_disp_split(RtdArgs& a, const UnitArgs& u) {
    static const bool off = std::getenv("NGRTD_NO_DISP_SPLIT") != nullptr;
    static const double frac = [] {   // NGRTD_DISP_SPLIT_FRAC: the theta waves' share of the ages (A/B)
        const char* e = std::getenv("NGRTD_DISP_SPLIT_FRAC");
        const double f = e ? std::atof(e) : 0.55;
        return (f > 0.0 && f < 1.0) ? f : 0.55;
    }();
    a.disp_split = 0;
    if (off || a.disp_pre || !a.disp_aux || !(a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP) || a.N < 2) return;
    a.disp_split = std::max(1, std::min(a.N - 1, (int)(a.N * frac)));
    if (fused_lds(a, u) > kFusedMaxLds) a.disp_split = 0;
}
static int gen_mix(const RtdArgs& a, const UnitArgs& u) {
    const bool disp = a.disp_aux && (a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP);   // the dispersion instances
    return 64 | (disp ? 128 : 0) | (a.row_thalf >= 0 ? 32 : 0) | (full_plan(a, u) && (u.flags & NGRTD_WANT_JACOBIAN) ? 4 : 0);
}
static bool gen_path(const RtdArgs& a0, const UnitArgs& u) {
    static const bool disabled = std::getenv("NGRTD_NO_GEN") != nullptr;
    if (disabled || !gen_mods(a0) || fused_path(a0, u)) return false;
    RtdArgs a = a0;
    gen_cheb_window(a, u);
    gen_disp_split(a, u);
    const bool exp_c = a.mod[0] == MOD_EXP || a.mod[1] == MOD_EXP;
    const bool epm_c = a.mod[0] == MOD_EPM || a.mod[1] == MOD_EPM;
    const bool disp_c = a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP;
    if ((exp_c && !a.cheb) || (epm_c && !a.epm) || (disp_c && (!a.disp_aux || !a.disp_rows))) return false;
    return a.C >= 1 && a.C <= 5 && lw_ok(a, u) && u.L >= 1 && u.L <= kFusedUnits &&
           fused_lds(a, u) <= kFusedMaxLds && gen_instance_exists(a.C, full_plan(a, u), gen_mix(a, u));
}
// one launch for the plan's log-prob / forward outputs: a specialised or a generic instance
static bool single_path(const RtdArgs& a, const UnitArgs& u) { return fused_path(a, u) || gen_path(a, u); }

// Waves per unit group (logp_fused_kernel ROLES): 2 = theta-only and RTD blocks in separate
// waves (default), 1 = one wave runs the whole unit.  NGRTD_FUSED_ROLES overrides (A/B runs).
static int fused_roles() {
    static const int r = [] {
        const char* e = std::getenv("NGRTD_FUSED_ROLES");
        return (e && std::atoi(e) == 1) ? 1 : 2;
    }();
    return r;
}
template <int C, bool FULL, int ROLES, int MIX>
static void launch_fused_cfr(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                             const DemcAccept& da, hipStream_t st) {
    static const bool attr = [] {   // dynamic LDS above 64 KiB (many wells) needs the opt-in
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&logp_fused_kernel<C, FULL, ROLES, MIX>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFusedMaxLds);
        return true;
    }();
    (void)attr;
    // DZ step, transformed chains: the chains'-space proposal rows
    const int dz_p = ((MIX & 8) && (MIX & 4)) ? da.P : 0;
    hipLaunchKernelGGL((logp_fused_kernel<C, FULL, ROLES, MIX>), dim3((unsigned)cdiv(W, WB)),
                       dim3(64 * kFusedWaves * ROLES), fused_lds(a, u, dz_p), st, a, u, WB, logp, da);
}
template <int C, bool FULL>
static void launch_fused_cf(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                            const DemcAccept& da, hipStream_t st) {
    const int mix = (a.mod[1] == MOD_PISTON ? 1 : 0) | (a.mod[0] == MOD_EPM ? 2 : 0);
    switch (mix) {
    case 1: launch_fused_cfr<C, FULL, 2, 1>(a, u, WB, W, logp, da, st); break;
    case 2: launch_fused_cfr<C, FULL, 2, 2>(a, u, WB, W, logp, da, st); break;
    case 3: launch_fused_cfr<C, FULL, 2, 3>(a, u, WB, W, logp, da, st); break;
    default:
        if (fused_roles() == 2) launch_fused_cfr<C, FULL, 2, 0>(a, u, WB, W, logp, da, st);
        else launch_fused_cfr<C, FULL, 1, 0>(a, u, WB, W, logp, da, st);
    }
}
// FULL instances: CE + RTD blocks, priors and likelihoods on (the joint model), without or
// -- single-component RTD -- with the transform Jacobians (the transformed-space sampler)
template <int C>
static void launch_fused_c(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                           const DemcAccept& da, hipStream_t st) {
    const bool joint = full_plan(a, u);
    const bool jac = (u.flags & NGRTD_WANT_JACOBIAN) != 0;
    if (joint && !jac) launch_fused_cf<C, true>(a, u, WB, W, logp, da, st);
    else if (joint && a.mod[1] == MOD_NONE && a.mod[0] == MOD_EXP) launch_fused_cfr<C, true, 2, 4>(a, u, WB, W, logp, da, st);
    else if (joint && a.mod[1] == MOD_NONE && a.mod[0] == MOD_EPM) launch_fused_cfr<C, true, 2, 6>(a, u, WB, W, logp, da, st);
    else if (C == 5 && joint && a.mod[1] == MOD_PISTON) {   // the BMMs' transformed-space log-prob (c4: 5 channels)
        if (a.mod[0] == MOD_EXP) launch_fused_cfr<C, true, 2, 5>(a, u, WB, W, logp, da, st);
        else launch_fused_cfr<C, true, 2, 7>(a, u, WB, W, logp, da, st);
    } else launch_fused_cf<C, false>(a, u, WB, W, logp, da, st);
}
// Single-launch DEMetropolisZ step (logp_fused_kernel MIX bit 3): the joint plan on a
// FULL instance with C = 5 channels (the c3 / c4 / published-model workloads), the role-split
// layout, at most kDzMaxP parameter rows, and the proposals fitting in LDS.  -1: not
// available (ngrtd_demcz_run then runs the proposal kernel + log-prob kernel pair).
// The generic model pairs (gen_path: dispersion, piston first, exponential / exp_pist_flow
// seconds) step on the generic DZ instances (MIX 64 | 8, + 128 with a dispersion component)
// when they carry no sampled half-life.
static void dz_window(RtdArgs& a, const UnitArgs& u, bool gen) {
    if (gen) {
        gen_cheb_window(a, u);
        gen_disp_split(a, u);
    } else {
        cheb_window(a, u);
    }
}
static int dz_mix(const RtdArgs& a0, const UnitArgs& u, int P, bool transformed) {
    RtdArgs a = a0;
    const bool joint = full_plan(a, u);
    const bool jac = (u.flags & NGRTD_WANT_JACOBIAN) != 0;
    // transformed chains <=> the Jacobian instance (its proposals go through backward())
    if (!joint || jac != transformed || a.C != 5 || fused_roles() != 2 || P < 1 || P > kDzMaxP) return -1;
    const bool gen = !fused_path(a0, u) && gen_path(a0, u);
    dz_window(a, u, gen);
    if (gen) {
        // (a small-ensemble dispersion plan sums its ages in disp_wide_kernel ahead of the log-prob
        // launch: its steps run the proposal / log-prob / accept kernels)
        if (a.row_thalf >= 0 || a.disp_pre || fused_lds(a, u, transformed ? P : 0) > kFusedMaxLds) return -1;
        const int r = 8 | (jac ? 4 : 0) | (gen_mix(a, u) & (64 | 128));
        return fused_dz_instance_exists(r) ? r : -1;
    }
    if (!fused_path(a, u) || fused_lds(a, u, transformed ? P : 0) > kFusedMaxLds) return -1;
    const int mix = (a.mod[1] == MOD_PISTON ? 1 : 0) | (a.mod[0] == MOD_EPM ? 2 : 0) | (a.row_thalf >= 0 ? 32 : 0);
    const int r = 8 | (jac ? 4 : 0) | mix;   // 12 (exponential), 13 / 15 (BMMs), 14 (exp_pist_flow) (+ 32: LW)
    return fused_dz_instance_exists(r) ? r : -1;
}
// The lane-chain step (ngrtd_dzc.hpp dz_chain_kernel) for the plans the reference itself
// samples: its RTD-only model (1 or 4 tracers, exponential / exp_pist_flow first component,
// optional piston second, the sampled CFC12 half-life) and its CE-only model; per-well chains,
// at most kDzcMaxP rows, the tables and the proposal rows fitting in LDS.  -1: none.
static int dzc_mix(const RtdArgs& a0, const UnitArgs& u, int P, bool transformed, size_t* lds) {
    const bool jac = (u.flags & NGRTD_WANT_JACOBIAN) != 0;
    if (jac != transformed || P < 1 || P > kDzcMaxP) return -1;
    RtdArgs a = a0;
    int mix, C = 1;
    if (u.ce_on && !u.rtd_on) {
        mix = 64 | (jac ? 4 : 0);
        a.cheb_np = 0;
        a.N = 0;
    } else if (u.rtd_on && !u.ce_on) {
        cheb_window(a, u);
        if (!fused_path(a, u)) return -1;
        C = a.C;
        mix = (a.mod[1] == MOD_PISTON ? 1 : 0) | (a.mod[0] == MOD_EPM ? 2 : 0) | (jac ? 4 : 0) |
              (a.row_thalf >= 0 ? 32 : 0);
    } else {
        return -1;
    }
    if (!dz_chain_instance_exists(C, mix)) return -1;
    *lds = dzc_lds_doubles(C, mix, (mix & 64) ? 0 : a.cheb_np, a.epm_nw, u.wd_n, P) * sizeof(double);
    return *lds <= kFusedMaxLds ? mix : -1;
}
// Every theta row a single-launch step reads is one of ThetaPre's (the 6 CE rows, tau1,
// nu_rtd: the joint exponential plan), all of them staged in the LDS proposal rows: no
// second RTD component, eta, D, f1, J, half-life or SF6 rows, no further Beta rows.
static bool dz_theta_all_lds(const RtdArgs& a, const UnitArgs& u, int P) {
    return P == 8 && a.row_tau[1] < 0 && a.row_eta[0] < 0 && a.row_eta[1] < 0 && a.row_D[0] < 0 && a.row_D[1] < 0 &&
           a.row_f1 < 0 && a.row_J < 0 && a.row_thalf < 0 && a.row_lamsf6 < 0 && u.bt_n <= 6;
}
static int launch_fused_dz(ngrtd_ctx* ctx, const RtdArgs& a0, const UnitArgs& u, int64_t W, int L, double* logp,
                           hipStream_t st, const DemcAccept& da, int mix) {
    const int WB = kFusedUnits / L;
    RtdArgs a = a0;
    dz_window(a, u, (mix & 64) != 0);
    const int dz_p = (mix & 4) ? da.P : 0;    // transformed chains: the chains'-space proposal rows
    size_t lds = fused_lds(a, u, dz_p);
    // the natural proposal rows in LDS too where they fit (not next to the EPM channel
    // table); NGRTD_DZ_PROP_GLOBAL=1 reads them back from dz_prop instead (A/B runs)
    DemcAccept d = da;
    // first the chains' state for the whole launch (DemcAccept::state_lds: rows [P][512] and
    // 3.5 per-chain doubles per slot; NGRTD_DZ_STATE_GLOBAL=1 keeps it in global memory, A/B)
    const size_t sb = ((size_t)da.P * kFusedUnits + 3 * kFusedUnits + kFusedUnits / 2) * sizeof(double);
    d.state_lds = (lds + sb <= kFusedMaxLds && !std::getenv("NGRTD_DZ_STATE_GLOBAL")) ? 1 : 0;
    const size_t pb = (size_t)da.P * kFusedUnits * sizeof(double);
    d.prop_lds = (lds + pb + (d.state_lds ? sb : 0) <= kFusedMaxLds && !std::getenv("NGRTD_DZ_PROP_GLOBAL")) ? 1 : 0;
    if (d.prop_lds) lds += pb;
    if (d.state_lds) lds += sb;   // after the proposal rows (logp_fused_kernel's carve-up)
    // no global proposal rows when nothing reads them (NGRTD_DZ_PROP_WRITE=1 writes them, A/B)
    d.prop_skip = (d.prop_lds && dz_theta_all_lds(a, u, da.P) && !std::getenv("NGRTD_DZ_PROP_WRITE")) ? 1 : 0;
    if (!fused_dz_instance_exists(mix)) return set_err(ctx, NGRTD_EINVAL, "no single-launch DEMetropolisZ instance %d", mix);
    HIP_TRY(ctx, launch_fused_dz_instance(mix, a, u, WB, W, logp, d, lds, kFusedMaxLds, st));
    return NGRTD_OK;
}
// Walkers per block of a log-prob launch: kFusedUnits / L fills all 8 unit waves of every
// block, but a small ensemble then leaves most CUs idle (a c5 shard, 256 walkers x 64 wells:
// 32 blocks on 256 CUs; c3, 2048 walkers x 1 well: 4).  Fewer walkers per block (halving)
// until the grid covers the CUs; the blocks' unit waves past WB L units skip their body.
// NGRTD_FUSED_WB=max keeps kFusedUnits / L (A/B runs).
constexpr int kCUs = 256;
static int fused_wb(int64_t W, int L) {
    static const bool fixed = [] {
        const char* e = std::getenv("NGRTD_FUSED_WB");
        return e && std::strcmp(e, "max") == 0;
    }();
    int wb = kFusedUnits / L;
    if (fixed) return wb;
    while (wb > 1 && cdiv(W, wb) < kCUs) wb /= 2;
    return wb;
}
// Small ensembles with a dispersion component (the reference's own runs: one well, 3 chains,
// N = 25 256): the component's ages go across the lanes of disp_wide_kernel (G blocks of
// kDispWideThreads per unit) instead of along one lane per unit, and the generic log-prob
// launch reads the sums (RtdArgs::disp_pre).  A plan-time choice -- the sums' order then does
// not depend on the launch's walker count: plans of at most kDispWideUnits units (L x
// max_walkers) with exactly one dispersion component and the interleaved rows; the flags
// NGRTD_DISP_WIDE / NGRTD_DISP_LANE force either geometry.  G: enough blocks to cover the CUs
// (kCUs / units), each lane summing at least kDispWideMinAges ages.  Returns G (0: lane loop).
constexpr int64_t kDispWideUnits = 256;
constexpr int kDispWideMinAges = 8;
static int disp_wide_plan(const RtdArgs& a, int32_t flags, int64_t Umax) {
    const int nd = (a.mod[0] == MOD_DISP ? 1 : 0) + (a.mod[1] == MOD_DISP ? 1 : 0);
    if (nd != 1 || !a.disp_aux || !a.disp_rows || a.C < 1 || a.C > 5 || a.N < 1 || (flags & NGRTD_DISP_LANE)) return 0;
    if (!(flags & NGRTD_DISP_WIDE) && Umax > kDispWideUnits) return 0;
    const int64_t gmax = std::max<int64_t>(1, a.N / ((int64_t)kDispWideThreads * kDispWideMinAges));
    const int64_t want = std::max<int64_t>(1, cdiv(kCUs, std::max<int64_t>(Umax, 1)));
    return (int)std::min<int64_t>({want, gmax, 64});
}
template <int C>
static void launch_disp_wide_c(const RtdArgs& a, int comp, hipStream_t st) {
    const dim3 grid((unsigned)a.disp_pre_g, (unsigned)a.U);
    if (a.row_thalf >= 0)
        hipLaunchKernelGGL((disp_wide_kernel<C, true>), grid, dim3(kDispWideThreads), 0, st, a, comp, a.disp_pre_g,
                           const_cast<double*>(a.disp_pre));
    else
        hipLaunchKernelGGL((disp_wide_kernel<C, false>), grid, dim3(kDispWideThreads), 0, st, a, comp, a.disp_pre_g,
                           const_cast<double*>(a.disp_pre));
}
// the dispersion sums ahead of a generic log-prob / forward launch of a wide plan (no-op otherwise)
static int launch_disp_wide(ngrtd_ctx* ctx, const RtdArgs& a, const UnitArgs& u, hipStream_t st) {
    if (!a.disp_pre || a.U <= 0 || fused_path(a, u)) return NGRTD_OK;
    if (a.U > 65535) return set_err(ctx, NGRTD_EINVAL, "disp_wide_kernel: %lld units", (long long)a.U);
    const int comp = a.mod[0] == MOD_DISP ? 0 : 1;
    switch (a.C) {
    case 1: launch_disp_wide_c<1>(a, comp, st); break;
    case 2: launch_disp_wide_c<2>(a, comp, st); break;
    case 3: launch_disp_wide_c<3>(a, comp, st); break;
    case 4: launch_disp_wide_c<4>(a, comp, st); break;
    default: launch_disp_wide_c<5>(a, comp, st); break;
    }
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}
static int launch_fused(ngrtd_ctx* ctx, const RtdArgs& a0, const UnitArgs& u, int64_t W, int L, double* logp,
                        hipStream_t st, const DemcAccept* dap = nullptr) {
    const int WB = fused_wb(W, L);
    RtdArgs a = a0;
    const DemcAccept da = dap ? *dap : DemcAccept{};
    if (!fused_path(a0, u)) {   // the generic instances (gen_path)
        gen_cheb_window(a, u);
        gen_disp_split(a, u);
        HIP_TRY(ctx, launch_fused_gen_instance(a.C, full_plan(a, u), gen_mix(a, u), a, u, WB, W, logp, da, fused_lds(a, u),
                                               kFusedMaxLds, st));
        return NGRTD_OK;
    }
    cheb_window(a, u);
    if (a.row_thalf >= 0) {   // the sampled CFC12 half-life (ngrtd_lw.hip, lw_ok)
        const bool joint = full_plan(a, u);
        const bool jac = (u.flags & NGRTD_WANT_JACOBIAN) != 0;
        const bool single = a.mod[1] == MOD_NONE;
        const bool full = joint && (!jac || single);
        const int mix = 32 | (a.mod[1] == MOD_PISTON ? 1 : 0) | (a.mod[0] == MOD_EPM ? 2 : 0) | (full && jac ? 4 : 0);
        HIP_TRY(ctx, launch_fused_lw_instance(a.C, full, mix, a, u, WB, W, logp, da, fused_lds(a, u), kFusedMaxLds, st));
        return NGRTD_OK;
    }
    switch (a.C) {
    case 1: launch_fused_c<1>(a, u, WB, W, logp, da, st); break;
    case 2: launch_fused_c<2>(a, u, WB, W, logp, da, st); break;
    case 3: launch_fused_c<3>(a, u, WB, W, logp, da, st); break;
    case 4: launch_fused_c<4>(a, u, WB, W, logp, da, st); break;
    default: launch_fused_c<5>(a, u, WB, W, logp, da, st); break;
    }
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}

// Enqueue the RTD kernel.  On the MFMA path with `ua` non-null the kernel also evaluates
// the per-unit log-prob (fused epilogue); *fused reports whether it did.
static int launch_rtd(ngrtd_ctx* ctx, RtdArgs a, bool lamw, hipStream_t st, const UnitArgs* ua = nullptr,
                      bool* fused = nullptr) {
    if (fused) *fused = false;
    if (a.U <= 0) return NGRTD_OK;
    if (mfma_path(a, lamw)) {
        UnitArgs u{};
        int32_t fuse = 0;
        if (ua) { u = *ua; fuse = 1; }
        switch (a.C) {
        case 1: launch_mfma<1>(a, u, fuse, st); break;
        case 2: launch_mfma<2>(a, u, fuse, st); break;
        case 3: launch_mfma<3>(a, u, fuse, st); break;
        case 4: launch_mfma<4>(a, u, fuse, st); break;
        case 5: launch_mfma<5>(a, u, fuse, st); break;
        case 6: launch_mfma<6>(a, u, fuse, st); break;
        case 7: launch_mfma<7>(a, u, fuse, st); break;
        default: launch_mfma<8>(a, u, fuse, st); break;
        }
        HIP_TRY(ctx, hipGetLastError());
        if (fused) *fused = fuse != 0;
        return NGRTD_OK;
    }
    const RtdGeom g = rtd_geometry(a.U, a.N, a.C, lamw);
    RtdKernel k = pick_rtd(g.R, a.C, lamw);
    if (!k) return set_err(ctx, NGRTD_EINVAL, "no RTD kernel for R=%d C=%d", g.R, a.C);
    a.LW = g.LW;
    hipLaunchKernelGGL(k, dim3(g.blocks), dim3(64 * g.NW), g.lds, st, a);
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}

static hipStream_t S(ngrtd_ctx* c) { return c->stream; }

// Staging: host pointers are copied into ctx buffers; device pointers pass through.
static int stage_in(ngrtd_ctx* ctx, int slot, const double* src, int64_t n, int32_t mem, const double** out) {
    if (!src) { *out = nullptr; return NGRTD_OK; }
    if (mem == NGRTD_MEM_DEVICE) { *out = src; return NGRTD_OK; }
    HIP_TRY(ctx, ctx->stage[slot].ensure((size_t)n * sizeof(double)));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->stage[slot].p, src, (size_t)n * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    *out = ctx->stage[slot].d();
    return NGRTD_OK;
}

#define NG_CHECK(x)                 \
    do {                            \
        int _r = (x);               \
        if (_r != NGRTD_OK) return _r; \
    } while (0)

extern "C" {

int ngrtd_abi_version(void) { return NGRTD_ABI_VERSION; }

int ngrtd_create(ngrtd_ctx** out, int device) {
    if (!out) return NGRTD_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return NGRTD_EDEVICE;
    if (device < 0 || device >= n) return NGRTD_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return NGRTD_EDEVICE;
    auto* c = new (std::nothrow) ngrtd_ctx;
    if (!c) return NGRTD_ENOMEM;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return NGRTD_EDEVICE; }
    c->stream = c->own;
    *out = c;
    return NGRTD_OK;
}

int ngrtd_destroy(ngrtd_ctx* ctx) {
    if (!ctx) return NGRTD_ESTATE;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    ctx->event_pool.clear();
    ctx->tables.clear();
    for (auto& b : ctx->stage) { if (b.p) (void)hipFree(b.p); b.p = nullptr; b.cap = 0; }
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    delete ctx;
    return NGRTD_OK;
}

const char* ngrtd_last_error(const ngrtd_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ngrtd_set_stream(ngrtd_ctx* ctx, void* s) {
    if (!ctx) return NGRTD_ESTATE;
    ctx->stream = static_cast<hipStream_t>(s);   // NULL is HIP's null (default) stream
    return NGRTD_OK;
}

int ngrtd_synchronize(ngrtd_ctx* ctx) {
    if (!ctx) return NGRTD_ESTATE;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return NGRTD_OK;
}

int ngrtd_set_profiling(ngrtd_ctx* ctx, int on) {
    if (!ctx) return NGRTD_ESTATE;
    ctx->profiling = on != 0;
    return NGRTD_OK;
}

// ----------------------------------------------------------------- CE forward
int ngrtd_ce_forward(ngrtd_ctx* ctx, int32_t what, int32_t p_mode, const double* E, const double* T,
                     const double* Ae, const double* F, const double* P, const double* Sal, int64_t n,
                     const int32_t* gas_ids, int32_t n_gases, double* out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    if (n < 0 || !out) return set_err(ctx, NGRTD_EINVAL, "bad n/out");
    if (what < 0 || what > NGRTD_CE_PRESSURE) return set_err(ctx, NGRTD_EINVAL, "bad 'what' %d", what);
    if (p_mode < 0 || p_mode > 2) return set_err(ctx, NGRTD_EINVAL, "bad p_mode %d", p_mode);
    if (p_mode == NGRTD_P_GIVEN && !P) return set_err(ctx, NGRTD_EINVAL, "P required for NGRTD_P_GIVEN");
    const bool scalar_out = (what == NGRTD_CE_VAPOR_PRESSURE || what == NGRTD_CE_PRESSURE);
    if (!scalar_out && (n_gases < 1 || n_gases > kMaxGas || !gas_ids))
        return set_err(ctx, NGRTD_EINVAL, "n_gases must be 1..5");
    if (n == 0) return NGRTD_OK;
    CeArgs a{};
    a.what = what; a.p_mode = p_mode; a.G = scalar_out ? 1 : n_gases; a.n = n;
    for (int j = 0; j < (scalar_out ? 0 : n_gases); ++j) {
        if (gas_ids[j] < 0 || gas_ids[j] > 4) return set_err(ctx, NGRTD_EINVAL, "bad gas id %d", gas_ids[j]);
        a.gas[j] = gas_ids[j];
    }
    NG_CHECK(stage_in(ctx, 0, E, n, mem, &a.E));
    NG_CHECK(stage_in(ctx, 1, T, n, mem, &a.T));
    NG_CHECK(stage_in(ctx, 2, Ae, n, mem, &a.Ae));
    NG_CHECK(stage_in(ctx, 3, F, n, mem, &a.F));
    NG_CHECK(stage_in(ctx, 4, (p_mode == NGRTD_P_GIVEN) ? P : nullptr, n, mem, &a.P));
    NG_CHECK(stage_in(ctx, 5, Sal, n, mem, &a.S));
    const int64_t nout = n * a.G;
    if (mem == NGRTD_MEM_DEVICE) {
        a.out = out;
    } else {
        HIP_TRY(ctx, ctx->stage[6].ensure((size_t)nout * sizeof(double)));
        a.out = ctx->stage[6].d();
    }
    hipLaunchKernelGGL(ce_forward_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(ctx), a);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(out, a.out, (size_t)nout * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

// ---------------------------------------------------- prep ensemble propagation
int ngrtd_he_comps(ngrtd_ctx* ctx, const double* He4_obs, const double* He3_obs, const double* Ae,
                   const double* F, const double* E, const double* T, const double* Rterr, double Rterr_const,
                   int64_t n, double* out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    if (n < 0 || !out) return set_err(ctx, NGRTD_EINVAL, "bad n/out");
    if (!He4_obs || !He3_obs || !Ae || !F || !E || !T)
        return set_err(ctx, NGRTD_EINVAL, "He4_obs, He3_obs, Ae, F, E, T are required");
    if (n == 0) return NGRTD_OK;
    HeCompsArgs a{};
    a.n = n;
    a.Rterr_c = Rterr_const;
    NG_CHECK(stage_in(ctx, 0, He4_obs, n, mem, &a.He4));
    NG_CHECK(stage_in(ctx, 1, He3_obs, n, mem, &a.He3));
    NG_CHECK(stage_in(ctx, 2, Ae, n, mem, &a.Ae));
    NG_CHECK(stage_in(ctx, 3, F, n, mem, &a.F));
    NG_CHECK(stage_in(ctx, 4, E, n, mem, &a.E));
    NG_CHECK(stage_in(ctx, 5, T, n, mem, &a.T));
    NG_CHECK(stage_in(ctx, 6, Rterr, n, mem, &a.Rterr));
    const int64_t nout = n * NGRTD_HE_NOUT;
    if (mem == NGRTD_MEM_DEVICE) {
        a.out = out;
    } else {
        HIP_TRY(ctx, ctx->stage[7].ensure((size_t)nout * sizeof(double)));
        a.out = ctx->stage[7].d();
    }
    hipLaunchKernelGGL(he_comps_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(ctx), a);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(out, a.out, (size_t)nout * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

int ngrtd_cfc_corr(ngrtd_ctx* ctx, int32_t what, const int32_t* species, int32_t n_species, const double* E,
                   const double* T, const double* Ae, const double* F, const double* Sal, const double* P,
                   const double* x, int64_t n, double* out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    if (n < 0 || !out) return set_err(ctx, NGRTD_EINVAL, "bad n/out");
    if (what < 0 || what > NGRTD_CFC_LAPSE_RATE_ATM) return set_err(ctx, NGRTD_EINVAL, "bad 'what' %d", what);
    const bool scalar_out = (what == NGRTD_CFC_VAPOR_PRESSURE_ATM || what == NGRTD_CFC_LAPSE_RATE_ATM);
    if (!scalar_out) {
        if (n_species < 1 || n_species > NGRTD_MAX_CFC || !species)
            return set_err(ctx, NGRTD_EINVAL, "n_species must be 1..%d", NGRTD_MAX_CFC);
        if ((what == NGRTD_CFC_EQUIL_AIR || what == NGRTD_CFC_EQUIL_AQ || what == NGRTD_CFC_CE_EXC) && !x)
            return set_err(ctx, NGRTD_EINVAL, "x (C_meas / z_i) required");
        if (what == NGRTD_CFC_CE_EXC && !P) return set_err(ctx, NGRTD_EINVAL, "P (self.P, atm) required for ce_exc");
    }
    if (what == NGRTD_CFC_LAPSE_RATE_ATM ? !E : !T) return set_err(ctx, NGRTD_EINVAL, "E / T required");
    if (!scalar_out && (!E || !Ae || !F)) return set_err(ctx, NGRTD_EINVAL, "E, T, Ae, F are required");
    if (n == 0) return NGRTD_OK;
    CfcArgs a{};
    a.what = what;
    a.ns = scalar_out ? 1 : n_species;
    a.n = n;
    for (int j = 0; j < (scalar_out ? 0 : n_species); ++j) {
        if (species[j] < 0 || species[j] > NGRTD_SF6) return set_err(ctx, NGRTD_EINVAL, "bad species %d", species[j]);
        a.sp[j] = species[j];
    }
    NG_CHECK(stage_in(ctx, 0, E, n, mem, &a.E));
    NG_CHECK(stage_in(ctx, 1, T, n, mem, &a.T));
    NG_CHECK(stage_in(ctx, 2, scalar_out ? nullptr : Ae, n, mem, &a.Ae));
    NG_CHECK(stage_in(ctx, 3, scalar_out ? nullptr : F, n, mem, &a.F));
    NG_CHECK(stage_in(ctx, 4, scalar_out ? nullptr : Sal, n, mem, &a.S));
    NG_CHECK(stage_in(ctx, 5, what == NGRTD_CFC_CE_EXC ? P : nullptr, n, mem, &a.P));
    const bool reads_x = (what == NGRTD_CFC_EQUIL_AIR || what == NGRTD_CFC_EQUIL_AQ || what == NGRTD_CFC_CE_EXC);
    NG_CHECK(stage_in(ctx, 6, reads_x ? x : nullptr, n * a.ns, mem, &a.x));
    const int64_t nout = n * a.ns;
    if (mem == NGRTD_MEM_DEVICE) {
        a.out = out;
    } else {
        HIP_TRY(ctx, ctx->stage[7].ensure((size_t)nout * sizeof(double)));
        a.out = ctx->stage[7].d();
    }
    hipLaunchKernelGGL(cfc_corr_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(ctx), a);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(out, a.out, (size_t)nout * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

// --------------------------------------------------------------------- series
int ngrtd_series_create(ngrtd_ctx* ctx, const double* c_by_age, const double* idx_by_age, int64_t n,
                        double dtp, int32_t* series_id) {
    if (!ctx) return NGRTD_ESTATE;
    if (!c_by_age || n <= 0 || n > (int64_t)1 << 30 || !series_id)
        return set_err(ctx, NGRTD_EINVAL, "bad series arguments");
    SeriesHost s;
    s.n = n;
    s.dtp = dtp;
    s.c.assign(c_by_age, c_by_age + n);
    s.idx.resize(n);
    for (int64_t k = 0; k < n; ++k) s.idx[k] = idx_by_age ? idx_by_age[k] : (double)k;
    const int id = ctx->next_series++;
    ctx->series[id] = std::move(s);
    *series_id = id;
    return NGRTD_OK;
}

int ngrtd_series_destroy(ngrtd_ctx* ctx, int32_t id) {
    if (!ctx) return NGRTD_ESTATE;
    if (!ctx->series.erase(id)) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", id);
    for (auto it = ctx->tables.begin(); it != ctx->tables.end();)
        it = (std::get<0>(it->first) == id) ? ctx->tables.erase(it) : std::next(it);
    return NGRTD_OK;
}

static const SeriesHost* find_series(ngrtd_ctx* ctx, int id) {
    auto it = ctx->series.find(id);
    return it == ctx->series.end() ? nullptr : &it->second;
}

// --------------------------------------------------------- single-tracer conv
int ngrtd_conv(ngrtd_ctx* ctx, int32_t series_id, int32_t mod_type, int32_t accum, const double* tau,
               const double* eta, const double* D, const double* t_half, double t_half_const,
               const double* J, double J_const, int64_t n, double* out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    const SeriesHost* s = find_series(ctx, series_id);
    if (!s) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", series_id);
    if (mod_type < NGRTD_MOD_PISTON || mod_type > NGRTD_MOD_DISPERSION)
        return set_err(ctx, NGRTD_EINVAL, "bad mod_type %d", mod_type);
    if (accum < 0 || accum > 3) return set_err(ctx, NGRTD_EINVAL, "bad accum %d", accum);
    if (!tau || !out || n < 0) return set_err(ctx, NGRTD_EINVAL, "tau/out required");
    if (mod_type == NGRTD_MOD_EXP_PIST_FLOW && !eta) return set_err(ctx, NGRTD_EINVAL, "eta required");
    if (mod_type == NGRTD_MOD_DISPERSION && !D) return set_err(ctx, NGRTD_EINVAL, "D required");
    if (n == 0) return NGRTD_OK;
    const bool lamw = t_half != nullptr;
    const double lam = lamw ? 0.0 : lam_of(t_half_const);
    uint64_t lb;
    std::memcpy(&lb, &lam, 8);
    auto key = std::make_tuple((int)series_id, lb, (int)accum, (int)lamw);
    auto it = ctx->tables.find(key);
    if (it == ctx->tables.end()) {
        auto t = std::make_unique<TableDev>();
        NG_CHECK(build_table(ctx, {TracerBuild{s, accum, lam, lamw}}, *t));
        it = ctx->tables.emplace(key, std::move(t)).first;
    }
    const TableDev& tab = *it->second;
    // theta rows: 0 tau, 1 eta, 2 D, 3 t_half, 4 J (device, [5][n])
    HIP_TRY(ctx, ctx->stage[0].ensure((size_t)5 * n * sizeof(double)));
    double* th = ctx->stage[0].d();
    const double* rows[5] = {tau, eta, D, t_half, J};
    const hipMemcpyKind kind = (mem == NGRTD_MEM_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    for (int r = 0; r < 5; ++r)
        if (rows[r]) HIP_TRY(ctx, hipMemcpyAsync(th + (size_t)r * n, rows[r], (size_t)n * sizeof(double), kind, S(ctx)));
    RtdArgs a{};
    a.theta = th; a.U = n;
    a.row_tau[0] = 0; a.row_tau[1] = -1;
    a.row_eta[0] = eta ? 1 : -1; a.row_eta[1] = -1;
    a.row_D[0] = D ? 2 : -1; a.row_D[1] = -1;
    a.row_f1 = -1; a.row_lamsf6 = -1;
    a.row_thalf = lamw ? 3 : -1; a.thalf_a = 1.0; a.thalf_b = 0.0;
    a.row_J = J ? 4 : -1; a.J_is_log10 = 0;
    a.tab = tab.buf.d(); a.N = (int)s->n; a.C = tab.C; a.CP = tab.CP;
    a.tp0 = (0.0 + 1e-5) + s->dtp; a.dtp = s->dtp;
    a.mod[0] = mod_type; a.mod[1] = MOD_NONE;
    a.K = 1;
    for (int c = 0; c < tab.C; ++c) { a.chan_tracer[c] = tab.chan_tracer[c]; a.chan_isB[c] = tab.chan_isB[c]; a.chan_lamw[c] = tab.chan_lamw[c]; }
    a.tr_sf6[0] = 0; a.tr_J[0] = J_const;
    set_frag(a, tab);
    if (mem == NGRTD_MEM_DEVICE) {
        a.conc = out;
    } else {
        HIP_TRY(ctx, ctx->stage[1].ensure((size_t)n * sizeof(double)));
        a.conc = ctx->stage[1].d();
    }
    NG_CHECK(launch_rtd(ctx, a, lamw, S(ctx)));
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(out, a.conc, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

int ngrtd_rtd_weights(ngrtd_ctx* ctx, int32_t series_id, int32_t mod_type, double tau, double eta, double D,
                      double* g_out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    const SeriesHost* s = find_series(ctx, series_id);
    if (!s) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", series_id);
    if (mod_type < NGRTD_MOD_PISTON || mod_type > NGRTD_MOD_DISPERSION || !g_out)
        return set_err(ctx, NGRTD_EINVAL, "bad mod_type/g_out");
    double* g = g_out;
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, ctx->stage[2].ensure((size_t)s->n * sizeof(double)));
        g = ctx->stage[2].d();
    }
    hipLaunchKernelGGL(rtd_weights_kernel, dim3(1), dim3(1024), 0, S(ctx), mod_type, tau, eta, D,
                       (0.0 + 1e-5) + s->dtp, s->dtp, (int)s->n, g);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(g_out, g, (size_t)s->n * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

int ngrtd_conv_dot(ngrtd_ctx* ctx, int32_t series_id, const double* g, double t_half, int32_t accum, double J,
                   double* out, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    const SeriesHost* s = find_series(ctx, series_id);
    if (!s) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", series_id);
    if (!g || !out || accum < 0 || accum > 3) return set_err(ctx, NGRTD_EINVAL, "bad arguments");
    const int64_t n = s->n;
    HIP_TRY(ctx, ctx->stage[3].ensure((size_t)2 * n * sizeof(double)));
    double* cs = ctx->stage[3].d();
    HIP_TRY(ctx, hipMemcpyAsync(cs, s->c.data(), n * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    HIP_TRY(ctx, hipMemcpyAsync(cs + n, s->idx.data(), n * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    const double* gd;
    NG_CHECK(stage_in(ctx, 4, g, n, mem, &gd));
    double* o = out;
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, ctx->stage[5].ensure(sizeof(double)));
        o = ctx->stage[5].d();
    }
    hipLaunchKernelGGL(conv_dot_kernel, dim3(1), dim3(1024), 0, S(ctx), cs, cs + n, gd, lam_of(t_half), accum, J,
                       (0.0 + 1e-5) + s->dtp, s->dtp, (int)n, o);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        HIP_TRY(ctx, hipMemcpyAsync(out, o, sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

// ------------------------------------------------------- frac_inf_diff RTD
int ngrtd_frac_conv(ngrtd_ctx* ctx, int32_t series_id, int32_t accum, const double* tau, const double* D,
                    const double* bbar, const double* Phi_im, const double* f_tadv_ext, int64_t ext_stride,
                    const double* t_half, double t_half_const, const double* J, double J_const, int64_t n,
                    double* conc, double* g_out, double* fm_mu, int32_t mem) {
    if (!ctx) return NGRTD_ESTATE;
    const SeriesHost* s = find_series(ctx, series_id);
    if (!s) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", series_id);
    if (n < 0 || accum < 0 || accum > 3) return set_err(ctx, NGRTD_EINVAL, "bad n/accum");
    if (!bbar || !Phi_im) return set_err(ctx, NGRTD_EINVAL, "bbar and Phi_im are required");
    if (!f_tadv_ext && (!tau || !D)) return set_err(ctx, NGRTD_EINVAL, "tau and D are required without f_tadv_ext");
    if (f_tadv_ext && ext_stride != 0 && ext_stride < s->n)
        return set_err(ctx, NGRTD_EINVAL, "ext_stride must be 0 or >= N");
    if (!conc && !g_out && !fm_mu) return set_err(ctx, NGRTD_EINVAL, "no output requested");
    if (s->n < 2) return set_err(ctx, NGRTD_EINVAL, "series too short");
    if (n == 0) return NGRTD_OK;
    const int64_t N = s->n;
    if (n * N > ((int64_t)1 << 40)) return set_err(ctx, NGRTD_EINVAL, "n * N too large");
    FracArgs a{};
    a.N = (int32_t)N;
    a.n = n;
    a.dtp = s->dtp;
    a.tp0 = (0.0 + 1e-5) + s->dtp;
    a.ext_stride = ext_stride;
    NG_CHECK(stage_in(ctx, 0, f_tadv_ext ? nullptr : tau, n, mem, &a.tau));
    NG_CHECK(stage_in(ctx, 1, f_tadv_ext ? nullptr : D, n, mem, &a.D));
    NG_CHECK(stage_in(ctx, 2, bbar, n, mem, &a.bbar));
    NG_CHECK(stage_in(ctx, 3, Phi_im, n, mem, &a.Phi));
    NG_CHECK(stage_in(ctx, 4, f_tadv_ext, ext_stride ? (n - 1) * ext_stride + N : N, mem, &a.ext));
    FracFinish b{};
    NG_CHECK(stage_in(ctx, 5, t_half, n, mem, &b.t_half));
    NG_CHECK(stage_in(ctx, 6, J, n, mem, &b.J));
    // series by age + index (device copy per call, as ngrtd_conv_dot)
    HIP_TRY(ctx, ctx->stage[7].ensure((size_t)2 * N * sizeof(double)));
    double* cs = ctx->stage[7].d();
    HIP_TRY(ctx, hipMemcpyAsync(cs, s->c.data(), N * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    HIP_TRY(ctx, hipMemcpyAsync(cs + N, s->idx.data(), N * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    // f / g: the caller's device buffer or ctx scratch
    double* f = (mem == NGRTD_MEM_DEVICE && g_out) ? g_out : nullptr;
    if (!f) {
        HIP_TRY(ctx, ctx->stage[8].ensure((size_t)n * N * sizeof(double)));
        f = ctx->stage[8].d();
    }
    double *dconc = nullptr, *dfm = nullptr;
    if (mem == NGRTD_MEM_DEVICE) {
        dconc = conc;
        dfm = fm_mu;
    } else {
        HIP_TRY(ctx, ctx->stage[9].ensure((size_t)2 * n * sizeof(double)));
        dconc = conc ? ctx->stage[9].d() : nullptr;
        dfm = fm_mu ? ctx->stage[9].d() + n : nullptr;
    }
    a.f = f;
    // one wave per (set, age); chunks of sets keep a launch below 2^30 threads
    const int64_t chunk = std::max<int64_t>(1, ((int64_t)1 << 30) / (64 * N));
    for (int64_t p0 = 0; p0 < n; p0 += chunk) {
        a.p0 = p0;
        const int64_t waves = std::min(chunk, n - p0) * N;
        a.waves = waves;
        hipLaunchKernelGGL(frac_inner_kernel, dim3((unsigned)cdiv(waves, kFracWaves)), dim3(64 * kFracWaves), 0,
                           S(ctx), a);
        HIP_TRY(ctx, hipGetLastError());
    }
    b.c = cs;
    b.idx = cs + N;
    b.t_half_c = t_half_const;
    b.J_c = J_const;
    b.accum = accum;
    b.tp0 = a.tp0;
    b.dtp = a.dtp;
    b.N = a.N;
    b.n = n;
    b.f = f;
    b.conc = dconc;
    b.fm = dfm;
    hipLaunchKernelGGL(frac_finish_kernel, dim3((unsigned)n), dim3(256), 0, S(ctx), b);
    HIP_TRY(ctx, hipGetLastError());
    if (mem != NGRTD_MEM_DEVICE) {
        if (conc) HIP_TRY(ctx, hipMemcpyAsync(conc, dconc, n * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        if (fm_mu) HIP_TRY(ctx, hipMemcpyAsync(fm_mu, dfm, n * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        if (g_out) HIP_TRY(ctx, hipMemcpyAsync(g_out, f, (size_t)n * N * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
        HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    }
    return NGRTD_OK;
}

// ---------------------------------------------------------------------- plans
static int upload(ngrtd_ctx* ctx, DevBuf& b, const double* src, size_t n) {
    HIP_TRY(ctx, b.ensure(n * sizeof(double) + 16));
    if (n) HIP_TRY(ctx, hipMemcpy(b.p, src, n * sizeof(double), hipMemcpyHostToDevice));
    return NGRTD_OK;
}

// StudentT precision terms per observation: lam = sd^-2 and 0.5*log(lam), laid out as
// [lam(L*n) | hll(L*n)]; sd <= 0 (or NaN) stores lam = -1 so the bound gives -inf.
// ... followed by per-well sums of 0.5*log(lam) ([L]) for st_block.
static int upload_lam(ngrtd_ctx* ctx, DevBuf& b, const double* sd, size_t L, size_t n) {
    const size_t m = L * n;
    std::vector<double> h(2 * m + L, 0.0);
    for (size_t i = 0; i < m; ++i) {
        const double lam = std::pow(sd[i], -2.0);
        const bool ok = sd[i] > 0 && lam > 0;
        h[i] = ok ? lam : -1.0;
        h[m + i] = ok ? 0.5 * std::log(lam) : 0.0;
        h[2 * m + i / n] += h[m + i];
    }
    return upload(ctx, b, h.data(), h.size());
}

// a-1 / b-1 when both are small non-negative integers (beta_logp_fast), else -1
static void beta_int(double a, double b, int32_t* ia, int32_t* ib) {
    const double x = a - 1, y = b - 1;
    const bool ok = x >= 0 && y >= 0 && x <= 4 && y <= 4 && x == std::floor(x) && y == std::floor(y);
    *ia = ok ? (int32_t)x : -1;
    *ib = ok ? (int32_t)y : -1;
}

int ngrtd_plan_create(ngrtd_ctx* ctx, const ngrtd_model_desc* d, int64_t max_walkers, ngrtd_plan** out) {
    if (!ctx) return NGRTD_ESTATE;
    if (!d || !out || max_walkers <= 0) return set_err(ctx, NGRTD_EINVAL, "bad plan arguments");
    *out = nullptr;
    const int L = d->n_wells;
    if (L <= 0 || d->n_params <= 0) return set_err(ctx, NGRTD_EINVAL, "n_wells/n_params must be > 0");
    if (!d->ce_enabled && !d->rtd_enabled) return set_err(ctx, NGRTD_EINVAL, "plan needs a CE or an RTD block");
    const int* ri = d->role_index;
    for (int r = 0; r < NGRTD_ROLE_COUNT; ++r)
        if (ri[r] >= d->n_params) return set_err(ctx, NGRTD_EINVAL, "role %d row %d >= n_params", r, ri[r]);
    auto p = std::make_unique<ngrtd_plan>();
    p->ctx = ctx;
    p->desc = *d;
    p->max_w = max_walkers;
    const int64_t Umax = (int64_t)L * max_walkers;
    UnitArgs& u = p->unit;
    u.L = L;
    u.flags = d->flags;
    if (d->ce_enabled) {
        for (int r = NGRTD_ROLE_AE_BETA; r <= NGRTD_ROLE_NU_CE_BETA; ++r)
            if (ri[r] < 0) return set_err(ctx, NGRTD_EINVAL, "CE block needs role %d", r);
        if (d->ce_n_gases < 1 || d->ce_n_gases > kMaxGas) return set_err(ctx, NGRTD_EINVAL, "ce_n_gases must be 1..5");
        if (!d->ce_obs || !d->ce_sd || !d->ce_E_min) return set_err(ctx, NGRTD_EINVAL, "CE obs/sd/E_min required");
        const int G = d->ce_n_gases;
        NG_CHECK(upload(ctx, p->ce_obs, d->ce_obs, (size_t)L * G));
        NG_CHECK(upload(ctx, p->ce_sd, d->ce_sd, (size_t)L * G));
        NG_CHECK(upload(ctx, p->ce_emin, d->ce_E_min, (size_t)L));
        NG_CHECK(upload_lam(ctx, p->ce_lam, d->ce_sd, (size_t)L, (size_t)G));
        u.ce_lam = p->ce_lam.d(); u.ce_hll = p->ce_lam.d() + (size_t)L * G;
        u.ce_hll_sum = p->ce_lam.d() + (size_t)2 * L * G;
        u.ce_on = 1; u.G = G;
        for (int j = 0; j < G; ++j) {
            if (d->ce_gas_ids[j] < 0 || d->ce_gas_ids[j] > 4) return set_err(ctx, NGRTD_EINVAL, "bad gas id");
            u.gas[j] = d->ce_gas_ids[j];
        }
        for (int j = 0; j < kMaxGas; ++j) {
            const GasCoef gc = gas_coef(u.gas[j < G ? j : 0]);
            u.gz[j] = gc.z; u.gA0[j] = gc.A0; u.gA1[j] = gc.A1; u.gA2[j] = gc.A2; u.gA3[j] = gc.A3;
            u.g_he[j] = u.gas[j < G ? j : 0] == 0;
        }
        for (int i = 0; i < 6; ++i) u.row_ce[i] = ri[NGRTD_ROLE_AE_BETA + i];
        u.ce_obs = p->ce_obs.d(); u.ce_sd = p->ce_sd.d(); u.ce_Emin = p->ce_emin.d();
        u.E_max = d->ce_E_max; u.logA_min = d->ce_logA_min; u.logA_max = d->ce_logA_max;
        u.logF_min = d->ce_logF_min; u.logF_max = d->ce_logF_max; u.b_min = d->ce_b_min; u.b_max = d->ce_b_max;
        u.nu_min = d->ce_nu_min; u.nu_max = d->ce_nu_max;
        u.m_mu = d->ce_m_mu;
        u.m_tau = std::pow(d->ce_m_sd, -2.0);
        u.m_log_tau_2pi = std::log(u.m_tau / M_PI / 2.0);
        for (int i = 0; i < 5; ++i) {
            u.ce_ba[i] = d->ce_beta_a[i]; u.ce_bb[i] = d->ce_beta_b[i];
            u.ce_betaln[i] = host_betaln(d->ce_beta_a[i], d->ce_beta_b[i]);
            beta_int(d->ce_beta_a[i], d->ce_beta_b[i], &u.ce_bia[i], &u.ce_bib[i]);
        }
    }
    if (d->rtd_enabled) {
        const int K = d->n_tracers;
        if (K < 1 || K > kMaxTracer) return set_err(ctx, NGRTD_EINVAL, "n_tracers must be 1..8");
        if (ri[NGRTD_ROLE_TAU1] < 0 || ri[NGRTD_ROLE_NU_RTD_BETA] < 0)
            return set_err(ctx, NGRTD_EINVAL, "RTD block needs tau1 and nu roles");
        if (d->mod_type1 < 0 || d->mod_type1 > 3 || d->mod_type2 < -1 || d->mod_type2 > 3)
            return set_err(ctx, NGRTD_EINVAL, "bad RTD model types");
        if (d->mod_type2 >= 0 && ri[NGRTD_ROLE_TAU2] < 0) return set_err(ctx, NGRTD_EINVAL, "BMM needs tau2");
        if ((d->mod_type1 == NGRTD_MOD_EXP_PIST_FLOW && ri[NGRTD_ROLE_ETA1] < 0) ||
            (d->mod_type2 == NGRTD_MOD_EXP_PIST_FLOW && ri[NGRTD_ROLE_ETA2] < 0) ||
            (d->mod_type1 == NGRTD_MOD_DISPERSION && ri[NGRTD_ROLE_D1] < 0) ||
            (d->mod_type2 == NGRTD_MOD_DISPERSION && ri[NGRTD_ROLE_D2] < 0))
            return set_err(ctx, NGRTD_EINVAL, "model type needs its eta/D role");
        if (!d->rtd_obs || !d->rtd_sd) return set_err(ctx, NGRTD_EINVAL, "RTD obs/sd required");
        std::vector<TracerBuild> trs;
        const bool thalf_role = ri[NGRTD_ROLE_THALF_BETA] >= 0;
        bool any_lamw = false;
        for (int t = 0; t < K; ++t) {
            const ngrtd_tracer_desc& td = d->tracers[t];
            const SeriesHost* s = find_series(ctx, td.series_id);
            if (!s) return set_err(ctx, NGRTD_ESTATE, "unknown series %d", td.series_id);
            if (td.accum < 0 || td.accum > 3) return set_err(ctx, NGRTD_EINVAL, "bad accum");
            const bool lamw = thalf_role && td.is_cfc12;
            any_lamw |= lamw;
            trs.push_back(TracerBuild{s, td.accum, lamw ? 0.0 : lam_of(td.t_half), lamw});
        }
        NG_CHECK(build_table(ctx, trs, p->table));
        p->N = (int)trs[0].s->n;
        p->dtp = trs[0].s->dtp;
        for (auto& tb : trs)
            if (tb.s->dtp != p->dtp) return set_err(ctx, NGRTD_EINVAL, "tracers must share dtp");
        p->tp0 = (0.0 + 1e-5) + p->dtp;
        NG_CHECK(upload(ctx, p->rtd_obs, d->rtd_obs, (size_t)L * K));
        NG_CHECK(upload(ctx, p->rtd_sd, d->rtd_sd, (size_t)L * K));
        NG_CHECK(upload_lam(ctx, p->rtd_lam, d->rtd_sd, (size_t)L, (size_t)K));
        u.rtd_lam = p->rtd_lam.d(); u.rtd_hll = p->rtd_lam.d() + (size_t)L * K;
        u.rtd_hll_sum = p->rtd_lam.d() + (size_t)2 * L * K;
        HIP_TRY(ctx, p->conc.ensure((size_t)K * Umax * sizeof(double)));
        RtdArgs& a = p->rtd;
        a.row_tau[0] = ri[NGRTD_ROLE_TAU1]; a.row_tau[1] = ri[NGRTD_ROLE_TAU2];
        a.row_eta[0] = ri[NGRTD_ROLE_ETA1]; a.row_eta[1] = ri[NGRTD_ROLE_ETA2];
        a.row_D[0] = ri[NGRTD_ROLE_D1]; a.row_D[1] = ri[NGRTD_ROLE_D2];
        a.row_f1 = ri[NGRTD_ROLE_F1];
        a.row_J = ri[NGRTD_ROLE_J]; a.J_is_log10 = 1;
        a.row_thalf = any_lamw ? ri[NGRTD_ROLE_THALF_BETA] : -1;
        a.thalf_a = d->thalf_hi - d->thalf_lo; a.thalf_b = d->thalf_lo;
        a.row_lamsf6 = ri[NGRTD_ROLE_LAMSF6];
        a.tab = p->table.buf.d(); a.N = p->N; a.C = p->table.C; a.CP = p->table.CP;
        a.tp0 = p->tp0; a.dtp = p->dtp;
        a.mod[0] = d->mod_type1; a.mod[1] = d->mod_type2 >= 0 ? d->mod_type2 : MOD_NONE;
        a.K = K;
        for (int c = 0; c < p->table.C; ++c) {
            a.chan_tracer[c] = p->table.chan_tracer[c]; a.chan_isB[c] = p->table.chan_isB[c];
            a.chan_lamw[c] = p->table.chan_lamw[c];
        }
        for (int t = 0; t < K; ++t) { a.tr_sf6[t] = d->tracers[t].is_sf6; a.tr_J[t] = d->tracers[t].J; }
        a.conc_ident = p->table.C == K ? 1 : 0;
        for (int c = 0; c < p->table.C; ++c)
            if (a.chan_tracer[c] != c) a.conc_ident = 0;
        a.conc = p->conc.d();
        set_frag(a, p->table);
        a.cheb = nullptr;
        // (a per-unit CFC12 half-life leaves its channel undecayed: the same surrogate serves it
        // at tau_eff, lw_decay)
        // (generic instances: any exponential component, gen_path)
        if ((a.mod[0] == MOD_EXP || a.mod[1] == MOD_EXP) && p->table.C <= 5 && p->dtp >= 0.0 &&
            !(d->flags & NGRTD_EXACT_RTD)) {
            NG_CHECK(cheb_prepare(ctx, p->table, (1.0 + p->dtp) - p->tp0));
            if (p->table.cheb_ok) a.cheb = p->table.cheb.d();
        }
        a.epm = nullptr;
        a.epm_nb = a.epm_p0 = a.epm_np = 0;
        a.epm_nw = (int)cdiv(p->N, kEpmBlock) * kEpmBlock;   // the whole table (epm_window narrows it per launch)
        a.ew_on = 0;
        a.ew_tau_lo = a.ew_tau_hi = a.ew_eta_lo = a.ew_eta_hi = 0.0;
        {
            const char* e = std::getenv("NGRTD_EPM_DIAG");     // timing diagnostics only
            a.epm_diag = e ? std::atoi(e) : 0;
        }
        const bool epm1 = a.mod[0] == MOD_EPM && ri[NGRTD_ROLE_ETA1] >= 0;
        const bool epm2 = a.mod[1] == MOD_EPM && ri[NGRTD_ROLE_ETA2] >= 0;
        if ((epm1 || epm2) && p->table.C <= 5 && p->dtp >= 0.0 && !(d->flags & NGRTD_EXACT_RTD)) {
            // block-tail surrogates over every tau' = tau / eta >= the priors' lower end (the
            // table reaches 2^kEpmOct0); lanes below it or NaN sum their tails exactly.  A
            // per-unit CFC12 half-life reads its channel at tau'_w = 1 / (eta / tau + lam) as well.
            // (generic instances: either component exp_pist_flow, the window over both)
            static const bool disabled = std::getenv("NGRTD_NO_CHEB") != nullptr;
            double x;
            double plo = HUGE_VAL;
            const double tmin = std::min(a.thalf_b, a.thalf_a + a.thalf_b);
            auto low = [&](double tau_lo, double eta_hi) {
                double v = tau_lo / eta_hi;
                if (any_lamw) v = tmin > 0.0 ? std::min(v, 1.0 / (eta_hi / tau_lo + kLn2Ref / tmin)) : 0.0;
                plo = std::min(plo, v);
            };
            if (epm1) low(d->tau1_lo, d->eta1_hi);
            if (epm2) low(d->tau2_lo, d->eta2_hi);
            const double lo = std::max(1.0 / (1 << -kEpmOct0), plo);
            const int pa = epm_piece(lo, x), pb = kEpmPieces - 1;
            // a table too long for LDS serves windowed launches only (epm_window): the blocks the
            // window's units reach, or nothing when the priors bound no window
            int nb_cap = 0;
            if ((size_t)epm_lds_doubles(p->N, cheb_cp(p->table.C)) * sizeof(double) > kFusedMaxLds) {
                const int rows = (epm1 && !epm2 && (d->flags & NGRTD_WANT_PRIOR))
                                     ? epm_window_rows(d->tau1_hi, d->eta1_hi, p->dtp, p->N) : -1;
                nb_cap = rows > 0 ? rows / kEpmBlock : -1;
            }
            if (!disabled && pa >= 0 && pb >= pa && nb_cap >= 0) {
                // mixed-precision pieces for every plan (kEpmMixedAll; LW plans always)
                NG_CHECK(epm_prepare(ctx, p->table, p->N, pa, pb + 1, nb_cap, a.row_thalf >= 0 || kEpmMixedAll));
                if (p->table.epm_ok) {
                    a.epm = p->table.epm.d();
                    a.epm_nb = p->table.epm_nb; a.epm_p0 = p->table.epm_p0; a.epm_np = p->table.epm_np;
                }
            }
        }
        a.disp_aux = nullptr;
        a.disp_rows = nullptr;
        if (a.mod[0] == MOD_DISP || a.mod[1] == MOD_DISP) {   // gen_exact's per-age factors
            std::vector<double> aux(2 * (size_t)p->N + kDispExpTab);
            for (int k = 0; k < p->N; ++k) {
                const double tp = k == 0 ? p->tp0 : (double)k + p->dtp;
                aux[k] = 1.0 / tp;
                aux[p->N + k] = std::pow(tp, -1.5);
            }
            // the dispersion loop's exponential table (fexp_tab): 2^(j / T), long double rounded
            for (int j = 0; j < kDispExpTab; ++j) aux[2 * (size_t)p->N + j] = (double)exp2l((long double)j / kDispExpTab);
            NG_CHECK(upload(ctx, p->table.disp, aux.data(), aux.size()));
            a.disp_aux = p->table.disp.d();
            if (p->table.C <= kDispRow - 3) {   // the single-launch loop's interleaved rows
                std::vector<double> rows((size_t)p->N * kDispRow, 0.0);
                for (int k = 0; k < p->N; ++k) {
                    for (int c = 0; c < p->table.C; ++c) rows[(size_t)k * kDispRow + c] = p->table.cols_host[c][k];
                    rows[(size_t)k * kDispRow + kDispRow - 3] = k == 0 ? p->tp0 : (double)k + p->dtp;
                    rows[(size_t)k * kDispRow + kDispRow - 2] = aux[k];
                    rows[(size_t)k * kDispRow + kDispRow - 1] = aux[p->N + k];
                }
                NG_CHECK(upload(ctx, p->table.disp_rows, rows.data(), rows.size()));
                a.disp_rows = p->table.disp_rows.d();
            }
        }
        a.disp_pre = nullptr;
        a.disp_pre_g = 0;
        const int dg = disp_wide_plan(a, d->flags, Umax);
        if (dg > 0) {
            HIP_TRY(ctx, p->disp_pre.ensure((size_t)dg * (a.C + 1) * Umax * sizeof(double)));
            a.disp_pre = p->disp_pre.d();
            a.disp_pre_g = dg;
        }
        u.rtd_on = 1; u.K = K;
        u.rtd_obs = p->rtd_obs.d(); u.rtd_sd = p->rtd_sd.d(); u.conc = p->conc.d();
        u.row_tau1 = ri[NGRTD_ROLE_TAU1]; u.row_nu = ri[NGRTD_ROLE_NU_RTD_BETA]; u.row_tau2 = ri[NGRTD_ROLE_TAU2];
        u.row_f1 = ri[NGRTD_ROLE_F1]; u.row_eta1 = ri[NGRTD_ROLE_ETA1]; u.row_eta2 = ri[NGRTD_ROLE_ETA2];
        u.row_D1 = ri[NGRTD_ROLE_D1]; u.row_D2 = ri[NGRTD_ROLE_D2]; u.row_J = ri[NGRTD_ROLE_J];
        u.row_thalf = ri[NGRTD_ROLE_THALF_BETA]; u.row_lamsf6 = ri[NGRTD_ROLE_LAMSF6];
        auto nlw = [](double lo, double hi) { return -std::log(hi - lo); };
        u.tau1_lo = d->tau1_lo; u.tau1_hi = d->tau1_hi; u.tau1_nlw = nlw(d->tau1_lo, d->tau1_hi);
        u.tau2_lo = d->tau2_lo; u.tau2_hi = d->tau2_hi; u.tau2_nlw = nlw(d->tau2_lo, d->tau2_hi);
        u.f1_lo = d->f1_lo; u.f1_hi = d->f1_hi; u.f1_nlw = nlw(d->f1_lo, d->f1_hi);
        u.eta1_lo = d->eta1_lo; u.eta1_hi = d->eta1_hi; u.eta1_nlw = nlw(d->eta1_lo, d->eta1_hi);
        u.eta2_lo = d->eta2_lo; u.eta2_hi = d->eta2_hi; u.eta2_nlw = nlw(d->eta2_lo, d->eta2_hi);
        u.D1_lo = d->D1_lo; u.D1_hi = d->D1_hi; u.D1_nlw = nlw(d->D1_lo, d->D1_hi);
        u.D2_lo = d->D2_lo; u.D2_hi = d->D2_hi; u.D2_nlw = nlw(d->D2_lo, d->D2_hi);
        u.J_mu = d->J_mu; u.J_tau = std::pow(d->J_sd, -2.0); u.J_log_tau_2pi = std::log(u.J_tau / M_PI / 2.0);
        u.th_a = d->thalf_a; u.th_b = d->thalf_b; u.th_betaln = host_betaln(d->thalf_a, d->thalf_b);
        u.ls_tau = std::pow(d->lamsf6_sd, -2.0); u.ls_half_log = 0.5 * std::log(u.ls_tau * 2.0 / M_PI);
        u.rnu_min = d->rtd_nu_min; u.rnu_max = d->rtd_nu_max; u.rnu_a = d->rtd_nu_a; u.rnu_b = d->rtd_nu_b;
        u.rnu_betaln = host_betaln(d->rtd_nu_a, d->rtd_nu_b);
        beta_int(d->rtd_nu_a, d->rtd_nu_b, &u.rnu_ia, &u.rnu_ib);
        beta_int(d->thalf_a, d->thalf_b, &u.th_ia, &u.th_ib);
    }
    // Beta-prior slots (beta_block): exponents a-1, b-1 (+1 each with the logodds Jacobian)
    // split into integer parts (0..7, one shared product) and non-integer coefficients
    {
        const bool jac = d->flags & NGRTD_WANT_JACOBIAN;
        auto add_beta = [&](int row, double A, double B) {
            const int i = u.bt_n++;
            u.bt_row[i] = row;
            const double ca = (A - 1) + (jac ? 1.0 : 0.0), cb = (B - 1) + (jac ? 1.0 : 0.0);
            const bool ia_ok = ca >= 0 && ca <= 7 && ca == std::floor(ca);
            const bool ib_ok = cb >= 0 && cb <= 7 && cb == std::floor(cb);
            u.bt_ia[i] = ia_ok ? (int)ca : 0; u.bt_fa[i] = ia_ok ? 0.0 : ca;
            u.bt_ib[i] = ib_ok ? (int)cb : 0; u.bt_fb[i] = ib_ok ? 0.0 : cb;
            u.bt_betaln += host_betaln(A, B);
        };
        u.bt_n = 0; u.bt_betaln = 0.0;
        if (d->ce_enabled) {
            const int rows[5] = {ri[NGRTD_ROLE_AE_BETA], ri[NGRTD_ROLE_F_BETA], ri[NGRTD_ROLE_E_BETA],
                                 ri[NGRTD_ROLE_B_BETA], ri[NGRTD_ROLE_NU_CE_BETA]};
            for (int i = 0; i < 5; ++i) add_beta(rows[i], d->ce_beta_a[i], d->ce_beta_b[i]);
        }
        if (d->rtd_enabled) {
            add_beta(ri[NGRTD_ROLE_NU_RTD_BETA], d->rtd_nu_a, d->rtd_nu_b);
            if (ri[NGRTD_ROLE_THALF_BETA] >= 0) add_beta(ri[NGRTD_ROLE_THALF_BETA], d->thalf_a, d->thalf_b);
        }
    }
    // per-well data packed for the single-launch kernel's LDS copy (UnitArgs.wd_src)
    {
        std::vector<double> wd;
        auto add = [&](const DevBuf& b, size_t off, size_t n) {
            std::vector<double> h(n);
            if (n) (void)hipMemcpy(h.data(), b.d() + off, n * sizeof(double), hipMemcpyDeviceToHost);
            wd.insert(wd.end(), h.begin(), h.end());
        };
        if (d->ce_enabled) {
            const size_t LG = (size_t)L * d->ce_n_gases;
            wd.insert(wd.end(), d->ce_obs, d->ce_obs + LG);
            add(p->ce_lam, 0, LG);
            add(p->ce_lam, 2 * LG, (size_t)L);
            wd.insert(wd.end(), d->ce_E_min, d->ce_E_min + L);
        }
        if (d->rtd_enabled) {
            const size_t LK = (size_t)L * d->n_tracers;
            wd.insert(wd.end(), d->rtd_obs, d->rtd_obs + LK);
            add(p->rtd_lam, 0, LK);
            add(p->rtd_lam, 2 * LK, (size_t)L);
        }
        // Student-t normaliser table over every nu the priors' supports allow
        static const bool no_c0 = std::getenv("NGRTD_NO_C0TAB") != nullptr;
        double lo = HUGE_VAL, hi = -HUGE_VAL;
        if (d->ce_enabled) { lo = std::min(lo, u.nu_min); hi = std::max(hi, u.nu_max); }
        if (d->rtd_enabled) { lo = std::min(lo, u.rnu_min); hi = std::max(hi, u.rnu_max); }
        std::vector<double> c0t;
        int e0 = 0, np = 0;
        size_t c0_off = 0;
        if (!no_c0 && c0_build(lo, hi, c0t, e0, np) <= kC0Tol) {
            if (wd.size() & 1) wd.push_back(0.0);   // 16-B aligned table rows in LDS
            c0_off = wd.size();
            wd.insert(wd.end(), c0t.begin(), c0t.end());
        } else {
            np = 0;
        }
        NG_CHECK(upload(ctx, p->welldata, wd.data(), wd.size()));
        u.wd_src = p->welldata.d();
        u.wd_n = (int32_t)wd.size();
        u.c0_tab = np > 0 ? p->welldata.d() + c0_off : nullptr;
        u.c0_e0 = e0;
        u.c0_np = np;
    }
    HIP_TRY(ctx, p->ulogp.ensure((size_t)Umax * sizeof(double)));
    u.ulogp = p->ulogp.d();
    *out = p.release();
    return NGRTD_OK;
}

int ngrtd_plan_destroy(ngrtd_plan* p) {
    if (!p) return NGRTD_ESTATE;
    (void)hipStreamSynchronize(p->ctx->stream);
    (void)drain_timings(p);
    for (hipEvent_t e : p->region)
        if (e) p->ctx->event_pool.push_back(e);
    delete p;
    return NGRTD_OK;
}

// Enqueue the plan's kernels for theta (device) -> logp (device) / forward outputs.
// Timing without host synchronisation: each profiled launch is bracketed by two events
// recorded on the launch stream; ngrtd_plan_kernel_stats() reads them back later.
static int timed_begin(ngrtd_plan* p, bool prof, hipStream_t st, hipEvent_t* a) {
    if (!prof) return NGRTD_OK;
    *a = p->ctx->take_event();
    HIP_TRY(p->ctx, hipEventRecord(*a, st));
    return NGRTD_OK;
}
static int timed_end(ngrtd_plan* p, bool prof, hipStream_t st, int kind, hipEvent_t a) {
    if (!prof) return NGRTD_OK;
    hipEvent_t b = p->ctx->take_event();
    HIP_TRY(p->ctx, hipEventRecord(b, st));
    p->pending.push_back(PendingTiming{kind, a, b});
    return NGRTD_OK;
}

static int drain_timings(ngrtd_plan* p) {
    for (auto& t : p->pending) {
        HIP_TRY(p->ctx, hipEventSynchronize(t.b));
        float ms = 0.f;
        HIP_TRY(p->ctx, hipEventElapsedTime(&ms, t.a, t.b));
        p->stats.ms[t.kind] += ms;
        p->stats.n[t.kind] += 1;
        p->ctx->event_pool.push_back(t.a);
        p->ctx->event_pool.push_back(t.b);
    }
    p->pending.clear();
    return NGRTD_OK;
}

// Enqueue the plan's kernels for theta (device) -> logp (device) / forward outputs.
static int plan_run(ngrtd_plan* p, const double* theta, int64_t W, double* logp, double* ce_out, double* rtd_out,
                    const DemcAccept* dap = nullptr) {
    ngrtd_ctx* ctx = p->ctx;
    const int64_t U = (int64_t)p->desc.n_wells * W;
    const bool prof = ctx->profiling;
    hipStream_t st = S(ctx);
    hipEvent_t ev = nullptr;
    if (prof && p->pending.size() > 4096) NG_CHECK(drain_timings(p));
    UnitArgs u = p->unit;
    u.theta = theta; u.U = U; u.W = W;
    u.ce_out = ce_out;
    if (!logp) u.flags = 0;
    bool fused = false;
    // single launch: the log-prob, or the forward outputs (posterior predictive,
    // run_age_mcmc.py:251-319: concentrations from the same surrogate / exact paths)
    if (p->desc.rtd_enabled && ((logp && !ce_out && !rtd_out) || (!logp && (ce_out || rtd_out)))) {
        RtdArgs a = p->rtd;
        a.theta = theta; a.U = U; a.conc = logp ? nullptr : rtd_out;
        if (single_path(a, u)) {
            if (a.disp_pre) {   // a small-ensemble dispersion plan's sums (counted as an RTD launch)
                NG_CHECK(timed_begin(p, prof, st, &ev));
                NG_CHECK(launch_disp_wide(ctx, a, u, st));
                NG_CHECK(timed_end(p, prof, st, 0, ev));
            }
            NG_CHECK(timed_begin(p, prof, st, &ev));
            NG_CHECK(launch_fused(ctx, a, u, W, p->desc.n_wells, logp, st, dap));
            NG_CHECK(timed_end(p, prof, st, 3, ev));
            return NGRTD_OK;
        }
    }
    if (dap) {   // accept after the generic kernels: log-prob into logp, then one thread per walker
        NG_CHECK(plan_run(p, theta, W, logp, nullptr, nullptr));
        hipLaunchKernelGGL(demc_accept_kernel, dim3((unsigned)cdiv(W, 256)), dim3(256), 0, st, *dap,
                           (const double*)logp, W, (int64_t)p->desc.n_params * p->desc.n_wells);
        HIP_TRY(ctx, hipGetLastError());
        return NGRTD_OK;
    }
    if (p->desc.rtd_enabled) {
        RtdArgs a = p->rtd;
        a.theta = theta; a.U = U;
        if (rtd_out) a.conc = rtd_out;
        if (rtd_out) u.conc = rtd_out;
        // Fusing the per-unit CE / likelihood epilogue into the MFMA kernel saves the
        // concentration round trip but runs that VALU-bound epilogue at the MFMA kernel's
        // occupancy (2 waves/SIMD at c4); measured slower than two kernels, so
        // it is opt-in (NGRTD_FUSE=1).
        static const bool fuse_env = std::getenv("NGRTD_FUSE") != nullptr;
        const bool want_unit = fuse_env && (logp || ce_out);
        // the fused MFMA kernel keeps concentrations in registers: store them only on request
        if (want_unit && !rtd_out && mfma_path(a, a.row_thalf >= 0)) a.conc = nullptr;
        NG_CHECK(timed_begin(p, prof, st, &ev));
        NG_CHECK(launch_rtd(ctx, a, a.row_thalf >= 0, st, want_unit ? &u : nullptr, &fused));
        NG_CHECK(timed_end(p, prof, st, 0, ev));
    }
    if ((logp || ce_out) && fused) {
        if (logp) {
            NG_CHECK(timed_begin(p, prof, st, &ev));
            hipLaunchKernelGGL(walker_reduce_kernel, dim3((unsigned)cdiv(W, 64)), dim3(1024), 0, st,
                               (const double*)p->ulogp.d(), W, p->desc.n_wells, logp);
            HIP_TRY(ctx, hipGetLastError());
            NG_CHECK(timed_end(p, prof, st, 2, ev));
        }
    } else if (logp && p->desc.n_wells <= 512) {
        // per-unit log-prob + per-walker sum over wells, one launch.  Blocks of one wave
        // while the grid would not cover the CUs at 512 threads (the c2 CE plan: 2048
        // walkers x 3 wells are 16 blocks of 512 threads on 16 CUs, 128 one-wave blocks
        // on 128): each lane runs one unit's long dependent chain, so spreading the waves
        // over the CUs is what shortens the launch.
        int LS = 1;
        while (LS < p->desc.n_wells) LS *= 2;
        int TB = 512;
        while (TB > 64 && TB > LS && cdiv(W, (int64_t)(TB / LS)) < 256) TB /= 2;
        const int WB = TB / LS;
        NG_CHECK(timed_begin(p, prof, st, &ev));
        hipLaunchKernelGGL(unit_walker_kernel, dim3((unsigned)cdiv(W, WB)), dim3(TB), (size_t)TB * sizeof(double),
                           st, u, WB, LS, logp);
        HIP_TRY(ctx, hipGetLastError());
        NG_CHECK(timed_end(p, prof, st, 1, ev));
    } else if (logp || ce_out) {
        NG_CHECK(timed_begin(p, prof, st, &ev));
        hipLaunchKernelGGL(unit_logp_kernel, dim3((unsigned)cdiv(U, 256)), dim3(256), 0, st, u);
        HIP_TRY(ctx, hipGetLastError());
        NG_CHECK(timed_end(p, prof, st, 1, ev));
        if (logp) {
            NG_CHECK(timed_begin(p, prof, st, &ev));
            hipLaunchKernelGGL(walker_reduce_kernel, dim3((unsigned)cdiv(W, 64)), dim3(1024), 0, st,
                               (const double*)p->ulogp.d(), W, p->desc.n_wells, logp);
            HIP_TRY(ctx, hipGetLastError());
            NG_CHECK(timed_end(p, prof, st, 2, ev));
        }
    }
    return NGRTD_OK;
}

int ngrtd_logp(ngrtd_plan* p, const double* theta, int64_t W, double* logp, int32_t mem) {
    if (!p) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (!theta || !logp || W < 0 || W > p->max_w) return set_err(ctx, NGRTD_EINVAL, "bad theta/logp/W (max %lld)", (long long)p->max_w);
    if (W == 0) return NGRTD_OK;
    const int64_t nth = (int64_t)p->desc.n_params * p->desc.n_wells * W;
    if (mem == NGRTD_MEM_DEVICE) return plan_run(p, theta, W, logp, nullptr, nullptr);
    HIP_TRY(ctx, p->theta_stage.ensure((size_t)nth * sizeof(double)));
    HIP_TRY(ctx, p->out_stage.ensure((size_t)W * sizeof(double)));
    HIP_TRY(ctx, hipMemcpyAsync(p->theta_stage.p, theta, nth * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    NG_CHECK(plan_run(p, p->theta_stage.d(), W, p->out_stage.d(), nullptr, nullptr));
    HIP_TRY(ctx, hipMemcpyAsync(logp, p->out_stage.p, W * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
    HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    return NGRTD_OK;
}

int ngrtd_logp_n(ngrtd_plan* p, const double* theta, int64_t W, double* logp, int64_t n) {
    if (!p) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (!theta || !logp || W < 0 || W > p->max_w || n < 0)
        return set_err(ctx, NGRTD_EINVAL, "bad theta/logp/W (max %lld)/n", (long long)p->max_w);
    if (W == 0) return NGRTD_OK;
    // one event pair around the n launches (ngrtd_plan_region_ms): the launches' device
    // time back to back, recorded here so that the caller's timed region pays no
    // event-object round trips of its own
    for (hipEvent_t& e : p->region)
        if (!e) e = ctx->take_event();
    HIP_TRY(ctx, hipEventRecord(p->region[0], S(ctx)));
    for (int64_t i = 0; i < n; ++i) NG_CHECK(plan_run(p, theta, W, logp, nullptr, nullptr));
    HIP_TRY(ctx, hipEventRecord(p->region[1], S(ctx)));
    p->region_set = true;
    return NGRTD_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ RCCL (multi-GPU walker blocks)
// The RCCL entry points are resolved with dlsym from the library the caller names (the one torch
// already loaded, so one RCCL instance serves both) -- libngrtd has no link-time RCCL dependency.
struct RcclApi {
    void* lib = nullptr;
    RcclApi() = default;
    RcclApi(const RcclApi&) = delete;
    RcclApi& operator=(const RcclApi&) = delete;
    ~RcclApi() {
        if (lib) dlclose(lib);   // (a library torch loaded stays loaded: dlclose drops our reference)
    }
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    bool load(const char* path) {
        lib = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!lib) return false;
        get_id = reinterpret_cast<decltype(get_id)>(dlsym(lib, "ncclGetUniqueId"));
        init = reinterpret_cast<decltype(init)>(dlsym(lib, "ncclCommInitRank"));
        all_gather = reinterpret_cast<decltype(all_gather)>(dlsym(lib, "ncclAllGather"));
        destroy = reinterpret_cast<decltype(destroy)>(dlsym(lib, "ncclCommDestroy"));
        err = reinterpret_cast<decltype(err)>(dlsym(lib, "ncclGetErrorString"));
        return get_id && init && all_gather && destroy && err;
    }
};

struct ngrtd_comm {
    ngrtd_ctx* ctx = nullptr;
    RcclApi api;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    hipStream_t gs = nullptr;               // the gathers' stream
    hipEvent_t eval[2] = {nullptr, nullptr}, gath[2] = {nullptr, nullptr};
    bool pending[2] = {false, false};       // a gather of buffer s may still run
    ~ngrtd_comm() {                         // (also the cleanup of a half-built communicator)
        if (gs) (void)hipStreamSynchronize(gs);
        if (comm) (void)api.destroy(comm);
        for (int s = 0; s < 2; ++s) {
            if (eval[s]) (void)hipEventDestroy(eval[s]);
            if (gath[s]) (void)hipEventDestroy(gath[s]);
        }
        if (gs) (void)hipStreamDestroy(gs);
    }
};

extern "C" {

int ngrtd_comm_unique_id(const char* rccl_path, uint8_t* id128) {
    if (!id128) return NGRTD_EINVAL;
    RcclApi api;
    if (!api.load(rccl_path)) return NGRTD_EDEVICE;
    ncclUniqueId id;
    if (api.get_id(&id) != ncclSuccess) return NGRTD_EDEVICE;
    std::memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return NGRTD_OK;
}

int ngrtd_comm_create(ngrtd_ctx* ctx, const char* rccl_path, const uint8_t* id128, int32_t nranks, int32_t rank,
                      ngrtd_comm** out) {
    if (!ctx || !id128 || !out || nranks < 1 || rank < 0 || rank >= nranks) return NGRTD_EINVAL;
    *out = nullptr;
    std::unique_ptr<ngrtd_comm> c(new ngrtd_comm);
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    if (!c->api.load(rccl_path)) return set_err(ctx, NGRTD_EDEVICE, "cannot load RCCL (%s): %s", rccl_path ? rccl_path : "librccl.so.1", dlerror());
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ncclUniqueId id;
    std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = c->api.init(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) return set_err(ctx, NGRTD_EDEVICE, "ncclCommInitRank: %s", c->api.err(r));
    HIP_TRY(ctx, hipStreamCreateWithFlags(&c->gs, hipStreamNonBlocking));
    for (int s = 0; s < 2; ++s) {
        HIP_TRY(ctx, hipEventCreateWithFlags(&c->eval[s], hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&c->gath[s], hipEventDisableTiming));
    }
    *out = c.release();
    return NGRTD_OK;
}

int ngrtd_comm_destroy(ngrtd_comm* c) {
    if (!c) return NGRTD_ESTATE;
    delete c;
    return NGRTD_OK;
}

int ngrtd_logp_gather_n(ngrtd_plan* p, ngrtd_comm* c, const double* theta, int64_t W, int64_t per, double* bufs,
                        double* gathered, int64_t n) {
    if (!p || !c) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (c->ctx != ctx) return set_err(ctx, NGRTD_EINVAL, "communicator of another context");
    if (!theta || !bufs || !gathered || W < 1 || W > p->max_w || per < W || n < 0)
        return set_err(ctx, NGRTD_EINVAL, "bad theta/bufs/gathered/W (max %lld)/per/n", (long long)p->max_w);
    for (hipEvent_t& e : p->region)
        if (!e) e = ctx->take_event();
    hipStream_t st = S(ctx);
    HIP_TRY(ctx, hipEventRecord(p->region[0], st));
    for (int64_t i = 0; i < n; ++i) {
        const int s = (int)(i & 1);
        double* b = bufs + (int64_t)s * per;
        double* g = gathered + (int64_t)s * per * c->nranks;
        if (c->pending[s]) HIP_TRY(ctx, hipStreamWaitEvent(st, c->gath[s], 0));   // buffer s is free again
        NG_CHECK(plan_run(p, theta, W, b, nullptr, nullptr));
        HIP_TRY(ctx, hipEventRecord(c->eval[s], st));
        HIP_TRY(ctx, hipStreamWaitEvent(c->gs, c->eval[s], 0));
        const ncclResult_t r = c->api.all_gather(b, g, (size_t)per, ncclDouble, c->comm, c->gs);
        if (r != ncclSuccess) return set_err(ctx, NGRTD_EDEVICE, "ncclAllGather: %s", c->api.err(r));
        HIP_TRY(ctx, hipEventRecord(c->gath[s], c->gs));
        c->pending[s] = true;
    }
    for (int s = 0; s < 2; ++s)      // the plan's stream waits for the gathers in flight
        if (c->pending[s]) HIP_TRY(ctx, hipStreamWaitEvent(st, c->gath[s], 0));
    HIP_TRY(ctx, hipEventRecord(p->region[1], st));
    p->region_set = true;
    return NGRTD_OK;
}

int ngrtd_plan_region_ms(ngrtd_plan* p, float* ms) {
    if (!p || !ms) return NGRTD_EINVAL;
    if (!p->region_set) return set_err(p->ctx, NGRTD_ESTATE, "no ngrtd_logp_n call to time");
    HIP_TRY(p->ctx, hipEventSynchronize(p->region[1]));
    HIP_TRY(p->ctx, hipEventElapsedTime(ms, p->region[0], p->region[1]));
    return NGRTD_OK;
}

// Per-unit log-probs out[l][w] (device): the single-launch kernel writing each unit's
// value before the per-walker sum, else the RTD kernel + unit_logp_kernel.
static int plan_run_units(ngrtd_plan* p, const double* theta, int64_t W, double* out) {
    ngrtd_ctx* ctx = p->ctx;
    const int L = p->desc.n_wells;
    const int64_t U = (int64_t)L * W;
    hipStream_t st = S(ctx);
    UnitArgs u = p->unit;
    u.theta = theta; u.U = U; u.W = W; u.ce_out = nullptr;
    if (p->desc.rtd_enabled) {
        RtdArgs a = p->rtd;
        a.theta = theta; a.U = U; a.conc = nullptr;
        if (single_path(a, u)) {
            u.unit_out = out;
            NG_CHECK(launch_disp_wide(ctx, a, u, st));
            return launch_fused(ctx, a, u, W, L, out, st);
        }
        a.conc = p->conc.d();
        NG_CHECK(launch_rtd(ctx, a, a.row_thalf >= 0, st));
    }
    u.ulogp = out;
    hipLaunchKernelGGL(unit_logp_kernel, dim3((unsigned)cdiv(U, 256)), dim3(256), 0, st, u);
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}

int ngrtd_logp_units(ngrtd_plan* p, const double* theta, int64_t W, double* out, int32_t mem) {
    if (!p) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (!theta || !out || W < 0 || W > p->max_w) return set_err(ctx, NGRTD_EINVAL, "bad theta/out/W (max %lld)", (long long)p->max_w);
    if (W == 0) return NGRTD_OK;
    const int64_t U = (int64_t)p->desc.n_wells * W, nth = (int64_t)p->desc.n_params * U;
    if (mem == NGRTD_MEM_DEVICE) return plan_run_units(p, theta, W, out);
    HIP_TRY(ctx, p->theta_stage.ensure((size_t)nth * sizeof(double)));
    HIP_TRY(ctx, p->out_stage.ensure((size_t)U * sizeof(double)));
    HIP_TRY(ctx, hipMemcpyAsync(p->theta_stage.p, theta, nth * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    NG_CHECK(plan_run_units(p, p->theta_stage.d(), W, p->out_stage.d()));
    HIP_TRY(ctx, hipMemcpyAsync(out, p->out_stage.p, U * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
    HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    return NGRTD_OK;
}

int ngrtd_forward(ngrtd_plan* p, const double* theta, int64_t W, double* ce_out, double* rtd_out, int32_t mem) {
    if (!p) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (!theta || W < 0 || W > p->max_w) return set_err(ctx, NGRTD_EINVAL, "bad theta/W");
    if (ce_out && !p->desc.ce_enabled) return set_err(ctx, NGRTD_EINVAL, "plan has no CE block");
    if (rtd_out && !p->desc.rtd_enabled) return set_err(ctx, NGRTD_EINVAL, "plan has no RTD block");
    if (W == 0) return NGRTD_OK;
    const int64_t U = (int64_t)p->desc.n_wells * W;
    if (mem == NGRTD_MEM_DEVICE) return plan_run(p, theta, W, nullptr, ce_out, rtd_out);
    const int64_t nth = (int64_t)p->desc.n_params * U;
    const int G = p->desc.ce_n_gases, K = p->desc.n_tracers;
    HIP_TRY(ctx, p->theta_stage.ensure((size_t)nth * sizeof(double)));
    HIP_TRY(ctx, hipMemcpyAsync(p->theta_stage.p, theta, nth * sizeof(double), hipMemcpyHostToDevice, S(ctx)));
    double* dce = nullptr;
    if (ce_out) {
        HIP_TRY(ctx, p->ce_stage.ensure((size_t)G * U * sizeof(double)));
        dce = p->ce_stage.d();
    }
    double* drtd = (rtd_out && p->desc.rtd_enabled) ? p->conc.d() : nullptr;
    NG_CHECK(plan_run(p, p->theta_stage.d(), W, nullptr, dce, drtd));
    if (ce_out) HIP_TRY(ctx, hipMemcpyAsync(ce_out, dce, (size_t)G * U * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
    if (drtd) HIP_TRY(ctx, hipMemcpyAsync(rtd_out, drtd, (size_t)K * U * sizeof(double), hipMemcpyDeviceToHost, S(ctx)));
    HIP_TRY(ctx, hipStreamSynchronize(S(ctx)));
    return NGRTD_OK;
}

int ngrtd_plan_kernel_stats(ngrtd_plan* p, double* times_ms, int64_t* counts, int32_t n, int32_t reset) {
    if (!p) return NGRTD_ESTATE;
    NG_CHECK(drain_timings(p));
    for (int i = 0; i < n && i < 4; ++i) {
        if (times_ms) times_ms[i] = p->stats.ms[i];
        if (counts) counts[i] = p->stats.n[i];
    }
    if (reset) p->stats = LaunchStats{};
    return NGRTD_OK;
}

int ngrtd_demcz_run(ngrtd_plan* p, double* theta, double* logp, int64_t W, int64_t n_steps,
                    ngrtd_demcz_state* z, uint8_t* accepted_log, double* logp_log, uint64_t* n_accepted) {
    if (!p) return NGRTD_ESTATE;
    ngrtd_ctx* ctx = p->ctx;
    if (!theta || !logp || !z || W < 1 || W > p->max_w || n_steps < 0)
        return set_err(ctx, NGRTD_EINVAL, "bad theta/logp/state/W (1 <= W <= %lld)/n_steps", (long long)p->max_w);
    if (!z->lamb || !z->scaling || !z->n_acc_tune || !z->hist || z->hist_cap < 1 || z->hist_len < 0 ||
        z->hist_lo < 0 || z->hist_lo > z->hist_len || z->steps_done < 0 || z->tune_interval < 1 ||
        z->tune_target < 0 || z->tune_target > 2 || !(z->drop_fraction >= 0.0 && z->drop_fraction <= 1.0) ||
        z->chain0 < 0 || (z->n_chains_total != 0 && z->chain0 + W > z->n_chains_total) ||
        (z->per_well != 0 && z->per_well != 1) || z->well0 < 0 || z->n_wells_total < 0)
        return set_err(ctx, NGRTD_EINVAL, "bad DEMetropolisZ state");
    if (z->n_wells_total > 0 && z->well0 + p->desc.n_wells > z->n_wells_total)
        return set_err(ctx, NGRTD_EINVAL, "wells [%lld, %lld) outside the run's %d wells", (long long)z->well0,
                       (long long)(z->well0 + p->desc.n_wells), z->n_wells_total);
    const bool pw = z->per_well != 0;
    const int64_t Wg = z->n_chains_total ? z->n_chains_total : W;
    if (z->hist_len + n_steps > z->hist_cap)
        return set_err(ctx, NGRTD_EINVAL, "history full: %lld entries + %lld steps > capacity %lld",
                       (long long)z->hist_len, (long long)n_steps, (long long)z->hist_cap);
    if (n_steps == 0) return NGRTD_OK;
    hipStream_t st = S(ctx);
    const int64_t R = (int64_t)p->desc.n_params * p->desc.n_wells, E = R * W;
    const int64_t U = (int64_t)p->desc.n_wells * W, NC = pw ? U : W;   // chains
    HIP_TRY(ctx, p->demc_prop[0].ensure((size_t)E * sizeof(double)));
    HIP_TRY(ctx, p->demc_lp.ensure((size_t)NC * sizeof(double)));
    HIP_TRY(ctx, p->demc_acc.ensure((size_t)NC * sizeof(int32_t)));
    // acceptances are counted only on request (n_accepted NULL: no atomics at all)
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(n_accepted);
    int32_t* acc = static_cast<int32_t*>(p->demc_acc.p);
    const bool tr = z->theta_u != nullptr;
    if (tr && !(p->desc.flags & NGRTD_WANT_JACOBIAN))
        return set_err(ctx, NGRTD_EINVAL, "transformed-space chains need a plan with NGRTD_WANT_JACOBIAN");
    if (tr) HIP_TRY(ctx, p->demc_prop[1].ensure((size_t)E * sizeof(double)));
    double* prop = p->demc_prop[0].d();                   // proposal in the chains' space
    double* prop_x = tr ? p->demc_prop[1].d() : prop;     // ... and in theta's (natural) space
    double* state = tr ? z->theta_u : theta;              // what the history records
    DemczArgs base{};
    base.x = state; base.prop = prop; base.hist = z->hist; base.lamb = z->lamb; base.scaling = z->scaling;
    base.W = W; base.R = R; base.chain0 = z->chain0; base.Wg = Wg; base.S = z->S;
    base.prop_x = tr ? prop_x : nullptr; base.L = p->desc.n_wells;
    base.per_well = pw ? 1 : 0; base.well0 = z->well0; base.P = p->desc.n_params;
    for (int i = 0; i < kRoleCount; ++i) {
        base.tr_kind[i] = z->tr_kind[i]; base.tr_a[i] = z->tr_a[i]; base.tr_b[i] = z->tr_b[i];
    }
    const dim3 grid((unsigned)cdiv(W, kZTileW), (unsigned)cdiv(R, kZTileR));
    // one launch per step where the plan has a single-launch DEMetropolisZ instance
    int dzm = -1;
    const char* dz_env = std::getenv("NGRTD_DZ_DIAG");
    const int32_t dz_diag = dz_env ? std::atoi(dz_env) : 0;
    UnitArgs du = p->unit;
    RtdArgs dr = p->rtd;
    if (p->desc.rtd_enabled) {
        du.theta = prop_x; du.U = (int64_t)p->desc.n_wells * W; du.W = W;   // the launch's theta: the
        dr.theta = prop_x; dr.U = du.U; dr.conc = nullptr;                   // proposals it forms
        // NGRTD_DZ_MODE=pair: the proposal kernel + log-prob kernel pair even where a
        // single-launch instance exists (A/B runs, tests/test_gpu_demc.py)
        const char* m_env = std::getenv("NGRTD_DZ_MODE");
        if (!(m_env && std::strcmp(m_env, "pair") == 0)) dzm = dz_mix(dr, du, p->desc.n_params, tr);
        if (dzm >= 0 && pw) dzm |= 16;   // per-well chains: one decision per unit
    }
    // the lane-chain step (RTD-only / CE-only models, per-well chains), where no logp_fused_kernel
    // instance steps the plan
    int dzc = -1;
    size_t dzc_lds = 0;
    {
        const char* m_env = std::getenv("NGRTD_DZ_MODE");
        if (dzm < 0 && pw && !(m_env && std::strcmp(m_env, "pair") == 0)) {
            du.theta = prop_x; du.U = (int64_t)p->desc.n_wells * W; du.W = W;
            dr.theta = prop_x; dr.U = du.U; dr.conc = nullptr;
            dzc = dzc_mix(dr, du, p->desc.n_params, tr, &dzc_lds);
        }
    }
    const bool multi = dzm >= 0 || dzc >= 0;   // one launch per chunk of steps
    const dim3 gpw((unsigned)cdiv(U, 256));   // per-well proposal / accept kernels
    // single-launch instance: chunks of up to NGRTD_DZ_CHUNK (default 256) steps per launch,
    // each block running its own chains through the chunk (DemcAccept::Sched / dz_step)
    const char* chunk_env = std::getenv("NGRTD_DZ_CHUNK");
    const int64_t chunk = std::max<int64_t>(1, chunk_env ? std::atoll(chunk_env) : 256);
    // the multi-step launch keeps the state walker-major ([P][W][L], a chain's rows contiguous
    // like its history entries) for the whole call: transposed in here, back after the loop
    const int Lw = p->desc.n_wells;
    double* xw[2] = {nullptr, nullptr};
    if (multi) {
        for (int i = 0; i < (tr ? 2 : 1); ++i) {
            HIP_TRY(ctx, p->demc_xw[i].ensure((size_t)E * sizeof(double)));
            xw[i] = p->demc_xw[i].d();
        }
        const dim3 g((unsigned)cdiv(W, 32), (unsigned)cdiv(Lw, 32), (unsigned)p->desc.n_params);
        hipLaunchKernelGGL(dz_layout_kernel, g, dim3(256), 0, st, theta, xw[0], (int64_t)Lw, W);
        if (tr) hipLaunchKernelGGL(dz_layout_kernel, g, dim3(256), 0, st, z->theta_u, xw[1], (int64_t)Lw, W);
        HIP_TRY(ctx, hipGetLastError());
    }
    // per-well chains: their lp / lamb / scaling / tuning counters walker-major too ([W][L],
    // the launch's unit order) for the whole call, so a wave's per-chain loads and stores are
    // contiguous runs; the logs stay [n][L][W]
    double* cl = logp;
    double* clamb = z->lamb;
    double* cscal = z->scaling;
    int32_t* cnat = z->n_acc_tune;
    const dim3 g1((unsigned)cdiv(W, 32), (unsigned)cdiv(Lw, 32), 1u), g1b((unsigned)cdiv(Lw, 32), (unsigned)cdiv(W, 32), 1u);
    if (multi && pw) {
        HIP_TRY(ctx, p->demc_pw.ensure((size_t)U * (3 * sizeof(double) + sizeof(int32_t))));
        cl = p->demc_pw.d(); clamb = cl + U; cscal = clamb + U;
        cnat = reinterpret_cast<int32_t*>(cscal + U);
        hipLaunchKernelGGL(dz_layout_kernel, g1, dim3(256), 0, st, logp, cl, (int64_t)Lw, W);
        hipLaunchKernelGGL(dz_layout_kernel, g1, dim3(256), 0, st, z->lamb, clamb, (int64_t)Lw, W);
        hipLaunchKernelGGL(dz_layout_kernel, g1, dim3(256), 0, st, z->scaling, cscal, (int64_t)Lw, W);
        hipLaunchKernelGGL(dz_layout_i32_kernel, g1, dim3(256), 0, st, z->n_acc_tune, cnat, (int64_t)Lw, W);
        HIP_TRY(ctx, hipGetLastError());
    }
    for (int64_t j = 0; multi && j < n_steps;) {
        const int64_t k = std::min(chunk, n_steps - j);
        DemcAccept da{cl, acc, cnt, xw[0], nullptr, p->desc.n_params, 0, cnat, clamb, cscal,
                      0, z->tune_target, z->tune_interval, accepted_log ? accepted_log + j * NC : nullptr,
                      logp_log ? logp_log + j * NC : nullptr, z->chain0, tr ? xw[1] : nullptr, nullptr};
        da.per_well = pw ? 1 : 0; da.well0 = z->well0;
        da.ar_log = z->accept_log ? z->accept_log + j * NC : nullptr;
        da.zx = tr ? xw[1] : xw[0]; da.dz_prop = prop_x; da.hist = z->hist;
        da.Wg = Wg; da.S = z->S; da.L = p->desc.n_wells;
        da.dz_diag = dz_diag;
        for (int i = 0; i < kRoleCount; ++i) {
            da.tr_kind[i] = z->tr_kind[i]; da.tr_a[i] = z->tr_a[i]; da.tr_b[i] = z->tr_b[i];
        }
        da.n_steps = (int32_t)k;
        da.sch.seed = z->seed; da.sch.s0 = z->steps_done;
        da.sch.h_len0 = z->hist_len; da.sch.h_lo0 = z->hist_lo; da.sch.append0 = j > 0 ? 1 : 0;
        da.sch.n_tune = z->n_tune; da.sch.drop = z->drop_fraction;
        da.sch.tune_target = z->tune_target; da.sch.tune_interval = z->tune_interval;
        hipEvent_t ev = nullptr;
        NG_CHECK(timed_begin(p, ctx->profiling, st, &ev));
        if (dzc >= 0) {
            RtdArgs dwin = dr;
            if (!(dzc & 64)) cheb_window(dwin, du);
            da.state_lds = 0; da.prop_lds = 0; da.prop_skip = 0;
            // up to 64 chains (the reference's own runs: 3 or 4): a theta wave beside the chain
            // wave (NGRTD_DZC_THETA_WAVE=0: off, A/B runs)
            static const bool tw_off = [] {
                const char* e = std::getenv("NGRTD_DZC_THETA_WAVE");
                return e && std::atoi(e) == 0;
            }();
            da.theta_wave = (!tw_off && du.U <= 64 && !(dzc & 64)) ? 1 : 0;   // (the CE-only model: no RTD half)
            HIP_TRY(ctx, launch_dz_chain(dwin.C, dzc, dwin, du, da, du.U, dzc_lds, kFusedMaxLds, st));
        } else {
            NG_CHECK(launch_fused_dz(ctx, dr, du, W, p->desc.n_wells, p->demc_lp.d(), st, da, dzm));
        }
        NG_CHECK(timed_end(p, ctx->profiling, st, 3, ev));
        // the host state after the chunk's last step (the kernel's own schedule)
        const DzStep last = dz_step(da.sch, k - 1);
        z->hist_len = last.len;
        z->hist_lo = last.lo;
        z->steps_done += k;
        j += k;
    }
    if (multi) {
        const dim3 g((unsigned)cdiv(Lw, 32), (unsigned)cdiv(W, 32), (unsigned)p->desc.n_params);
        hipLaunchKernelGGL(dz_layout_kernel, g, dim3(256), 0, st, xw[0], theta, W, (int64_t)Lw);
        if (tr) hipLaunchKernelGGL(dz_layout_kernel, g, dim3(256), 0, st, xw[1], z->theta_u, W, (int64_t)Lw);
        if (pw) {
            hipLaunchKernelGGL(dz_layout_kernel, g1b, dim3(256), 0, st, cl, logp, W, (int64_t)Lw);
            hipLaunchKernelGGL(dz_layout_kernel, g1b, dim3(256), 0, st, clamb, z->lamb, W, (int64_t)Lw);
            hipLaunchKernelGGL(dz_layout_kernel, g1b, dim3(256), 0, st, cscal, z->scaling, W, (int64_t)Lw);
            hipLaunchKernelGGL(dz_layout_i32_kernel, g1b, dim3(256), 0, st, cnat, z->n_acc_tune, W, (int64_t)Lw);
        }
        HIP_TRY(ctx, hipGetLastError());
    }
    // step j's bookkeeping (the host restatement dz_step mirrors): the previous step's state
    // becomes history entry s - 1 (the previous call appended its own last state), then
    // proposals draw from [hist_lo, hist_len)
    auto step_args = [&](int64_t j) {
        const int64_t s = z->steps_done;
        const int64_t append_at = j > 0 ? z->hist_len : -1;
        if (j > 0) z->hist_len += 1;
        if (s == z->n_tune && z->n_tune > 0)   // stop_tuning before the first draw: drop the
            z->hist_lo += (int64_t)(z->drop_fraction * (double)(z->hist_len - z->hist_lo));   // oldest
        DemczArgs d = base;
        d.propose = 1; d.append_at = append_at; d.lo = z->hist_lo; d.it = z->hist_len - z->hist_lo;
        d.key = demc_key(z->seed, (uint64_t)s);
        return d;
    };
    // per-well chains: step j's accept and step j + 1's append + proposal (after the last step:
    // the final append) in one launch (demc_accept_propose_pw_kernel; NGRTD_DZ_NO_FUSE=1: the
    // separate kernels, A/B runs)
    static const bool no_fuse = [] {
        const char* e = std::getenv("NGRTD_DZ_NO_FUSE");
        return e && std::atoi(e) != 0;
    }();
    const bool fuse = pw && !no_fuse;
    bool staged = false;                   // this step's proposal ran in the previous launch
    DemczArgs d = base;
    for (int64_t j = 0; !multi && j < n_steps; ++j) {
        if (!staged) {
            d = step_args(j);
            if (pw) hipLaunchKernelGGL(demcz_propose_pw_kernel, gpw, dim3(256), 0, st, d);
            else hipLaunchKernelGGL(demcz_propose_kernel, grid, dim3(kZThreads), 0, st, d);
            HIP_TRY(ctx, hipGetLastError());
        }
        staged = false;
        const int64_t s = z->steps_done;
        const uint64_t key = d.key;
        const int64_t next = s + 1;
        const int32_t tune_now = (z->tune_target != NGRTD_TUNE_NONE && next < z->n_tune &&
                                  next % z->tune_interval == 0) ? 1 : 0;
        DemcAccept da{logp, acc, cnt, theta, prop_x, p->desc.n_params, key, z->n_acc_tune, z->lamb, z->scaling,
                      tune_now, z->tune_target, z->tune_interval,
                      accepted_log ? accepted_log + j * NC : nullptr, logp_log ? logp_log + j * NC : nullptr,
                      z->chain0, tr ? z->theta_u : nullptr, tr ? prop : nullptr};
        da.ar_log = z->accept_log ? z->accept_log + j * NC : nullptr;
        if (pw) {   // per-unit log-probs of the proposal, then one decision per unit
            da.L = p->desc.n_wells; da.Wg = Wg; da.per_well = 1; da.well0 = z->well0;
            NG_CHECK(plan_run_units(p, prop_x, W, p->demc_lp.d()));
            z->steps_done = next;
            if (fuse) {
                if (j + 1 < n_steps) {
                    d = step_args(j + 1);
                } else {                       // the last step's state: history entry steps_done - 1
                    d = base;
                    d.propose = 0; d.append_at = z->hist_len;
                }
                hipLaunchKernelGGL(demc_accept_propose_pw_kernel, gpw, dim3(256), 0, st, da,
                                   (const double*)p->demc_lp.d(), W, d);
                staged = true;
            } else {
                hipLaunchKernelGGL(demc_accept_pw_kernel, gpw, dim3(256), 0, st, da, (const double*)p->demc_lp.d(), W);
            }
            HIP_TRY(ctx, hipGetLastError());
        } else {
            NG_CHECK(plan_run(p, prop_x, W, p->demc_lp.d(), nullptr, nullptr, &da));
            z->steps_done = next;
        }
    }
    if (!staged) {   // the last step's state: history entry steps_done - 1
        d = base;
        d.propose = 0; d.append_at = z->hist_len;
        if (pw) hipLaunchKernelGGL(demcz_propose_pw_kernel, gpw, dim3(256), 0, st, d);
        else hipLaunchKernelGGL(demcz_propose_kernel, grid, dim3(kZThreads), 0, st, d);
        HIP_TRY(ctx, hipGetLastError());
    }
    z->hist_len += 1;
    return NGRTD_OK;
}

int ngrtd_pymc3_backward(ngrtd_ctx* ctx, const double* u, double* x, int64_t lead, int32_t P, int64_t inner,
                         const int32_t* kind, const double* a, const double* b) {
    if (!ctx) return NGRTD_ESTATE;
    if (!u || !x || !kind || lead < 0 || inner < 0 || P < 1 || P > kRoleCount)
        return set_err(ctx, NGRTD_EINVAL, "bad pymc3_backward arguments");
    TrRows t{};
    for (int p = 0; p < P; ++p) {
        if (kind[p] < NGRTD_TR_NONE || kind[p] > NGRTD_TR_LOG) return set_err(ctx, NGRTD_EINVAL, "bad transform kind");
        t.kind[p] = kind[p];
        t.a[p] = a ? a[p] : 0.0;
        t.b[p] = b ? b[p] : 0.0;
    }
    const int64_t n = lead * P * inner;
    if (n == 0) return NGRTD_OK;
    hipLaunchKernelGGL(pymc3_backward_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(ctx), u, x, n, P,
                       inner, t);
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}

int ngrtd_fm_log(ngrtd_ctx* ctx, const double* in, double* out, int64_t n) {
    if (!ctx) return NGRTD_ESTATE;
    if (!in || !out || n < 0) return set_err(ctx, NGRTD_EINVAL, "bad fm_log arguments");
    if (n == 0) return NGRTD_OK;
    hipLaunchKernelGGL(fm_log_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, S(ctx), in, out, n);
    HIP_TRY(ctx, hipGetLastError());
    return NGRTD_OK;
}

int ngrtd_surrogate_check(const double* cols, int32_t C, int64_t N, double dtp, double* coef, double* max_rel_err) {
    if (!cols || C < 1 || C > kMaxChan || N < 2 || !max_rel_err) return NGRTD_EINVAL;
    std::vector<std::vector<double>> cv((size_t)C);
    for (int c = 0; c < C; ++c) cv[c].assign(cols + (size_t)c * N, cols + (size_t)(c + 1) * N);
    std::vector<double> co;
    *max_rel_err = cheb_build(cv, C, (1.0 + dtp) - ((0.0 + 1e-5) + dtp), co);
    if (coef) std::copy(co.begin(), co.end(), coef);
    return NGRTD_OK;
}

int ngrtd_epm_window_check(double tau_hi, double eta_hi, double dtp, int32_t N, int32_t* rows) {
    if (!rows || N < 1) return NGRTD_EINVAL;
    *rows = epm_window_rows(tau_hi, eta_hi, dtp, N);
    return NGRTD_OK;
}

int ngrtd_c0_check(double nu_lo, double nu_hi, double* coef, int32_t* e0, int32_t* n_pieces, double* max_abs_err) {
    if (!e0 || !n_pieces || !max_abs_err) return NGRTD_EINVAL;
    std::vector<double> t;
    int e = 0, np = 0;
    *max_abs_err = c0_build(nu_lo, nu_hi, t, e, np);
    *e0 = e;
    *n_pieces = np;
    if (coef) std::copy(t.begin(), t.end(), coef);
    return NGRTD_OK;
}

int ngrtd_plan_info(ngrtd_plan* p, int64_t W, int64_t* info, int32_t n) {
    if (!p) return NGRTD_ESTATE;
    const int64_t U = (int64_t)p->desc.n_wells * W;
    int64_t v[16] = {0};
    v[13] = p->unit.c0_np;
    v[14] = p->rtd.disp_pre_g;   // disp_wide_kernel partials per unit (0: the lane loop)
    if (p->desc.rtd_enabled) {
        RtdArgs a = p->rtd;
        v[11] = a.cheb != nullptr ? 1 : (a.epm != nullptr ? 2 : 0);
        const double err = a.epm != nullptr ? p->table.epm_err : p->table.cheb_err;
        v[12] = (err >= 0 && err < 1.0) ? (int64_t)llround(err * 1e18) : -1;
        a.U = U;
        const bool lamw = a.row_thalf >= 0;
        if (mfma_path(a, lamw)) {
            v[0] = mfma_tiles(a.C); v[1] = mfma_waves(a.C); v[2] = cdiv(U, kMfmaUnitsPerBlock); v[3] = a.Lseg;
            v[6] = (int64_t)mfma_lds(a);
            v[8] = mfma_rows(a.C); v[9] = a.S_seg; v[10] = a.nsteps;
        } else {
            const RtdGeom g = rtd_geometry(U, p->N, p->table.C, lamw);
            v[0] = g.R; v[1] = g.NW; v[2] = g.blocks; v[3] = (int64_t)g.LW * g.NW; v[6] = (int64_t)g.lds;
        }
        v[4] = p->table.C; v[5] = p->N;
    }
    v[7] = U;
    for (int i = 0; i < n && i < 16; ++i) info[i] = v[i];
    return NGRTD_OK;
}

}  // extern "C"

#ifdef NGRTD_SECTION_PROBE
// probe build only (tools/section_probe.py): copy the s_memtime stamps of the last launch
extern "C" int ngrtd_probe_read(unsigned long long* dst, int64_t n) {
    if (n > (int64_t)(sizeof(g_probe) / sizeof(g_probe[0]))) n = sizeof(g_probe) / sizeof(g_probe[0]);
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_probe), (size_t)n * sizeof(unsigned long long)) == hipSuccess ? 0 : -2;
}
#endif
