// Probe for the exponential-RTD MFMA kernel (rtd_exp_mfma_kernel): variants of the block
// shape (NT tiles per wave, waves per block) and of the LDS staging of the fragment
// table, on the c4 geometry (U = 131072 units, C = 5 channels, 3 age segments, 25 steps).
// Each block's wave 0 records wall-clock stamps (100 MHz) at start / after staging / after
// the MFMA loop / end, and the shader clock at start/end, so the kernel time splits into
// prologue, matrix loop and epilogue, and the effective core clock is visible.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 \
//         -o /tmp/mfma_probe tools/mfma_probe.hip && /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef double v4d __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int C = 5, S = 3, NSTEPS = 25, LSEG = 400;

struct Stamp { unsigned long long w0, w1, w2, w3, c0, c3; };
struct WaveRec { unsigned long long t0, t1; unsigned hw, xcc; };
__device__ WaveRec g_waves[1 << 14];

// STAGE 0: one double2 per thread per iteration (production); 1: all loads issued first;
// 2: no LDS staging, A operands read from global (L2/L1 hits) each step
template <int NT, int NWAVE, int STAGE>
__global__ void __launch_bounds__(64 * NWAVE) probe(const double* __restrict__ theta, const double* __restrict__ frag,
                                                    int64_t U, double* __restrict__ conc, Stamp* st) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 15, tq = lane >> 4;
    Stamp s{};
    if (lane == 0) { s.w0 = wall_clock64(); s.c0 = clock64(); }
    const int64_t u0 = ((int64_t)blockIdx.x * NWAVE + wave) * (16 * NT);
    const int64_t Umax = U - 1;
    constexpr int NTH = 64 * NWAVE;
    constexpr int NV2 = NSTEPS * 128;                 // double2 in the table
    constexpr int PER = (NV2 + NTH - 1) / NTH;
    double2 stash[STAGE == 1 ? PER : 1];
    if (STAGE == 1) {
        const double2* src = reinterpret_cast<const double2*>(frag);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * NTH;
            if (i < NV2) stash[j] = src[i];
        }
    }
    double q16[NT], pw[NT][4];
    v4d acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        int64_t u = u0 + 16 * t + col;
        u = u < Umax ? u : Umax;
        const double beta = 1. / theta[u];
        const double q = exp(-beta);
        const double q2 = q * q, q4 = q2 * q2;
        const double qt = (tq == 0) ? 1.0 : (tq == 1) ? q : (tq == 2) ? q2 : q2 * q;
        pw[t][0] = qt;
        pw[t][1] = qt * q4;
        pw[t][2] = pw[t][1] * q4;
        pw[t][3] = pw[t][2] * q4;
        const double q8 = q4 * q4;
        q16[t] = q8 * q8;
        acc[t] = v4d{0.0, 0.0, 0.0, 0.0};
    }
    if (STAGE == 0) {
        const double2* src = reinterpret_cast<const double2*>(frag);
        double2* dst = reinterpret_cast<double2*>(lds);
        for (int i = threadIdx.x; i < NV2; i += NTH) dst[i] = src[i];
    } else if (STAGE == 1) {
        double2* dst = reinterpret_cast<double2*>(lds);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * NTH;
            if (i < NV2) dst[i] = stash[j];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) s.w1 = wall_clock64();
    const double* f = (STAGE == 2 ? frag : lds) + lane;
    for (int step = 0; step < NSTEPS; ++step, f += 256) {
        const double A0 = f[0], A1 = f[64], A2 = f[128], A3 = f[192];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(A0, pw[t][0], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(A1, pw[t][1], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(A2, pw[t][2], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(A3, pw[t][3], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int mm = 0; mm < 4; ++mm) pw[t][mm] *= q16[t];
    }
    if (threadIdx.x == 0) s.w2 = wall_clock64();
    if (lane == 0) {
        WaveRec r;
        r.t0 = s.w0; r.t1 = wall_clock64();
        r.hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        r.xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        g_waves[blockIdx.x * NWAVE + wave] = r;
    }
    __syncthreads();
    double (*sh)[NT * 16][17] = reinterpret_cast<double (*)[NT * 16][17]>(lds);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sh[wave][16 * t + col][tq + 4 * r] = acc[t][r];
    __syncthreads();
    if (lane < 16 * NT) {
        const int64_t u = u0 + lane;
        if (u <= Umax) {
            const double beta = 1. / theta[u];
            const double Qs = exp(-beta * (double)LSEG);
            const double* P = sh[wave][lane];
            const double s01 = exp(-beta * 0.5);
            const double G = expm1(-beta * 1199.0) / expm1(-beta);
            const double den = 1.0 + s01 * G;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                double y = P[c * S + S - 1];
#pragma unroll
                for (int sg = S - 2; sg >= 0; --sg) y = fma(y, Qs, P[c * S + sg]);
                conc[(int64_t)c * U + u] = (1.0 + s01 * y) / den;
            }
        }
    }
    if (threadIdx.x == 0) { s.w3 = wall_clock64(); s.c3 = clock64(); st[blockIdx.x] = s; }
}

// Row-tiled layout (production rtd_exp_mfma_kernel since r1b): each B register (q^(4 step
// + kq) of 16 units) feeds R row tiles; 4-age steps.  MODE 0: A from LDS; 1: A from LDS
// with the next step's A loaded before this step's MFMAs; 2: A straight from global.
template <int R, int NT, int NWAVE, int MODE>
__global__ void __launch_bounds__(64 * NWAVE) probe_rt(const double* __restrict__ theta, const double* __restrict__ frag,
                                                       int64_t U, double* __restrict__ conc, Stamp* st, int nsteps) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 15, tq = lane >> 4;
    Stamp s{};
    if (lane == 0) { s.w0 = wall_clock64(); s.c0 = clock64(); }
    const int64_t u0 = ((int64_t)blockIdx.x * NWAVE + wave) * (16 * NT);
    const int64_t Umax = U - 1;
    double beta[NT], q4[NT], pw[NT];
    v4d acc[NT][R];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        int64_t u = u0 + 16 * t + col;
        u = u < Umax ? u : Umax;
        beta[t] = 1. / theta[u];
        const double q = exp(-beta[t]);
        const double q2 = q * q;
        q4[t] = q2 * q2;
        pw[t] = (tq == 0) ? 1.0 : (tq == 1) ? q : (tq == 2) ? q2 : q2 * q;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[t][r] = v4d{0.0, 0.0, 0.0, 0.0};
    }
    if (MODE != 2) {
        const double2* src = reinterpret_cast<const double2*>(frag);
        double2* dst = reinterpret_cast<double2*>(lds);
        for (int i = threadIdx.x; i < nsteps * R * 32; i += 64 * NWAVE) dst[i] = src[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) s.w1 = wall_clock64();
    const double* f = (MODE == 2 ? frag : lds) + lane;
    if (MODE == 3 || MODE == 4) {
        double A[R];
#pragma unroll
        for (int r = 0; r < R; ++r) A[r] = f[r * 64];
        for (int step = 0; step < nsteps; ++step) {
            if (MODE == 4) {
#pragma unroll
                for (int r = 0; r < R; ++r) A[r] = f[r * 64 + step * R * 64];
            }
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r) acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[r], pw[t], acc[t][r], 0, 0, 0);
            if (MODE == 3) {
#pragma unroll
                for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
            }
        }
    } else if (MODE == 5) {
        // two steps per iteration, A of the next pair loaded while this pair runs
        double A0[R], A1[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { A0[r] = f[r * 64]; A1[r] = f[R * 64 + r * 64]; }
        for (int step = 0; step < nsteps; step += 2) {
            f += 2 * R * 64;
            double B0[R], B1[R];
#pragma unroll
            for (int r = 0; r < R; ++r) { B0[r] = f[r * 64]; B1[r] = f[R * 64 + r * 64]; }
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r) acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A0[r], pw[t], acc[t][r], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r) acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A1[r], pw[t], acc[t][r], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
#pragma unroll
            for (int r = 0; r < R; ++r) { A0[r] = B0[r]; A1[r] = B1[r]; }
        }
    } else if (MODE == 1) {
        double A[R];
#pragma unroll
        for (int r = 0; r < R; ++r) A[r] = f[r * 64];
        for (int step = 0; step < nsteps; ++step) {
            f += R * 64;
            double An[R];
#pragma unroll
            for (int r = 0; r < R; ++r) An[r] = (step + 1 < nsteps) ? f[r * 64] : 0.0;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r) acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[r], pw[t], acc[t][r], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
#pragma unroll
            for (int r = 0; r < R; ++r) A[r] = An[r];
        }
    } else {
        for (int step = 0; step < nsteps; ++step, f += R * 64) {
            double A[R];
#pragma unroll
            for (int r = 0; r < R; ++r) A[r] = f[r * 64];
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < R; ++r) acc[t][r] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[r], pw[t], acc[t][r], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) pw[t] *= q4[t];
        }
    }
    if (threadIdx.x == 0) s.w2 = wall_clock64();
    if (lane == 0) {
        WaveRec r;
        r.t0 = s.w0; r.t1 = wall_clock64();
        r.hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        r.xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        g_waves[blockIdx.x * NWAVE + wave] = r;
    }
    constexpr int CC = 5, SG = 4 * R / CC;
    double y[NT][CC];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const double Q = exp(-beta[t] * 76.0);
        const double Q2 = Q * Q, Q4 = Q2 * Q2;
        const double Qt = (tq == 0) ? 1.0 : (tq == 1) ? Q : (tq == 2) ? Q2 : Q2 * Q;
#pragma unroll
        for (int c = 0; c < CC; ++c) {
            double v = 0.0;
#pragma unroll
            for (int m = SG - 1; m >= 0; --m) {
                const int g = c + CC * m;
                v = fma(v, Q4, acc[t][g >> 2][g & 3]);
            }
            v *= Qt;
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            y[t][c] = v;
        }
    }
    if (tq < NT) {
        double yy[CC], bu = 0.0;
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (t == tq) {
                bu = beta[t];
#pragma unroll
                for (int c = 0; c < CC; ++c) yy[c] = y[t][c];
            }
        const int64_t u = u0 + 16 * tq + col;
        if (u <= Umax) {
            const double s01 = exp(-bu * 0.5);
            const double G = expm1(-bu * 1199.0) / expm1(-bu);
            const double den = 1.0 + s01 * G;
#pragma unroll
            for (int c = 0; c < CC; ++c) conc[(int64_t)c * U + u] = (1.0 + s01 * yy[c]) / den;
        }
    }
    if (threadIdx.x == 0) { s.w3 = wall_clock64(); s.c3 = clock64(); st[blockIdx.x] = s; }
}

template <typename F>
void run_any(const char* name, F launch, int blocks, int NWAVE, int64_t U, Stamp* dst, int reps) {
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<Stamp> h(blocks);
    CK(hipMemcpy(h.data(), dst, blocks * sizeof(Stamp), hipMemcpyDeviceToHost));
    unsigned long long lo = ~0ull, hi = 0;
    double p0 = 0, p1 = 0, p2 = 0, clk = 0, latest_start = 0, dmax = 0;
    for (auto& s : h) {
        dmax = std::max(dmax, (double)(s.w3 - s.w0));
        lo = std::min(lo, s.w0); hi = std::max(hi, s.w3);
        p0 += (s.w1 - s.w0); p1 += (s.w2 - s.w1); p2 += (s.w3 - s.w2);
        clk += (double)(s.c3 - s.c0) / (double)(s.w3 - s.w0);
    }
    for (auto& s : h) latest_start = std::max(latest_start, (double)(s.w0 - lo));
    const double n = (double)blocks;
    {   // waves per SIMD and loop-end spread
        const int nw = blocks * NWAVE;
        std::vector<WaveRec> wv(nw);
        CK(hipMemcpyFromSymbol(wv.data(), HIP_SYMBOL(g_waves), nw * sizeof(WaveRec)));
        std::vector<int> cnt(8 * 4 * 2 * 16 * 4, 0);
        unsigned long long wlo = ~0ull;
        for (auto& r : wv) wlo = std::min(wlo, r.t0);
        int hist[8] = {0};
        double end_by_load[8] = {0};
        int n_by_load[8] = {0};
        std::vector<int> key(nw);
        for (int i = 0; i < nw; ++i) {
            const unsigned hw = wv[i].hw;
            const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 3;
            key[i] = ((((wv[i].xcc & 7) * 4 + se) * 2 + sh) * 16 + cu) * 4 + simd;
            cnt[key[i]]++;
        }
        int used = 0;
        for (int c : cnt) if (c) { used++; hist[std::min(c, 7)]++; }
        for (int i = 0; i < nw; ++i) {
            const int c = std::min(cnt[key[i]], 7);
            end_by_load[c] += (wv[i].t1 - wlo) / 100.0;
            n_by_load[c]++;
        }
        double xs[8] = {0}, xm[8] = {0};
        int xn[8] = {0};
        std::vector<double> ends(nw);
        for (int i = 0; i < nw; ++i) {
            const int x = wv[i].xcc & 7;
            const double e = (wv[i].t1 - wlo) / 100.0;
            ends[i] = e;
            xs[x] += e; xm[x] = std::max(xm[x], e); xn[x]++;
        }
        std::sort(ends.begin(), ends.end());
        printf("   loop end p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f us; per XCC mean/max:",
               ends[nw / 10], ends[nw / 2], ends[nw * 9 / 10], ends[nw * 99 / 100], ends[nw - 1]);
        for (int x = 0; x < 8; ++x) if (xn[x]) printf(" %d:%.1f/%.1f", x, xs[x] / xn[x], xm[x]);
        printf("\n");
        printf("   SIMDs used %d; waves/SIMD histogram:", used);
        for (int c = 1; c < 8; ++c) if (hist[c]) printf(" %d:%d (loop end %.1f us)", c, hist[c], end_by_load[c] / n_by_load[c]);
        printf("\n");
    }
    const double flop = 2.0 * U * C * 1199.0;
    printf("%-26s blocks %4d  %7.2f us/launch  %6.1f TF(alg)  span %6.2f us  max-block %6.2f  last-start %5.2f us | "
           "stage %5.2f  loop %5.2f  epi %5.2f us | clk %.2f GHz\n",
           name, blocks, 1e3 * ms / reps, flop / (1e-3 * ms / reps) / 1e12, (hi - lo) / 100.0, dmax / 100.0, latest_start / 100.0,
           p0 / n / 100.0, p1 / n / 100.0, p2 / n / 100.0, clk / n * 0.1);
}

template <int NT, int NWAVE, int STAGE>
void run(const char* name, const double* th, const double* fr, int64_t U, double* conc, Stamp* dst, int reps,
         size_t pad = 0) {
    const int blocks = (int)((U + 16 * NT * NWAVE - 1) / (16 * NT * NWAVE));
    size_t lds = std::max<size_t>(STAGE == 2 ? 0 : (size_t)NSTEPS * 2048, (size_t)NWAVE * NT * 16 * 17 * 8);
    lds = std::max(lds, pad);          // pad > 160K/(k+1) caps the blocks per CU at k
    auto k = probe<NT, NWAVE, STAGE>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    run_any(name, [&] { hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * NWAVE), lds, 0, th, fr, U, conc, dst); },
            blocks, NWAVE, U, dst, reps);
}

template <int R, int NT, int NWAVE, int MODE>
void run_rt(const char* name, const double* th, const double* fr, int64_t U, double* conc, Stamp* dst, int reps,
            size_t pad = 56 << 10) {
    const int nsteps = 19;
    const int blocks = (int)((U + 16 * NT * NWAVE - 1) / (16 * NT * NWAVE));
    size_t lds = std::max<size_t>(MODE == 2 ? 0 : (size_t)nsteps * R * 512, pad);
    auto k = probe_rt<R, NT, NWAVE, MODE>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    run_any(name, [&] { hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * NWAVE), lds, 0, th, fr, U, conc, dst, nsteps); },
            blocks, NWAVE, U, dst, reps);
}

int main(int argc, char** argv) {
    const int64_t U = 131072;
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    std::vector<double> th(U), fr((size_t)32 * 256 * 8);
    srand(7);
    for (auto& v : th) v = 1.0 + 999.0 * (rand() / (double)RAND_MAX);
    for (auto& v : fr) v = rand() / (double)RAND_MAX;
    double *dth, *dfr, *dconc;
    Stamp* dst;
    CK(hipMalloc(&dth, U * 8)); CK(hipMalloc(&dfr, fr.size() * 8)); CK(hipMalloc(&dconc, U * C * 8));
    CK(hipMalloc(&dst, 8192 * sizeof(Stamp)));
    CK(hipMemcpy(dth, th.data(), U * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dfr, fr.data(), fr.size() * 8, hipMemcpyHostToDevice));
    run_rt<5, 4, 4, 0>("W4 lds56K (prod)", dth, dfr, U, dconc, dst, reps);
    run_rt<5, 4, 4, 0>("W4 lds96K", dth, dfr, U, dconc, dst, reps, 96 << 10);
    run_rt<5, 4, 8, 0>("W8 lds56K", dth, dfr, U, dconc, dst, reps, 56 << 10);
    run_rt<5, 4, 8, 0>("W8 lds64K", dth, dfr, U, dconc, dst, reps, 64 << 10);
    run_rt<5, 4, 8, 0>("W8 lds80K", dth, dfr, U, dconc, dst, reps, 80 << 10);
    run_rt<5, 4, 8, 0>("W8 lds96K", dth, dfr, U, dconc, dst, reps, 96 << 10);
    run_rt<5, 4, 16, 0>("W16 lds96K", dth, dfr, U, dconc, dst, reps, 96 << 10);
    run_rt<5, 4, 4, 0>("W4 lds56K (prod) again", dth, dfr, U, dconc, dst, reps);
    return 0;
}
