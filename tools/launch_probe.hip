// Dead time between back-to-back kernels vs block shape: each wave spins for a fixed
// number of shader cycles; per-launch time minus the spin is the dispatch/drain cost.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int NTH, int VG>
__global__ void __launch_bounds__(NTH) spin(double* out, long long cycles) {
    extern __shared__ double lds[];
    double v[VG];
#pragma unroll
    for (int i = 0; i < VG; ++i) v[i] = out[(threadIdx.x + i) & 1023];
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
#pragma unroll
        for (int i = 0; i < VG; ++i) v[i] = v[i] * 1.0000001;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < VG; ++i) s += v[i];
    if (s == 12345.0) { lds[threadIdx.x] = s; out[threadIdx.x] = lds[(threadIdx.x + 1) % NTH]; }
}

template <int NTH, int VG>
void run(const char* name, int blocks, size_t lds, long long cycles, double* d) {
    auto k = spin<NTH, VG>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(NTH), lds, 0, d, cycles);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int reps = 200;
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(NTH), lds, 0, d, cycles);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-34s blocks %5d lds %6zu  spin %.2f us  per launch %.2f us\n", name, blocks, lds, cycles / 2.4e3,
           1e3 * ms / reps);
}

template <int NTH, int VG>
void run2(const char* name, int blocks, size_t lds, long long cycles, double* d, int nsplit) {
    auto k = spin<NTH, VG>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipStream_t s0, s[4];
    hipStreamCreate(&s0);
    for (int i = 0; i < nsplit; ++i) hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    hipEvent_t fork[64], join[4][64];
    for (int i = 0; i < 64; ++i) { hipEventCreateWithFlags(&fork[i], hipEventDisableTiming);
        for (int j = 0; j < 4; ++j) hipEventCreateWithFlags(&join[j][i], hipEventDisableTiming); }
    auto step = [&](int it) {
        hipEventRecord(fork[it & 63], s0);
        for (int i = 0; i < nsplit; ++i) {
            hipStreamWaitEvent(s[i], fork[it & 63], 0);
            hipLaunchKernelGGL(k, dim3(blocks / nsplit), dim3(NTH), lds, s[i], d, cycles);
            hipEventRecord(join[i][it & 63], s[i]);
            hipStreamWaitEvent(s0, join[i][it & 63], 0);
        }
    };
    for (int i = 0; i < 5; ++i) step(i);
    hipDeviceSynchronize();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int reps = 200;
    hipEventRecord(a, s0);
    for (int i = 0; i < reps; ++i) step(i);
    hipEventRecord(b, s0); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-34s blocks %5d split %d  spin %.2f us  per step %.2f us\n", name, blocks, nsplit, cycles / 2.4e3,
           1e3 * ms / reps);
}

int main(int argc, char** argv) {
    double* d; hipMalloc(&d, 1 << 20); hipMemset(d, 0, 1 << 20);
    if (argc > 1) {   // the single-launch log-prob kernel's shape: 256 blocks x 512 threads, 35 KB LDS
        for (long long cyc : {0LL, 2400LL, 12000LL, 24000LL, 36000LL})
            run<512, 48>("512thr VG48 1 stream", 256, 35 * 1024, cyc, d);
        // same 2048 waves in other block shapes / LDS sizes
        run<1024, 48>("1024thr VG48 1 stream", 128, 35 * 1024, 0, d);
        run<256, 48>("256thr VG48 1 stream", 512, 35 * 1024, 0, d);
        run<512, 48>("512thr VG48 nolds", 256, 0, 0, d);
        run<512, 48>("512thr VG48 1 stream", 128, 35 * 1024, 0, d);
        run<512, 48>("512thr VG48 1 stream", 64, 35 * 1024, 0, d);
        run<64, 48>("64thr VG48 1 stream", 2048, 0, 0, d);
        // the same launches replayed from a hipGraph (1 and 10 launches per graph)
        for (int per : {1, 10}) {
            for (long long cyc : {0LL, 24000LL}) {
                auto k = spin<512, 48>;
                hipStream_t s; hipStreamCreate(&s);
                hipGraph_t g; hipGraphExec_t ge;
                hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
                for (int i = 0; i < per; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(512), 35 * 1024, s, d, cyc);
                hipStreamEndCapture(s, &g);
                hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
                for (int i = 0; i < 3; ++i) hipGraphLaunch(ge, s);
                hipStreamSynchronize(s);
                hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
                const int reps = 200 / per;
                hipEventRecord(a, s);
                for (int i = 0; i < reps; ++i) hipGraphLaunch(ge, s);
                hipEventRecord(b, s); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                printf("graph of %2d launches             spin %.2f us  per launch %.2f us\n", per, cyc / 2.4e3,
                       1e3 * ms / (reps * per));
            }
        }
        return 0;
    }
    const long long cyc = 48000;   // ~20 us at 2.4 GHz
    run<256, 96>("256thr VG96 1 stream", 512, 57344, cyc, d);
    run2<256, 96>("256thr VG96 streams", 512, 57344, cyc, d, 1);
    run2<256, 96>("256thr VG96 streams", 512, 57344, cyc, d, 2);
    run2<256, 96>("256thr VG96 streams", 512, 57344, cyc, d, 4);
    run<256, 96>("256thr VG96 1 stream nospin", 512, 57344, 0, d);
    run2<256, 96>("256thr VG96 streams nospin", 512, 57344, 0, d, 2);
    return 0;
}
