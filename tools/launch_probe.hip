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

int main() {
    double* d; hipMalloc(&d, 1 << 20); hipMemset(d, 0, 1 << 20);
    const long long cyc = 48000;   // ~20 us at 2.4 GHz
    (void)cyc;
    run<256, 8>("256thr VG8", 512, 0, 0, d);
    run<256, 16>("256thr VG16", 512, 0, 0, d);
    run<256, 32>("256thr VG32", 512, 0, 0, d);
    run<256, 48>("256thr VG48", 512, 0, 0, d);
    run<256, 64>("256thr VG64", 512, 0, 0, d);
    run<256, 96>("256thr VG96", 512, 0, 0, d);
    run<256, 8>("256thr VG8 x4 blocks", 2048, 0, 0, d);
    run<256, 32>("256thr VG32 x4 blocks", 2048, 0, 0, d);
    run<256, 48>("256thr VG48 x4 blocks", 2048, 0, 0, d);
    run<256, 8>("256thr VG8 x16 blocks", 8192, 0, 0, d);
    return 0;
}
