#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long* o, int n) {
    unsigned long long w0 = wall_clock64(), c0 = clock64();
    double x = 1.0;
    for (int i = 0; i < n; ++i) x = fma(x, 1.0000001, 1e-9);
    unsigned long long w1 = wall_clock64(), c1 = clock64();
    if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = w1 - w0; o[1] = c1 - c0; o[2] = (unsigned long long)x; }
}
int main() {
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("wall clock rate attr = %d kHz, clock rate attr = %d kHz\n", rate, clk);
    unsigned long long* d; hipMalloc(&d, 64);
    unsigned long long h[3];
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int n : {1000000, 10000000}) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, n);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("n=%d event %.3f ms, wall ticks %llu (%.3f ms at 100MHz), clock64 %llu -> %.3f GHz vs event\n", n, ms, h[0], h[0] / 1e5, h[1], h[1] / (ms * 1e6));
    }
}
