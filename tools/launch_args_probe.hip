// Per-launch cost of an empty kernel in the fused log-prob's shape (256 blocks x 1024
// threads, 41 KB dynamic LDS) against the size of its by-value kernel arguments: 16 B
// (a pointer) vs ~2 KB (the RtdArgs + UnitArgs blocks).  Back-to-back launches on one
// stream, HIP events around 400 of them.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_args_probe tools/launch_args_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big {
    double v[256];
};

__global__ void __launch_bounds__(1024) k_small(double* out) {
    extern __shared__ double lds[];
    lds[threadIdx.x] = out[threadIdx.x & 255];
    __syncthreads();
    if (lds[(threadIdx.x + 1) & 1023] == 12345.0) out[threadIdx.x & 255] = 1.0;
}

__global__ void __launch_bounds__(1024) k_big(const Big b, double* out) {
    extern __shared__ double lds[];
    lds[threadIdx.x] = b.v[threadIdx.x & 255];
    __syncthreads();
    if (lds[(threadIdx.x + 1) & 1023] == 12345.0) out[threadIdx.x & 255] = 1.0;
}

__global__ void __launch_bounds__(1024) k_ptr(const Big* b, double* out) {
    extern __shared__ double lds[];
    lds[threadIdx.x] = b->v[threadIdx.x & 255];
    __syncthreads();
    if (lds[(threadIdx.x + 1) & 1023] == 12345.0) out[threadIdx.x & 255] = 1.0;
}

template <class F>
static void time(const char* name, F launch) {
    for (int i = 0; i < 10; ++i) launch();
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 400;
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-40s %.2f us per launch\n", name, 1e3 * ms / reps);
}

int main() {
    double* d;
    hipMalloc(&d, 1 << 20);
    hipMemset(d, 0, 1 << 20);
    Big h{};
    Big* dp;
    hipMalloc(&dp, sizeof(Big));
    hipMemcpy(dp, &h, sizeof(Big), hipMemcpyHostToDevice);
    const size_t lds = 41 * 1024;
    hipFuncSetAttribute((const void*)k_small, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)k_big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)k_ptr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int rep = 0; rep < 2; ++rep) {
        time("8-B args (pointer), 256 x 1024, 41 KB", [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), lds, 0, d); });
        time("2-KB args by value, 256 x 1024, 41 KB", [&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), lds, 0, h, d); });
        time("args in device memory, 256 x 1024, 41 KB", [&] { hipLaunchKernelGGL(k_ptr, dim3(256), dim3(1024), lds, 0, dp, d); });
        time("8-B args, 256 x 1024, no LDS", [&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, 0, d); });
        time("8-B args, 512 x 512, 41 KB", [&] { hipLaunchKernelGGL(k_small, dim3(512), dim3(512), lds, 0, d); });
    }
    return 0;
}
