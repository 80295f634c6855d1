// Microbenchmark: FP64 throughput on gfx950 -- VALU v_fma_f64 vs MFMA v_mfma_f64_16x16x4f64,
// alone and co-issued.  Decides how the RTD Horner evaluation should be mapped.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_fp64 tools/ubench_fp64.hip && /tmp/ubench_fp64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int CH>
__global__ void valu_fma(double* out, double q, int iters) {
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], q, 1e-7 * c);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    if (s == 1234.5) out[threadIdx.x] = s;
}

template <int NA>
__global__ void mfma_f64(double* out, double a0, double b0, int iters) {
    v4d acc[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) acc[j] = v4d{0.0, 0.0, 0.0, 0.0};
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < NA; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    if (s == 1234.5) out[threadIdx.x] = s;
}

// waves with even id do MFMA, odd do VALU FMA (same SIMD pairs share pipes)
template <int CH, int NA>
__global__ void mixed(double* out, double q, int iters_v, int iters_m) {
    const int wave = threadIdx.x >> 6;
    if (wave & 1) {
        double acc[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
        for (int i = 0; i < iters_v; ++i) {
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], q, 1e-7 * c);
        }
        double s = 0;
#pragma unroll
        for (int c = 0; c < CH; ++c) s += acc[c];
        if (s == 1234.5) out[threadIdx.x] = s;
    } else {
        v4d acc[NA];
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[j] = v4d{0.0, 0.0, 0.0, 0.0};
        double a = q + threadIdx.x * 1e-9, b = q - threadIdx.x * 1e-9;
        for (int i = 0; i < iters_m; ++i) {
#pragma unroll
            for (int j = 0; j < NA; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
        }
        double s = 0;
#pragma unroll
        for (int j = 0; j < NA; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
        if (s == 1234.5) out[threadIdx.x] = s;
    }
}

// one wave interleaves MFMA and VALU FMA in its own stream
template <int CH, int NA>
__global__ void interleaved(double* out, double q, int iters) {
    double acc[CH];
    v4d m[NA];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
#pragma unroll
    for (int j = 0; j < NA; ++j) m[j] = v4d{0.0, 0.0, 0.0, 0.0};
    double a = q + threadIdx.x * 1e-9, b = q - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NA; ++j) m[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m[j], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], q, 1e-7 * c);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
#pragma unroll
    for (int j = 0; j < NA; ++j) s += m[j][0] + m[j][1] + m[j][2] + m[j][3];
    if (s == 1234.5) out[threadIdx.x] = s;
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <typename F>
static float timeit(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    double* out; CHECK(hipMalloc(&out, 1 << 20));
    const int CUs = 256;
    const int iters = 4096;
    for (int wps : {1, 2, 4, 8}) {   // waves per SIMD
        const int blocks = CUs * wps, threads = 256;  // 4 waves per block -> 1 per SIMD
        float ms = timeit([&] { hipLaunchKernelGGL(valu_fma<16>, dim3(blocks), dim3(threads), 0, 0, out, 0.999, iters); });
        double flop = 2.0 * 16 * iters * (double)blocks * threads;
        printf("VALU fma_f64 16 chains  waves/SIMD=%d: %.3f ms  %.1f TFLOP/s\n", wps, ms, flop / ms / 1e9);
    }
    for (int wps : {1, 2, 4}) {
        const int blocks = CUs * wps, threads = 256;
        float ms = timeit([&] { hipLaunchKernelGGL(mfma_f64<4>, dim3(blocks), dim3(threads), 0, 0, out, 0.5, 0.25, iters / 4); });
        double flop = 2.0 * 16 * 16 * 4 * 4 * (iters / 4) * (double)blocks * (threads / 64);
        printf("MFMA f64 16x16x4 (4 acc) waves/SIMD=%d: %.3f ms  %.1f TFLOP/s\n", wps, ms, flop / ms / 1e9);
    }
    {
        // 8 waves per block: waves 0,2,4,6 MFMA; 1,3,5,7 VALU; two blocks per CU
        const int blocks = CUs * 2, threads = 512;
        const int iv = 4096, im = 1024;
        float ms = timeit([&] { hipLaunchKernelGGL((mixed<16, 4>), dim3(blocks), dim3(threads), 0, 0, out, 0.999, iv, im); });
        double fv = 2.0 * 16 * iv * 64 * 4 * (double)blocks;
        double fm = 2.0 * 16 * 16 * 4 * 4 * im * 4 * (double)blocks;
        float msv = timeit([&] { hipLaunchKernelGGL((mixed<16, 4>), dim3(blocks), dim3(threads), 0, 0, out, 0.999, iv, 0); });
        float msm = timeit([&] { hipLaunchKernelGGL((mixed<16, 4>), dim3(blocks), dim3(threads), 0, 0, out, 0.999, 0, im); });
        printf("mixed waves: both %.3f ms (%.1f TF total)  valu-only %.3f ms  mfma-only %.3f ms\n", ms,
               (fv + fm) / ms / 1e9, msv, msm);
    }
    {
        const int blocks = CUs * 2, threads = 256;
        float ms = timeit([&] { hipLaunchKernelGGL((interleaved<16, 2>), dim3(blocks), dim3(threads), 0, 0, out, 0.999, 2048); });
        double f = (2.0 * 16 * 64 + 2.0 * 16 * 16 * 4 * 2) * 2048 * (double)blocks * 4;
        printf("interleaved in one wave (16 fma + 2 mfma / iter): %.3f ms %.1f TF\n", ms, f / ms / 1e9);
    }
    return 0;
}
