// FETCH_SIZE calibration for the access widths the ngrtd kernels use (MI355X_MICROARCH.md
// 'HBM': only 16 B/lane streaming reads are calibrated there, at 1/2).  Each kernel reads a
// known byte count once; run under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` and divide.
//   read8   : one double per lane, consecutive lanes consecutive (theta rows of the
//             log-prob kernels: 512 B per wave instruction)
//   read16  : one double2 per lane (the LDS staging copies of the fragment tables)
// Sizes: 8 MiB (theta-sized, L3-resident) and 512 MiB (past the 256 MiB Infinity Cache).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void read8(const double* __restrict__ x, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += x[i];
    if (s == 12345.678) out[0] = s;
}

__global__ void read16(const double2* __restrict__ x, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = x[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s;
}

int main() {
    const size_t sizes[2] = {(size_t)8 << 20, (size_t)512 << 20};
    double* out;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    for (size_t bytes : sizes) {
        void* buf;
        if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
        if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
        // evict: stream a different 512 MiB buffer between runs so every run starts cold
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, (const double*)buf, bytes / 8, out);
            hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, (const double2*)buf, bytes / 16, out);
        }
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        printf("bytes %zu (%.1f KiB)\n", bytes, bytes / 1024.0);
        (void)hipFree(buf);
    }
    (void)hipFree(out);
    return 0;
}
