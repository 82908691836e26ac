// tools/pmc_calib.hip — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the
// access width the SIFT kernels use (8 bytes per lane, global_load_dwordx2 /
// global_store_dwordx2), on a buffer larger than the 256 MiB Infinity Cache.
// The copy moves exactly N*8 bytes in and N*8 bytes out per launch; run it
// under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`,
// and divide the known byte counts by the counter values.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void copy_f64_x2(const double* __restrict__ a,
                                                   double* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

int main() {
    const size_t n = (size_t)96 << 20;  // 96 Mi doubles = 768 MiB per buffer
    double *a, *b;
    if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) return 1;
    hipMemset(a, 0, n * 8);
    hipMemset(b, 0, n * 8);
    for (int it = 0; it < 3; ++it) {
        hipLaunchKernelGGL(copy_f64_x2, dim3(8192), dim3(256), 0, 0, a, b, n);
        hipDeviceSynchronize();
    }
    std::printf("copy_f64_x2: %zu bytes read, %zu bytes written per launch\n", n * 8, n * 8);
    hipFree(a);
    hipFree(b);
    return 0;
}
