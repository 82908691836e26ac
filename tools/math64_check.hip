// math64_check.hip — accuracy of the descriptor's f64 sqrt / atan2 / exp
// (sift-project_amd/csrc/sift_math64.h) against the device's own sqrt
// (correctly rounded), ocml's atan2 / exp, and the host's glibc, on the
// argument ranges the descriptor feeds them (src/sift.cpp:660-672):
// sqrt of dx^2 + dy^2, atan2(dy, dx), exp of -(row_rot^2 + col_rot^2) / 8.
//
//   math64_check [n]   ->  one line per function:
//   <fn> n=<n> ulp_max_dev=<u> diff_frac_dev=<f> ulp_max_glibc=<u> diff_frac_glibc=<f>
//
// Built by __graft_entry__.build(); run by tests/test_gpu_math64.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../sift-project_amd/csrc/sift_device.h"
#include "../sift-project_amd/csrc/sift_math64.h"

using namespace sift_amd;

__global__ void k_eval(const double* a, const double* b, int n, double* mine, double* dev, int fn) {
    __shared__ double2 tab[17];
    if (threadIdx.x < 17) tab[threadIdx.x] = kAtanTab[threadIdx.x];
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (fn == 0) {
        const double s = a[i] * a[i] + b[i] * b[i];
        mine[i] = sqrt_f64(s);
        dev[i] = sqrt(s);
    } else if (fn == 1 || fn == 4) {
        mine[i] = atan2_f64(a[i], b[i], tab);
        dev[i] = atan2(a[i], b[i]);
    } else if (fn == 2) {
        mine[i] = exp_f64(a[i]);
        dev[i] = exp(a[i]);
    } else {  // the f32 atan2 of the orientation bins, error in radians
        mine[i] = (double)atan2_f32((float)a[i], (float)b[i]);
        dev[i] = atan2(a[i], b[i]);
    }
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {  // splitmix64
    uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni() { return (next_u64() >> 11) * 0x1.0p-53; }

static int64_t ulp_diff(double x, double y) {
    if (x == y) return 0;
    int64_t a, b;
    std::memcpy(&a, &x, 8);
    std::memcpy(&b, &y, 8);
    if (a < 0) a = INT64_MIN - a;
    if (b < 0) b = INT64_MIN - b;
    return a > b ? a - b : b - a;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : (1 << 22);
    std::vector<double> a(n), b(n), mine(n), dev(n);
    double *da, *db, *dm, *dd;
    if (hipMalloc(&da, n * 8) || hipMalloc(&db, n * 8) || hipMalloc(&dm, n * 8) ||
        hipMalloc(&dd, n * 8)) {
        std::fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    // atan2_tiny: atan2_f64 on gradients below the f32 normal range (2^-700
    // scale) and subnormal ones (2^-1040): never produced by image data, the
    // out-of-line fallback keeps them correct
    const char* names[5] = {"sqrt", "atan2", "exp", "atan2_f32", "atan2_tiny"};
    for (int fn = 0; fn < 5; ++fn) {
        for (int i = 0; i < n; ++i) {
            if (fn == 2) {
                a[i] = -1.6 * uni();
                b[i] = 0.0;
                continue;
            }
            // gradients of blurred 0..255 images: differences of doubles,
            // with exact zeros, axis-aligned and diagonal cases mixed in
            const int kind = (int)(next_u64() % 16);
            double x = (uni() - 0.5) * 100.0, y = (uni() - 0.5) * 100.0;
            if (kind == 0) x = 0.0;
            if (kind == 1) y = 0.0;
            if (kind == 2) x = y = 0.0;
            if (kind == 3) y = x;
            if (kind == 4) y = -x;
            if (kind == 5) x *= 1e-6;
            if (kind == 6) y *= 1e-9;
            if (kind == 7) {  // a = y/x near a table point k/16
                const double k = (double)(next_u64() % 17) / 16.0;
                y = x * k * (1.0 + (uni() - 0.5) * 1e-6);
            }
            if (fn == 4) {  // below the f32 range, and subnormal
                const double s = (next_u64() & 1) ? 0x1p-700 : 0x1p-1040;
                x *= s;
                y *= s;
            }
            a[i] = y;
            b[i] = x;
        }
        if (hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice) ||
            hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice)) {
            std::fprintf(stderr, "hipMemcpy failed\n");
            return 1;
        }
        hipLaunchKernelGGL(k_eval, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, n, dm, dd, fn);
        if (hipDeviceSynchronize() || hipMemcpy(mine.data(), dm, n * 8, hipMemcpyDeviceToHost) ||
            hipMemcpy(dev.data(), dd, n * 8, hipMemcpyDeviceToHost)) {
            std::fprintf(stderr, "kernel failed\n");
            return 1;
        }
        if (fn == 3) {
            double emax = 0.0;
            for (int i = 0; i < n; ++i) emax = std::max(emax, std::fabs(mine[i] - dev[i]));
            std::printf("%s n=%d abs_err_max_rad=%.3e\n", names[fn], n, emax);
            continue;
        }
        int64_t umax_dev = 0, umax_ref = 0;
        long ndiff_dev = 0, ndiff_ref = 0;
        for (int i = 0; i < n; ++i) {
            double ref;
            if (fn == 0) ref = std::sqrt(a[i] * a[i] + b[i] * b[i]);
            else if (fn == 1 || fn == 4) ref = std::atan2(a[i], b[i]);
            else ref = std::exp(a[i]);
            const int64_t ud = ulp_diff(mine[i], dev[i]), ur = ulp_diff(mine[i], ref);
            umax_dev = ud > umax_dev ? ud : umax_dev;
            umax_ref = ur > umax_ref ? ur : umax_ref;
            ndiff_dev += ud != 0;
            ndiff_ref += ur != 0;
        }
        std::printf("%s n=%d ulp_max_dev=%lld diff_frac_dev=%.3e ulp_max_glibc=%lld "
                    "diff_frac_glibc=%.3e\n",
                    names[fn], n, (long long)umax_dev, (double)ndiff_dev / n, (long long)umax_ref,
                    (double)ndiff_ref / n);
    }
    return 0;
}
