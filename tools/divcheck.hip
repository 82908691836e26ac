// tools/divcheck.hip — evidence for the blur normaliser: the
// pyramid kernels compute a / sum_w as Markstein's correction of a * inv
// (inv = RN(1/sum_w) from the host; q = a*inv; r = fma(-q, s, a);
// q' = fma(r, inv, q)). This tool compares that against IEEE division on
// random operands for every normaliser the default pyramids use
// (intervals 1..5, init_sigma 1.6, double_image_size) plus generic sigmas.
// Not part of the product.
//
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/divcheck tools/divcheck.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

// reference src/image.cpp:226-235 taps; sum_w as the blur loops accumulate it
static double sum_w_of(double sigma, int* radius) {
    const int ks = (int)std::ceil(3 * sigma) + 1;
    const double d = 2 * sigma * sigma, coef = 1 / (std::sqrt(2 * M_PI) * sigma);
    double s = std::exp(0.0) * coef;
    for (int u = 1; u < ks; ++u) s += 2.0 * (std::exp(-u * u / d) * coef);
    *radius = ks - 1;
    return s;
}

__global__ void k_divcheck(double s, double inv, uint64_t seed, int per_thread,
                           unsigned long long* bad, double* first_bad) {
    uint64_t st = seed ^ (0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1));
    unsigned nbad = 0;
    for (int i = 0; i < per_thread; ++i) {
        st ^= st >> 12;
        st ^= st << 25;
        st ^= st >> 27;
        const uint64_t r = st * 2685821657736338717ull;
        // positive doubles with exponents spanning [2^-20, 2^12)
        const uint64_t mant = r & ((1ull << 52) - 1);
        const uint64_t ex = 1023 - 20 + ((r >> 52) % 32);
        const double a = __longlong_as_double((long long)((ex << 52) | mant));
        const double q = a * inv;
        const double rr = __builtin_fma(-q, s, a);
        const double f = __builtin_fma(rr, inv, q);
        if (f != a / s) {
            ++nbad;
            *first_bad = a;
        }
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

int main() {
    std::vector<double> sig = {1.2489995996796797, 2.0, 2.5, 3.5, 4.0, 5.0, 6.5};
    for (int iv = 1; iv <= 5; ++iv) {
        const double k = std::pow(2.0, 1.0 / iv);
        for (int i = 1; i < iv + 3; ++i) sig.push_back(std::pow(k, i - 1) * 1.6 * std::sqrt(k * k - 1));
    }
    unsigned long long* d_bad;
    double* d_first;
    CK(hipMalloc(&d_bad, 8));
    CK(hipMalloc(&d_first, 8));
    unsigned long long total_bad = 0;
    for (double sg : sig) {
        int R;
        const double s = sum_w_of(sg, &R), inv = 1.0 / s;
        CK(hipMemset(d_bad, 0, 8));
        const int blocks = 4096, per = 4096, reps = 16;
        for (int rep = 0; rep < reps; ++rep)
            hipLaunchKernelGGL(k_divcheck, dim3(blocks), dim3(256), 0, 0, s, inv,
                               (uint64_t)rep * 7919 + 1, per, d_bad, d_first);
        CK(hipDeviceSynchronize());
        unsigned long long bad;
        CK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
        total_bad += bad;
        std::printf("divcheck sigma=%.7f R=%d s=%a inv=%a samples=%.3g mismatches=%llu%s\n", sg, R,
                    s, inv, (double)reps * blocks * 256.0 * per, bad, bad ? " FAIL" : "");
        std::fflush(stdout);
    }
    return total_bad ? 1 : 0;
}
