// synth.cpp — portable synthetic SIFT workload generator.
//
// the survey's images used std::mt19937 +
// uniform_real_distribution + libm sin/cos/exp, which are not portable by
// spec. This generator is defined ONLY through integer arithmetic
// (splitmix64) and IEEE-754 basic operations (+ - * / floor, no FMA
// contraction: build with -ffp-contract=off), so it produces the same bits on
// this container, on the GPU box and anywhere else. It defines the workload
// class of BASELINE configs 2-5: a 128+40*sin(x/37)*cos(y/53) background plus
// N Gaussian blobs (sigma in [1.5, 1.5+smax], amplitude in [-100, 100]),
// clamped to [0,255] and rounded to integers.
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>

#include "../../include/sift_hip.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    // uniform in [0,1): top 53 bits times 2^-53 (exact).
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// 2^n for integer n in the normal range, built from bits (exact).
double pow2i(int n) {
    if (n < -1022) return 0.0;
    uint64_t bits = (uint64_t)(n + 1023) << 52;
    double d;
    std::memcpy(&d, &bits, sizeof d);
    return d;
}

// exp(x) for x <= 0 from basic operations only (Cody-Waite + Taylor).
double det_exp(double x) {
    if (x < -700.0) return 0.0;
    const double inv_ln2 = 1.4426950408889634;
    const double ln2_hi = 0.6931471803691238;      // 0x3FE62E42FEE00000
    const double ln2_lo = 1.9082149292705877e-10;  // ln2 - ln2_hi
    double n = std::floor(x * inv_ln2 + 0.5);
    double r = (x - n * ln2_hi) - n * ln2_lo;
    double p = 1.0;
    for (int k = 13; k >= 1; --k) p = 1.0 + p * r / (double)k;
    return p * pow2i((int)n);
}

// sin/cos from basic operations only (range reduction to [-pi, pi]).
double det_reduce(double x) {
    const double inv_2pi = 0.15915494309189535;
    const double two_pi_hi = 6.283185307179586;
    const double two_pi_lo = 2.4492935982947064e-16;
    double k = std::floor(x * inv_2pi + 0.5);
    return (x - k * two_pi_hi) - k * two_pi_lo;
}

double det_sin(double x) {
    double r = det_reduce(x);
    double r2 = r * r;
    // sin r = r * sum_{k>=0} (-1)^k r^(2k) / (2k+1)!
    double p = 1.0;
    for (int k = 14; k >= 1; --k) p = 1.0 - p * r2 / (double)((2 * k) * (2 * k + 1));
    return r * p;
}

double det_cos(double x) {
    double r = det_reduce(x);
    double r2 = r * r;
    double p = 1.0;
    for (int k = 14; k >= 1; --k) p = 1.0 - p * r2 / (double)((2 * k - 1) * (2 * k));
    return p;
}

double clamp_round(double v) {
    if (v < 0.0) v = 0.0;
    if (v > 255.0) v = 255.0;
    return std::floor(v + 0.5);
}

}  // namespace

extern "C" int sift_synth_image(int w, int h, int channels, int64_t nblobs,
                                double smax, uint64_t seed, double* out) {
    if (w <= 0 || h <= 0 || out == nullptr || nblobs < 0 || smax < 0.0)
        return SIFT_ERR_ARG;
    if (channels != 1 && channels != 3) return SIFT_ERR_CHANNELS;

    const size_t n = (size_t)w * (size_t)h;
    std::vector<double> acc(n);
    std::vector<double> cx(w);
    for (int x = 0; x < w; ++x) cx[x] = det_sin((double)x / 37.0);
    for (int y = 0; y < h; ++y) {
        double cy = det_cos((double)y / 53.0);
        for (int x = 0; x < w; ++x) acc[(size_t)y * w + x] = 128.0 + 40.0 * cx[x] * cy;
    }

    SplitMix64 rng(seed);
    std::vector<double> ex, ey;
    for (int64_t b = 0; b < nblobs; ++b) {
        const double bx = rng.uniform() * (double)w;
        const double by = rng.uniform() * (double)h;
        const double sigma = 1.5 + rng.uniform() * smax;
        const double amp = (rng.uniform() * 2.0 - 1.0) * 100.0;
        const int r = (int)std::ceil(3.0 * sigma);
        const double denom = 2.0 * sigma * sigma;
        const int x0 = (int)std::floor(bx) - r, x1 = (int)std::floor(bx) + r;
        const int y0 = (int)std::floor(by) - r, y1 = (int)std::floor(by) + r;
        const int xa = x0 < 0 ? 0 : x0, xb = x1 >= w ? w - 1 : x1;
        const int ya = y0 < 0 ? 0 : y0, yb = y1 >= h ? h - 1 : y1;
        if (xa > xb || ya > yb) continue;
        ex.resize(xb - xa + 1);
        ey.resize(yb - ya + 1);
        for (int x = xa; x <= xb; ++x) {
            double d = (double)x - bx;
            ex[x - xa] = det_exp(-(d * d) / denom);
        }
        for (int y = ya; y <= yb; ++y) {
            double d = (double)y - by;
            ey[y - ya] = amp * det_exp(-(d * d) / denom);
        }
        for (int y = ya; y <= yb; ++y) {
            double* row = &acc[(size_t)y * w];
            const double fy = ey[y - ya];
            for (int x = xa; x <= xb; ++x) row[x] += fy * ex[x - xa];
        }
    }

    if (channels == 1) {
        for (size_t i = 0; i < n; ++i) out[i] = clamp_round(acc[i]);
    } else {
        for (size_t i = 0; i < n; ++i) {
            double v = clamp_round(acc[i]);
            out[3 * i + 0] = v;
            out[3 * i + 1] = clamp_round(0.8 * v + 20.0);
            out[3 * i + 2] = clamp_round(255.0 - v);
        }
    }
    return SIFT_OK;
}
