// blur_lab.hip — octave-0 blur variants against the library's k_blur on the
// GPU box: bit-exactness (every output and decimated pixel) and per-launch
// time along a level chain like the pyramid's (plane l -> plane l+1, the
// decimation on the level `dec_at`), so each launch reads what the previous
// one just wrote, as in compute_gaussian_octave (reference sift.cpp:161-174,
// image.cpp:156-214).
//
//   blur_lab VARIANT W H dec_at R1 R2 ...   (e.g. pc:1:64 3840 2160 2 4 5 6 8 10)
// VARIANT = kind:C:rows, kind pc / ud (tools/blur_variants.h), pair (the
// library's k_blur_pair at that shape) or strip (the
// library's k_blur at that shape); the baseline is the library's launch_blur.
//
// Test tooling only: includes the library's kernel translation unit.
#include "../sift-project_amd/csrc/sift_kernels.hip"
#include "blur_variants.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace sift_amd;

namespace {

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                         hipGetErrorString(e_));                                      \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

BlurTaps taps_for_radius(int R) {
    // sigma with ceil(3 sigma) == R (image.cpp:226): the taps' values do not
    // matter for the comparison, only that both kernels use the same ones
    const double sigma = (R - 0.5) / 3.0;
    BlurTaps t{};
    t.R = R;
    double sw = 0.0;
    for (int u = 0; u <= R; ++u) {
        t.k[u] = std::exp(-(double)(u * u) / (2.0 * sigma * sigma)) / (std::sqrt(2 * M_PI) * sigma);
        sw += u ? 2.0 * t.k[u] : t.k[u];
    }
    t.sum_w = sw;
    t.inv = 1.0 / sw;
    return t;
}

using Launch = hipError_t (*)(const double*, double*, int, int, const BlurTaps&, double*, int,
                              int, hipStream_t, hipEvent_t, hipEvent_t);

hipError_t run_base(const double* src, double* dst, int W, int H, const BlurTaps& t, double* dec,
                    int Wd, int Hd, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    return launch_blur(src, 0, dst, 0, 1, W, H, t, dec, Wd, Hd, nullptr, s, e0, e1, (size_t)1 << 21);
}

char g_kind[16];
int g_C = 2, g_rows = 32;

hipError_t run_walk(const double* src, double* dst, int W, int H, const BlurTaps& t, double* dec,
                    int Wd, int Hd, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    lab::VarFn f = lab::pick(g_kind, g_C, t.R);
    if (!f) {
        std::fprintf(stderr, "no variant %s C=%d R=%d\n", g_kind, g_C, t.R);
        std::exit(2);
    }
    return f(src, dst, W, H, g_rows, t, dec, Wd, Hd, s, e0, e1);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s kind:C:rows W H dec_at R1 [R2 ...]\n", argv[0]);
        return 2;
    }
    if (std::sscanf(argv[1], "%15[a-z]:%d:%d", g_kind, &g_C, &g_rows) != 3) return 2;
    ++argv;
    --argc;
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]), dec_at = std::atoi(argv[3]);
    std::vector<int> radii;
    for (int i = 4; i < argc; ++i) radii.push_back(std::atoi(argv[i]));
    const int L = (int)radii.size();
    const size_t N = (size_t)W * H;
    const int Wd = W / 2, Hd = H / 2;
    std::vector<double> h0(N);
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < N; ++i) {  // smooth-ish 0..255 plane with noise
        z ^= z << 13;
        z ^= z >> 7;
        z ^= z << 17;
        const double x = (double)(i % W), y = (double)(i / W);
        h0[i] = 128.0 + 60.0 * std::sin(x / 23.0) * std::cos(y / 31.0) +
                (double)(z >> 40) / (double)(1ull << 24) * 60.0;
    }
    struct Chain {
        std::vector<double*> p;
        double* dec = nullptr;
    };
    auto alloc = [&](Chain& c) {
        c.p.resize(L + 1);
        for (auto& q : c.p) CK(hipMalloc(&q, N * 8));
        CK(hipMalloc(&c.dec, (size_t)Wd * Hd * 8));
        CK(hipMemcpy(c.p[0], h0.data(), N * 8, hipMemcpyHostToDevice));
    };
    Chain base, walk;
    alloc(base);
    alloc(walk);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<hipEvent_t> e0(L), e1(L);
    for (int l = 0; l < L; ++l) {
        CK(hipEventCreate(&e0[l]));
        CK(hipEventCreate(&e1[l]));
    }
    auto chain = [&](Chain& c, Launch f, std::vector<double>& ms, int reps) {
        ms.assign(L, 0.0);
        for (int r = 0; r < reps; ++r) {
            for (int l = 0; l < L; ++l) {
                const BlurTaps t = taps_for_radius(radii[l]);
                const bool dec = l == dec_at;
                CK(f(c.p[l], c.p[l + 1], W, H, t, dec ? c.dec : nullptr, dec ? Wd : 0, dec ? Hd : 0,
                     s, e0[l], e1[l]));
            }
            CK(hipStreamSynchronize(s));
            for (int l = 0; l < L; ++l) {
                float m = 0.f;
                CK(hipEventElapsedTime(&m, e0[l], e1[l]));
                ms[l] += m / reps;
            }
        }
    };
    std::vector<double> mb, mw;
    chain(base, run_base, mb, 3);
    chain(walk, run_walk, mw, 3);
    // exactness: every level and the decimated plane
    bool exact = true;
    std::vector<double> a(N), b(N);
    for (int l = 1; l <= L; ++l) {
        CK(hipMemcpy(a.data(), base.p[l], N * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), walk.p[l], N * 8, hipMemcpyDeviceToHost));
        size_t bad = 0, first = N;
        for (size_t i = 0; i < N; ++i)
            if (std::memcmp(&a[i], &b[i], 8)) {
                if (!bad) first = i;
                ++bad;
            }
        if (bad) {
            exact = false;
            std::printf("MISMATCH level %d (R=%d): %zu px, first (%zu, %zu): %.17g vs %.17g\n", l,
                        radii[l - 1], bad, first % W, first / W, a[first], b[first]);
        }
    }
    if (dec_at >= 0 && dec_at < L) {
        const size_t nd = (size_t)Wd * Hd;
        CK(hipMemcpy(a.data(), base.dec, nd * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), walk.dec, nd * 8, hipMemcpyDeviceToHost));
        if (std::memcmp(a.data(), b.data(), nd * 8)) {
            exact = false;
            std::printf("MISMATCH decimated plane\n");
        }
    }
    const int reps = 20;
    chain(base, run_base, mb, reps);
    chain(walk, run_walk, mw, reps);
    chain(base, run_base, mb, reps);  // again, interleaved
    std::vector<double> mb2 = mb;
    chain(walk, run_walk, mw, reps);
    double tb = 0, tw = 0;
    std::printf("%s:%d:%d %dx%d %s\n", g_kind, g_C, g_rows, W, H, exact ? "EXACT" : "NOT EXACT");
    for (int l = 0; l < L; ++l) {
        const double bytes = 16.0 * N + (l == dec_at ? 8.0 * Wd * Hd : 0.0);
        std::printf("  R=%2d base %7.2f us (%5.2f TB/s)  var %7.2f us (%5.2f TB/s)  %+6.1f %%\n",
                    radii[l], mb2[l] * 1e3, bytes / (mb2[l] * 1e-3) / 1e12, mw[l] * 1e3,
                    bytes / (mw[l] * 1e-3) / 1e12, 100.0 * (mw[l] / mb2[l] - 1.0));
        tb += mb2[l];
        tw += mw[l];
    }
    std::printf("  total base %.2f us  var %.2f us  %+.1f %%\n", tb * 1e3, tw * 1e3,
                100.0 * (tw / tb - 1.0));
    return exact ? 0 : 1;
}
