// flow_lab.hip — k_octaves_flow (the small octaves in flight) against the
// per-level launches on the GPU box: every level and decimated plane
// bit-identical, the band counters complete, the give-up flag clear, and the
// time of both (reference sift.cpp:161-202, image.cpp:156-214).
//
//   flow_lab W0 H0 o_first o_last n_img wgs [reps]
// W0 x H0: octave 0 (planes of octave o are (W0 >> o) x (H0 >> o)); the
// octaves o_first..o_last run in one launch of `wgs` workgroups, level radii
// 4 5 6 8 10 (intervals 3), level 3 decimated into the next octave's base.
//
// Test tooling only: includes the library's kernel translation unit.
#include "../sift-project_amd/csrc/sift_kernels.hip"

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

}  // namespace

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s W0 H0 o_first o_last n_img wgs [reps]\n", argv[0]);
        return 2;
    }
    const int W0 = std::atoi(argv[1]), H0 = std::atoi(argv[2]);
    const int o_first = std::atoi(argv[3]), o_last = std::atoi(argv[4]);
    const int n_img = std::atoi(argv[5]), wgs = std::atoi(argv[6]);
    const int reps = argc > 7 ? std::atoi(argv[7]) : 20;
    const int n_gauss = 6, dec_level = 3;
    const int radii[6] = {0, 4, 5, 6, 8, 10};
    const int n_oct = o_last + 2;  // the last flow octave decimates into one more
    std::vector<BlurTaps> taps(kMaxLevels);
    for (int l = 1; l < n_gauss; ++l) taps[l] = taps_for_radius(radii[l]);
    BlurTaps* d_taps;
    CK(hipMalloc(&d_taps, sizeof(BlurTaps) * kMaxLevels));
    CK(hipMemcpy(d_taps, taps.data(), sizeof(BlurTaps) * kMaxLevels, hipMemcpyHostToDevice));
    // one arena per pyramid copy: octave-major levels, image b img_stride later
    size_t img_stride = 0;
    std::vector<size_t> off(n_oct * n_gauss);
    for (int o = 0; o < n_oct; ++o)
        for (int l = 0; l < n_gauss; ++l) {
            off[o * n_gauss + l] = img_stride;
            img_stride += (size_t)(W0 >> o) * (H0 >> o);
        }
    struct Copy {
        double* arena;
        PyrTable pt;
        PyrTable* d_pt;
    };
    auto make = [&](Copy& c) {
        CK(hipMalloc(&c.arena, img_stride * n_img * 8));
        CK(hipMemset(c.arena, 0, img_stride * n_img * 8));
        std::memset(&c.pt, 0, sizeof c.pt);
        for (int o = 0; o < n_oct; ++o) {
            c.pt.w[o] = W0 >> o;
            c.pt.h[o] = H0 >> o;
            for (int l = 0; l < n_gauss; ++l) c.pt.lvl[o][l] = c.arena + off[o * n_gauss + l];
        }
        c.pt.img_stride = img_stride;
        c.pt.n_img = n_img;
        c.pt.n_oct = n_oct;
        CK(hipMalloc(&c.d_pt, sizeof(PyrTable)));
        CK(hipMemcpy(c.d_pt, &c.pt, sizeof(PyrTable), hipMemcpyHostToDevice));
    };
    Copy base, flow;
    make(base);
    make(flow);
    // octave o_first's base level: a smooth-ish plane with noise, per image
    {
        const int W = W0 >> o_first, H = H0 >> o_first;
        std::vector<double> h0((size_t)W * H);
        uint64_t z = 0x9E3779B97F4A7C15ull;
        for (int b = 0; b < n_img; ++b) {
            for (size_t i = 0; i < h0.size(); ++i) {
                z ^= z << 13;
                z ^= z >> 7;
                z ^= z << 17;
                const double x = (double)(i % W), y = (double)(i / W);
                h0[i] = 128.0 + 60.0 * std::sin(x / 7.0 + b) * std::cos(y / 11.0) +
                        (double)(z >> 40) / (double)(1ull << 24) * 60.0;
            }
            for (Copy* c : {&base, &flow})
                CK(hipMemcpy(c->pt.lvl[o_first][0] + b * img_stride, h0.data(), h0.size() * 8,
                             hipMemcpyHostToDevice));
        }
    }
    // the flow grid as sift_ctx builds it
    FlowGrid fg;
    std::memset(&fg, 0, sizeof fg);
    fg.n_img = n_img;
    fg.err = 1;
    int words = 2;
    for (int o = o_first; o <= o_last; ++o)
        for (int l = 1; l < n_gauss; ++l) {
            FlowGroup& G = fg.g[fg.n_groups];
            G.o = o;
            G.l = l;
            G.W = W0 >> o;
            G.H = H0 >> o;
            G.nbx = (G.W + 63) / 64;
            G.nby = (G.H + 31) / 32;
            G.first = fg.total;
            fg.total += G.nby * n_img * G.nbx;
            G.cnt = words;
            words += n_img * G.nby;
            G.dep = l >= 2 ? fg.n_groups - 1
                           : (o > o_first ? (o - 1 - o_first) * (n_gauss - 1) + dec_level - 1 : -1);
            G.dep_dec = l == 1 && o > o_first;
            G.dec = l == dec_level;
            ++fg.n_groups;
        }
    unsigned* d_ctr;
    CK(hipMalloc(&d_ctr, words * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run_base = [&]() {
        for (int o = o_first; o <= o_last; ++o)
            for (int l = 1; l < n_gauss; ++l) {
                const bool dec = l == dec_level;
                CK(launch_blur(base.pt.lvl[o][l - 1], img_stride, base.pt.lvl[o][l], img_stride,
                               n_img, W0 >> o, H0 >> o, taps[l],
                               dec ? base.pt.lvl[o + 1][0] : nullptr, dec ? W0 >> (o + 1) : 0,
                               dec ? H0 >> (o + 1) : 0, nullptr, s, nullptr, nullptr,
                               (size_t)1 << 21));
            }
    };
    auto run_flow = [&]() {
        CK(hipMemsetAsync(d_ctr, 0, words * 4, s));
        CK(launch_octaves_flow(flow.d_pt, fg, d_taps, d_ctr, wgs, s, nullptr, nullptr));
    };
    std::fprintf(stderr, "base launches\n");
    run_base();
    CK(hipStreamSynchronize(s));
    std::fprintf(stderr, "base done; flow: %d groups %d tasks %d counter words\n", fg.n_groups,
                 fg.total, words);
    run_flow();
    CK(hipStreamSynchronize(s));
    std::fprintf(stderr, "flow done\n");
    // counters: every band complete, no give-up
    std::vector<unsigned> h(words);
    CK(hipMemcpy(h.data(), d_ctr, words * 4, hipMemcpyDeviceToHost));
    bool ok = h[1] == 0 && h[0] >= (unsigned)fg.total;
    if (!ok) std::printf("ticket %u of %d tasks, give-up flag %u\n", h[0], fg.total, h[1]);
    for (int gi = 0; gi < fg.n_groups; ++gi) {
        const FlowGroup& G = fg.g[gi];
        for (int i = 0; i < n_img * G.nby; ++i)
            if (h[G.cnt + i] != (unsigned)G.nbx) {
                if (ok) std::printf("group %d (o %d l %d) band %d: %u of %d tiles\n", gi, G.o, G.l,
                                    i, h[G.cnt + i], G.nbx);
                ok = false;
            }
    }
    // planes: bit-identical
    for (int o = o_first; o <= o_last + 1; ++o)
        for (int l = (o == o_first ? 1 : 0); l < (o <= o_last ? n_gauss : 1); ++l) {
            const size_t n = (size_t)(W0 >> o) * (H0 >> o);
            for (int b = 0; b < n_img; ++b) {
                std::vector<double> a(n), c(n);
                CK(hipMemcpy(a.data(), base.pt.lvl[o][l] + b * img_stride, n * 8,
                             hipMemcpyDeviceToHost));
                CK(hipMemcpy(c.data(), flow.pt.lvl[o][l] + b * img_stride, n * 8,
                             hipMemcpyDeviceToHost));
                if (std::memcmp(a.data(), c.data(), n * 8)) {
                    size_t bad = 0;
                    for (size_t i = 0; i < n; ++i) bad += std::memcmp(&a[i], &c[i], 8) != 0;
                    std::printf("MISMATCH octave %d level %d image %d: %zu of %zu px\n", o, l, b,
                                bad, n);
                    ok = false;
                }
            }
        }
    std::printf("%dx%d octaves %d-%d images %d wgs %d tasks %d: %s\n", W0, H0, o_first, o_last,
                n_img, wgs, fg.total, ok ? "EXACT" : "WRONG");
    if (!ok) return 1;
    // time: per-level launches vs one flow launch (same stream, back to back)
    auto time = [&](auto&& f) {
        CK(hipStreamSynchronize(s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) f();
        CK(hipStreamSynchronize(s));
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                   .count() / reps;
    };
    const double tb = time(run_base), tf = time(run_flow), tb2 = time(run_base),
                 tf2 = time(run_flow);
    std::printf("  per-level launches %.1f / %.1f us, flow %.1f / %.1f us (incl. a counter memset)\n",
                tb, tb2, tf, tf2);
    return 0;
}
