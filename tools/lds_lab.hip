// lds_lab.hip — where k_octaves_lds (the small octaves, one workgroup) spends
// its time: the library kernel timed with events, and its body (octaves_lds_run)
// instantiated with a hook that records s_memtime after each phase. Octaves as a W0 x H0 image's
// pyramid from octave o_first on (intervals 3, sigma 1.6).
//
//   lds_lab W0 H0 o_first o_last [same_level]
//
// Test tooling only: includes the library's kernel translation unit.
#include "../sift-project_amd/csrc/sift_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
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

constexpr int kMaxStamps = 256;

// k_octaves_lds's body (octaves_lds_run) with a stamp after the taps + base
// load, every level and every octave (thread 0, vector store of a VGPR copy)
struct Stamp {
    unsigned long long* stamps;
    int* ns;
    __device__ void operator()() const {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) {
            volatile unsigned long long* p = stamps + *ns;
            *p = t;
        }
        ++*ns;
    }
};

__global__ __launch_bounds__(1024) void k_octaves_lds_stamped(const PyrTable* __restrict__ pt,
                                                              int o_first, int o_last,
                                                              int n_gauss,
                                                              const BlurTaps* __restrict__ taps,
                                                              unsigned long long* stamps,
                                                              unsigned long long* sub_stamps,
                                                              int cap, int dcap) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int ns = 0;
    const Stamp st{stamps, &ns};
    st();
    if (sub_stamps) {
        int ns2 = 0;
        const Stamp sub{sub_stamps, &ns2};
        octaves_lds_run(pt, o_first, o_last, n_gauss, taps, lds, cap, dcap, st, sub);
    } else {
        octaves_lds_run(pt, o_first, o_last, n_gauss, taps, lds, cap, dcap, st);
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s W0 H0 o_first o_last\n", argv[0]);
        return 2;
    }
    const int W0 = std::atoi(argv[1]), H0 = std::atoi(argv[2]);
    const int o_first = std::atoi(argv[3]), o_last = std::atoi(argv[4]);
    // optional: every level with the sigma of level `same` (same code path
    // for all levels: separates per-level instruction fetch from the work)
    const int same = argc > 5 ? std::atoi(argv[5]) : 0;
    const int n_gauss = 6;
    PyrTable h{};
    std::vector<double*> bufs;
    for (int o = 0; o <= o_last; ++o) {
        h.w[o] = W0 >> o;
        h.h[o] = H0 >> o;
        for (int l = 0; l < n_gauss; ++l) {
            if (o < o_first) continue;
            double* p;
            CK(hipMalloc(&p, (size_t)h.w[o] * h.h[o] * 8));
            std::vector<double> v((size_t)h.w[o] * h.h[o]);
            for (size_t i = 0; i < v.size(); ++i) v[i] = 100.0 + 50.0 * std::sin(0.37 * i);
            CK(hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
            h.lvl[o][l] = p;
            bufs.push_back(p);
        }
    }
    h.n_img = 1;
    h.n_oct = o_last + 1;
    // level sigmas of intervals 3 (sift.cpp:143-155): R = ceil(3 sigma)
    std::vector<BlurTaps> taps(n_gauss);
    const double s0 = 1.6, k = std::pow(2.0, 1.0 / 3.0);
    for (int l = 1; l < n_gauss; ++l) {
        const double sg = std::pow(k, (same ? same : l) - 1) * s0 * std::sqrt(k * k - 1);
        BlurTaps& t = taps[l];
        t.R = (int)std::ceil(3 * sg);
        double sw = 0;
        for (int u = 0; u <= t.R; ++u) {
            t.k[u] = std::exp(-(double)(u * u) / (2 * sg * sg));
            sw += u ? 2 * t.k[u] : t.k[u];
        }
        t.sum_w = sw;
        t.inv = 1.0 / sw;
    }
    PyrTable* d_pt;
    BlurTaps* d_taps;
    unsigned long long* d_st;
    CK(hipMalloc(&d_pt, sizeof h));
    CK(hipMalloc(&d_taps, taps.size() * sizeof(BlurTaps)));
    CK(hipMalloc(&d_st, kMaxStamps * 8));
    unsigned long long* d_sub;
    CK(hipMalloc(&d_sub, kMaxStamps * 8));
    CK(hipMemcpy(d_pt, &h, sizeof h, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_taps, taps.data(), taps.size() * sizeof(BlurTaps), hipMemcpyHostToDevice));
    CK(prepare_kernel_attributes());
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_octaves_lds_stamped),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsOctaveBytes));
    const LdsShape sh = lds_shape(h.w[o_first], h.h[o_first], o_first < o_last, n_gauss);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 50;
    for (int i = 0; i < 5; ++i)
        CK(launch_octaves_lds(d_pt, o_first, o_last, n_gauss, d_taps, 1, h.w[o_first],
                              h.h[o_first], 0, nullptr, nullptr));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i)
        CK(launch_octaves_lds(d_pt, o_first, o_last, n_gauss, d_taps, 1, h.w[o_first],
                              h.h[o_first], 0, nullptr, nullptr));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("k_octaves_lds %dx%d octaves %d-%d: %.2f us per launch (back to back)\n", W0, H0,
                o_first, o_last, ms * 1e3 / reps);
    // stamped copy
    std::vector<double> acc(kMaxStamps, 0.0);
    int n = 0;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_octaves_lds_stamped, dim3(1), dim3(1024), sh.bytes, 0, d_pt,
                           o_first, o_last, n_gauss, d_taps, d_st, nullptr, sh.cap, sh.dcap);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> st(kMaxStamps);
        CK(hipMemcpy(st.data(), d_st, kMaxStamps * 8, hipMemcpyDeviceToHost));
        n = 2 + (o_last - o_first + 1) * n_gauss;
        for (int i = 1; i < n; ++i) acc[i] += (double)(st[i] - st[i - 1]) / reps;
    }
    std::printf("stamped (s_memtime cycles, mean of %d): base load %.0f\n", reps, acc[1]);
    int i = 2;
    for (int o = o_first; o <= o_last; ++o) {
        std::printf("  octave %2d (%4dx%-4d):", o, h.w[o], h.h[o]);
        double tot = 0;
        for (int l = 1; l < n_gauss; ++l, ++i) {
            std::printf(" L%d(R%d) %6.0f", l, taps[l].R, acc[i]);
            tot += acc[i];
        }
        std::printf("  octave end %4.0f  sum %7.0f\n", acc[i], tot + acc[i]);
        ++i;
    }
    // phases inside the tiny levels: row pass, barrier, column pass, barrier
    std::vector<double> ph(4 * kMaxStamps, 0.0);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_octaves_lds_stamped, dim3(1), dim3(1024), sh.bytes, 0, d_pt,
                           o_first, o_last, n_gauss, d_taps, d_st, d_sub, sh.cap, sh.dcap);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> st(kMaxStamps), su(kMaxStamps);
        CK(hipMemcpy(st.data(), d_st, kMaxStamps * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(su.data(), d_sub, kMaxStamps * 8, hipMemcpyDeviceToHost));
        int q = 0;
        for (int o = o_first; o <= o_last; ++o) {
            if (h.w[o] * h.h[o] > kLdsTinyPx) continue;
            for (int l = 1; l < n_gauss; ++l, ++q) {
                const int e = 2 + (o - o_first) * n_gauss + (l - 1);
                const double t0 = (double)st[e - 1], t3 = (double)st[e];
                const double a = (double)su[3 * q], b = (double)su[3 * q + 1],
                             c = (double)su[3 * q + 2];
                ph[4 * q] += (a - t0) / reps;
                ph[4 * q + 1] += (b - a) / reps;
                ph[4 * q + 2] += (c - b) / reps;
                ph[4 * q + 3] += (t3 - c) / reps;
            }
        }
    }
    std::printf("tiny levels (cycles): row pass | barrier | column pass | barrier\n");
    int q = 0;
    for (int o = o_first; o <= o_last; ++o) {
        if (h.w[o] * h.h[o] > kLdsTinyPx) continue;
        for (int l = 1; l < n_gauss; ++l, ++q)
            std::printf("  octave %2d L%d (R%2d): %6.0f %6.0f %6.0f %6.0f\n", o, l, taps[l].R,
                        ph[4 * q], ph[4 * q + 1], ph[4 * q + 2], ph[4 * q + 3]);
    }
    for (double* p : bufs) (void)hipFree(p);
    return 0;
}
