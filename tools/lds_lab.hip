// lds_lab.hip — where k_octaves_lds (the small octaves, one workgroup) spends
// its time: the library kernel timed with events, and a stamped copy of its
// octave / level loop (same device functions: lds_level<R>, lds_level_any)
// that records s_memtime after each phase. Octaves as a W0 x H0 image's
// pyramid from octave o_first on (intervals 3, sigma 1.6).
//
//   lds_lab W0 H0 o_first o_last
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

// k_octaves_lds's loop with a stamp after the taps + base load, every level
// and every octave (thread 0, vector store of a VGPR copy)
__global__ __launch_bounds__(1024) void k_octaves_lds_stamped(const PyrTable* __restrict__ pt,
                                                              int o_first, int o_last,
                                                              int n_gauss,
                                                              const BlurTaps* __restrict__ taps,
                                                              unsigned long long* stamps) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int dec_level = n_gauss - 3;
    int ns = 0;
    auto stamp = [&]() {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (tid == 0) {
            volatile unsigned long long* p = stamps + ns;
            *p = t;
        }
        ++ns;
    };
    stamp();
    double* A = lds;
    double* T = lds + kLdsOctavePx;
    double* D = lds + 2 * kLdsOctavePx;
    double* const TP = lds + 2 * kLdsOctavePx + kLdsOctavePx / 4;
    for (int i = tid; i < n_gauss * kLdsTapStride; i += nt) {
        const int l = i / kLdsTapStride, j = i - l * kLdsTapStride;
        const BlurTaps& t = taps[l];
        double v = 0.0;
        if (j <= kMaxTemplR) v = j <= t.R ? t.k[j] : 0.0;
        else v = j == kMaxTemplR + 1 ? t.sum_w : t.inv;
        TP[i] = v;
    }
    {
        const int W = pt->w[o_first], H = pt->h[o_first], P = W | 1;
        const double* g0 = plane(pt, 0, o_first, 0);
        for (int i = tid; i < W * H; i += nt) {
            const int y = i / W;
            A[y * P + (i - y * W)] = g0[i];
        }
    }
    __syncthreads();
    stamp();
    for (int o = o_first; o <= o_last; ++o) {
        const bool has_next = o < o_last;
        LdsLevel L;
        L.A = A;
        L.T = T;
        L.D = D;
        L.W = pt->w[o];
        L.H = pt->h[o];
        L.P = L.W | 1;
        L.Wd = has_next ? pt->w[o + 1] : 0;
        L.Hd = has_next ? pt->h[o + 1] : 0;
        L.Pd = L.Wd | 1;
        L.gd = has_next ? const_cast<double*>(plane(pt, 0, o + 1, 0)) : nullptr;
        const bool tiny = L.W * L.H <= kLdsTinyPx;
        for (int l = 1; l < n_gauss; ++l) {
            L.g = const_cast<double*>(plane(pt, 0, o, l));
            L.dec = has_next && l == dec_level;
            const double* tp = TP + l * kLdsTapStride;
            switch (taps[l].R) {
                case 4: tiny ? lds_level_tiny<4>(L, tp) : lds_level<4>(L, tp); break;
                case 5: tiny ? lds_level_tiny<5>(L, tp) : lds_level<5>(L, tp); break;
                case 6: tiny ? lds_level_tiny<6>(L, tp) : lds_level<6>(L, tp); break;
                case 8: tiny ? lds_level_tiny<8>(L, tp) : lds_level<8>(L, tp); break;
                case 10: tiny ? lds_level_tiny<10>(L, tp) : lds_level<10>(L, tp); break;
                default: lds_level_any(L, taps[l]);
            }
            stamp();
        }
        double* t = A;
        A = D;
        D = t;
        stamp();
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
        const double sg = std::pow(k, l - 1) * s0 * std::sqrt(k * k - 1);
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
    CK(hipMemcpy(d_pt, &h, sizeof h, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_taps, taps.data(), taps.size() * sizeof(BlurTaps), hipMemcpyHostToDevice));
    CK(prepare_kernel_attributes());
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_octaves_lds_stamped),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsOctaveBytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 50;
    for (int i = 0; i < 5; ++i)
        CK(launch_octaves_lds(d_pt, o_first, o_last, n_gauss, d_taps, 1, 0, nullptr, nullptr));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i)
        CK(launch_octaves_lds(d_pt, o_first, o_last, n_gauss, d_taps, 1, 0, nullptr, nullptr));
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
        hipLaunchKernelGGL(k_octaves_lds_stamped, dim3(1), dim3(1024), kLdsOctaveBytes, 0, d_pt,
                           o_first, o_last, n_gauss, d_taps, d_st);
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
    for (double* p : bufs) (void)hipFree(p);
    return 0;
}
