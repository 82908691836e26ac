// tools/blur_variants.hip — design-space microbenchmark for the f64 blur
// kernel (not part of the product). Times variants of the sliding-window
// blur on one level shape, checks every variant against variant 0 bitwise.
//   P = rows prefetched ahead (register queue), C = columns per lane,
//   rows = strip height.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o blur_variants blur_variants.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

struct Taps {
    double k[32];
    double sum_w;
    int R;
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// C columns per lane (lane handles x0 + lane + 64*c), P rows prefetched.
template <int R, int P, int C>
__global__ __launch_bounds__(256) void k_blur_v(const double* __restrict__ src, double* __restrict__ dst,
                                                int W, int H, int rows, Taps taps) {
    constexpr int SEG = 64 * C + 2 * R;
    constexpr int NL = (SEG + 63) / 64;  // staged loads per lane
    __shared__ double sline[4][NL * 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64 * C;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;
    const int y_end = min(y_begin + rows, H);
    double* sl = sline[wv];
    int gx[NL];
    bool has[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
        gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
        has[q] = lane + 64 * q < SEG;
    }
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w;
    double win[C][2 * R + 1];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q <= 2 * R; ++q) win[c][q] = 0.0;
    const int yy0 = y_begin - R, yy_end = y_end + R;
    double pf[P][NL];
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const double* row = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = (has[q] && yy0 + p < yy_end) ? row[gx[q]] : 0.0;
    }
    for (int yb = yy0; yb < yy_end; yb += P) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const int yy = yb + p;
            if (yy < yy_end) {
#pragma unroll
                for (int q = 0; q < NL; ++q)
                    if (has[q]) sl[lane + 64 * q] = pf[p][q];
                const int ny = yy + P;
                if (ny < yy_end) {
                    const double* row = src + (size_t)clampi(ny, 0, H - 1) * W;
#pragma unroll
                    for (int q = 0; q < NL; ++q)
                        if (has[q]) pf[p][q] = row[gx[q]];
                }
                wave_sync();
                double t[C];
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int b = lane + 64 * c + R;
                    double acc = sl[b] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u) acc += k[u] * (sl[b + u] + sl[b - u]);
                    t[c] = acc / sw;
                }
                wave_sync();
#pragma unroll
                for (int c = 0; c < C; ++c) {
#pragma unroll
                    for (int q = 0; q < 2 * R; ++q) win[c][q] = win[c][q + 1];
                    win[c][2 * R] = t[c];
                }
                if (yy >= y_begin + R) {
                    const int y = yy - R;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double o = win[c][R] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u) o += k[u] * (win[c][R + u] + win[c][R - u]);
                        o = o / sw;
                        const int x = x0 + lane + 64 * c;
                        if (x < W) dst[(size_t)y * W + x] = o;
                    }
                }
            }
        }
    }
}


// rotating register window: loop unrolled by NW = 2R+1 rows so every window
// slot index is a compile-time constant (no per-row register moves)
template <int R>
__global__ __launch_bounds__(256) void k_blur_rot(const double* __restrict__ src, double* __restrict__ dst,
                                                  int W, int H, int rows, Taps taps) {
    constexpr int NW = 2 * R + 1;
    constexpr int SEG = 64 + 2 * R;
    __shared__ double sline[4][SEG];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;
    const int y_end = min(y_begin + rows, H);
    double* sl = sline[wv];
    const int x = x0 + lane;
    const int gx0 = clampi(x0 - R + lane, 0, W - 1);
    const bool has1 = lane < 2 * R;
    const int gx1 = clampi(x0 + 64 - R + lane, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w;
    double win[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) win[q] = 0.0;
    const int yy0 = y_begin - R, yy_end = y_end + R;
    const double* srow = src + (size_t)clampi(yy0, 0, H - 1) * W;
    double a0 = srow[gx0];
    double a1 = has1 ? srow[gx1] : 0.0;
    for (int yb = yy0; yb < yy_end; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy < yy_end) {
                sl[lane] = a0;
                if (has1) sl[64 + lane] = a1;
                if (yy + 1 < yy_end) {
                    const double* nrow = src + (size_t)clampi(yy + 1, 0, H - 1) * W;
                    a0 = nrow[gx0];
                    if (has1) a1 = nrow[gx1];
                }
                wave_sync();
                double acc = sl[lane + R] * k[0];
#pragma unroll
                for (int u = 1; u <= R; ++u) acc += k[u] * (sl[lane + R + u] + sl[lane + R - u]);
                win[s] = acc / sw;  // slot s holds source row yy (the newest)
                wave_sync();
                if (yy >= y_begin + R) {
                    // rows yy-2R..yy live in slots s+1..s (mod NW); centre yy-R
                    double o = win[(s + R + 1) % NW] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u)
                        o += k[u] * (win[(s + NW - R + u) % NW] + win[(s + 2 * NW - R - u) % NW]);
                    o = o / sw;
                    if (x < W) dst[(size_t)(yy - R) * W + x] = o;
                }
            }
        }
    }
}

template <int R>
float run_rot(const double* src, double* dst, int W, int H, int rows, const Taps& t, int iters) {
    dim3 grid((W + 63) / 64, ((H + rows - 1) / rows + 3) / 4);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_blur_rot<R>), grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_blur_rot<R>), grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1000.f;
}

template <int R, int P, int C>
float run(const double* src, double* dst, int W, int H, int rows, const Taps& t, int iters) {
    dim3 grid((W + 64 * C - 1) / (64 * C), ((H + rows - 1) / rows + 3) / 4);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_blur_v<R, P, C>), grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_blur_v<R, P, C>), grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1000.f;
}

Taps make_taps(double sigma) {
    Taps t;
    std::memset(&t, 0, sizeof t);
    int ks = (int)std::ceil(3 * sigma) + 1;
    double d = 2 * sigma * sigma, coef = 1 / (std::sqrt(2 * M_PI) * sigma);
    for (int i = 0; i < ks; ++i) t.k[i] = std::exp(-i * i / d) * coef;
    double s = t.k[0];
    for (int u = 1; u < ks; ++u) s += 2.0 * t.k[u];
    t.sum_w = s;
    t.R = ks - 1;
    return t;
}

template <int R>
void sweep(int W, int H, double sigma) {
    Taps t = make_taps(sigma);
    if (t.R != R) {
        std::printf("sigma %g gives R=%d not %d\n", sigma, t.R, R);
        return;
    }
    const size_t n = (size_t)W * H;
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (double)((i * 2654435761u) % 256);
    double *src, *dst, *ref;
    CK(hipMalloc(&src, n * 8));
    CK(hipMalloc(&dst, n * 8));
    CK(hipMalloc(&ref, n * 8));
    CK(hipMemcpy(src, h.data(), n * 8, hipMemcpyHostToDevice));
    std::vector<double> a(n), b(n);
    const double gb = 16.0 * n / 1e9;
    auto check = [&](const char* name, int rows, float us) {
        CK(hipMemcpy(b.data(), dst, n * 8, hipMemcpyDeviceToHost));
        bool ok = std::memcmp(a.data(), b.data(), n * 8) == 0;
        std::printf("  R=%2d %5dx%-5d %-10s rows=%4d %8.1f us %7.0f GB/s %s\n", R, W, H, name, rows, us,
                    gb / (us * 1e-6), ok ? "ok" : "MISMATCH");
    };
    // reference variant
    float us = run<R, 1, 1>(src, dst, W, H, 32, t, 20);
    CK(hipMemcpy(a.data(), dst, n * 8, hipMemcpyDeviceToHost));
    check("P1C1", 32, us);
    int rows_list[] = {4, 8, 16, 24, 32, 48, 64};
    for (int rows : rows_list) {
        if (rows > H) continue;
        check("P1C1", rows, run<R, 1, 1>(src, dst, W, H, rows, t, 20));
        check("ROT", rows, run_rot<R>(src, dst, W, H, rows, t, 20));
    }
    CK(hipFree(src));
    CK(hipFree(dst));
    CK(hipFree(ref));
}

int main() {
    // intervals=3 sigmas: 1.22627 (R=4), 1.54501 (R=5), 1.94659 (R=6), 2.45255 (R=8), 3.09002 (R=10)
    int shapes[][2] = {{3840, 2160}, {1920, 1080}, {960, 540}, {240, 135}, {60, 33}};
    for (auto& s : shapes) {
        sweep<4>(s[0], s[1], 1.22627);
        sweep<6>(s[0], s[1], 1.94659);
        sweep<10>(s[0], s[1], 3.09002);
    }
    return 0;
}
