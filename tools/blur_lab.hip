// tools/blur_lab.hip — design-space microbenchmark for the f64 pyramid blur
// (not part of the product). Every variant is checked bit for bit against
// the baseline (the product's rotating-window kernel, k_blur in
// sift_kernels.hip) on the same input; times are medians of 20 launches.
//
// Variants
//   ROT      baseline: wave per 64-column strip, LDS line for the row pass,
//            (2R+1)-deep register window for the column pass, divide by sum_w
//   ROT_FD   same with the correctly rounded division by the constant sum_w
//            done as q = a*inv; r = fma(-q, s, a); q = fma(r, inv, q)
//            (inv = RN(1/s) from the host; Markstein's correction step)
//   ROT_PF   ROT_FD with the source rows prefetched PF rows ahead
//   C2       two adjacent columns per lane (128-column strip), b128 LDS reads
//
// Also: `divcheck` — exhaustive-style random test of the fast division
// against IEEE division for the divisors the pyramid uses.
//
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/blur_lab tools/blur_lab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

struct Taps {
    double k[32];
    double sum_w;
    double inv;
    int R;
};

#ifndef LAB_FENCE
// LDS instructions of one wave execute in issue order in hardware; only the
// compiler must be kept from reordering them (no s_waitcnt is generated)
__device__ __forceinline__ void wave_sync() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
#else
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <bool FD>
__device__ __forceinline__ double divs(double a, double s, double inv) {
    if (!FD) return a / s;
    const double q = a * inv;
    const double r = __builtin_fma(-q, s, a);
    return __builtin_fma(r, inv, q);
}

// ---------------------------------------------------------------- ROT family
template <int R, bool FD, int PF>
__global__ __launch_bounds__(256) void k_rot(const double* __restrict__ src, double* __restrict__ dst,
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
    const double sw = taps.sum_w, inv = taps.inv;
    double win[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) win[q] = 0.0;
    const int yy0 = y_begin - R, yy_end = y_end + R;
    double pa[PF], pb[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
        pa[p] = r[gx0];
        pb[p] = has1 ? r[gx1] : 0.0;
    }
    for (int yb = yy0; yb < yy_end; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy < yy_end) {
                sl[lane] = pa[0];
                if (has1) sl[64 + lane] = pb[0];
#pragma unroll
                for (int p = 0; p + 1 < PF; ++p) {
                    pa[p] = pa[p + 1];
                    pb[p] = pb[p + 1];
                }
                {
                    const int ny = yy + PF;
                    if (ny < yy_end) {
                        const double* r = src + (size_t)clampi(ny, 0, H - 1) * W;
                        pa[PF - 1] = r[gx0];
                        if (has1) pb[PF - 1] = r[gx1];
                    }
                }
                wave_sync();
                double acc = sl[lane + R] * k[0];
#pragma unroll
                for (int u = 1; u <= R; ++u) acc += k[u] * (sl[lane + R + u] + sl[lane + R - u]);
                win[s] = divs<FD>(acc, sw, inv);
                wave_sync();
                if (yy >= y_begin + R) {
                    double o = win[(s + R + 1) % NW] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u)
                        o += k[u] * (win[(s + NW - R + u) % NW] + win[(s + 2 * NW - R - u) % NW]);
                    o = divs<FD>(o, sw, inv);
                    if (x < W) dst[(size_t)(yy - R) * W + x] = o;
                }
            }
        }
    }
}

// ---------------------------------------------------------------- C2: two columns per lane
template <int R, int PF>
__global__ __launch_bounds__(256) void k_c2(const double* __restrict__ src, double* __restrict__ dst,
                                            int W, int H, int rows, Taps taps) {
    constexpr int NW = 2 * R + 1;
    constexpr int SEG = 128 + 2 * R + 2;  // +2: b128 reads of the last pair stay inside
    constexpr int NL = (128 + 2 * R + 63) / 64;
    __shared__ __attribute__((aligned(16))) double sline[4][SEG];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 128;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;
    const int y_end = min(y_begin + rows, H);
    double* sl = sline[wv];
    int gx[NL];
    bool has[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
        gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
        has[q] = lane + 64 * q < 128 + 2 * R;
    }
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    double w0[NW], w1[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) w0[q] = w1[q] = 0.0;
    const int yy0 = y_begin - R, yy_end = y_end + R;
    double pf[PF][NL];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = has[q] ? r[gx[q]] : 0.0;
    }
    const int xa = x0 + 2 * lane;
    for (int yb = yy0; yb < yy_end; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy < yy_end) {
#pragma unroll
                for (int q = 0; q < NL; ++q)
                    if (has[q]) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
                for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
                    for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
                {
                    const int ny = yy + PF;
                    if (ny < yy_end) {
                        const double* r = src + (size_t)clampi(ny, 0, H - 1) * W;
#pragma unroll
                        for (int q = 0; q < NL; ++q)
                            if (has[q]) pf[PF - 1][q] = r[gx[q]];
                    }
                }
                wave_sync();
                // values sl[2*lane .. 2*lane + 2R + 1]
                double v[2 * R + 2];
                const double2* s2 = reinterpret_cast<const double2*>(sl + 2 * lane);
#pragma unroll
                for (int q = 0; q <= R; ++q) {
                    const double2 t = s2[q];
                    v[2 * q] = t.x;
                    v[2 * q + 1] = t.y;
                }
                double a0 = v[R] * k[0], a1 = v[R + 1] * k[0];
#pragma unroll
                for (int u = 1; u <= R; ++u) {
                    a0 += k[u] * (v[R + u] + v[R - u]);
                    a1 += k[u] * (v[R + 1 + u] + v[R + 1 - u]);
                }
                w0[s] = divs<true>(a0, sw, inv);
                w1[s] = divs<true>(a1, sw, inv);
                wave_sync();
                if (yy >= y_begin + R) {
                    double o0 = w0[(s + R + 1) % NW] * k[0];
                    double o1 = w1[(s + R + 1) % NW] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u) {
                        o0 += k[u] * (w0[(s + NW - R + u) % NW] + w0[(s + 2 * NW - R - u) % NW]);
                        o1 += k[u] * (w1[(s + NW - R + u) % NW] + w1[(s + 2 * NW - R - u) % NW]);
                    }
                    o0 = divs<true>(o0, sw, inv);
                    o1 = divs<true>(o1, sw, inv);
                    double* d = dst + (size_t)(yy - R) * W + xa;
                    if (xa + 1 < W) {
                        *reinterpret_cast<double2*>(d) = make_double2(o0, o1);
                    } else if (xa < W) {
                        d[0] = o0;
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------- ROT2 / C2B: branch-free
// Every lane issues every load and store (rows clamped, out-of-image outputs
// redirected to a trash line), strips are NB blocks of NW = 2R+1 rows, and
// the priming rows are peeled, so the waitcnt pass can count precisely
// (no vmcnt(0) per row behind the previous row's store).
template <int R, int PF, int NB>
__global__ __launch_bounds__(256) void k_rot2(const double* __restrict__ src, double* __restrict__ dst,
                                              int W, int H, int rows_unused, Taps taps) {
    constexpr int NW = 2 * R + 1;
    constexpr int ROWS = NB * NW;
    __shared__ double sline[4][128];
    __shared__ double trash[4][64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * 64;
    const int y_begin = (blockIdx.y * 4 + wv) * ROWS;
    if (y_begin >= H) return;
    double* sl = sline[wv];
    const int x = x0 + lane;
    const int gx0 = clampi(x0 - R + lane, 0, W - 1);
    const int gx1 = clampi(x0 + 64 - R + lane, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    double win[NW];
    const int yy0 = y_begin - R;
    double pa[PF], pb[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
        pa[p] = r[gx0];
        pb[p] = r[gx1];
    }
    auto step = [&](const int slot, const int yy, const bool store) __attribute__((always_inline)) {
        sl[lane] = pa[0];
        sl[64 + lane] = pb[0];
#pragma unroll
        for (int p = 0; p + 1 < PF; ++p) {
            pa[p] = pa[p + 1];
            pb[p] = pb[p + 1];
        }
        {
            const double* r = src + (size_t)clampi(yy + PF, 0, H - 1) * W;
            pa[PF - 1] = r[gx0];
            pb[PF - 1] = r[gx1];
        }
        wave_sync();
        double acc = sl[lane + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u) acc += k[u] * (sl[lane + R + u] + sl[lane + R - u]);
        win[slot] = divs<true>(acc, sw, inv);
        asm volatile("" : "+v"(win[slot]));  // materialise the row here (no sinking)
        wave_sync();
        if (store) {
            double o = win[(slot + R + 1) % NW] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u)
                o += k[u] * (win[(slot + NW - R + u) % NW] + win[(slot + 2 * NW - R - u) % NW]);
            o = divs<true>(o, sw, inv);
            const int y = yy - R;
            double* d = (y < H && x < W) ? dst + (size_t)y * W + x : &trash[wv][lane];
            *d = o;
        }
        __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int s = 0; s < 2 * R; ++s) step(s, yy0 + s, false);
    for (int b = 0; b < NB; ++b) {
        const int yb = yy0 + 2 * R + b * NW;
#pragma unroll
        for (int j = 0; j < NW; ++j) step((2 * R + j) % NW, yb + j, true);
    }
}

template <int R, int PF, int NB>
__global__ __launch_bounds__(256) void k_c2b(const double* __restrict__ src, double* __restrict__ dst,
                                             int W, int H, int rows_unused, Taps taps) {
    constexpr int NW = 2 * R + 1;
    constexpr int ROWS = NB * NW;
    constexpr int NL = (128 + 2 * R + 63) / 64;
    __shared__ __attribute__((aligned(16))) double sline[4][64 * NL + 2];
    __shared__ __attribute__((aligned(16))) double trash[4][128];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * 128;
    const int y_begin = (blockIdx.y * 4 + wv) * ROWS;
    if (y_begin >= H) return;
    double* sl = sline[wv];
    int gx[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    double w0[NW], w1[NW];
    const int yy0 = y_begin - R;
    double pf[PF][NL];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = r[gx[q]];
    }
    const int xa = x0 + 2 * lane;
    auto step = [&](const int slot, const int yy, const bool store) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
        for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
            for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
        {
            const double* r = src + (size_t)clampi(yy + PF, 0, H - 1) * W;
#pragma unroll
            for (int q = 0; q < NL; ++q) pf[PF - 1][q] = r[gx[q]];
        }
        wave_sync();
        double v[2 * R + 2];
        const double2* s2 = reinterpret_cast<const double2*>(sl + 2 * lane);
#pragma unroll
        for (int q = 0; q <= R; ++q) {
            const double2 t = s2[q];
            v[2 * q] = t.x;
            v[2 * q + 1] = t.y;
        }
        double a0 = v[R] * k[0], a1 = v[R + 1] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u) {
            a0 += k[u] * (v[R + u] + v[R - u]);
            a1 += k[u] * (v[R + 1 + u] + v[R + 1 - u]);
        }
        w0[slot] = divs<true>(a0, sw, inv);
        w1[slot] = divs<true>(a1, sw, inv);
        asm volatile("" : "+v"(w0[slot]), "+v"(w1[slot]));
        wave_sync();
        if (store) {
            double o0 = w0[(slot + R + 1) % NW] * k[0];
            double o1 = w1[(slot + R + 1) % NW] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u) {
                o0 += k[u] * (w0[(slot + NW - R + u) % NW] + w0[(slot + 2 * NW - R - u) % NW]);
                o1 += k[u] * (w1[(slot + NW - R + u) % NW] + w1[(slot + 2 * NW - R - u) % NW]);
            }
            o0 = divs<true>(o0, sw, inv);
            o1 = divs<true>(o1, sw, inv);
            const int y = yy - R;
            // W even in the lab shapes: a pair is inside or outside as a whole
            double* d = (y < H && xa + 1 < W) ? dst + (size_t)y * W + xa : &trash[wv][2 * lane];
            *reinterpret_cast<double2*>(d) = make_double2(o0, o1);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int s = 0; s < 2 * R; ++s) step(s, yy0 + s, false);
    for (int b = 0; b < NB; ++b) {
        const int yb = yy0 + 2 * R + b * NW;
#pragma unroll
        for (int j = 0; j < NW; ++j) step((2 * R + j) % NW, yb + j, true);
    }
}

// ---------------------------------------------------------------- ROT3: ROT with uniform control flow
template <int R, int PF>
__global__ __launch_bounds__(256) void k_rot3(const double* __restrict__ src, double* __restrict__ dst,
                                              int W, int H, int rows, Taps taps) {
    constexpr int NW = 2 * R + 1;
    __shared__ double sline[4][128];
    __shared__ double trash[4][64];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * 64;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;
    const int y_end = min(y_begin + rows, H);
    double* sl = sline[wv];
    const int x = x0 + lane;
    const int gx0 = clampi(x0 - R + lane, 0, W - 1);
    const int gx1 = clampi(x0 + 64 - R + lane, 0, W - 1);
    double* const tl = &trash[wv][lane];
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    double win[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) win[q] = 0.0;
    const int yy0 = y_begin - R, yy_end = y_end + R;
    double pa[PF], pb[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
        pa[p] = r[gx0];
        pb[p] = r[gx1];
    }
    for (int yb = yy0; yb < yy_end; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy < yy_end) {
                sl[lane] = pa[0];
                sl[64 + lane] = pb[0];
#pragma unroll
                for (int p = 0; p + 1 < PF; ++p) {
                    pa[p] = pa[p + 1];
                    pb[p] = pb[p + 1];
                }
                {
                    const double* r = src + (size_t)clampi(yy + PF, 0, H - 1) * W;
                    pa[PF - 1] = r[gx0];
                    pb[PF - 1] = r[gx1];
                }
                wave_sync();
                double acc = sl[lane + R] * k[0];
#pragma unroll
                for (int u = 1; u <= R; ++u) acc += k[u] * (sl[lane + R + u] + sl[lane + R - u]);
                win[s] = divs<true>(acc, sw, inv);
                wave_sync();
                if (yy >= y_begin + R) {
                    double o = win[(s + R + 1) % NW] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u)
                        o += k[u] * (win[(s + NW - R + u) % NW] + win[(s + 2 * NW - R - u) % NW]);
                    o = divs<true>(o, sw, inv);
                    double* d = (x < W) ? dst + (size_t)(yy - R) * W + x : tl;
                    *d = o;
                }
            }
        }
    }
}

// ---------------------------------------------------------------- IL: interleaved passes
// Step for source row yy computes the row pass of yy AND the column pass of
// output row yy-R-1 (rows yy-2R-1..yy-1, all already in the window): the two
// dependency chains are independent, so their f64 latencies overlap. The
// window is 2R+2 deep. C = adjacent columns per lane (1 or 2).
template <int R, int C, int PF>
__global__ __launch_bounds__(256) void k_il(const double* __restrict__ src, double* __restrict__ dst,
                                            int W, int H, int rows, Taps taps) {
    constexpr int NW = 2 * R + 2;
    constexpr int SPAN = 64 * C;
    constexpr int NL = (SPAN + 2 * R + 63) / 64;
    __shared__ __attribute__((aligned(16))) double sline[4][64 * NL + 2];
    __shared__ __attribute__((aligned(16))) double trash[4][64 * C];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x0 = blockIdx.x * SPAN;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;
    const int y_end = min(y_begin + rows, H);
    double* sl = sline[wv];
    int gx[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    double win[C][NW];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < NW; ++q) win[c][q] = 0.0;
    const int yy0 = y_begin - R, yy_last = y_end + R;  // inclusive: one drain step
    double pf[PF][NL];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const double* r = src + (size_t)clampi(yy0 + p, 0, H - 1) * W;
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = r[gx[q]];
    }
    const int xa = x0 + C * lane;
    for (int yb = yy0; yb <= yy_last; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy <= yy_last) {
#pragma unroll
                for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
                for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
                    for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
                {
                    const double* r = src + (size_t)clampi(yy + PF, 0, H - 1) * W;
#pragma unroll
                    for (int q = 0; q < NL; ++q) pf[PF - 1][q] = r[gx[q]];
                }
                wave_sync();
                // row pass of yy
                double v[C + 2 * R];
                if (C == 2) {
                    const double2* s2 = reinterpret_cast<const double2*>(sl + 2 * lane);
#pragma unroll
                    for (int q = 0; q < (C + 2 * R) / 2; ++q) {
                        const double2 t = s2[q];
                        v[2 * q] = t.x;
                        v[2 * q + 1] = t.y;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < C + 2 * R; ++q) v[q] = sl[lane + q];
                }
                double hn[C];
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    double acc = v[c + R] * k[0];
#pragma unroll
                    for (int u = 1; u <= R; ++u) acc += k[u] * (v[c + R + u] + v[c + R - u]);
                    hn[c] = divs<true>(acc, sw, inv);
                }
                // column pass of output row yy-R-1: rows yy-2R-1..yy-1 sit in
                // slots s+1..s-1 (mod NW); centre yy-R-1 at slot s+R+1
                if (yy >= y_begin + R + 1) {
                    const int y = yy - R - 1;
                    double o[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double a = win[c][(s + R + 1) % NW] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u)
                            a += k[u] * (win[c][(s + R + 1 + u) % NW] + win[c][(s + R + 1 + NW - u) % NW]);
                        o[c] = divs<true>(a, sw, inv);
                    }
                    if (C == 2) {
                        double* d = (xa + 1 < W) ? dst + (size_t)y * W + xa : &trash[wv][2 * lane];
                        *reinterpret_cast<double2*>(d) = make_double2(o[0], o[C - 1]);
                    } else {
                        double* d = (xa < W) ? dst + (size_t)y * W + xa : &trash[wv][lane];
                        *d = o[0];
                    }
                }
#pragma unroll
                for (int c = 0; c < C; ++c) win[c][s] = hn[c];
                wave_sync();
            }
        }
    }
}

// ---------------------------------------------------------------- harness
using KFn = void (*)(const double*, double*, int, int, int, Taps);

float time_kernel(KFn k, dim3 grid, const double* src, double* dst, int W, int H, int rows,
                  const Taps& t, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, src, dst, W, H, rows, t);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
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
    t.inv = 1.0 / s;
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
    uint64_t st = 0x9E3779B97F4A7C15ull ^ n;
    for (size_t i = 0; i < n; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        h[i] = (double)(st >> 11) * 0x1.0p-53 * 255.0;  // full-mantissa values
    }
    double *src, *dst;
    CK(hipMalloc(&src, n * 8));
    CK(hipMalloc(&dst, n * 8));
    CK(hipMemcpy(src, h.data(), n * 8, hipMemcpyHostToDevice));
    std::vector<double> a(n), b(n);
    const double gb = 16.0 * n / 1e9;
    auto report = [&](const char* name, int rows, float us) {
        CK(hipMemcpy(b.data(), dst, n * 8, hipMemcpyDeviceToHost));
        bool ok = std::memcmp(a.data(), b.data(), n * 8) == 0;
        std::printf("  R=%2d %5dx%-5d %-10s rows=%3d %8.2f us %7.0f GB/s %s\n", R, W, H, name, rows,
                    us, gb / (us * 1e-6), ok ? "ok" : "MISMATCH");
        std::fflush(stdout);
    };
    auto grid64 = [&](int rows) { return dim3((W + 63) / 64, ((H + rows - 1) / rows + 3) / 4); };
    auto grid128 = [&](int rows) { return dim3((W + 127) / 128, ((H + rows - 1) / rows + 3) / 4); };
    float us = time_kernel(k_rot<R, false, 1>, grid64(32), src, dst, W, H, 32, t, 20);
    CK(hipMemcpy(a.data(), dst, n * 8, hipMemcpyDeviceToHost));
    report("ROT", 32, us);
    const int rows_list[] = {16, 32};
    for (int rows : rows_list) {
        if (rows > H) continue;
        report("ROT", rows, time_kernel(k_rot<R, false, 1>, grid64(rows), src, dst, W, H, rows, t, 20));
        report("ROT_FD", rows, time_kernel(k_rot<R, true, 1>, grid64(rows), src, dst, W, H, rows, t, 20));
        report("C2_PF1", rows, time_kernel(k_c2<R, 1>, grid128(rows), src, dst, W, H, rows, t, 20));
    }
    auto g64 = [&](int rows) { return dim3((W + 63) / 64, ((H + rows - 1) / rows + 3) / 4); };
    auto g128 = [&](int rows) { return dim3((W + 127) / 128, ((H + rows - 1) / rows + 3) / 4); };
    constexpr int NW = 2 * R + 1;
    for (int rows : {16, 24, 32, 48}) {
        report("IL_C1P1", rows, time_kernel(k_il<R, 1, 1>, g64(rows), src, dst, W, H, rows, t, 20));
        report("IL_C1P2", rows, time_kernel(k_il<R, 1, 2>, g64(rows), src, dst, W, H, rows, t, 20));
        report("IL_C2P1", rows, time_kernel(k_il<R, 2, 1>, g128(rows), src, dst, W, H, rows, t, 20));
        report("IL_C2P2", rows, time_kernel(k_il<R, 2, 2>, g128(rows), src, dst, W, H, rows, t, 20));
    }
    report("ROT3_P1", 32, time_kernel(k_rot3<R, 1>, g64(32), src, dst, W, H, 32, t, 20));
    report("ROT3_P2", 32, time_kernel(k_rot3<R, 2>, g64(32), src, dst, W, H, 32, t, 20));
    report("ROT3_P1", 16, time_kernel(k_rot3<R, 1>, g64(16), src, dst, W, H, 16, t, 20));
    report("ROT3_P2", 16, time_kernel(k_rot3<R, 2>, g64(16), src, dst, W, H, 16, t, 20));
    report("ROT3_P1", 24, time_kernel(k_rot3<R, 1>, g64(24), src, dst, W, H, 24, t, 20));
    report("ROT3_P1", 48, time_kernel(k_rot3<R, 1>, g64(48), src, dst, W, H, 48, t, 20));
    report("ROT2_P1N1", NW, time_kernel(k_rot2<R, 1, 1>, g64(NW), src, dst, W, H, 0, t, 20));
    report("ROT2_P2N1", NW, time_kernel(k_rot2<R, 2, 1>, g64(NW), src, dst, W, H, 0, t, 20));
    report("ROT2_P1N2", 2 * NW, time_kernel(k_rot2<R, 1, 2>, g64(2 * NW), src, dst, W, H, 0, t, 20));
    report("ROT2_P2N2", 2 * NW, time_kernel(k_rot2<R, 2, 2>, g64(2 * NW), src, dst, W, H, 0, t, 20));
    report("ROT2_P1N3", 3 * NW, time_kernel(k_rot2<R, 1, 3>, g64(3 * NW), src, dst, W, H, 0, t, 20));
    report("ROT2_P2N3", 3 * NW, time_kernel(k_rot2<R, 2, 3>, g64(3 * NW), src, dst, W, H, 0, t, 20));
    report("C2B_P1N1", NW, time_kernel(k_c2b<R, 1, 1>, g128(NW), src, dst, W, H, 0, t, 20));
    report("C2B_P2N1", NW, time_kernel(k_c2b<R, 2, 1>, g128(NW), src, dst, W, H, 0, t, 20));
    report("C2B_P1N2", 2 * NW, time_kernel(k_c2b<R, 1, 2>, g128(2 * NW), src, dst, W, H, 0, t, 20));
    report("C2B_P2N2", 2 * NW, time_kernel(k_c2b<R, 2, 2>, g128(2 * NW), src, dst, W, H, 0, t, 20));
    CK(hipFree(src));
    CK(hipFree(dst));
}

// ---------------------------------------------------------------- division check
__global__ void k_divcheck(double s, double inv, uint64_t seed, int per_thread,
                           unsigned long long* bad, double* first_bad) {
    uint64_t st = seed ^ (0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1));
    unsigned nbad = 0;
    for (int i = 0; i < per_thread; ++i) {
        st ^= st >> 12;
        st ^= st << 25;
        st ^= st >> 27;
        const uint64_t r = st * 2685821657736338717ull;
        // random sign-free doubles with exponents spanning [2^-20, 2^12)
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

void divcheck() {
    // the blur normalisers of every sigma the default pyramids use
    // (intervals 2..5, init 1.6, double_image_size) plus the generic taps
    std::vector<double> sig = {1.2489995996796797, 1.2262735, 1.5450077, 1.9465878, 2.4525513,
                               3.0900155, 1.2262735 * 1.5, 2.0, 2.5, 3.5, 4.0, 5.0};
    for (int iv = 1; iv <= 5; ++iv) {
        const double k = std::pow(2.0, 1.0 / iv);
        for (int i = 1; i < iv + 3; ++i)
            sig.push_back(std::pow(k, i - 1) * 1.6 * std::sqrt(k * k - 1));
    }
    unsigned long long* d_bad;
    double* d_first;
    CK(hipMalloc(&d_bad, 8));
    CK(hipMalloc(&d_first, 8));
    for (double sg : sig) {
        const Taps t = make_taps(sg);
        CK(hipMemset(d_bad, 0, 8));
        const int blocks = 4096, per = 4096;
        for (int rep = 0; rep < 16; ++rep)
            hipLaunchKernelGGL(k_divcheck, dim3(blocks), dim3(256), 0, 0, t.sum_w, t.inv,
                               (uint64_t)rep * 7919 + 1, per, d_bad, d_first);
        CK(hipDeviceSynchronize());
        unsigned long long bad;
        double first;
        CK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&first, d_first, 8, hipMemcpyDeviceToHost));
        std::printf("divcheck sigma=%.7f R=%d s=%a inv=%a samples=%.3g mismatches=%llu%s\n", sg,
                    t.R, t.sum_w, t.inv, 16.0 * blocks * 256.0 * per, bad,
                    bad ? " FAIL" : "");
        std::fflush(stdout);
    }
}

int main(int argc, char** argv) {
    const bool only_div = argc > 1 && !std::strcmp(argv[1], "div");
    if (only_div) {
        divcheck();
        return 0;
    }
    const int shapes[][2] = {{3840, 2160}, {1920, 1080}, {960, 540}};
    for (auto& s : shapes) {
        sweep<4>(s[0], s[1], 1.2262735);
        sweep<5>(s[0], s[1], 1.5450077);
        sweep<6>(s[0], s[1], 1.9465878);
        sweep<8>(s[0], s[1], 2.4525513);
        sweep<10>(s[0], s[1], 3.0900155);
    }
    return 0;
}
