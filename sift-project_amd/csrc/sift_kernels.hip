// sift_kernels.hip — hand-written CDNA4 (gfx950) kernels for the SIFT hot
// path of ahmedhassayoune/sift-project (src/sift.cpp:712-776).
//
// Every kernel reproduces the reference's IEEE-754 double arithmetic in the
// reference's evaluation order; the library is built with -ffp-contract=off
// so no multiply-add is fused (contraction breaks the bit-exact
// extremum set). Division and sqrt lower to gfx950's correctly-rounded
// sequences (v_div_scale/fmas/fixup, v_rsq + Newton + residual fixup).
//
// Data layout in HBM: every Gaussian level G[o][l] is a dense row-major f64
// plane of W_o x H_o (idx = y*W_o + x), the reference's Image with channels=1
// (image_io.cpp:81-92). DoG planes are never materialised: D_l = G_{l+1} -
// G_l is one IEEE subtraction, recomputed bit-identically where needed
// (sift.cpp:209-225, image.cpp:30-36).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sift_pow2.h"
#include "sift_device.h"
#include "sift_math64.h"
#include "sift_kernels.h"

// compile-time A/B knobs (alternative builds, SIFT_HIP_LIB)
#ifndef SIFT_BLUR_PF
#define SIFT_BLUR_PF 2  // k_blur: source rows in flight ahead of the staged one
#endif
// wave issue priority (s_setprio) of the pyramid kernels, which share CUs
// with the keypoint kernels' gather-bound waves (of their own job and of the
// jobs in flight beside it): interleaved A/B, 1080p, single-image jobs four
// in flight, priority 1 for all three -3.6 % over 20-step runs and -8.6 %
// steady state; 3 for the LDS octaves and 2 for the tiles -3.5 / -6.3 %;
// 8-image jobs +-1 %
#ifndef SIFT_PRIO_STRIP
#define SIFT_PRIO_STRIP 1
#endif
#ifndef SIFT_PRIO_TILE
#define SIFT_PRIO_TILE 1
#endif
#ifndef SIFT_PRIO_LDS
#define SIFT_PRIO_LDS 1
#endif
#ifndef SIFT_BLUR_BIG_ROWS  // k_blur strip rows / columns per lane on planes >= 4 Mpx (A/B)
#define SIFT_BLUR_BIG_ROWS 32
#endif
#ifndef SIFT_BLUR_BIG_COLS
#define SIFT_BLUR_BIG_COLS 2
#endif
// Gaussian planes >= 4 Mpx: k_blur_pair (1) or the strip walk k_blur (0).
// Pair walk, 2 columns per lane, 32 rows per wave, against the strip walk
// (tools/blur_lab.hip, r05_lab6; every output bit-identical): 3840x2160
// levels R = 4..10 169.0 vs 174.8 us, 8192^2 R = 5..14 1086 vs 1207 us,
// 15360x8640 2349 vs 2507 us (the R = 10 levels -10..-12 %); one column per
// lane 171.0 / 1288 / 2688 us; driver's bench 0.557 vs 0.565 ms per step.
#ifndef SIFT_BLUR_PAIR
#define SIFT_BLUR_PAIR 1
#endif
#ifndef SIFT_BLUR_PAIR_COLS  // k_blur_pair: columns per lane (1 or 2)
#define SIFT_BLUR_PAIR_COLS 2
#endif
#ifndef SIFT_BLUR_PAIR_ROWS  // k_blur_pair: output rows per wave (a pair: twice that)
#define SIFT_BLUR_PAIR_ROWS 32
#endif
// k_blur_pair source rows: staged by LDS-DMA into a ring of this many lines
// per wave (k_blur_pair_dma), or 0: through registers (k_blur_pair) — on
// planes of at least 2^SIFT_BLUR_DMA_PX_LOG2 pixels and radii up to
// SIFT_BLUR_DMA_MAXR. Measured (tools/blur_lab.hip, r06_s1 / r06_s2, every
// plane bit-identical): 4096^2 R = 5 / 7 / 10 -4.8 / -13.8 / -3.8 %, 8192^2
// R = 5 / 7 -5.6 / -11.1 % but R = 10 +5.4 %, 15360x8640 R = 4..8 -3.6..-5.3 %
// but R = 10 +2.9 %, 3840x2160 (1080p's octave 0) +2.7..+6 % (below the
// 2^24-pixel threshold, so 1080p keeps k_blur_pair); ring depth 2 or 8 no
// better than 4. In the pipelined big-config legs (4 jobs in flight, r06_dma2)
// config 5 9.17 / 8.99 vs 9.42 / 9.29 ms per image, config 3 +-0.3 %;
// pyramid alone at 8K -1.6 %, at 4096^2 -4 %. (An earlier A/B, r06_s3, had it
// losing config 5, 10.01 vs 9.66, while the export buffers were mis-sized.)
#ifndef SIFT_BLUR_DMA
#define SIFT_BLUR_DMA 4
#endif
#ifndef SIFT_BLUR_DMA_MAXR
#define SIFT_BLUR_DMA_MAXR 8
#endif
#ifndef SIFT_BLUR_DMA_PX_LOG2
#define SIFT_BLUR_DMA_PX_LOG2 24
#endif
#ifndef SIFT_ORI_AHEAD  // k_orient_wave: steps of 64 samples whose loads are in flight
#define SIFT_ORI_AHEAD 1
#endif

namespace sift_amd {

namespace {

// XCD-aware block remap (bijective): workgroups are dealt round-robin over
// the 8 XCDs, so consecutive block ids land on different L2s. Renumber so
// every XCD owns one contiguous range of logical tiles; neighbouring strips
// (which re-read each other's halo columns / priming rows) then share an L2.
// Placement is a speed hint only; results do not depend on it.
__device__ __forceinline__ void xcd_remap(int& bx, int& by, int& bz) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int n = nx * ny * gridDim.z;
    const int orig = (blockIdx.z * ny + blockIdx.y) * nx + blockIdx.x;
    const int q = n / 8, r = n % 8, xcd = orig % 8;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    bx = id % nx;
    by = (id / nx) % ny;
    bz = id / (nx * ny);
}

// Source of the rows staged by k_blur: a Gaussian plane, or — for the
// initial blur — the reference's initial image computed on the fly from the
// input: convert_to_grayscale (image.cpp:8-24) and, with double_image_size,
// resize_inter_bilinear x2 (image.cpp:62-88); bit-identical to materialising
// it first (same expressions, evaluated once per staged pixel).
// kSrcUpsample: one-channel input, kSrcUpsampleRGB: three channels (the
// raw input ring holds 1 or 3 values per column and row)
enum BlurSrcMode { kSrcPlane = 0, kSrcGray = 1, kSrcUpsample = 2, kSrcUpsampleRGB = 3 };

template <int MODE>
__device__ __forceinline__ double fetch_src(const BlurSource& s, int W, int yy, int gx) {
    if (MODE == kSrcPlane) return s.p[(size_t)yy * W + gx];
    auto gray = [&](int x, int y) -> double {
        const double* q = s.p + ((size_t)y * s.w + x) * s.c;
        if (s.c == 1) return q[0];
        return 0.2126 * q[0] + 0.7152 * q[1] + 0.0722 * q[2];
    };
    if (MODE == kSrcGray) return gray(gx, yy);
    const double fx = gx / 2.0, fy = yy / 2.0;
    const int x0 = (int)fx, y0 = (int)fy;
    const int x1 = min(x0 + 1, s.w - 1), y1 = min(y0 + 1, s.h - 1);
    const double dx = fx - x0, dy = fy - y0;
    const double v0 = gray(x0, y0) * (1 - dx) + gray(x1, y0) * dx;
    const double v1 = gray(x0, y1) * (1 - dx) + gray(x1, y1) * dx;
    return v0 * (1 - dy) + v1 * dy;
}

}  // namespace

// ---------------------------------------------------------------------------
// k_prepare: compute_initial_image minus the blur (sift.cpp:113-122):
// convert_to_grayscale (image.cpp:8-24) then resize_inter_bilinear x2
// (image.cpp:62-88), fused; one thread per output pixel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prepare(const double* __restrict__ in, size_t in_bs,
                                                 int w, int h, int c, int dbl,
                                                 double* __restrict__ out, size_t out_bs,
                                                 int W0, int H0) {
    const int ox = blockIdx.x * blockDim.x + threadIdx.x;
    const int oy = blockIdx.y;
    if (ox >= W0 || oy >= H0) return;
    in += blockIdx.z * in_bs;
    out += blockIdx.z * out_bs;
    auto gray = [&](int x, int y) -> double {
        const double* p = in + ((size_t)y * w + x) * c;
        if (c == 1) return p[0];
        return 0.2126 * p[0] + 0.7152 * p[1] + 0.0722 * p[2];
    };
    if (!dbl) {
        out[(size_t)oy * W0 + ox] = gray(ox, oy);
        return;
    }
    const double fx = ox / 2.0, fy = oy / 2.0;
    const int x0 = (int)fx, y0 = (int)fy;
    const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
    const double dx = fx - x0, dy = fy - y0;
    const double v0 = gray(x0, y0) * (1 - dx) + gray(x1, y0) * dx;
    const double v1 = gray(x0, y1) * (1 - dx) + gray(x1, y1) * dx;
    out[(size_t)oy * W0 + ox] = v0 * (1 - dy) + v1 * dy;
}

// ---------------------------------------------------------------------------
// k_blur<R, C>: apply_gaussian_blur_fast / apply_double_convolution_1d
// (image.cpp:156-238), both passes in one kernel.
//
// One wavefront owns a strip of 64*C columns (C adjacent columns per lane)
// and `rows` output rows, and slides down it one source row per step:
//  * the source row (+R replicate halo each side) is staged in a per-wave
//    LDS line, the next PF rows are already in flight in registers;
//  * row pass of source row yy from LDS (C = 2: b128 reads of column pairs);
//  * in the same step, the column pass of output row yy-R-1 from a
//    (2R+2)-deep register window that does not include row yy — the two
//    f64 dependency chains are independent, so their latencies overlap
//    (measured: 20-30 % over computing the column pass of yy-R after the row
//    pass of yy; tools/blur_lab.hip IL variants);
//  * the window slot of every row is a compile-time constant (the step loop
//    is unrolled by the window depth), so the window never moves.
// Every lane issues every load (rows clamped); out-of-image lanes skip
// their store. Replicate borders: staged columns and
// source rows are clamped, i.e. the reference's min(x+u, W-1) / max(x-u, 0)
// (image.cpp:177-180, 200-203). DECIM also writes resize_inter_nearest
// (image.cpp:41-55) of the output, the next octave's base (sift.cpp:195-196).
// HBM traffic: one read of the source rows (+2R/rows priming overlap, mostly
// L2-served) and one write per output pixel.
// ---------------------------------------------------------------------------
template <int R, int C, bool DECIM, int MODE>
__global__ __launch_bounds__(256) void k_blur(BlurSource src, double* __restrict__ dst,
                                              size_t bs, int W, int H, int rows, BlurTaps taps,
                                              double* __restrict__ dec, int Wd, int Hd) {
    set_job_prio(taps.jp, SIFT_PRIO_STRIP);
    constexpr int PF = SIFT_BLUR_PF;               // rows in flight ahead of the staged one
    constexpr int NW = 2 * R + 2;                  // register window depth
    constexpr int SPAN = 64 * C;                   // strip width
    constexpr int NL = (SPAN + 2 * R + 63) / 64;   // staged loads per lane per row
    __shared__ __attribute__((aligned(16))) double sline[4][64 * NL + 2];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    // image bz of the batched launch
    src.p += bz * src.bstride;
    dst += bz * bs;
    if (DECIM) dec += bz * bs;
    const int x0 = bx * SPAN;
    const int y_begin = (by * 4 + wv) * rows;
    if (y_begin >= H) return;  // whole wave leaves; no block barriers below
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
    constexpr bool UP = MODE == kSrcUpsample || MODE == kSrcUpsampleRGB;
    if (!UP) {
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int ry = clampi(yy0 + p, 0, H - 1);
#pragma unroll
            for (int q = 0; q < NL; ++q) pf[p][q] = fetch_src<MODE>(src, W, ry, gx[q]);
        }
    }
    // kSrcUpsample (resize_inter_bilinear x2 of the gray input, image.cpp:
    // 62-88): staged row ry interpolates input rows y0 = ry/2 and
    // y1 = min(y0 + 1, h - 1) with dy in {0, 0.5}. Instead of 4 gathers per
    // staged pixel, a ring of input rows follows the walk: hx0 / hx1 hold the
    // horizontally interpolated rows y0 and y1 (v0, v1 of the reference), two
    // more rows are in flight as raw input (kUpAhead rows ahead), and each
    // input row is loaded once per strip. Same expressions, same operands:
    // bit-identical to fetch_src<kSrcUpsample>.
    constexpr int kUpAhead = 2;  // raw slots 0, 1
    constexpr int UC = (MODE == kSrcUpsampleRGB) ? 3 : 1;  // raw channel slots
    int ux0[NL], ux1[NL];
    double udx[NL], hx0[NL], hx1[NL], raw[kUpAhead][NL][2 * UC];
    int ci = 0;  // input row of hx0 (hx1: min(ci + 1, h - 1))
    // raw slot a <- input row r (clamped); hx <- gray + horizontal
    // interpolation of raw slot a: v = g0 * (1 - dx) + g1 * dx
#define SIFT_UP_LOAD(r, a)                                                             \
    {                                                                                  \
        const double* row_ = src.p + (size_t)min((r), src.h - 1) * src.w * src.c;    \
        _Pragma("unroll") for (int q = 0; q < NL; ++q) {                               \
            if (UC == 1 || src.c == 1) {                                               \
                raw[a][q][0] = row_[(size_t)ux0[q] * src.c];                           \
                raw[a][q][1] = row_[(size_t)ux1[q] * src.c];                           \
            } else {                                                                   \
                _Pragma("unroll") for (int ch = 0; ch < UC; ++ch) {                    \
                    raw[a][q][2 * ch] = row_[(size_t)ux0[q] * src.c + ch];             \
                    raw[a][q][2 * ch + 1] = row_[(size_t)ux1[q] * src.c + ch];         \
                }                                                                      \
            }                                                                          \
        }                                                                              \
    }
#define SIFT_UP_HX(a, hx)                                                              \
    {                                                                                  \
        _Pragma("unroll") for (int q = 0; q < NL; ++q) {                               \
            double g0 = raw[a][q][0], g1 = raw[a][q][1];                               \
            if (UC == 3 && src.c != 1) {                                               \
                g0 = 0.2126 * raw[a][q][0] + 0.7152 * raw[a][q][2] + 0.0722 * raw[a][q][4]; \
                g1 = 0.2126 * raw[a][q][1] + 0.7152 * raw[a][q][3] + 0.0722 * raw[a][q][5]; \
            }                                                                          \
            hx[q] = g0 * (1 - udx[q]) + g1 * udx[q];                                   \
        }                                                                              \
    }
    if (UP) {
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const double fx = gx[q] / 2.0;
            ux0[q] = (int)fx;
            ux1[q] = min(ux0[q] + 1, src.w - 1);
            udx[q] = fx - ux0[q];
        }
        ci = clampi(yy0, 0, H - 1) >> 1;
        SIFT_UP_LOAD(ci, 0)
        SIFT_UP_HX(0, hx0)
        SIFT_UP_LOAD(ci + 1, 0)
        SIFT_UP_HX(0, hx1)
        SIFT_UP_LOAD(ci + 2, 0)
        SIFT_UP_LOAD(ci + 3, 1)
    }
    const int xa = x0 + C * lane;
    for (int yb = yy0; yb <= yy_last; yb += NW) {
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            const int yy = yb + s;
            if (yy <= yy_last) {
                if (UP) {
                    const int ry = clampi(yy, 0, H - 1);
                    if ((ry >> 1) > ci) {  // advance the ring by one input row
#pragma unroll
                        for (int q = 0; q < NL; ++q) hx0[q] = hx1[q];
                        SIFT_UP_HX(0, hx1)
#pragma unroll
                        for (int q = 0; q < NL; ++q)
#pragma unroll
                            for (int e = 0; e < 2 * UC; ++e) raw[0][q][e] = raw[1][q][e];
                        SIFT_UP_LOAD(ci + 2 + kUpAhead, 1)
                        ++ci;
                    }
                    const double dy = (ry & 1) ? 0.5 : 0.0;  // ry / 2.0 - (int)(ry / 2.0)
#pragma unroll
                    for (int q = 0; q < NL; ++q)
                        sl[lane + 64 * q] = hx0[q] * (1 - dy) + hx1[q] * dy;
                } else {
#pragma unroll
                    for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
                    for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
                        for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
                    const int ry = clampi(yy + PF, 0, H - 1);
#pragma unroll
                    for (int q = 0; q < NL; ++q) pf[PF - 1][q] = fetch_src<MODE>(src, W, ry, gx[q]);
                }
                wave_sync();
                // row pass of source row yy (image.cpp:170-185)
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
                    hn[c] = div_sum_w(acc, sw, inv);
                }
                // column pass of output row yy-R-1 (image.cpp:193-208): rows
                // yy-2R-1..yy-1 sit in slots s+1..s-1 (mod NW), centre at s+R+1
                if (yy >= y_begin + R + 1) {
                    const int y = yy - R - 1;
                    double o[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double a = win[c][(s + R + 1) % NW] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u)
                            a += k[u] * (win[c][(s + R + 1 + u) % NW] +
                                         win[c][(s + R + 1 + NW - u) % NW]);
                        o[c] = div_sum_w(a, sw, inv);
                    }
                    // guarded global store (round 4: an LDS trash line for
                    // the out-of-image lanes made the store FLAT, which counts
                    // in lgkmcnt, so every step's LDS wait also waited for the
                    // store: octave 0 alone -1.3 %, latency -1.5 %, r04_ii)
                    if (xa < W) {
                        if (C == 2)  // W is even for C == 2 (launcher)
                            *reinterpret_cast<double2*>(dst + (size_t)y * W + xa) =
                                make_double2(o[0], o[C - 1]);
                        else
                            dst[(size_t)y * W + xa] = o[0];
                    }
                    if (DECIM && !(y & 1) && (y >> 1) < Hd) {
                        // the even column of the lane: xa for C == 2, x for C == 1
                        if ((C == 2 || !(xa & 1)) && (xa >> 1) < Wd)
                            dec[(size_t)(y >> 1) * Wd + (xa >> 1)] = o[0];
                    }
                }
#pragma unroll
                for (int c = 0; c < C; ++c) win[c][s] = hn[c];
                wave_sync();
            }
        }
    }
}

#undef SIFT_UP_LOAD
#undef SIFT_UP_HX

// ---------------------------------------------------------------------------
// k_blur_pair<R, C, DECIM>: the same level (image.cpp:156-214) for Gaussian
// planes of octave-0 size, walked by PAIRS of wavefronts. A workgroup's four
// waves are two pairs; a pair owns 2*rows output rows of a strip of 64*C
// columns, split at its boundary row b: the down wave produces rows
// [b, b+rows) walking down, the up wave rows [b-rows, b) walking up. Each
// wave first evaluates the row pass of the R source rows on its side of b —
// the first R rows of its own column window and the first R rows of its
// partner's — and hands them over through LDS (one workgroup barrier). A
// wave thus evaluates R + rows row passes for `rows` outputs where the strip
// walk of k_blur evaluates 2R + rows: at R = 10 and 32 rows, 42 instead of
// 52 (the walk's priming of 2R rows, halved).
//
// Walk position p of a wave is source row b - R + p (down) or b - 1 + R - p
// (up); positions [R, 2R) are its own prologue rows, [0, R) its partner's
// (partner position R + j = own position R - 1 - j), position 2R + k is
// staged at walk step k, and step k >= 1 produces the output at position
// R + k - 1 from window positions k - 1 .. k - 1 + 2R while the row pass of
// position 2R + k is in flight (the two dependency chains overlap as in
// k_blur). The PF rows in flight run on from the prologue into the walk.
// The column pass sums the pairs k[u] * (v[+u] + v[-u]), whose IEEE
// addition commutes, so the up wave's outputs are bit-identical to a
// downward walk's; borders replicate by clamping the source row.
// ---------------------------------------------------------------------------
template <int R, int C, bool DECIM>
__global__ __launch_bounds__(256) void k_blur_pair(const double* __restrict__ src, size_t src_bs,
                                                   double* __restrict__ dst, size_t bs, int W,
                                                   int H, int rows, BlurTaps taps,
                                                   double* __restrict__ dec, int Wd, int Hd) {
    set_job_prio(taps.jp, SIFT_PRIO_STRIP);
    constexpr int PF = SIFT_BLUR_PF;
    constexpr int NW = 2 * R + 2;
    constexpr int SPAN = 64 * C;
    constexpr int NL = (SPAN + 2 * R + 63) / 64;
    __shared__ __attribute__((aligned(16))) double sline[4][64 * NL + 2];
    __shared__ __attribute__((aligned(16))) double xch[4][R][SPAN];
    static_assert(sizeof(sline) + sizeof(xch) <= 64 * 1024, "k_blur_pair: static LDS");
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool down = (wv & 1) != 0;
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    if (by * 4 * rows >= H) return;  // the whole workgroup lies below the image
    src += bz * src_bs;
    dst += bz * bs;
    if (DECIM) dec += bz * bs;
    const int x0 = bx * SPAN;
    const int b = (2 * (by * 2 + (wv >> 1)) + 1) * rows;  // the pair's boundary row
    double* const sl = sline[wv];
    int gx[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    // source row of walk position p (clamped: replicate border)
    auto row_at = [&](int p) {
        return clampi(down ? b - R + p : b - 1 + R - p, 0, H - 1);
    };
    double pf[PF][NL];
    auto stage = [&](int p_next) {  // stage pf[0] in the LDS line, fetch position p_next
#pragma unroll
        for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
        for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
            for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
        const int ry = row_at(p_next);
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[PF - 1][q] = src[(size_t)ry * W + gx[q]];
    };
    auto row_pass = [&](double* hn) {  // of the row staged in the LDS line
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
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double acc = v[c + R] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u) acc += k[u] * (v[c + R + u] + v[c + R - u]);
            hn[c] = div_sum_w(acc, sw, inv);
        }
    };
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int ry = row_at(R + p);
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = src[(size_t)ry * W + gx[q]];
    }
    double win[C][NW];
    // prologue: own positions R .. 2R-1 (their rows' horizontal pass), also
    // handed to the partner
#pragma unroll
    for (int j = 0; j < R; ++j) {
        stage(R + j + PF);
        wave_sync();
        double hn[C];
        row_pass(hn);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            win[c][R + j] = hn[c];
            xch[wv][j][C * lane + c] = hn[c];
        }
        wave_sync();
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) win[c][R - 1 - j] = xch[wv ^ 1][j][C * lane + c];
    if (down ? b >= H : b - rows >= H) return;  // no output row of this wave in the image
    const int xa = x0 + C * lane;
    for (int kb = 0; kb <= rows; kb += NW) {
#pragma unroll
        for (int t = 0; t < NW; ++t) {
            const int kk = kb + t;
            if (kk <= rows) {
                // (the last step's row pass is not needed; evaluating it keeps
                // the row pass unconditional, so the compiler interleaves it
                // with the column pass: skipping it cost ~10 %)
                double hn[C];
                stage(2 * R + kk + PF);
                wave_sync();
                row_pass(hn);
                if (kk >= 1) {
                    const int y = down ? b + kk - 1 : b - kk;
                    double o[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double a = win[c][(t + R - 1 + NW) % NW] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u)
                            a += k[u] * (win[c][(t + R - 1 + u) % NW] +
                                         win[c][(t + R - 1 - u + 2 * NW) % NW]);
                        o[c] = div_sum_w(a, sw, inv);
                    }
                    if (y < H && xa < W) {
                        if (C == 2)  // W is even for C == 2 (launcher)
                            *reinterpret_cast<double2*>(dst + (size_t)y * W + xa) =
                                make_double2(o[0], o[C - 1]);
                        else
                            dst[(size_t)y * W + xa] = o[0];
                        if (DECIM && !(y & 1) && (y >> 1) < Hd && (C == 2 || !(xa & 1)) &&
                            (xa >> 1) < Wd)
                            dec[(size_t)(y >> 1) * Wd + (xa >> 1)] = o[0];
                    }
                }
#pragma unroll
                for (int c = 0; c < C; ++c) win[c][(2 * R + t) % NW] = hn[c];
                wave_sync();
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_blur_pair_dma<R, C, DECIM, NB>: k_blur_pair with its source rows staged
// by LDS-DMA (global_load_lds_dword: the loads write LDS directly, no VGPR
// destination). Each wave owns a ring of NB row lines; the row of walk step
// s + NB - 1 is issued into the line step s - 1 consumed, so NB - 1 rows are
// in flight while step s runs, at no VGPR cost (k_blur_pair holds its PF = 2
// rows in flight in registers, 12 VGPRs at C = 2, and stages each through a
// ds_write). A line holds source columns x0 - R .. x0 - R + LW - 1, clamped
// per double (replicate border) — each lane moves one 4-B half of a double,
// so the clamp is exact at both borders. The wait for step s's row is a
// counted vmcnt over the DMA instructions issued after it (loads complete in
// order; the column pass's stores only make the wait stricter). Same walk,
// same per-output arithmetic and order as k_blur_pair: bit-identical planes.
// LDS (dynamic): ring [4 waves][NB][LW] + hand-over [4][R][64 C] doubles.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One global_load_lds_dword: this lane's 4 bytes at `g` land at LDS address
// lds + 4 * lane. Issued as inline asm, so the compiler's wait insertion does
// not see an LDS write in flight (it would put vmcnt(0) before every LDS
// read); the kernels wait with counted vm_wait<N> instead.
__device__ __forceinline__ void dma_dword(const void* g, const double* lds) {
    // M0 (the DMA's LDS base) is compiler-reserved: saved and restored in the
    // same statement; s_nop 0 covers the M0 write -> LDS-DMA hazard
    const unsigned m0 = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) const void*)lds);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(m0)
        : "memory");
}

template <int R, int C>
constexpr int pair_dma_lw() {  // line width in doubles: 32-double DMA pieces
    return (64 * C + 2 * R + 31) / 32 * 32;
}
template <int R, int C, int NB>
constexpr size_t pair_dma_lds_bytes() {
    return ((size_t)4 * NB * pair_dma_lw<R, C>() + (size_t)4 * R * 64 * C) * sizeof(double);
}

template <int R, int C, bool DECIM, int NB>
__global__ __launch_bounds__(256) void k_blur_pair_dma(const double* __restrict__ src,
                                                       size_t src_bs, double* __restrict__ dst,
                                                       size_t bs, int W, int H, int rows,
                                                       BlurTaps taps, double* __restrict__ dec,
                                                       int Wd, int Hd) {
    set_job_prio(taps.jp, SIFT_PRIO_STRIP);
    constexpr int NW = 2 * R + 2;
    constexpr int SPAN = 64 * C;
    constexpr int LW = pair_dma_lw<R, C>();
    constexpr int NI = LW / 32;  // 4-B DMA instructions per row
    static_assert((NB & (NB - 1)) == 0 && NB >= 2, "ring depth: a power of two");
    static_assert(NI * (NB - 1) <= 63, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) double lds_pair[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool down = (wv & 1) != 0;
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    if (by * 4 * rows >= H) return;  // the whole workgroup lies below the image
    src += bz * src_bs;
    dst += bz * bs;
    if (DECIM) dec += bz * bs;
    const int x0 = bx * SPAN;
    const int b = (2 * (by * 2 + (wv >> 1)) + 1) * rows;  // the pair's boundary row
    double* const ring = lds_pair + wv * NB * LW;
    double* const xch = lds_pair + 4 * NB * LW;  // [4][R][SPAN]
    // byte offset, within a source row, of this lane's 4-B piece of DMA
    // instruction q: line double 32 q + lane / 2, half lane & 1
    unsigned gofs[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q)
        gofs[q] = (unsigned)clampi(x0 - R + 32 * q + (lane >> 1), 0, W - 1) * 8u + 4u * (lane & 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    const int last = R + rows;  // walk steps s = 0 .. last stage position R + s
    auto issue = [&](int s) {   // the row of step s (clamped to the last) into its line
        const int p = R + min(s, last);
        const int ry = clampi(down ? b - R + p : b - 1 + R - p, 0, H - 1);
        const char* rp = reinterpret_cast<const char*>(src + (size_t)ry * W);
        double* const line = ring + (s & (NB - 1)) * LW;
        asm volatile("" ::: "memory");  // after the previous reads of that line
#pragma unroll
        for (int q = 0; q < NI; ++q) dma_dword(rp + gofs[q], line + 32 * q);
    };
    auto row_pass = [&](int s, double* hn) {  // of the row of step s
        const double* const sl = ring + (s & (NB - 1)) * LW;
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
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double acc = v[c + R] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u) acc += k[u] * (v[c + R + u] + v[c + R - u]);
            hn[c] = div_sum_w(acc, sw, inv);
        }
    };
#pragma unroll
    for (int s = 0; s + 1 < NB; ++s) issue(s);
    double win[C][NW];
    // prologue: own positions R .. 2R-1 (steps 0 .. R-1), also handed to the partner
#pragma unroll
    for (int j = 0; j < R; ++j) {
        issue(j + NB - 1);
        vm_wait<(NB - 1) * NI>();
        double hn[C];
        row_pass(j, hn);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            win[c][R + j] = hn[c];
            xch[(wv * R + j) * SPAN + C * lane + c] = hn[c];
        }
    }
    // workgroup barrier that leaves the DMAs in flight (__syncthreads would
    // drain them: vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) win[c][R - 1 - j] = xch[((wv ^ 1) * R + j) * SPAN + C * lane + c];
    if (down ? b >= H : b - rows >= H) {  // no output row of this wave in the image
        vm_wait<0>();
        return;
    }
    const int xa = x0 + C * lane;
    for (int kb = 0; kb <= rows; kb += NW) {
#pragma unroll
        for (int t = 0; t < NW; ++t) {
            const int kk = kb + t;
            if (kk <= rows) {
                const int s = R + kk;
                issue(s + NB - 1);
                vm_wait<(NB - 1) * NI>();
                double hn[C];
                row_pass(s, hn);
                if (kk >= 1) {
                    const int y = down ? b + kk - 1 : b - kk;
                    double o[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double a = win[c][(t + R - 1 + NW) % NW] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u)
                            a += k[u] * (win[c][(t + R - 1 + u) % NW] +
                                         win[c][(t + R - 1 - u + 2 * NW) % NW]);
                        o[c] = div_sum_w(a, sw, inv);
                    }
                    if (y < H && xa < W) {
                        if (C == 2)  // W is even for C == 2 (launcher)
                            *reinterpret_cast<double2*>(dst + (size_t)y * W + xa) =
                                make_double2(o[0], o[C - 1]);
                        else
                            dst[(size_t)y * W + xa] = o[0];
                        if (DECIM && !(y & 1) && (y >> 1) < Hd && (C == 2 || !(xa & 1)) &&
                            (xa >> 1) < Wd)
                            dec[(size_t)(y >> 1) * Wd + (xa >> 1)] = o[0];
                    }
                }
#pragma unroll
                for (int c = 0; c < C; ++c) win[c][(2 * R + t) % NW] = hn[c];
            }
        }
    }
    vm_wait<0>();  // the ring's last (unused) rows land before the wave ends
}

// ---------------------------------------------------------------------------
// k_blur_tile<R, DECIM>: the same level (image.cpp:156-214) for planes small
// enough to be cache-resident (octaves >= 1 of a 1080p image), where the
// strip walk of k_blur is latency-bound (2R+1+rows serial steps per wave).
// One workgroup per 64 x 32 output tile: the (32+2R) x (64+2R) source
// region (replicate border by clamping) is staged in LDS with one round of
// loads, the row pass writes (32+2R) x 64 row-pass values to LDS, the column
// pass produces the tile. Each thread evaluates runs of outputs (4 along x in
// the row pass, 8 along y in the column pass) from one register window, so
// an output costs ~(run+2R)/run LDS reads instead of 2R+1. Same arithmetic
// and order as k_blur per output (acc = v*k0, acc += k[u]*(v[+u]+v[-u]),
// Markstein-corrected division by sum_w), hence bit-identical planes. LDS
// row strides are odd in doubles so lane-per-row accesses are conflict-free.
// ---------------------------------------------------------------------------
constexpr int kTileW = 64, kTileH = 32;

// Plane access of a tile: plain, or (SC1, k_octaves_flow) sc1 loads and
// stores — write-through stores and L1-bypassing loads, the hand-off form of
// the flow kernel (MI355X_MICROARCH "Valid forms", row 1)
template <bool SC1>
__device__ __forceinline__ double tile_ld(const double* p) {
    if (SC1) {
        const unsigned long long b =
            __hip_atomic_load((const __attribute__((address_space(1))) unsigned long long*)p,
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return __longlong_as_double((long long)b);
    }
    return *gbl(p);
}
template <bool SC1>
__device__ __forceinline__ void tile_st(double* p, double v) {
    if (SC1)
        __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)p,
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// One 64 x 32 output tile (bx, by) of a level; sin_ holds (32+2R) x
// ((64+2R) | 1) doubles of LDS. Every thread of the 256 takes part.
template <int R, bool DECIM, bool SC1>
__device__ __forceinline__ void blur_tile_body(const double* __restrict__ src,
                                               double* __restrict__ dst, int W, int H,
                                               const BlurTaps& taps, double* __restrict__ dec,
                                               int Wd, int Hd, int bx, int by, double* sin_) {
    constexpr int SH = kTileH + 2 * R;             // staged rows
    constexpr int SWp = (kTileW + 2 * R) | 1;      // staged row stride (odd)
    constexpr int RX = 4, RY = 8;                  // output runs per task
    double* const tmp = sin_;
    constexpr int TS = SWp;  // row-pass row stride (odd)
    const int tid = threadIdx.x;
    const int x0 = bx * kTileW, y0 = by * kTileH;
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    // stage: all loads of a thread in flight before the LDS stores
    {
        constexpr int N = SH * (kTileW + 2 * R);
        constexpr int NIT = (N + 255) / 256;
        double v[NIT];
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int i = tid + 256 * it;
            const int r = i / (kTileW + 2 * R), c = i - r * (kTileW + 2 * R);
            const int gy = clampi(y0 - R + r, 0, H - 1), gx = clampi(x0 - R + c, 0, W - 1);
            v[it] = (i < N) ? tile_ld<SC1>(src + (size_t)gy * W + gx) : 0.0;
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int i = tid + 256 * it;
            const int r = i / (kTileW + 2 * R), c = i - r * (kTileW + 2 * R);
            if (i < N) sin_[r * SWp + c] = v[it];
        }
    }
    __syncthreads();
    // row pass (image.cpp:170-185): task = (row r, columns c0..c0+RX-1);
    // consecutive lanes take consecutive rows
    constexpr int NTASK = SH * (kTileW / RX);
    constexpr int NT = (NTASK + 255) / 256;
    double res[NT][RX];
#pragma unroll
    for (int it = 0; it < NT; ++it) {
        const int t = tid + 256 * it;
        if (t < NTASK) {
            const int r = t % SH, c0 = (t / SH) * RX;
            const double* row = sin_ + r * SWp + c0;
            double v[RX + 2 * R];
#pragma unroll
            for (int j = 0; j < RX + 2 * R; ++j) v[j] = row[j];
#pragma unroll
            for (int j = 0; j < RX; ++j) res[it][j] = v[j + R] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u)
#pragma unroll
                for (int j = 0; j < RX; ++j) res[it][j] += k[u] * (v[j + R + u] + v[j + R - u]);
#pragma unroll
            for (int j = 0; j < RX; ++j) res[it][j] = div_sum_w(res[it][j], sw, inv);
        }
    }
    __syncthreads();  // every staged value has been read
#pragma unroll
    for (int it = 0; it < NT; ++it) {
        const int t = tid + 256 * it;
        if (t < NTASK) {
            const int r = t % SH, c0 = (t / SH) * RX;
#pragma unroll
            for (int j = 0; j < RX; ++j) tmp[r * TS + c0 + j] = res[it][j];
        }
    }
    __syncthreads();
    // column pass (image.cpp:193-208): task = (column c, rows r0..r0+RY-1)
    {
        const int c = tid % kTileW, r0 = (tid / kTileW) * RY;
        double v[RY + 2 * R];
#pragma unroll
        for (int j = 0; j < RY + 2 * R; ++j) v[j] = tmp[(r0 + j) * TS + c];
        double acc[RY];
#pragma unroll
        for (int j = 0; j < RY; ++j) acc[j] = v[j + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
#pragma unroll
            for (int j = 0; j < RY; ++j) acc[j] += k[u] * (v[j + R + u] + v[j + R - u]);
        const int x = x0 + c;
#pragma unroll
        for (int j = 0; j < RY; ++j) {
            const int y = y0 + r0 + j;
            if (x < W && y < H) {
                const double o = div_sum_w(acc[j], sw, inv);
                tile_st<SC1>(dst + (size_t)y * W + x, o);
                if (DECIM && !(x & 1) && !(y & 1) && (x >> 1) < Wd && (y >> 1) < Hd)
                    tile_st<SC1>(dec + (size_t)(y >> 1) * Wd + (x >> 1), o);
            }
        }
    }
}

template <int R, bool DECIM>
__global__ __launch_bounds__(256) void k_blur_tile(const double* __restrict__ src, size_t src_bs,
                                                   double* __restrict__ dst, size_t bs, int W,
                                                   int H, BlurTaps taps,
                                                   double* __restrict__ dec, int Wd, int Hd) {
    set_job_prio(taps.jp, SIFT_PRIO_TILE);
    // one LDS region: the staged source, overwritten in place by the row
    // pass (results held in registers across a barrier), so a tile workgroup
    // takes 23-35 KB instead of 44-62 KB and more of them (and of other jobs'
    // kernels) fit on a CU
    __shared__ double sin_[(kTileH + 2 * R) * ((kTileW + 2 * R) | 1)];
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    if (DECIM) dec += bz * bs;
    blur_tile_body<R, DECIM, false>(src + bz * src_bs, dst + bz * bs, W, H, taps, dec, Wd, Hd, bx,
                                    by, sin_);
}
static_assert(kTileH == 4 * 8, "column pass: 256 threads = 64 columns x 4 runs of 8 rows");

// ---------------------------------------------------------------------------
// k_octaves_flow: the levels of consecutive small octaves (1080p: octaves
// 2/3-5) in ONE launch instead of one launch per level. Levels that small
// are latency-bound (~5 us per dependent launch alone for a few hundred KB,
// and, in a job alone, each launch waits for CU slots behind the keypoint
// chains), so the launch boundaries, not the bytes, set their time.
// Persistent workgroups take 64 x 32 tiles (blur_tile_body, the arithmetic
// of k_blur_tile: bit-identical planes) from a ticket in topological order:
// octave, level, band of 32 rows, image, tile. A tile of level l waits until
// the bands it reads of level l-1 (its own band +-1: R <= 32) — or, for
// level 1, the bands of the previous octave's level `intervals` whose even
// rows the decimated plane holds — have all their tiles; a tile waits only
// on tiles with smaller tickets, held by running workgroups, so the launch
// cannot deadlock. Hand-off (MI355X_MICROARCH "Valid forms", row 1): every
// plane value is stored and loaded sc1 (write-through / L1-bypassing); each
// wave drains its stores (vmcnt 0), the workgroup's barrier, then one lane's
// agent-scope add to the band counter; the consumer's one lane polls the
// counters with sc1 loads, the workgroup's barrier, then the loads. Dynamic
// LDS pads each workgroup above half a CU's LDS: one per CU, the measured
// configuration of that form. Waits are bounded (ctr[fg.err] = 1: never
// expected; the planes are then wrong, never a hang).
// ---------------------------------------------------------------------------
constexpr int kFlowLdsDoubles = (kTileH + 2 * kFlowMaxR) * ((kTileW + 2 * kFlowMaxR) | 1);
#ifndef SIFT_FLOW_PAD_KB
#define SIFT_FLOW_PAD_KB 48
#endif
constexpr size_t kFlowPadBytes = SIFT_FLOW_PAD_KB * 1024;  // static + pad > 80 KB: one workgroup per CU
constexpr unsigned long long kFlowGiveUp = 5000000;  // s_memrealtime ticks (100 MHz): 50 ms

// (not inlined: one body per radius with its own registers; inlined into
// the kernel's radius switch they shared one allocation and spilled)
#ifdef SIFT_FLOW_INLINE
#define SIFT_FLOW_TILE_ATTR __forceinline__
#else
#define SIFT_FLOW_TILE_ATTR __attribute__((noinline))
#endif
template <int R>
__device__ SIFT_FLOW_TILE_ATTR void flow_tile(const double* src, double* dst, int W, int H,
                                          const BlurTaps& taps, double* dec, int Wd, int Hd,
                                          int bx, int by, double* lds) {
    if (dec)
        blur_tile_body<R, true, true>(src, dst, W, H, taps, dec, Wd, Hd, bx, by, lds);
    else
        blur_tile_body<R, false, true>(src, dst, W, H, taps, nullptr, 0, 0, bx, by, lds);
}

__global__ __launch_bounds__(256) void k_octaves_flow(const PyrTable* __restrict__ pt, FlowGrid fg,
                                                      const BlurTaps* __restrict__ taps,
                                                      unsigned* __restrict__ ctr) {
    set_job_prio(pt->jp, SIFT_PRIO_TILE);
    __shared__ __attribute__((aligned(16))) double lds[kFlowLdsDoubles];
    extern __shared__ double flow_pad[];  // occupancy only (never touched)
    __shared__ int s_task;
    typedef __attribute__((address_space(1))) unsigned gu32;
    // Lane 0's work sits in ONE block per task, at its end (publish, then
    // the next ticket), followed by the barrier: with a lane-0 block at the
    // loop head as well, the compiler merged the two across the back edge
    // and the other lanes looped on the same task without a new ticket. The
    // task index is made wave-uniform (readfirstlane), so the exit is a
    // scalar branch.
    if (threadIdx.x == 0) s_task = (int)atomicAdd(&ctr[0], 1u);
    __syncthreads();
    for (;;) {
        const int t = __builtin_amdgcn_readfirstlane(s_task);
        if (t >= fg.total) break;
        int gi = 0;
        while (gi + 1 < fg.n_groups && t >= fg.g[gi + 1].first) ++gi;
        const FlowGroup& G = fg.g[gi];
        const int r = t - G.first;
        const int per_band = fg.n_img * G.nbx;
        const int by = r / per_band, rem = r - by * per_band;
        const int im = rem / G.nbx, bx = rem - im * G.nbx;
        const BlurTaps& tp = taps[G.l];
        const int R = tp.R;
#ifdef SIFT_FLOW_DEBUG
        if (threadIdx.x == 0)
            printf("wg %d task %d group %d (o %d l %d) band %d img %d tile %d R %d dep %d\n",
                   (int)blockIdx.x, t, gi, G.o, G.l, by, im, bx, R, G.dep);
#endif
        if (threadIdx.x == 0 && G.dep >= 0) {
            const FlowGroup& D = fg.g[G.dep];
            int lo, hi;
            if (!G.dep_dec) {  // rows [32 by - R, 32 by + 32 + R) of a same-size plane
                lo = max(by - 1, 0);
                hi = min(by + 1, D.nby - 1);
            } else {  // decimated rows d come from the producer's rows 2 d
                const int d0 = max(kTileH * by - R, 0), d1 = min(kTileH * by + kTileH - 1 + R, G.H - 1);
                lo = min(2 * d0 / kTileH, D.nby - 1);
                hi = min(2 * d1 / kTileH, D.nby - 1);
            }
            const unsigned need = (unsigned)D.nbx;
            const unsigned long long t_give_up = __builtin_amdgcn_s_memrealtime() + kFlowGiveUp;
            for (int b2 = lo; b2 <= hi; ++b2) {
                gu32* c = (gu32*)&ctr[D.cnt + im * D.nby + b2];
                while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() > t_give_up) {  // flag it, go on
                        __hip_atomic_store((gu32*)&ctr[fg.err], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
        }
        __syncthreads();
        const double* src = plane(pt, im, G.o, G.l - 1);
        double* dst = pt->lvl[G.o][G.l] + (size_t)im * pt->img_stride;
        double* dec = G.dec ? pt->lvl[G.o + 1][0] + (size_t)im * pt->img_stride : nullptr;
        const int Wd = G.dec ? pt->w[G.o + 1] : 0, Hd = G.dec ? pt->h[G.o + 1] : 0;
        switch (R) {
#define SIFT_FLOW_R(RR)                                                            \
    case RR:                                                                       \
        flow_tile<RR>(src, dst, G.W, G.H, tp, dec, Wd, Hd, bx, by, lds);           \
        break;
            SIFT_FLOW_R(1) SIFT_FLOW_R(2) SIFT_FLOW_R(3) SIFT_FLOW_R(4) SIFT_FLOW_R(5)
            SIFT_FLOW_R(6) SIFT_FLOW_R(7) SIFT_FLOW_R(8) SIFT_FLOW_R(9) SIFT_FLOW_R(10)
            SIFT_FLOW_R(11) SIFT_FLOW_R(12)
#undef SIFT_FLOW_R
            default:
                break;  // the host never builds such a group (kFlowMaxR)
        }
        // publish: this wave's sc1 stores have completed, every wave's
        // (barrier), then one add for the workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add((gu32*)&ctr[G.cnt + im * G.nby + by], 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#ifdef SIFT_FLOW_DEBUG
            printf("wg %d task %d done: ctr[%d] = %u\n", (int)blockIdx.x, t,
                   G.cnt + im * G.nby + by, ctr[G.cnt + im * G.nby + by]);
#endif
            s_task = (int)atomicAdd(&ctr[0], 1u);
        }
        __syncthreads();
    }
    (void)flow_pad;
}

hipError_t launch_octaves_flow(const PyrTable* d_pt, const FlowGrid& fg, const BlurTaps* d_taps,
                               unsigned* ctr, int wgs, hipStream_t s, hipEvent_t e0,
                               hipEvent_t e1) {
    static bool attr = false;  // (benign race: idempotent)
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&k_octaves_flow),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFlowPadBytes);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int n = std::max(1, std::min(wgs, fg.total));
    return launch_timed(k_octaves_flow, dim3(n), dim3(256), kFlowPadBytes, s, e0, e1, d_pt, fg,
                        d_taps, ctr);
}

// ---------------------------------------------------------------------------
// k_octaves_lds: every remaining small octave (W*H <= kLdsOctavePx) in ONE
// launch of ONE workgroup. A level and the horizontal-pass temporary both
// live in LDS, so each level is two barrier-separated LDS sweeps instead of
// a latency-bound launch; each finished level is streamed to its global
// plane (needed later by extrema/orientation/descriptor), and the decimated
// level `intervals` becomes the next octave's base in LDS. Same arithmetic
// and order as k_blur (image.cpp:156-214), replicate borders by clamping.
// Every level's taps, sum_w and 1/sum_w are staged in LDS once at the start
// (a level used to load them from global memory inside its loops: a fixed
// ~3,500-cycle cost per level that dominated the tiny octaves; stamped
// copy in tools/lds_lab.hip, round 5); the radius is a template parameter,
// so the taps of a level sit in registers.
// ---------------------------------------------------------------------------
struct LdsLevel {
    double* A;  // current level (in: previous level, out: this level), row stride P
    double* T;  // horizontal-pass temporary, row stride P
    double* D;  // next octave base (when dec), row stride Pd
    double* g;  // global plane of this level (row stride W)
    double* gd; // global plane of the next octave's base (when dec, row stride Wd)
    int W, H, Wd, Hd, P, Pd;
    bool dec;
};

// A level's output pixel: the plane in LDS and in global memory, and the
// next octave's base (resize_inter_nearest, image.cpp:41-55) when due.
// (global-address-space stores: generic ones are FLAT stores, which count in
// lgkmcnt as well, so later LDS waits of the wave would also wait for them)
__device__ __forceinline__ void lds_put(const LdsLevel& L, int x, int y, double o) {
    L.A[y * L.P + x] = o;
    gbl_w(L.g)[y * L.W + x] = o;
    if (L.dec && !(x & 1) && !(y & 1) && (x >> 1) < L.Wd && (y >> 1) < L.Hd) {
        L.D[(y >> 1) * L.Pd + (x >> 1)] = o;
        gbl_w(L.gd)[(y >> 1) * L.Wd + (x >> 1)] = o;
    }
}

// Levels of more than kLdsTinyPx pixels: every thread takes runs of kLdsRun
// consecutive outputs (along x in the row pass, along y in the column pass),
// loads the run plus its 2R halo once from LDS and evaluates the kLdsRun
// independent dependency chains interleaved. Row-pass tasks go lane-per-row
// and the odd stride P keeps those lanes on different banks. Runs of 4 (not
// 8) put twice the waves on the level's FP64 work.
constexpr int kLdsRun = 4;
#ifndef SIFT_LDS_TINY_PX
#define SIFT_LDS_TINY_PX 600
#endif
constexpr int kLdsTinyPx = SIFT_LDS_TINY_PX;
// threads of k_octaves_lds: with ~120 VGPRs a wave, 1024 threads (4 waves
// per SIMD) take a CU's whole register file, so the launch waited at
// dispatch for a CU with no other wave resident (~25 us beside a job's
// keypoint chains); 512 take half of it: 34 -> 36 us alone, synchronous
// latency -1.2 %, pipelined step +-0 (r05_l512)
#ifndef SIFT_LDS_THREADS
#define SIFT_LDS_THREADS 512
#endif

template <int R>
__device__ void lds_level(const LdsLevel& L, const double* __restrict__ tp) {
    constexpr int NV = kLdsRun + 2 * R;
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = tp[u];
    const double sw = tp[kMaxTemplR + 1], inv = tp[kMaxTemplR + 2];
    const int W = L.W, H = L.H, P = L.P;
    // row pass (image.cpp:170-185): task = (row y, run of columns from x0)
    const int rx = (W + kLdsRun - 1) / kLdsRun;
    for (int task = threadIdx.x; task < H * rx; task += blockDim.x) {
        const int x0 = (task / H) * kLdsRun;
        const int y = task - (x0 / kLdsRun) * H;
        const double* row = L.A + y * P;
        double v[NV];
        if (x0 >= R && x0 + kLdsRun + R <= W) {  // interior run: no clamping
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = row[x0 - R + i];
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = row[clampi(x0 - R + i, 0, W - 1)];
        }
        double acc[kLdsRun];
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j) acc[j] = v[j + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
#pragma unroll
            for (int j = 0; j < kLdsRun; ++j) acc[j] += k[u] * (v[j + R + u] + v[j + R - u]);
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j)
            if (x0 + j < W) L.T[y * P + x0 + j] = div_sum_w(acc[j], sw, inv);
    }
    __syncthreads();
    // column pass (image.cpp:193-208): task = (column x, run of rows from y0);
    // consecutive threads take consecutive columns (conflict-free LDS reads)
    const int ry = (H + kLdsRun - 1) / kLdsRun;
    for (int task = threadIdx.x; task < W * ry; task += blockDim.x) {
        const int yr = task / W;
        const int x = task - yr * W;
        const int y0 = yr * kLdsRun;
        double v[NV];
        if (y0 >= R && y0 + kLdsRun + R <= H) {  // interior run: no clamping
            const double* col = L.T + (y0 - R) * P + x;
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = col[i * P];
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = L.T[clampi(y0 - R + i, 0, H - 1) * P + x];
        }
        double acc[kLdsRun];
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j) acc[j] = v[j + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
#pragma unroll
            for (int j = 0; j < kLdsRun; ++j) acc[j] += k[u] * (v[j + R + u] + v[j + R - u]);
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j)
            if (y0 + j < H) lds_put(L, x, y0 + j, div_sum_w(acc[j], sw, inv));
    }
    __syncthreads();
}

// diagnostics hook of the LDS-octave kernel: called at phase boundaries (a
// no-op here; tools/lds_lab.hip stamps s_memtime there)
struct LdsNoHook {
    __device__ void operator()() const {}
};

// Levels of at most kLdsTinyPx pixels (1080p: 30x16 and below): one output
// per thread, a pass is a single short task per thread
template <int R, class Hook = LdsNoHook>
__device__ void lds_level_tiny(const LdsLevel& L, const double* __restrict__ tp,
                               Hook sub = Hook{}) {
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = tp[u];
    const double sw = tp[kMaxTemplR + 1], inv = tp[kMaxTemplR + 2];
    const int W = L.W, H = L.H, P = L.P;
    for (int i = threadIdx.x; i < W * H; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        const double* row = L.A + y * P;
        double acc = row[x] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u) acc += k[u] * (row[min(x + u, W - 1)] + row[max(x - u, 0)]);
        L.T[y * P + x] = div_sum_w(acc, sw, inv);
    }
    sub();
    __syncthreads();
    sub();
    for (int i = threadIdx.x; i < W * H; i += blockDim.x) {
        const int y = i / W, x = i - y * W;
        double acc = L.T[y * P + x] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
            acc += k[u] * (L.T[min(y + u, H - 1) * P + x] + L.T[max(y - u, 0) * P + x]);
        lds_put(L, x, y, div_sum_w(acc, sw, inv));
    }
    sub();
    __syncthreads();
}

// kernels wider than kMaxTemplR (unusual sigmas): runtime radius, taps and
// IEEE division from the global table
__device__ void lds_level_any(const LdsLevel& L, const BlurTaps& t) {
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int W = L.W, H = L.H, R = t.R, P = L.P;
    for (int y = ty; y < H; y += nw) {
        const double* row = L.A + y * P;
        for (int x = tx; x < W; x += 64) {
            double acc = row[x] * t.k[0];
            for (int u = 1; u <= R; ++u) acc += t.k[u] * (row[min(x + u, W - 1)] + row[max(x - u, 0)]);
            L.T[y * P + x] = acc / t.sum_w;
        }
    }
    __syncthreads();
    for (int y = ty; y < H; y += nw) {
        for (int x = tx; x < W; x += 64) {
            double acc = L.T[y * P + x] * t.k[0];
            for (int u = 1; u <= R; ++u)
                acc += t.k[u] * (L.T[min(y + u, H - 1) * P + x] + L.T[max(y - u, 0) * P + x]);
            lds_put(L, x, y, acc / t.sum_w);
        }
    }
    __syncthreads();
}

// per-lane tables of the launch (every wave holds them; v_readlane gives a
// level's values with no memory access in the level loop)
struct LdsTables {
    // lane i + 64 j of pl<j>: plane (octave o_first + (i + 64 j) / n_gauss,
    // level (i + 64 j) % n_gauss)
    const double *pl0, *pl1, *pl2;
    int w, h;  // lane i: dims of octave o_first + i
    int r;     // lane l: radius of level l
    __device__ const double* plane_of(int idx) const {
        const int j = idx >> 6, i = idx & 63;
        return readlane_ptr(j == 0 ? pl0 : (j == 1 ? pl1 : pl2), i);
    }
};

// the kernel's body; `hook()` runs after the base load, every level and
// every octave, `sub()` inside the tiny levels (no-ops here; tools/
// lds_lab.hip stamps s_memtime there)
// `cap` / `dcap`: doubles of the level regions (the first octave's level,
// (W | 1) * H) and of the next-base region ((W / 2 | 1) * (H / 2)), so the
// launch takes only the LDS its octaves need (1080p octaves 6-10: 37 KB) and
// shares a CU with other workgroups instead of waiting for a whole CU's LDS
// to drain (a job alone: up to ~35 us at dispatch beside its keypoint
// chains, r05_s kernel trace)
template <class Hook, class Sub = LdsNoHook>
__device__ __forceinline__ void octaves_lds_run(const PyrTable* __restrict__ pt, int o_first,
                                                int o_last, int n_gauss,
                                                const BlurTaps* __restrict__ taps, double* lds,
                                                int cap, int dcap, Hook hook, Sub sub = Sub{}) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    const int dec_level = n_gauss - 3;
    const int b = blockIdx.x;                           // image of the job
    const int n_oct = o_last - o_first + 1;             // <= kMaxOctaves
    LdsTables tb;
    auto entry = [&](int i) -> const double* {
        return i < n_oct * n_gauss ? plane(pt, b, o_first + i / n_gauss, i % n_gauss) : nullptr;
    };
    tb.pl0 = entry(lane);
    tb.pl1 = entry(lane + 64);
    tb.pl2 = entry(lane + 128);
    tb.w = lane < n_oct ? pt->w[o_first + lane] : 0;
    tb.h = lane < n_oct ? pt->h[o_first + lane] : 0;
    tb.r = lane < n_gauss ? taps[lane].R : 0;
    // the level's plane lives in the large region A, the next octave's base
    // in the quarter region D; the roles swap from octave to octave (the
    // next octave's levels fit in the quarter region), so no copy
    double* A = lds;                                    // current level
    double* T = lds + cap;                              // horizontal-pass temporary
    double* D = lds + 2 * cap;                          // next octave's base
    double* const TP = lds + 2 * cap + dcap;            // staged taps
    for (int i = tid; i < n_gauss * kLdsTapStride; i += nt) {
        const int l = i / kLdsTapStride, j = i - l * kLdsTapStride;
        const BlurTaps& t = taps[l];
        double v = 0.0;
        if (j <= kMaxTemplR) v = j <= t.R ? t.k[j] : 0.0;
        else v = j == kMaxTemplR + 1 ? t.sum_w : t.inv;
        TP[i] = v;
    }
    {
        const int W = readlane_i32(tb.w, 0), H = readlane_i32(tb.h, 0), P = W | 1;
        gdouble* g0 = gbl(tb.plane_of(0));
        for (int i = tid; i < W * H; i += nt) {
            const int y = i / W;
            A[y * P + (i - y * W)] = g0[i];
        }
    }
    __syncthreads();
    hook();
    for (int o = o_first; o <= o_last; ++o) {
        const int oi = o - o_first;
        const bool has_next = o < o_last;
        LdsLevel L;
        L.A = A;
        L.T = T;
        L.D = D;
        L.W = readlane_i32(tb.w, oi);
        L.H = readlane_i32(tb.h, oi);
        L.P = L.W | 1;
        L.Wd = has_next ? readlane_i32(tb.w, oi + 1) : 0;
        L.Hd = has_next ? readlane_i32(tb.h, oi + 1) : 0;
        L.Pd = L.Wd | 1;
        L.gd = has_next ? const_cast<double*>(tb.plane_of((oi + 1) * n_gauss)) : nullptr;
        const bool tiny = L.W * L.H <= kLdsTinyPx;
        for (int l = 1; l < n_gauss; ++l) {
            L.g = const_cast<double*>(tb.plane_of(oi * n_gauss + l));
            L.dec = has_next && l == dec_level;
            const double* tp = TP + l * kLdsTapStride;
            switch (readlane_i32(tb.r, l)) {
#define SIFT_LDS_CASE(RR)                                      \
    case RR:                                                   \
        if (tiny) lds_level_tiny<RR>(L, tp, sub);              \
        else lds_level<RR>(L, tp);                             \
        break;
                SIFT_LDS_CASE(1) SIFT_LDS_CASE(2) SIFT_LDS_CASE(3) SIFT_LDS_CASE(4)
                SIFT_LDS_CASE(5) SIFT_LDS_CASE(6) SIFT_LDS_CASE(7) SIFT_LDS_CASE(8)
                SIFT_LDS_CASE(9) SIFT_LDS_CASE(10) SIFT_LDS_CASE(11) SIFT_LDS_CASE(12)
#undef SIFT_LDS_CASE
                default:  // R > 12 (intervals <= 2, larger sigmas): templated
                          // radii beyond 12 would push the kernel past 128
                          // VGPRs into scratch
                    lds_level_any(L, taps[l]);
            }
            hook();
        }
        // the next octave's base (row stride Pd) becomes the current level
        double* t = A;
        A = D;
        D = t;
        hook();
    }
}

__global__ __launch_bounds__(SIFT_LDS_THREADS) void k_octaves_lds(const PyrTable* __restrict__ pt,
                                                      int o_first, int o_last, int n_gauss,
                                                      const BlurTaps* __restrict__ taps, int cap,
                                                      int dcap) {
    set_job_prio(pt->jp, SIFT_PRIO_LDS);
    extern __shared__ __attribute__((aligned(16))) double lds[];
    octaves_lds_run(pt, o_first, o_last, n_gauss, taps, lds, cap, dcap, LdsNoHook{});
}

// ---------------------------------------------------------------------------
// k_octave_fused: levels [l_first, l_last] of ONE mid-sized octave (1080p:
// 960x540 down to 120x67) in one launch, tiled with recomputed halos,
// instead of one launch per level (the levels of these octaves are a few
// microseconds of work each, so per-level launches run at the
// dependent-launch floor, ~5 us: VERDICT r05 "small octaves"). The job
// launches an octave as two groups like its per-level launches: the
// decimation chain (levels 1 .. intervals) and the tail (the two levels
// after it, on the second pyramid stream), so each group's halo is only its
// own levels' radii. Workgroup = (tile of tw x th output pixels, image).
// Level l of the tile is evaluated over its core grown by
// halo[l] = R_{l+1} + ... + R_{l_last} (clipped to the image), exactly what
// the group's later levels of the tile read, so a tile never needs another
// workgroup's pixels: the base level's region comes in from global memory
// once, then each level is a row pass into LDS and a column pass back into
// the level buffer, two barriers, no global round trip. Each level's core
// goes to its global plane (extrema, orientation and descriptor read them)
// and the decimated level `intervals` to the next octave's base. Per output
// pixel the arithmetic and its order are k_blur's (image.cpp:156-214):
// replicate borders by clamping to the image, never to the tile, and a
// pixel of a halo is computed from the same clamped inputs as in its own
// tile, so every plane is bit-identical to the per-level launches.
// ---------------------------------------------------------------------------
template <int R>
__device__ void fused_level(const double* __restrict__ tp, double* S, double* T,
                            const FusedOctave& f, int ax, int ay, int aw, int ah, int bx, int by,
                            int bw, int bh, int cx0, int cy0, int cx1, int cy1,
                            double* __restrict__ g, double* __restrict__ gd) {
    constexpr int NV = kLdsRun + 2 * R;
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = tp[u];
    const double sw = tp[kMaxTemplR + 1], inv = tp[kMaxTemplR + 2];
    const int W = f.W, H = f.H;
    const int Pa = aw | 1, PT = bw | 1;
    // row pass of every source row (the column pass needs rows
    // [by - R, by + bh + R) clipped = the source region's rows) over the
    // level region's columns: task = (row, run of kLdsRun columns),
    // lane-per-row (odd stride)
    const int rx = (bw + kLdsRun - 1) / kLdsRun;
    for (int task = threadIdx.x; task < ah * rx; task += blockDim.x) {
        const int xr = task / ah;
        const int yy = task - xr * ah;
        const int x0 = bx + xr * kLdsRun;  // image column of the run
        const double* row = S + yy * Pa;
        double v[NV];
        if (x0 >= R && x0 + kLdsRun + R <= W) {  // no clamping: inside the region
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = row[x0 - R - ax + i];
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = row[clampi(x0 - R + i, 0, W - 1) - ax];
        }
        double acc[kLdsRun];
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j) acc[j] = v[j + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
#pragma unroll
            for (int j = 0; j < kLdsRun; ++j) acc[j] += k[u] * (v[j + R + u] + v[j + R - u]);
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j)
            if (xr * kLdsRun + j < bw) T[yy * PT + xr * kLdsRun + j] = div_sum_w(acc[j], sw, inv);
    }
    __syncthreads();
    // column pass into the level buffer (now the level region, stride
    // bw | 1) and the core to global memory: task = (column, run of rows),
    // consecutive threads on consecutive columns
    const int Pb = bw | 1;
    const int ry = (bh + kLdsRun - 1) / kLdsRun;
    gdouble_w* gw = gbl_w(g);
    for (int task = threadIdx.x; task < bw * ry; task += blockDim.x) {
        const int yr = task / bw;
        const int xx = task - yr * bw;
        const int y0 = by + yr * kLdsRun;  // image row of the run
        double v[NV];
        if (y0 >= R && y0 + kLdsRun + R <= H) {
            const double* col = T + (y0 - R - ay) * PT + xx;
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = col[i * PT];
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) v[i] = T[(clampi(y0 - R + i, 0, H - 1) - ay) * PT + xx];
        }
        double acc[kLdsRun];
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j) acc[j] = v[j + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u)
#pragma unroll
            for (int j = 0; j < kLdsRun; ++j) acc[j] += k[u] * (v[j + R + u] + v[j + R - u]);
        const int x = bx + xx;
        const bool core_x = x >= cx0 && x < cx1;
#pragma unroll
        for (int j = 0; j < kLdsRun; ++j) {
            if (yr * kLdsRun + j >= bh) break;
            const int y = y0 + j;
            const double o = div_sum_w(acc[j], sw, inv);
            S[(y - by) * Pb + xx] = o;
            if (core_x && y >= cy0 && y < cy1) {
                gw[(size_t)y * W + x] = o;
                if (gd && !(x & 1) && !(y & 1) && (x >> 1) < f.Wd && (y >> 1) < f.Hd)
                    gbl_w(gd)[(size_t)(y >> 1) * f.Wd + (x >> 1)] = o;
            }
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(1024) void k_octave_fused(const PyrTable* __restrict__ pt,
                                                       FusedOctave f,
                                                       const BlurTaps* __restrict__ taps) {
    set_job_prio(pt->jp, SIFT_PRIO_TILE);
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* const S = lds;                    // level region (row stride width | 1)
    double* const T = lds + f.capS;           // row-pass temporary
    double* const TP = lds + f.capS + f.capT; // staged taps
    const int b = blockIdx.y;
    const int tx = blockIdx.x % f.ntx, ty = blockIdx.x / f.ntx;
    const int cx0 = tx * f.tw, cy0 = ty * f.th;
    const int cx1 = min(cx0 + f.tw, f.W), cy1 = min(cy0 + f.th, f.H);
    for (int i = threadIdx.x; i < f.n_gauss * kLdsTapStride; i += blockDim.x) {
        const int l = i / kLdsTapStride, j = i - l * kLdsTapStride;
        const BlurTaps& t = taps[l];
        double v = 0.0;
        if (j <= kMaxTemplR) v = j <= t.R ? t.k[j] : 0.0;
        else v = j == kMaxTemplR + 1 ? t.sum_w : t.inv;
        TP[i] = v;
    }
    const int h0 = f.halo[f.l_first - 1];
    int ax = max(0, cx0 - h0), ay = max(0, cy0 - h0);
    int aw = min(f.W, cx1 + h0) - ax, ah = min(f.H, cy1 + h0) - ay;
    {
        gdouble* g0 = gbl(plane(pt, b, f.o, f.l_first - 1));
        const int Pa = aw | 1;
        for (int i = threadIdx.x; i < aw * ah; i += blockDim.x) {
            const int yy = i / aw, xx = i - yy * aw;
            S[yy * Pa + xx] = g0[(size_t)(ay + yy) * f.W + ax + xx];
        }
    }
    __syncthreads();
    for (int l = f.l_first; l <= f.l_last; ++l) {
        const int h = f.halo[l];
        const int bx = max(0, cx0 - h), by = max(0, cy0 - h);
        const int bw = min(f.W, cx1 + h) - bx, bh = min(f.H, cy1 + h) - by;
        double* g = const_cast<double*>(plane(pt, b, f.o, l));
        double* gd = (l == f.dec_level && f.Wd > 0) ? const_cast<double*>(plane(pt, b, f.o + 1, 0))
                                                     : nullptr;
        const double* tp = TP + l * kLdsTapStride;
        switch (f.R[l]) {
#define SIFT_FUSED_CASE(RR)                                                                     \
    case RR:                                                                                    \
        fused_level<RR>(tp, S, T, f, ax, ay, aw, ah, bx, by, bw, bh, cx0, cy0, cx1, cy1, g, gd); \
        break;
            SIFT_FUSED_CASE(1) SIFT_FUSED_CASE(2) SIFT_FUSED_CASE(3) SIFT_FUSED_CASE(4)
            SIFT_FUSED_CASE(5) SIFT_FUSED_CASE(6) SIFT_FUSED_CASE(7) SIFT_FUSED_CASE(8)
            SIFT_FUSED_CASE(9) SIFT_FUSED_CASE(10) SIFT_FUSED_CASE(11) SIFT_FUSED_CASE(12)
#undef SIFT_FUSED_CASE
            default:
                break;  // plan_octave_fused admits radii 1..12 only
        }
        ax = bx;
        ay = by;
        aw = bw;
        ah = bh;
    }
}

// Generic fallbacks for kernels wider than kMaxTemplR (unusual sigmas): a
// plain horizontal pass into `tmp`, then a vertical pass, one thread per px.
__global__ __launch_bounds__(256) void k_blur_rows_any(const double* __restrict__ src,
                                                       size_t src_bs, double* __restrict__ tmp,
                                                       int W, int H, BlurTaps tp) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    src += blockIdx.z * src_bs;
    tmp += blockIdx.z * (size_t)W * H;
    const double* row = src + (size_t)y * W;
    double acc = row[x] * tp.k[0];
    for (int u = 1; u <= tp.R; ++u)
        acc += tp.k[u] * (row[min(x + u, W - 1)] + row[max(x - u, 0)]);
    tmp[(size_t)y * W + x] = acc / tp.sum_w;
}

__global__ __launch_bounds__(256) void k_blur_cols_any(const double* __restrict__ tmp,
                                                       double* __restrict__ dst, size_t bs,
                                                       int W, int H, BlurTaps tp,
                                                       double* __restrict__ dec, int Wd,
                                                       int Hd) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    tmp += blockIdx.z * (size_t)W * H;
    dst += blockIdx.z * bs;
    if (dec) dec += blockIdx.z * bs;
    double acc = tmp[(size_t)y * W + x] * tp.k[0];
    for (int u = 1; u <= tp.R; ++u)
        acc += tp.k[u] * (tmp[(size_t)min(y + u, H - 1) * W + x] +
                           tmp[(size_t)max(y - u, 0) * W + x]);
    const double o = acc / tp.sum_w;
    dst[(size_t)y * W + x] = o;
    if (dec && !(x & 1) && !(y & 1) && (x >> 1) < Wd && (y >> 1) < Hd)
        dec[(size_t)(y >> 1) * Wd + (x >> 1)] = o;
}

// ---------------------------------------------------------------------------
// refine_one: compute_keypoints (sift.cpp:330-436) for one candidate, with
// get_pixel_cube, compute_gradient, compute_hessian, fit_quadratic
// (sift.cpp:32-106); bit-exact (no libm: the size's pow(2, t) is glibc's
// algorithm, sift_pow2.h).
// ---------------------------------------------------------------------------
// The pyramid table in LDS: the plane bases every refine step looks up per
// lane (a candidate's octave and layer vary across the wave), so a step
// costs one round trip to memory (its 36 pixels), not two.
struct RefineLds {
    const double* lvl[kMaxOctaves][kMaxLevels];
    int w[kMaxOctaves], h[kMaxOctaves];
};

__device__ bool refine_one(const RefineLds& T, size_t img_stride, const DevParams& P, int ex,
                           int ey, int ez, int o, int im, RawKp* out) {
    const int b = P.window_size / 2;
    const int W = T.w[o], H = T.h[o], depth = P.n_dog;
    double x = ex, y = ey;
    int layer = ez;
    double off0 = 0, off1 = 0, off2 = 0;
    int step;
    for (step = 0; step < kMaxSteps; ++step) {
        // the 3x3x3 DoG cube from the four Gaussian planes layer-1..layer+2:
        // all 36 loads in flight together
        const int xi = (int)x, yi = (int)y;
        double g[4][3][3];  // [plane][dy][dx]
#pragma unroll
        for (int pl = 0; pl < 4; ++pl) {
            gdouble* gp = gbl(T.lvl[o][layer - 1 + pl] + (size_t)im * img_stride);
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx)
                    g[pl][dy + 1][dx + 1] = gp[(size_t)(yi + dy) * W + (xi + dx)];
        }
        double c[3][3][3];  // get_pixel_cube (sift.cpp:32-44): [layer][x][y], /255
#pragma unroll
        for (int dz = 0; dz < 3; ++dz)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
                    c[dz][dx][dy] = (g[dz + 1][dy][dx] - g[dz][dy][dx]) / 255.0;
        const double g0 = 0.5 * (c[2][1][1] - c[0][1][1]);
        const double g1 = 0.5 * (c[1][2][1] - c[1][0][1]);
        const double g2 = 0.5 * (c[1][1][2] - c[1][1][0]);
        const double h00 = c[0][1][1] - 2 * c[1][1][1] + c[2][1][1];
        const double h11 = c[1][0][1] - 2 * c[1][1][1] + c[1][2][1];
        const double h22 = c[1][1][0] - 2 * c[1][1][1] + c[1][1][2];
        const double h01 = 0.25 * (c[2][2][1] - c[2][0][1] - c[0][2][1] + c[0][0][1]);
        const double h02 = 0.25 * (c[2][1][2] - c[2][1][0] - c[0][1][2] + c[0][1][0]);
        const double h12 = 0.25 * (c[1][0][0] - c[1][2][0] - c[1][0][2] + c[1][2][2]);
        const double det = h00 * h11 * h22 + 2 * (h01 * h12 * h02) - h02 * h11 * h02 -
                           h00 * h12 * h12 - h01 * h01 * h22;
        const double i00 = (h11 * h22 - h12 * h12) / det;
        const double i01 = (h02 * h12 - h01 * h22) / det;
        const double i02 = (h01 * h12 - h02 * h11) / det;
        const double i11 = (h00 * h22 - h02 * h02) / det;
        const double i12 = (h02 * h01 - h00 * h12) / det;
        const double i22 = (h00 * h11 - h01 * h01) / det;
        off0 = -i00 * g0 - i01 * g1 - i02 * g2;
        off1 = -i01 * g0 - i11 * g1 - i12 * g2;
        off2 = -i02 * g0 - i12 * g1 - i22 * g2;
        const double m = fmax(fabs(off0), fmax(fabs(off1), fabs(off2)));
        if (m < kConvThr) {
            const double dot = g0 * off0 + g1 * off1 + g2 * off2;
            const double val = c[1][1][1] + 0.5 * dot;
            if (!((fabs(val) * P.intervals) >= P.contrast_threshold)) return false;
            const double tr = h11 + h22;
            const double dt = h11 * h22 - h12 * h12;
            if (tr <= 0) return false;
            const double er = P.eigen_ratio;
            if ((tr * tr * er) >= ((er + 1) * (er + 1) * dt)) return false;
            break;
        }
        layer = (int)((double)layer + round(off0));
        x += round(off1);
        y += round(off2);
        if (x < b || x >= (W - b) || y < b || y >= (H - b) || layer < b || layer >= (depth - b))
            return false;
    }
    if (step >= kMaxSteps) return false;
    const double scale = pow2i(o);
    out->x = scale * (x + off1);
    out->y = scale * (y + off2);
    // glibc's pow(2, t), bit for bit (sift_pow2.h): the size sets the
    // orientation and descriptor windows, so it must be the reference's
    out->size = P.init_sigma * scale * pow2_glibc(((double)layer + off0) / P.intervals);
    out->off0 = off0;
    out->octave = o;
    out->layer = layer;
    out->img = im;
    out->pad = 0;
    return true;
}

// k_refine: candidates [cand_begin, n_cand), one thread each (the dependent
// gathers of all candidates in flight together). NT = 64 (default): one
// wavefront per workgroup, so a batch's few thousand candidates spread over
// ~100 CUs instead of ~25, and each CU's address units serve one wave's 36
// scattered loads per step instead of four waves'.
template <int NT, int CPW>
__global__ __launch_bounds__(NT) void k_refine(const PyrTable* __restrict__ pt, DevParams P,
                                               const sift_extremum* __restrict__ cand,
                                               const unsigned* __restrict__ cand_begin,
                                               const unsigned* __restrict__ n_cand,
                                               unsigned cap_cand, RawKp* __restrict__ out,
                                               unsigned* __restrict__ n_out,
                                               unsigned cap_out, unsigned* __restrict__ snap0) {
    set_job_prio(pt->jp, 0);
    // the chain's candidate end (the extrema launch has completed) for the
    // next chain on this lane
    if (snap0 && blockIdx.x == 0 && threadIdx.x == 0) *snap0 = *n_cand;
    __shared__ RefineLds T;
    const unsigned n = min(*n_cand, cap_cand);
    const unsigned i0 = min(*cand_begin, n);
    // CPW candidates per wavefront (lanes >= CPW idle): fewer per wave
    // spreads a batch over more CUs
    constexpr int WPB = NT / 64;
    const unsigned stride = gridDim.x * WPB * CPW;
    if (i0 + blockIdx.x * WPB * CPW >= n) return;  // no candidate for this workgroup
    // grid-stride over whole waves (wave-uniform trip count), so the kept
    // keypoints of a wave take one counter atomic (ballot + prefix)
    const int lane = threadIdx.x & 63;
    for (int k = threadIdx.x; k < kMaxOctaves * kMaxLevels; k += NT)
        T.lvl[k / kMaxLevels][k % kMaxLevels] = pt->lvl[k / kMaxLevels][k % kMaxLevels];
    if (threadIdx.x < kMaxOctaves) {
        T.w[threadIdx.x] = pt->w[threadIdx.x];
        T.h[threadIdx.x] = pt->h[threadIdx.x];
    }
    const size_t img_stride = pt->img_stride;
    __syncthreads();
    for (unsigned i0w = i0 + (blockIdx.x * WPB + threadIdx.x / 64) * CPW; i0w < n;
         i0w += stride) {
        const unsigned i = i0w + lane;
        RawKp r;
        bool keep = false;
        if (lane < CPW && i < n) {
            const sift_extremum e = cand[i];
            const int o = e.octave & ((1 << kOctBits) - 1), im = e.octave >> kOctBits;
            keep = refine_one(T, img_stride, P, e.x, e.y, e.z, o, im, &r);
        }
        const unsigned long long m = __ballot(keep);
        if (m) {
            unsigned base = 0;
            if (lane == 0) base = atomicAdd(n_out, (unsigned)__popcll(m));
            base = __shfl(base, 0);
            const unsigned idx = base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            if (keep && idx < cap_out) out[idx] = r;
        }
    }
}

// ---------------------------------------------------------------------------
// Orientation: compute_orientations (sift.cpp:447-533), one record per
// orientation peak (the descriptors are in sift_desc.hip). Describing every
// oriented keypoint before clean_keypoints (sift.cpp:762, host) gives the
// same final records: std::unique only drops records equal in (x, y, size,
// pori), and the kept one is described from its own fields. (One fused
// orientation+descriptor kernel was measured slower: 242 VGPRs, 2 waves/SIMD.)
// ---------------------------------------------------------------------------
// lane i <- lane i-1 (DPP wavefront shift right); lane 0 <- fill
__device__ __forceinline__ double wave_shr1_f64(double v, double fill) {
    const unsigned long long u = __double_as_longlong(v), f = __double_as_longlong(fill);
    const unsigned lo =
        __builtin_amdgcn_update_dpp((unsigned)f, (unsigned)u, 0x138, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp((unsigned)(f >> 32), (unsigned)(u >> 32),
                                                    0x138, 0xf, 0xf, false);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------------------
// k_orient_wave: compute_orientations (sift.cpp:447-533) with one WAVEFRONT
// per refined keypoint, four independent waves per workgroup pulling
// keypoints from the work counter; no workgroup barrier.
//  * The (2r+1)^2 window is swept 64 samples at a time (lanes along x, so
//    the four gradient loads coalesce).
//  * The bin of a sample comes from an f32 atan2 (atan2_f32, error below
//    3.1e-7 rad) and a correctly rounded sqrt; whenever it lies within
//    nb * 3e-6 of a rounding boundary (10x the f32 path's error bound) or
//    |dx|, |dy| is tiny, the f64 atan2 decides, so the bin index equals the
//    f64 one. Gaussian weights come from a per-keypoint table of the same
//    ocml exp of the same argument (bit-identical to evaluating per sample).
//  * weight * magnitude goes into lane-interleaved f64 replicas of the
//    histogram (ds_add_f64), summed in a fixed order: reproducible run to
//    run. The per-bin summation order differs from the reference's scan
//    order: the bins move by a few ulps, the same order of effect as ocml's
//    atan2/exp against glibc's, far below what a peak decision resolves.
//  * The in-place circular smoothing (sift.cpp:496-504) is a Gauss-Seidel
//    recurrence, run in registers (lane = bin); peaks are tested one bin per
//    lane. (A 256-thread-workgroup-per-keypoint variant repeated the setup,
//    table, smoothing and peak search in every wave; removed in round 4.)
// Per-wave dynamic LDS: the histogram replicas, the weight table (kOriWTab
// doubles), and for num_bins > 64 the smoothed histogram.
// ---------------------------------------------------------------------------
#ifndef SIFT_ORIW_TAB
#define SIFT_ORIW_TAB 512
#endif
constexpr int kOriWTab = SIFT_ORIW_TAB;

// SIFT_ORIW_REPS replica-interleaved copies of the histogram per wave (bin b
// of replica r at hist[b * reps + r], r = lane % reps). 16 make the atomics
// conflict-free (see k_descriptor_wave) but the larger footprint measured
// +2.3 % on the bench (8: +1 %) against 4 (profiles/r03_h/bench_ab.json)
#ifndef SIFT_ORIW_REPS
#define SIFT_ORIW_REPS 4
#endif
constexpr int kOriWReps = SIFT_ORIW_REPS;

// records a wave buffers (keypoint index, orientation) before one counter
// atomic appends them: the peaks of every keypoint a wave handles
constexpr int kOriEmit = 64;

__host__ __device__ constexpr int ori_wave_lds_doubles(int nb) {
    return kOriWReps * nb + kOriWTab + (nb > 64 ? nb : 0) + 2 * kOriEmit;
}

// the rare exact-bin path (f64 atan2, sift.cpp:489), out of line so its
// registers do not count against the sample loop's
__device__ __noinline__ int ori_bin_exact(double dy, double dx, int nb) {
    return (int)round(nb * (atan2(dy, dx) + kPi) / kTwoPi);
}

__global__ __launch_bounds__(256, 4) void k_orient_wave(
    const PyrTable* __restrict__ pt, DevParams P, const RawKp* __restrict__ raw,
    const unsigned* __restrict__ raw_begin, const unsigned* __restrict__ n_raw, unsigned cap_raw,
    sift_kp* __restrict__ recs, RecSide* __restrict__ rec_side, unsigned* __restrict__ n_rec,
    unsigned cap_rec, unsigned* __restrict__ work, bool static_walk) {
    extern __shared__ double ori_wdyn[];
    set_job_prio(pt->jp, 0);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned n = min(*n_raw, cap_raw);
    const unsigned k0 = min(*raw_begin, n);
    const int nb = P.num_bins;
    double* const hist = ori_wdyn + wv * ori_wave_lds_doubles(nb);
    double* const rep = hist + (lane & (kOriWReps - 1));  // bin b at rep[b * kOriWReps]
    double* const wtab = hist + kOriWReps * nb;
    double* const hs = wtab + kOriWTab;  // num_bins > 64 only
    double* const eori = hs + (nb > 64 ? nb : 0);                   // buffered records:
    unsigned* const ekp = reinterpret_cast<unsigned*>(eori + kOriEmit);  // orientation, keypoint
    const double bin_guard = nb * 3e-6;  // f32 bin error bound x 10 (see above)
    const float nbf = (float)nb;
    unsigned nbuf = 0;  // wave-uniform
    // the buffered records go out at `base`; a record's fields come from its
    // keypoint (sift.cpp:515-528)
    auto write_out = [&](unsigned base) {
        for (unsigned i = lane; i < nbuf; i += 64) {
            const unsigned rec = base + i;
            if (rec >= cap_rec) continue;
            const RawKp q = raw[ekp[i]];
            double rx = q.x, ry = q.y, rs = q.size;
            if (P.double_image) {  // sift.cpp:522-526
                rx /= 2;
                ry /= 2;
                rs /= 2;
            }
            sift_kp& r = recs[rec];
            r.x = rx;
            r.y = ry;
            r.octave = q.octave;
            r.layer = q.layer;
            r.size = rs;
            r.pori = eori[i];
            rec_side[rec] = RecSide{q.off0, q.img, 0};
        }
    };
    auto flush = [&]() {  // a full buffer: one counter atomic
        wave_sync();
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(n_rec, nbuf);
        write_out(__builtin_amdgcn_readfirstlane(base));
        wave_sync();
        nbuf = 0;
    };
    // wave g's first keypoint is g of the launch's range, the later ones come
    // from the work counter (offset by the grid's waves): same-address
    // atomics serialise at one L2 channel (~10 ns each), and every wave
    // claiming at once at the start cost the last one ~20 us. static_walk
    // (a launch alone on the chip, ~2 keypoints per wave): g, g + waves, ...
    // with no counter at all (1080p alone 92 -> 75 us; sharing the chip with
    // fewer waves, ~9 keypoints each, the dynamic balance wins by 1 %)
    const unsigned n_waves = gridDim.x * 4;
    for (unsigned k = k0 + blockIdx.x * 4 + wv; k < n;) {
        const RawKp kp = raw[k];
        const int o = kp.octave;
        const double inv = 1.0 / pow2i(o);
        const int x = (int)round(kp.x * inv);
        const int y = (int)round(kp.y * inv);
        const double scale = P.ori_sigma_factor * (kp.size * inv);
        const int radius = (int)round(3.0 * scale);
        const double denom = 2.0 * scale * scale;
        gdouble* img = gbl(plane(pt, kp.img, o, kp.layer));
        const int W = pt->w[o], H = pt->h[o];
        const int side = 2 * radius + 1;
        const int kmax = 2 * radius * radius;
        const bool use_tab = kmax < kOriWTab;
        for (int i = lane; i < kOriWReps * nb; i += 64) hist[i] = 0.0;
        if (use_tab)
            for (int q = lane; q <= kmax; q += 64) wtab[q] = exp(-q / denom);
        wave_sync();
        // the side x side window flattened, 64 samples per step; sample s
        // at (i, j) = (s % side, s / side) - radius
        const int nsamp = side * side;
        const int dj = 64 / side, di = 64 - dj * side;
        int ci_ = lane % side - radius, cj_ = lane / side - radius;
        auto advance = [&](int& i, int& j) {
            i += di;
            j += dj;
            if (i > radius) {
                i -= side;
                ++j;
            }
        };
        auto fetch = [&](int s, int i, int j, double* v) -> bool {
            const bool ok =
                !(s >= nsamp || x + i - 1 < 0 || x + i + 1 >= W || y + j - 1 < 0 || y + j + 1 >= H);
            const size_t r0 = ok ? (size_t)(y + j) * W + x + i : (size_t)W + 1;
            v[0] = img[r0 + 1];
            v[1] = img[r0 - 1];
            v[2] = img[r0 - W];
            v[3] = img[r0 + W];
            return ok;
        };
        // a ring of A + 1 steps of 64 samples: step s0 is processed while
        // the loads of the next A steps are in flight
        constexpr int A = SIFT_ORI_AHEAD;
        int qi[A + 1], qj[A + 1];
        bool qok[A + 1];
        double qv[A + 1][4];
        int pi_ = ci_, pj_ = cj_;  // position of the next step to fetch
#pragma unroll
        for (int a = 0; a < A; ++a) {
            qi[a] = pi_;
            qj[a] = pj_;
            qok[a] = fetch(64 * a + lane, pi_, pj_, qv[a]);
            advance(pi_, pj_);
        }
        for (int s0 = 0; s0 < nsamp; s0 += 64) {
            qi[A] = pi_;
            qj[A] = pj_;
            qok[A] = fetch(s0 + 64 * A + lane, pi_, pj_, qv[A]);
            advance(pi_, pj_);
            if (qok[0]) {
                const double* cv = qv[0];
                ci_ = qi[0];
                cj_ = qj[0];
                const double dx = cv[0] - cv[1];
                const double dy = cv[2] - cv[3];
                const double mag = sqrt_f64(dx * dx + dy * dy);  // correctly rounded
                const float at = atan2_f32((float)dy, (float)dx);
                const int k2 = ci_ * ci_ + cj_ * cj_;
                const double wgt = use_tab ? wtab[k2] : exp(-k2 / denom);
                const float t = nbf * (at + (float)kPi) * (float)(1.0 / kTwoPi);
                int hidx = (int)rintf(t);
                const bool tiny = (dx != 0.0 && fabs(dx) < 1e-30) || (dy != 0.0 && fabs(dy) < 1e-30);
                if (fabs((double)t - floor((double)t) - 0.5) < bin_guard || tiny)
                    hidx = ori_bin_exact(dy, dx, nb);  // exact path
                hidx = (hidx < nb) ? hidx : 0;
                atomicAdd(&rep[hidx * kOriWReps], wgt * mag);
            }
#pragma unroll
            for (int a = 0; a < A; ++a) {
                qi[a] = qi[a + 1];
                qj[a] = qj[a + 1];
                qok[a] = qok[a + 1];
#pragma unroll
                for (int q = 0; q < 4; ++q) qv[a][q] = qv[a + 1][q];
            }
        }
        wave_sync();
        // smoothing (sift.cpp:496-504) and peaks (sift.cpp:507-531)
        auto emit = [&](bool peak, double ori) {  // into the wave's buffer
            const unsigned long long m = __ballot(peak);
            if (!m) return;
            const unsigned c = (unsigned)__popcll(m);  // <= 64 = kOriEmit
            if (nbuf + c > kOriEmit) flush();  // rare: 64 records
            if (peak) {
                const unsigned i = nbuf + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
                eori[i] = ori;
                ekp[i] = k;
            }
            nbuf += c;
        };
        auto interp = [&](int i, double h0, double h1, double h2) {
            double fi = i + 0.5 * (h0 - h2) / (h0 - 2 * h1 + h2);
            fi = fmod(fi + nb, (double)nb);
            double ori = kTwoPi * fi / nb;
            return fmod(ori + kTwoPi, kTwoPi);
        };
        if (nb <= 64) {
            // lane b holds bin b; the Gauss-Seidel chain runs through
            // wave-uniform values, one dependent fma+add per bin
            double h = 0.0;
            if (lane < nb)  // fixed order per bin, rotated by lane (banks)
#pragma unroll
                for (int q = 0; q < kOriWReps; ++q)
                    h += hist[lane * kOriWReps + ((q + lane) & (kOriWReps - 1))];
            // The recurrence runs across the lanes: every step, lane i
            // re-evaluates fma(0.25, h_new[i-1], c_i) + d_i from lane i-1's
            // current value (DPP wavefront shift; lane 0 takes the old
            // h[nb-1]), so lane i is final from step i on: nb steps of 4
            // VALU instructions instead of ~10 (readlanes and a select per
            // bin); the same operands in the same order, bit-identical.
            for (int it = 0; it < kSmoothIters; ++it) {
                const double hn = __shfl(h, lane + 1 < nb ? lane + 1 : 0);  // old h[i+1]
                const double c = 0.5 * h;
                double d = 0.25 * hn;
                const double hlast = readlane_f64(h, nb - 1);  // h[i-1] for i = 0: old
                double v = h;
                for (int i = 0; i < nb; ++i) {
                    v = fma(0.25, wave_shr1_f64(v, hlast), c) + d;
                    if (i == 0 && nb > 1) {
                        // in place: the last bin's h[i+1] is the new h[0]
                        const double first_new = readlane_f64(v, 0);
                        if (lane == nb - 1) d = 0.25 * first_new;
                    }
                }
                h = v;
            }
            double mx = lane < nb ? h : 0.0;  // bins >= 0
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
            const double h0 = __shfl(h, lane == 0 ? nb - 1 : lane - 1);
            const double h2 = __shfl(h, lane + 1 >= nb ? 0 : lane + 1);
            const bool peak = lane < nb && h > h0 && h > h2 && h > (P.peak_ratio * mx);
            emit(peak, peak ? interp(lane, h0, h, h2) : 0.0);
        } else {
            for (int b = lane; b < nb; b += 64) {
                double v = 0.0;
                for (int q = 0; q < kOriWReps; ++q)
                    v += hist[b * kOriWReps + ((q + b) & (kOriWReps - 1))];
                hs[b] = v;
            }
            wave_sync();
            if (lane == 0) {
                for (int it = 0; it < kSmoothIters; ++it) {
                    double prev = hs[nb - 1];  // h[i-1] for i = 0: not yet updated
                    const double h0_old = hs[0];
                    double first_new = 0.0;
                    for (int i = 0; i < nb; ++i) {
                        const double h1 = hs[i];
                        const double h2 = (i + 1 < nb) ? hs[i + 1] : (i == 0 ? h0_old : first_new);
                        const double v = fma(0.25, prev, 0.5 * h1) + 0.25 * h2;
                        hs[i] = v;
                        prev = v;
                        if (i == 0) first_new = v;
                    }
                }
            }
            wave_sync();
            double mx = 0.0;
            for (int b = lane; b < nb; b += 64) mx = fmax(mx, hs[b]);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
            for (int b0 = 0; b0 < nb; b0 += 64) {
                const int i = b0 + lane;
                bool peak = false;
                double ori = 0.0;
                if (i < nb) {
                    const double h0 = hs[i == 0 ? nb - 1 : i - 1];
                    const double h1 = hs[i];
                    const double h2 = hs[i + 1 == nb ? 0 : i + 1];
                    peak = h1 > h0 && h1 > h2 && h1 > (P.peak_ratio * mx);
                    if (peak) ori = interp(i, h0, h1, h2);
                }
                emit(peak, ori);
            }
        }
        wave_sync();
        if (static_walk) {
            k += n_waves;
        } else {
            unsigned claim = 0;
            if (lane == 0) claim = atomicAdd(work, 1u);
            k = k0 + n_waves + __builtin_amdgcn_readfirstlane(claim);
        }
    }
    // the workgroup's remaining records: one counter atomic
    __shared__ unsigned wg_n[4], wg_base[4];
    if (lane == 0) wg_n[wv] = nbuf;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = wg_n[0] + wg_n[1] + wg_n[2] + wg_n[3];
        const unsigned base = t ? atomicAdd(n_rec, t) : 0u;
        wg_base[0] = base;
        wg_base[1] = base + wg_n[0];
        wg_base[2] = wg_base[1] + wg_n[1];
        wg_base[3] = wg_base[2] + wg_n[2];
    }
    __syncthreads();
    write_out(wg_base[wv]);
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------

template <int R, int C, int MODE>
static hipError_t launch_blur_r(const BlurSource& src, double* dst, size_t bs, int n_img, int W,
                                int H, int rows, const BlurTaps& taps, double* dec, int Wd,
                                int Hd, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    dim3 grid((W + 64 * C - 1) / (64 * C), ((H + rows - 1) / rows + 3) / 4, n_img);
    if (MODE == kSrcPlane && dec)
        return launch_timed(k_blur<R, C, true, kSrcPlane>, grid, dim3(256), 0, s, e0, e1, src,
                            dst, bs, W, H, rows, taps, dec, Wd, Hd);
    return launch_timed(k_blur<R, C, false, MODE>, grid, dim3(256), 0, s, e0, e1, src, dst, bs,
                        W, H, rows, taps, dec, Wd, Hd);
}

template <int R, int C, int NB>
static hipError_t launch_pair_dma_r(const double* src, size_t src_bs, double* dst, size_t bs,
                                    int n_img, int W, int H, int rows, const BlurTaps& taps,
                                    double* dec, int Wd, int Hd, hipStream_t s, hipEvent_t e0,
                                    hipEvent_t e1) {
    const dim3 grid((W + 64 * C - 1) / (64 * C), (H + 4 * rows - 1) / (4 * rows), n_img);
    constexpr size_t lds = pair_dma_lds_bytes<R, C, NB>();
    static_assert(lds <= 160 * 1024, "k_blur_pair_dma: LDS");
    static bool attr = false;  // above 64 KB of dynamic LDS (benign race: idempotent)
    if (!attr) {
        const hipError_t e = (lds > 64 * 1024)
            ? hipFuncSetAttribute(reinterpret_cast<const void*>(&k_blur_pair_dma<R, C, true, NB>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
            : hipSuccess;
        const hipError_t e2 = (lds > 64 * 1024)
            ? hipFuncSetAttribute(reinterpret_cast<const void*>(&k_blur_pair_dma<R, C, false, NB>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
            : hipSuccess;
        if (e != hipSuccess) return e;
        if (e2 != hipSuccess) return e2;
        attr = true;
    }
    if (dec)
        return launch_timed(k_blur_pair_dma<R, C, true, NB>, grid, dim3(256), lds, s, e0, e1, src,
                            src_bs, dst, bs, W, H, rows, taps, dec, Wd, Hd);
    return launch_timed(k_blur_pair_dma<R, C, false, NB>, grid, dim3(256), lds, s, e0, e1, src,
                        src_bs, dst, bs, W, H, rows, taps, dec, Wd, Hd);
}

template <int R, int C>
static hipError_t launch_pair_r(const double* src, size_t src_bs, double* dst, size_t bs,
                                int n_img, int W, int H, int rows, const BlurTaps& taps,
                                double* dec, int Wd, int Hd, hipStream_t s, hipEvent_t e0,
                                hipEvent_t e1) {
    if constexpr (SIFT_BLUR_DMA > 0 && R <= SIFT_BLUR_DMA_MAXR) {
        if ((size_t)W * H >= ((size_t)1 << SIFT_BLUR_DMA_PX_LOG2))
            return launch_pair_dma_r<R, C, (SIFT_BLUR_DMA > 0 ? SIFT_BLUR_DMA : 2)>(
                src, src_bs, dst, bs, n_img, W, H, rows, taps, dec, Wd, Hd, s, e0, e1);
    }
    const dim3 grid((W + 64 * C - 1) / (64 * C), (H + 4 * rows - 1) / (4 * rows), n_img);
    if (dec)
        return launch_timed(k_blur_pair<R, C, true>, grid, dim3(256), 0, s, e0, e1, src, src_bs,
                            dst, bs, W, H, rows, taps, dec, Wd, Hd);
    return launch_timed(k_blur_pair<R, C, false>, grid, dim3(256), 0, s, e0, e1, src, src_bs, dst,
                        bs, W, H, rows, taps, dec, Wd, Hd);
}
using PairFn = hipError_t (*)(const double*, size_t, double*, size_t, int, int, int, int,
                              const BlurTaps&, double*, int, int, hipStream_t, hipEvent_t,
                              hipEvent_t);
template <int C, int... Rs>
struct PairTable {
    static constexpr PairFn fns[sizeof...(Rs)] = {&launch_pair_r<Rs, C>...};
};
template <int C, int... Rs>
constexpr PairFn PairTable<C, Rs...>::fns[sizeof...(Rs)];
using BlurPair1 = PairTable<1, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;
// two columns per lane: the hand-over buffer (4 waves x R rows x 128
// columns) fits the 64 KB of static LDS up to R = 14
using BlurPair2 = PairTable<2, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14>;

using BlurFn = hipError_t (*)(const BlurSource&, double*, size_t, int, int, int, int,
                              const BlurTaps&, double*, int, int, hipStream_t, hipEvent_t,
                              hipEvent_t);

template <int C, int MODE, int... Rs>
struct BlurTable {
    static constexpr BlurFn fns[sizeof...(Rs)] = {&launch_blur_r<Rs, C, MODE>...};
};
template <int C, int MODE, int... Rs>
constexpr BlurFn BlurTable<C, MODE, Rs...>::fns[sizeof...(Rs)];

#define SIFT_R_LIST 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16
using BlurPlane1 = BlurTable<1, kSrcPlane, SIFT_R_LIST>;
using BlurPlane2 = BlurTable<2, kSrcPlane, SIFT_R_LIST>;
using BlurGray1 = BlurTable<1, kSrcGray, SIFT_R_LIST>;
using BlurGray2 = BlurTable<2, kSrcGray, SIFT_R_LIST>;
using BlurUps1 = BlurTable<1, kSrcUpsample, SIFT_R_LIST>;
using BlurUps2 = BlurTable<2, kSrcUpsample, SIFT_R_LIST>;
using BlurUpsRGB1 = BlurTable<1, kSrcUpsampleRGB, SIFT_R_LIST>;
using BlurUpsRGB2 = BlurTable<2, kSrcUpsampleRGB, SIFT_R_LIST>;
#undef SIFT_R_LIST
static_assert(kMaxTemplR == 16, "blur tables must cover 1..kMaxTemplR");

// Strip shape per level (measured on MI355X, tools/blur_lab.hip): two
// columns per lane and 32-row strips on octave-0-sized levels (the initial
// blur fused with the input staging; the other octave-0 levels take
// k_blur_pair), two columns and 16 rows around 2 Mpx, one column and 16 rows
// below (more, shorter strips: the small levels are latency-bound).
BlurShape blur_shape_for(int W, int H, int R) {
    const size_t px = (size_t)W * H;
    BlurShape b;
    b.cols = (!(W & 1) && px >= ((size_t)1 << 20)) ? 2 : 1;
    if (px >= ((size_t)4 << 20)) b.cols = std::min(b.cols, SIFT_BLUR_BIG_COLS);
    b.rows = px >= ((size_t)4 << 20) ? SIFT_BLUR_BIG_ROWS : 16;  // 48 / 64 / 96 rows measured slower;
    // round 4: 24 / 48 / 64 rows for R >= 6 only: octave 0 alone within 1 %;
    // R > 12 (config 3's R = 14 level) also at 32 rows: 8192^2 alone 546 ->
    // 415 us against the 16 rows it used to take (tools/blur_lab.hip, round 5)
    if (b.rows > H) b.rows = H;
    return b;
}

static hipError_t launch_blur_shaped(int MODE, const BlurSource& bs, double* dst, size_t dst_bs,
                                     int n_img, int W, int H, const BlurTaps& taps, double* dec,
                                     int Wd, int Hd, hipStream_t s, hipEvent_t e0,
                                     hipEvent_t e1) {
    const BlurShape sh = blur_shape_for(W, H, taps.R);
    const int i = taps.R - 1;
    BlurFn f;
    if (MODE == kSrcPlane)
        f = sh.cols == 2 ? BlurPlane2::fns[i] : BlurPlane1::fns[i];
    else if (MODE == kSrcGray)
        f = sh.cols == 2 ? BlurGray2::fns[i] : BlurGray1::fns[i];
    else if (MODE == kSrcUpsample)
        f = sh.cols == 2 ? BlurUps2::fns[i] : BlurUps1::fns[i];
    else
        f = sh.cols == 2 ? BlurUpsRGB2::fns[i] : BlurUpsRGB1::fns[i];
    return f(bs, dst, dst_bs, n_img, W, H, sh.rows, taps, dec, Wd, Hd, s, e0, e1);
}

template <int R, bool DECIM>
static hipError_t launch_tile_r(const double* src, size_t src_bs, double* dst, size_t bs,
                                int n_img, int W, int H, const BlurTaps& taps, double* dec,
                                int Wd, int Hd, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const dim3 grid((W + kTileW - 1) / kTileW, (H + kTileH - 1) / kTileH, n_img);
    return launch_timed(k_blur_tile<R, DECIM>, grid, dim3(256), 0, s, e0, e1, src, src_bs, dst,
                        bs, W, H, taps, dec, Wd, Hd);
}
using TileFn = hipError_t (*)(const double*, size_t, double*, size_t, int, int, int,
                              const BlurTaps&, double*, int, int, hipStream_t, hipEvent_t,
                              hipEvent_t);
template <bool DECIM, int... Rs>
struct TileTable {
    static constexpr TileFn fns[sizeof...(Rs)] = {&launch_tile_r<Rs, DECIM>...};
};
template <bool DECIM, int... Rs>
constexpr TileFn TileTable<DECIM, Rs...>::fns[sizeof...(Rs)];
using TileDec = TileTable<true, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;
using TileNoDec = TileTable<false, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;

hipError_t launch_blur(const double* src, size_t src_bs, double* dst, size_t bs, int n_img, int W,
                       int H, const BlurTaps& taps, double* dec, int Wd, int Hd, double* tmp,
                       hipStream_t s, hipEvent_t e0, hipEvent_t e1, size_t tile_max_px) {
    const int R = taps.R;
    if (R >= 1 && R <= kMaxTemplR && (size_t)W * H <= tile_max_px)
        return (dec ? TileDec::fns[R - 1] : TileNoDec::fns[R - 1])(src, src_bs, dst, bs, n_img, W,
                                                                   H, taps, dec, Wd, Hd, s, e0,
                                                                   e1);
    if (R >= 1 && R <= kMaxTemplR && SIFT_BLUR_PAIR && (size_t)W * H >= ((size_t)4 << 20)) {
        const int rows = std::min(SIFT_BLUR_PAIR_ROWS, (H + 1) / 2);
        const bool two = SIFT_BLUR_PAIR_COLS == 2 && !(W & 1) && R <= 14;
        return (two ? BlurPair2::fns : BlurPair1::fns)[R - 1](src, src_bs, dst, bs, n_img, W, H,
                                                              rows, taps, dec, Wd, Hd, s, e0, e1);
    }
    if (R >= 1 && R <= kMaxTemplR) {
        const BlurSource src_desc{src, src_bs, W, H, 1};
        return launch_blur_shaped(kSrcPlane, src_desc, dst, bs, n_img, W, H, taps, dec, Wd, Hd,
                                  s, e0, e1);
    }
    // wide kernels (or R == 0): generic two-pass path through `tmp`
    // (n_img * W * H doubles)
    dim3 grid((W + 255) / 256, H, n_img);
    if (e0) {
        hipError_t e = hipEventRecord(e0, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_blur_rows_any, grid, dim3(256), 0, s, src, src_bs, tmp, W, H, taps);
    hipLaunchKernelGGL(k_blur_cols_any, grid, dim3(256), 0, s, tmp, dst, bs, W, H, taps, dec,
                       Wd, Hd);
    if (e1) {
        hipError_t e = hipEventRecord(e1, s);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

bool launch_blur_initial_fused(const double* in, size_t in_bs, int w, int h, int c, int dbl,
                               double* dst, size_t bs, int n_img, int W0, int H0,
                               const BlurTaps& taps, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                               hipError_t* err) {
    const int R = taps.R;
    if (R < 1 || R > kMaxTemplR || (c == 1 && !dbl)) return false;
    const BlurSource src_desc{in, in_bs, w, h, c};
    *err = launch_blur_shaped(dbl ? (c == 1 ? kSrcUpsample : kSrcUpsampleRGB) : kSrcGray, src_desc, dst, bs, n_img, W0, H0,
                              taps, nullptr, 0, 0, s, e0, e1);
    return true;
}

hipError_t prepare_kernel_attributes() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_octaves_lds),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kLdsOctaveBytes);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_octave_fused),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFusedMaxBytes);
}

bool plan_octave_fused(int o, int n_gauss, int l_first, int l_last, int W, int H, int Wd, int Hd,
                       const int* radii, int tile, int threads, FusedOctave* f) {
    if (n_gauss < 2 || n_gauss > kMaxLevels || l_first < 1 || l_last < l_first ||
        l_last >= n_gauss || tile < 8 || W < 1 || H < 1 || threads < 64 || threads > 1024 ||
        threads % 64)
        return false;
    std::memset(f, 0, sizeof *f);
    for (int l = l_first; l <= l_last; ++l) {
        if (radii[l] < 1 || radii[l] > 12) return false;
        f->R[l] = radii[l];
    }
    f->l_first = l_first;
    f->l_last = l_last;
    f->halo[l_last] = 0;
    for (int l = l_last - 1; l >= l_first - 1; --l) f->halo[l] = f->halo[l + 1] + radii[l + 1];
    f->o = o;
    f->n_gauss = n_gauss;
    f->W = W;
    f->H = H;
    f->Wd = Wd;
    f->Hd = Hd;
    f->dec_level = (Wd > 0 && n_gauss - 3 >= l_first && n_gauss - 3 <= l_last) ? n_gauss - 3 : -1;
    f->tw = f->th = tile;
    f->ntx = (W + tile - 1) / tile;
    f->nty = (H + tile - 1) / tile;
    // the level buffer holds the largest region (the base's), the temporary
    // the base's rows x level 1's columns
    const int hb = f->halo[l_first - 1], h1 = f->halo[l_first];
    const int w0 = std::min(W, tile + 2 * hb), h0 = std::min(H, tile + 2 * hb);
    const int w1 = std::min(W, tile + 2 * h1);
    f->capS = (((w0 | 1) * h0) + 1) & ~1;
    f->capT = (((w1 | 1) * h0) + 1) & ~1;
    f->threads = threads;
    f->bytes = ((size_t)f->capS + f->capT + (size_t)n_gauss * kLdsTapStride) * sizeof(double);
    return f->bytes <= kFusedMaxBytes && (long)f->ntx * f->nty < (1L << 30);
}

hipError_t launch_octave_fused(const PyrTable* d_pt, const FusedOctave& f, const BlurTaps* d_taps,
                               int n_img, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (f.bytes > kFusedMaxBytes || f.ntx < 1 || f.nty < 1) return hipErrorInvalidValue;
    return launch_timed(k_octave_fused, dim3(f.ntx * f.nty, n_img), dim3(f.threads), f.bytes, s,
                        e0, e1, d_pt, f, d_taps);
}

LdsShape lds_shape(int W_first, int H_first, bool has_next, int n_gauss) {
    LdsShape sh;
    sh.cap = (((W_first | 1) * H_first) + 1) & ~1;  // even: 16-B aligned regions
    sh.dcap = has_next ? ((((W_first / 2) | 1) * (H_first / 2)) + 1) & ~1 : 2;
    sh.bytes = ((size_t)2 * sh.cap + sh.dcap + (size_t)n_gauss * kLdsTapStride) * sizeof(double);
    return sh;
}

hipError_t launch_octaves_lds(const PyrTable* d_pt, int o_first, int o_last, int n_gauss,
                              const BlurTaps* d_taps, int n_img, int W_first, int H_first,
                              hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (!lds_octave_fits(W_first, H_first) || n_gauss > kMaxLevels) return hipErrorInvalidValue;
    const LdsShape sh = lds_shape(W_first, H_first, o_first < o_last, n_gauss);
    return launch_timed(k_octaves_lds, dim3(n_img), dim3(SIFT_LDS_THREADS), sh.bytes, s, e0, e1, d_pt,
                        o_first, o_last, n_gauss, d_taps, sh.cap, sh.dcap);
}

hipError_t launch_prepare(const double* in, size_t in_bs, int w, int h, int c, int dbl,
                          double* out, size_t out_bs, int W0, int H0, int n_img, hipStream_t s) {
    dim3 grid((W0 + 255) / 256, H0, n_img);
    hipLaunchKernelGGL(k_prepare, grid, dim3(256), 0, s, in, in_bs, w, h, c, dbl, out, out_bs,
                       W0, H0);
    return hipGetLastError();
}

// Image bytes -> doubles (exact: every uint8 is a double), 8 per thread.
__global__ __launch_bounds__(256) void k_u8_to_f64(const uint8_t* __restrict__ in,
                                                   double* __restrict__ out, size_t n) {
    const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i0 + 8 <= n && !((uintptr_t)(in + i0) & 7)) {
        const uint64_t v = *reinterpret_cast<const uint64_t*>(in + i0);
        double2* o = reinterpret_cast<double2*>(out + i0);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = make_double2((double)((v >> (16 * k)) & 0xFF), (double)((v >> (16 * k + 8)) & 0xFF));
    } else {
        for (size_t i = i0; i < n && i < i0 + 8; ++i) out[i] = (double)in[i];
    }
}

// A job's first device work besides its pyramid: zero its counters and set
// its age rank in the (otherwise unchanged) device copy of its tables — one
// small launch instead of a table upload (a copy kernel reading pinned host
// memory, ~8 us) and a memset (~5 us) ahead of the first blur.
__global__ __launch_bounds__(256) void k_job_begin(PyrTable* __restrict__ pt, JobPrio jp,
                                                   unsigned* __restrict__ ctr, int n_ctr,
                                                   unsigned* __restrict__ ctr2, int n_ctr2) {
    for (int i = threadIdx.x; i < n_ctr; i += blockDim.x) ctr[i] = 0u;
    for (int i = threadIdx.x; i < n_ctr2; i += blockDim.x) ctr2[i] = 0u;
    if (threadIdx.x == 0) pt->jp = jp;
}

hipError_t launch_job_begin(PyrTable* pt, const JobPrio& jp, unsigned* ctr, int n_ctr,
                            unsigned* ctr2, int n_ctr2, hipStream_t s) {
    hipLaunchKernelGGL(k_job_begin, dim3(1), dim3(256), 0, s, pt, jp, ctr, n_ctr, ctr2,
                       ctr2 ? n_ctr2 : 0);
    return hipGetLastError();
}

hipError_t launch_u8_to_f64(const uint8_t* in, double* out, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t threads = (n + 7) / 8;
    hipLaunchKernelGGL(k_u8_to_f64, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, in,
                       out, n);
    return hipGetLastError();
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Final records of a job gathered into the caller's HBM buffer
// (sift_hip_fetch_device): out[i] = recs[items[i].src] with the host's
// glibc-exact size (sift.cpp:427-429) at byte 24; `items` is mapped host
// memory (read over PCIe once per record, no copy launch). With `checksum`,
// the wrapping 64-bit sum of every word written goes to *checksum so a
// receiver can verify the records: one atomic per workgroup into `acc`
// (zeroed with the job's counters), the last workgroup (`done`) writes the
// total, so *checksum needs no memset launch. Grid-stride over the 21 words
// of every record (consecutive threads write consecutive words), at most
// kGatherWgs workgroups: a wave per record with one atomic per workgroup of
// 4 records put ~1,500 same-address atomics (~10 ns each at one L2 channel)
// on a 1080p job.
constexpr unsigned kGatherWgs = 128;

__global__ __launch_bounds__(256) void k_gather_records(const sift_kp* __restrict__ recs,
                                                        const GatherItem* __restrict__ items,
                                                        unsigned n, sift_kp* __restrict__ out,
                                                        unsigned long long* __restrict__ checksum,
                                                        unsigned long long* __restrict__ acc,
                                                        unsigned* __restrict__ done) {
    __shared__ unsigned long long part[4];
    constexpr unsigned kWords = sizeof(sift_kp) / 8;  // 21
    const unsigned words = n * kWords;
    unsigned long long sum = 0;
    for (unsigned w = blockIdx.x * 256 + threadIdx.x; w < words; w += gridDim.x * 256) {
        const unsigned i = w / kWords, j = w - i * kWords;
        const GatherItem it = items[i];
        const double v = (j == 3) ? it.size : reinterpret_cast<const double*>(recs + it.src)[j];
        reinterpret_cast<double*>(out + i)[j] = v;
        sum += (unsigned long long)__double_as_longlong(v);
    }
    if (!checksum) return;
    sum = wave_sum_u64(sum);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        // the partial sum is published by the acq_rel done increment
        // (release); the last workgroup's increment also acquires every
        // other workgroup's add before it reads the total
        __hip_atomic_fetch_add(acc, part[0] + part[1] + part[2] + part[3], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
            gridDim.x - 1)
            *checksum = __hip_atomic_load(acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

hipError_t launch_gather_records(const sift_kp* recs, const GatherItem* items, unsigned n,
                                 sift_kp* out, unsigned long long* checksum,
                                 unsigned long long* acc, unsigned* done, hipStream_t s) {
    if (n == 0) return hipSuccess;
    static_assert(sizeof(sift_kp) == 168, "21 words per record");
    const unsigned wgs = std::min<unsigned>(kGatherWgs, (n * 21u + 1023u) / 1024u);
    hipLaunchKernelGGL(k_gather_records, dim3(wgs), dim3(256), 0, s, recs, items, n, out,
                       checksum, acc, done);
    return hipGetLastError();
}

// Exchange verification (sift_hip_verify_slots): slot r of `slots` holds,
// at word `count_word`, the number of 168-B records after `hdr_rows` header
// rows, and at words [sum_word, sum_word + n_sums) the sender's checksums of
// consecutive pieces of them (k_gather_records, one per step); the records'
// wrapping word sum must equal the checksums' sum; a mismatch increments *bad.
// One launch: each workgroup sums kVerifyChunk words of one slot (four loads
// per thread in flight) into the slot's accumulator with one 64-bit atomic;
// the slot's last workgroup (done count) compares and resets the
// accumulator and count for the next call (calls on a context are chained,
// sift_hip_verify_slots). Summing a slot of ~70 K records in one workgroup
// took 2.1 ms per bucket (profiles/r03_m); a memset + sum + check launch
// triple per bucket: world-1 exchange step 1.036 -> 1.028x the plain step.
constexpr int kVerifyChunk = 256 * 16;

__global__ __launch_bounds__(256) void k_verify_slots(const unsigned long long* __restrict__ slots,
                                                      size_t slot_words, int hdr_rows,
                                                      int count_word, int sum_word, int n_sums,
                                                      size_t cap_rows,
                                                      unsigned long long* __restrict__ scratch,
                                                      unsigned long long* __restrict__ bad) {
    __shared__ unsigned long long part[4];
    const unsigned slot = blockIdx.y;
    const unsigned long long* sl = slots + (size_t)slot * slot_words;
    const unsigned long long n = sl[count_word];
    const size_t words = (size_t)(n < cap_rows ? n : cap_rows) * 21;
    const size_t k0 = (size_t)blockIdx.x * kVerifyChunk;
    unsigned long long v = 0;
    if (k0 < words) {
        const unsigned long long* rec = sl + (size_t)hdr_rows * 21;
        const size_t k1 = words - k0 < (size_t)kVerifyChunk ? words : k0 + kVerifyChunk;
        for (size_t k = k0 + threadIdx.x; k < k1; k += 4 * 256) {
            unsigned long long a[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = k + q * 256 < k1 ? rec[k + q * 256] : 0ull;
#pragma unroll
            for (int q = 0; q < 4; ++q) v += a[q];
        }
    }
    v = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x != 0) return;
    unsigned long long* acc = scratch + 2 * slot;
    unsigned long long* done = acc + 1;
    // published by the acq_rel done count; the last workgroup acquires all
    __hip_atomic_fetch_add(acc, part[0] + part[1] + part[2] + part[3], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(done, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) !=
        gridDim.x - 1)
        return;
    const unsigned long long total = __hip_atomic_load(acc, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long want = 0;
    for (int k = 0; k < n_sums; ++k) want += sl[sum_word + k];
    if (n > cap_rows || total != want) atomicAdd(bad, 1ull);
    *acc = 0;  // ready for the next call (kernel boundary)
    *done = 0;
}

hipError_t launch_verify_slots(const void* slots, int n_slots, size_t slot_bytes, int hdr_rows,
                               int count_word, int sum_word, int n_sums, size_t cap_rows,
                               unsigned long long* bad, unsigned long long* scratch,
                               hipStream_t s) {
    if (n_slots <= 0) return hipSuccess;
    const auto* sl = static_cast<const unsigned long long*>(slots);
    const unsigned chunks =
        (unsigned)std::max<size_t>(1, (cap_rows * 21 + kVerifyChunk - 1) / kVerifyChunk);
    hipLaunchKernelGGL(k_verify_slots, dim3(chunks, n_slots), dim3(256), 0, s, sl, slot_bytes / 8,
                       hdr_rows, count_word, sum_word, n_sums, cap_rows, scratch, bad);
    return hipGetLastError();
}

__global__ void k_snapshot(const unsigned* __restrict__ ctr, unsigned* __restrict__ snap, int w0,
                           int w1) {
    if ((int)threadIdx.x >= w0 && (int)threadIdx.x < w1) snap[threadIdx.x] = ctr[threadIdx.x];
}

__global__ void k_job_done(unsigned* done) { atomicAdd(done, 1u); }

hipError_t launch_job_done(unsigned* done, hipStream_t s) {
    hipLaunchKernelGGL(k_job_done, dim3(1), dim3(1), 0, s, done);
    return hipGetLastError();
}

hipError_t launch_snapshot(const unsigned* ctr, unsigned* snap, hipStream_t s, int w0, int w1) {
    hipLaunchKernelGGL(k_snapshot, dim3(1), dim3(64), 0, s, ctr, snap, w0, w1);
    return hipGetLastError();
}

hipError_t launch_refine(const PyrTable* d_pt, const DevParams& P, const sift_extremum* cand,
                         const unsigned* cand_begin, const unsigned* n_cand, unsigned cap_cand,
                         RawKp* out, unsigned* n_out, unsigned cap_out, unsigned* snap0,
                         hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    // one wavefront per workgroup, a candidate per lane: a batch's few
    // thousand candidates spread over ~100 CUs (256-thread workgroups, 16 or
    // 32 candidates per wave measured slower)
    constexpr unsigned kPerWg = 64;
    unsigned blocks = (cap_cand + kPerWg - 1) / kPerWg;
    blocks = std::max(1u, std::min(blocks, 262144u / kPerWg));
    return launch_timed(k_refine<64, 64>, dim3(blocks), dim3(64), 0, s, e0, e1, d_pt, P, cand,
                        cand_begin, n_cand, cap_cand, out, n_out, cap_out, snap0);
}

hipError_t launch_orient(const PyrTable* d_pt, const DevParams& P, const RawKp* raw,
                         const unsigned* raw_begin, const unsigned* n_raw, unsigned cap_raw,
                         sift_kp* recs, RecSide* rec_side, unsigned* n_rec, unsigned cap_rec,
                         unsigned* work, unsigned wgs, bool static_walk, hipStream_t s,
                         hipEvent_t e0, hipEvent_t e1) {
    // persistent: four waves per workgroup, a keypoint per wave
    const unsigned blocks = std::min<unsigned>(wgs, cap_raw > 0 ? (cap_raw + 3) / 4 : 1);
    const size_t lds = (size_t)4 * ori_wave_lds_doubles(P.num_bins) * sizeof(double);
    return launch_timed(k_orient_wave, dim3(blocks), dim3(256), lds, s, e0, e1, d_pt, P, raw,
                        raw_begin, n_raw, cap_raw, recs, rec_side, n_rec, cap_rec, work,
                        static_walk);
}

}  // namespace sift_amd
