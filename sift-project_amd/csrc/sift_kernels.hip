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
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sift_kernels.h"

namespace sift_amd {

namespace {

constexpr double kTwoPi = 6.283185307179586;  // M_PI2 (sift.hh:5)
constexpr double kPi = 3.14159265358979323846;  // M_PI

// Compiler-level ordering for LDS traffic exchanged between the lanes of ONE
// wavefront (a wave's LDS instructions execute in order in hardware).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

// 2^e for small integer e, exact (the reference uses std::pow(2, int)).
__device__ __forceinline__ double pow2i(int e) { return ldexp(1.0, e); }

}  // namespace

// ---------------------------------------------------------------------------
// k_prepare: compute_initial_image minus the blur (sift.cpp:113-122):
// convert_to_grayscale (image.cpp:8-24) then resize_inter_bilinear x2
// (image.cpp:62-88), fused; one thread per output pixel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prepare(const double* __restrict__ in, int w,
                                                 int h, int c, int dbl,
                                                 double* __restrict__ out, int W0, int H0) {
    const int ox = blockIdx.x * blockDim.x + threadIdx.x;
    const int oy = blockIdx.y;
    if (ox >= W0 || oy >= H0) return;
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
// k_blur<R>: apply_gaussian_blur_fast / apply_double_convolution_1d
// (image.cpp:156-238), both passes in one kernel.
//
// One wavefront owns a 64-column strip of `rows` output rows. It slides down
// the strip one source row at a time: the row (plus an R-pixel replicate
// halo each side) is staged in a per-wave LDS line, every lane computes the
// horizontal pass for its column from LDS (2R+1 reads), and pushes the f64
// result into a (2R+1)-deep register window; once primed, the vertical pass
// runs entirely in registers. HBM traffic is one read of the source rows
// (+2R/rows priming overlap, L2-served) and one write per output pixel.
// Replicate borders: staged columns and source rows are clamped, which is
// exactly the reference's min(x+u, W-1) / max(x-u, 0) (image.cpp:177-180,
// 200-203). DECIM additionally writes resize_inter_nearest (image.cpp:41-55)
// of the output, i.e. the next octave's base (sift.cpp:195-196).
// ---------------------------------------------------------------------------
template <int R, bool DECIM>
__global__ __launch_bounds__(256) void k_blur(const double* __restrict__ src,
                                              double* __restrict__ dst, int W, int H,
                                              int rows, BlurTaps taps,
                                              double* __restrict__ dec, int Wd, int Hd) {
    constexpr int SEG = 64 + 2 * R;
    __shared__ double sline[4][SEG];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64;
    const int y_begin = (blockIdx.y * 4 + wv) * rows;
    if (y_begin >= H) return;  // whole wave leaves; no block barriers below
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

    double win[2 * R + 1];
#pragma unroll
    for (int q = 0; q <= 2 * R; ++q) win[q] = 0.0;

    int yy = y_begin - R;
    const int yy_end = y_end + R;
    const double* srow = src + (size_t)clampi(yy, 0, H - 1) * W;
    double a0 = srow[gx0];
    double a1 = has1 ? srow[gx1] : 0.0;
    for (; yy < yy_end; ++yy) {
        sl[lane] = a0;
        if (has1) sl[64 + lane] = a1;
        if (yy + 1 < yy_end) {  // prefetch the next source row
            const double* nrow = src + (size_t)clampi(yy + 1, 0, H - 1) * W;
            a0 = nrow[gx0];
            if (has1) a1 = nrow[gx1];
        }
        wave_sync();
        // horizontal pass (image.cpp:170-185)
        double acc = sl[lane + R] * k[0];
#pragma unroll
        for (int u = 1; u <= R; ++u) acc += k[u] * (sl[lane + R + u] + sl[lane + R - u]);
        const double t = acc / sw;
        wave_sync();
#pragma unroll
        for (int q = 0; q < 2 * R; ++q) win[q] = win[q + 1];
        win[2 * R] = t;
        if (yy >= y_begin + R) {
            // vertical pass for output row yy-R (image.cpp:193-208)
            const int y = yy - R;
            double o = win[R] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u) o += k[u] * (win[R + u] + win[R - u]);
            o = o / sw;
            if (x < W) {
                dst[(size_t)y * W + x] = o;
                if (DECIM && !(x & 1) && !(y & 1) && (x >> 1) < Wd && (y >> 1) < Hd)
                    dec[(size_t)(y >> 1) * Wd + (x >> 1)] = o;
            }
        }
    }
}

// Generic fallbacks for kernels wider than kMaxTemplR (unusual sigmas): a
// plain horizontal pass into `tmp`, then a vertical pass, one thread per px.
__global__ __launch_bounds__(256) void k_blur_rows_any(const double* __restrict__ src,
                                                       double* __restrict__ tmp, int W,
                                                       int H, BlurTaps tp) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const double* row = src + (size_t)y * W;
    double acc = row[x] * tp.k[0];
    for (int u = 1; u <= tp.R; ++u)
        acc += tp.k[u] * (row[min(x + u, W - 1)] + row[max(x - u, 0)]);
    tmp[(size_t)y * W + x] = acc / tp.sum_w;
}

__global__ __launch_bounds__(256) void k_blur_cols_any(const double* __restrict__ tmp,
                                                       double* __restrict__ dst, int W,
                                                       int H, BlurTaps tp,
                                                       double* __restrict__ dec, int Wd,
                                                       int Hd) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
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
// Extrema: detect_octave_extrema + is_extremum (sift.cpp:227-291) for
// window_size 3 (border 1). A pixel is kept iff |D_z| > threshold (the int
// threshold of sift.cpp:266,279) and it is a NON-strict maximum or minimum
// of its 3x3x3 cube, i.e. v == max(cube) or v == min(cube) (v is in the
// cube, so the centre comparison is vacuous, sift.cpp:241-246).
//
// One wavefront slides down a 64-column strip; per source row it stages the
// DoG row segments (66 values per DoG level, computed as G_{l+1}-G_l on the
// fly) in LDS, reduces them to 3-wide row max/min, and keeps three rows of
// those in registers, so the 3x3 max/min of every level is 2+2 max ops per
// row. Candidates are compacted per wave with a 64-bit ballot and one atomic.
// ---------------------------------------------------------------------------
template <int NL>
__global__ __launch_bounds__(256) void k_extrema3(const PyrTable* __restrict__ pt, int o,
                                                  int thr, int rows,
                                                  sift_extremum* __restrict__ out,
                                                  unsigned* __restrict__ counter,
                                                  unsigned cap) {
    constexpr int ND = NL - 1;  // DoG layers
    __shared__ double sd[4][ND][66];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int W = pt->w[o], H = pt->h[o];
    const int x0 = blockIdx.x * 64;
    const int yc_begin = 1 + (blockIdx.y * 4 + wv) * rows;  // first centre row
    if (yc_begin >= H - 1) return;
    const int yc_end = min(yc_begin + rows, H - 1);
    const double* G[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) G[l] = pt->lvl[o][l];
    const int x = x0 + lane;
    const int gxa = clampi(x0 - 1 + lane, 0, W - 1);
    const bool hasb = lane < 2;
    const int gxb = clampi(x0 + 63 + lane, 0, W - 1);
    const bool xin = (x >= 1) && (x < W - 1);
    const double dthr = (double)thr;

    double rmax[ND][3], rmin[ND][3], cen[ND][2];
#pragma unroll
    for (int l = 0; l < ND; ++l) {
        rmax[l][0] = rmax[l][1] = rmax[l][2] = 0.0;
        rmin[l][0] = rmin[l][1] = rmin[l][2] = 0.0;
        cen[l][0] = cen[l][1] = 0.0;
    }
    for (int yy = yc_begin - 1; yy <= yc_end; ++yy) {
        const size_t ro = (size_t)yy * W;
        double ga[NL], gb[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            ga[l] = G[l][ro + gxa];
            gb[l] = hasb ? G[l][ro + gxb] : 0.0;
        }
#pragma unroll
        for (int l = 0; l < ND; ++l) {
            sd[wv][l][lane] = ga[l + 1] - ga[l];
            if (hasb) sd[wv][l][64 + lane] = gb[l + 1] - gb[l];
        }
        wave_sync();
#pragma unroll
        for (int l = 0; l < ND; ++l) {
            const double a = sd[wv][l][lane], b = sd[wv][l][lane + 1], c = sd[wv][l][lane + 2];
            rmax[l][0] = rmax[l][1];
            rmax[l][1] = rmax[l][2];
            rmax[l][2] = fmax(fmax(a, b), c);
            rmin[l][0] = rmin[l][1];
            rmin[l][1] = rmin[l][2];
            rmin[l][2] = fmin(fmin(a, b), c);
            cen[l][0] = cen[l][1];
            cen[l][1] = b;  // D_l(yy, x)
        }
        wave_sync();
        if (yy < yc_begin + 1) continue;
        const int yc = yy - 1;  // centre row: its D values are cen[l][0]
        double cmax[ND], cmin[ND];
#pragma unroll
        for (int l = 0; l < ND; ++l) {
            cmax[l] = fmax(fmax(rmax[l][0], rmax[l][1]), rmax[l][2]);
            cmin[l] = fmin(fmin(rmin[l][0], rmin[l][1]), rmin[l][2]);
        }
#pragma unroll
        for (int z = 1; z < ND - 1; ++z) {
            const double v = cen[z][0];
            bool cand = false;
            if (xin && fabs(v) > dthr) {
                const double mx = fmax(fmax(cmax[z - 1], cmax[z]), cmax[z + 1]);
                const double mn = fmin(fmin(cmin[z - 1], cmin[z]), cmin[z + 1]);
                cand = (v == mx) || (v == mn);
            }
            const unsigned long long m = __ballot(cand);
            if (m) {
                unsigned base = 0;
                if (lane == 0) base = atomicAdd(counter, (unsigned)__popcll(m));
                base = __shfl(base, 0);
                const unsigned idx = base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
                if (cand && idx < cap) out[idx] = sift_extremum{x, yc, z, o};
            }
        }
    }
}

// Generic border b (window_size 4..7): one thread per (x, y), direct cube.
__global__ __launch_bounds__(256) void k_extrema_any(const PyrTable* __restrict__ pt, int o,
                                                     int thr, int b, int nd,
                                                     sift_extremum* __restrict__ out,
                                                     unsigned* __restrict__ counter,
                                                     unsigned cap) {
    const int W = pt->w[o], H = pt->h[o];
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x < b || x >= W - b || y < b || y >= H - b) return;
    for (int z = b; z < nd - b; ++z) {
        const size_t c = (size_t)y * W + x;
        const double v = pt->lvl[o][z + 1][c] - pt->lvl[o][z][c];
        if (fabs(v) <= (double)thr) continue;
        bool mx = true, mn = true;
        for (int dz = -b; dz <= b; ++dz)
            for (int dy = -b; dy <= b; ++dy)
                for (int dx = -b; dx <= b; ++dx) {
                    const size_t q = (size_t)(y + dy) * W + (x + dx);
                    const double n = pt->lvl[o][z + dz + 1][q] - pt->lvl[o][z + dz][q];
                    if (v < n) mx = false;
                    if (v > n) mn = false;
                }
        if (mx || mn) {
            const unsigned idx = atomicAdd(counter, 1u);
            if (idx < cap) out[idx] = sift_extremum{x, y, z, o};
        }
    }
}

// ---------------------------------------------------------------------------
// k_refine: compute_keypoints (sift.cpp:330-436) with get_pixel_cube,
// compute_gradient, compute_hessian, fit_quadratic (sift.cpp:32-106), one
// thread per candidate, bit-exact (no libm except the size's pow(2, t),
// which the host recomputes with glibc for the final records).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_refine(const PyrTable* __restrict__ pt, DevParams P,
                                                const sift_extremum* __restrict__ cand,
                                                const unsigned* __restrict__ n_cand,
                                                unsigned cap_cand, RawKp* __restrict__ out,
                                                unsigned* __restrict__ n_out,
                                                unsigned cap_out) {
    const unsigned n = min(*n_cand, cap_cand);
    const int b = P.window_size / 2;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += gridDim.x * blockDim.x) {
        const sift_extremum e = cand[i];
        const int o = e.octave;
        const int W = pt->w[o], H = pt->h[o], depth = P.n_dog;
        double x = e.x, y = e.y;
        int layer = e.z;
        double off0 = 0, off1 = 0, off2 = 0;
        int step;
        for (step = 0; step < kMaxSteps; ++step) {
            double c[3][3][3];
            const int xi = (int)x, yi = (int)y;
#pragma unroll
            for (int dz = -1; dz <= 1; ++dz) {
                const double* ga = pt->lvl[o][layer + dz + 1];
                const double* gb = pt->lvl[o][layer + dz];
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx)
#pragma unroll
                    for (int dy = -1; dy <= 1; ++dy) {
                        const size_t q = (size_t)(yi + dy) * W + (xi + dx);
                        c[dz + 1][dx + 1][dy + 1] = (ga[q] - gb[q]) / 255.0;
                    }
            }
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
                if (!((fabs(val) * P.intervals) >= P.contrast_threshold)) {
                    step = kMaxSteps;
                    break;
                }
                const double tr = h11 + h22;
                const double dt = h11 * h22 - h12 * h12;
                if (tr <= 0) {
                    step = kMaxSteps;
                    break;
                }
                const double er = P.eigen_ratio;
                if ((tr * tr * er) >= ((er + 1) * (er + 1) * dt)) step = kMaxSteps;
                break;
            }
            layer = (int)((double)layer + round(off0));
            x += round(off1);
            y += round(off2);
            if (x < b || x >= (W - b) || y < b || y >= (H - b) || layer < b ||
                layer >= (depth - b)) {
                step = kMaxSteps;
                break;
            }
        }
        if (step >= kMaxSteps) continue;
        const double scale = pow2i(o);
        RawKp r;
        r.x = scale * (x + off1);
        r.y = scale * (y + off2);
        r.size = P.init_sigma * scale * pow(2.0, ((double)layer + off0) / P.intervals);
        r.off0 = off0;
        r.octave = o;
        r.layer = layer;
        const unsigned idx = atomicAdd(n_out, 1u);
        if (idx < cap_out) out[idx] = r;
    }
}

// ---------------------------------------------------------------------------
// k_orient: compute_orientations (sift.cpp:447-533), one wavefront per
// refined keypoint. Samples of the (2r+1)^2 window are evaluated 64-wide in
// chunks and staged in LDS in the reference's scan order (i outer, j inner);
// each lane then owns up to 4 bins and adds that chunk's values for its bins
// sequentially, so every bin is summed in exactly the reference order
// (sift.cpp:491). The in-place circular smoothing (sift.cpp:496-504) is a
// Gauss-Seidel recurrence and runs sequentially on lane 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_orient(const PyrTable* __restrict__ pt, DevParams P,
                                                const RawKp* __restrict__ raw,
                                                const unsigned* __restrict__ n_raw,
                                                unsigned cap_raw, sift_kp* __restrict__ out,
                                                double* __restrict__ out_off0,
                                                unsigned* __restrict__ n_out,
                                                unsigned cap_out) {
    constexpr int CH = 512;
    __shared__ double sval[4][CH];
    __shared__ short sbin[4][CH];
    __shared__ double shist[4][kMaxBins];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const unsigned n = min(*n_raw, cap_raw);
    const int nb = P.num_bins;
    const int nbq = (nb + 63) >> 6;
    for (unsigned k = blockIdx.x * 4 + wv; k < n; k += gridDim.x * 4) {
        const RawKp kp = raw[k];
        const int o = kp.octave;
        const double inv = 1.0 / pow2i(o);
        const int x = (int)round(kp.x * inv);
        const int y = (int)round(kp.y * inv);
        const double size = kp.size * inv;
        const double scale = P.ori_sigma_factor * size;
        const int radius = (int)round(3.0 * scale);
        const double denom = 2.0 * scale * scale;
        const double* img = pt->lvl[o][kp.layer];
        const int W = pt->w[o], H = pt->h[o];
        const int side = 2 * radius + 1;
        const int ns = side * side;
        double hb[4] = {0.0, 0.0, 0.0, 0.0};
        for (int base = 0; base < ns; base += CH) {
            const int cnt = min(CH, ns - base);
            for (int s = lane; s < cnt; s += 64) {
                const int si = base + s;
                const int i = si / side - radius;
                const int j = si % side - radius;
                short bin = -1;
                double val = 0.0;
                if (!(x + i - 1 < 0 || x + i + 1 >= W || y + j - 1 < 0 || y + j + 1 >= H)) {
                    const size_t r0 = (size_t)(y + j) * W;
                    const double dx = img[r0 + x + i + 1] - img[r0 + x + i - 1];
                    const double dy = img[r0 - W + x + i] - img[r0 + W + x + i];
                    const double mag = sqrt(dx * dx + dy * dy);
                    const double ang = atan2(dy, dx);
                    const double wgt = exp(-(i * i + j * j) / denom);
                    int hidx = (int)round(nb * (ang + kPi) / kTwoPi);
                    hidx = (hidx < nb) ? hidx : 0;
                    bin = (short)hidx;
                    val = wgt * mag;
                }
                sval[wv][s] = val;
                sbin[wv][s] = bin;
            }
            wave_sync();
            for (int t = 0; t < cnt; ++t) {
                const int bsel = sbin[wv][t];
                const double v = sval[wv][t];
                for (int q = 0; q < nbq; ++q)
                    if (bsel == lane + 64 * q) hb[q] += v;
            }
            wave_sync();
        }
        for (int q = 0; q < nbq; ++q)
            if (lane + 64 * q < nb) shist[wv][lane + 64 * q] = hb[q];
        wave_sync();
        if (lane == 0) {
            double* hs = shist[wv];
            for (int it = 0; it < kSmoothIters; ++it)
                for (int i = 0; i < nb; ++i)
                    hs[i] = 0.25 * hs[(i - 1 + nb) % nb] + 0.5 * hs[i] +
                            0.25 * hs[(i + 1) % nb];
        }
        wave_sync();
        double mx = 0.0;  // histogram entries are >= 0
        for (int q = 0; q < nbq; ++q)
            if (lane + 64 * q < nb) mx = fmax(mx, shist[wv][lane + 64 * q]);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
        for (int q = 0; q < nbq; ++q) {
            const int i = lane + 64 * q;
            bool peak = false;
            double ori = 0.0;
            if (i < nb) {
                const double h0 = shist[wv][(i - 1 + nb) % nb];
                const double h1 = shist[wv][i];
                const double h2 = shist[wv][(i + 1) % nb];
                if (h1 > h0 && h1 > h2 && h1 > (P.peak_ratio * mx)) {
                    double fi = i + 0.5 * (h0 - h2) / (h0 - 2 * h1 + h2);
                    fi = fmod(fi + nb, (double)nb);
                    ori = kTwoPi * fi / nb;
                    ori = fmod(ori + kTwoPi, kTwoPi);
                    peak = true;
                }
            }
            if (peak) {
                const unsigned idx = atomicAdd(n_out, 1u);
                if (idx < cap_out) {
                    sift_kp r;
                    r.x = kp.x;
                    r.y = kp.y;
                    r.octave = kp.octave;
                    r.layer = kp.layer;
                    r.size = kp.size;
                    r.pori = ori;
                    if (P.double_image) {
                        r.x /= 2;
                        r.y /= 2;
                        r.size /= 2;
                    }
                    out[idx].x = r.x;
                    out[idx].y = r.y;
                    out[idx].octave = r.octave;
                    out[idx].layer = r.layer;
                    out[idx].size = r.size;
                    out[idx].pori = r.pori;
                    out_off0[idx] = kp.off0;
                }
            }
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// k_descriptor: compute_descriptors + update_histogram + convert_hist_to_desc
// (sift.cpp:541-682), one wavefront per oriented keypoint. Window samples are
// strided over the lanes; each accepted sample's trilinear split adds into a
// per-wave 4x4x8 f64 histogram in LDS (ds_add_f64; one wave per histogram,
// so the result is reproducible run to run). The two normalisation sums run
// sequentially on lane 0 in index order (sift.cpp:583-596).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_descriptor(const PyrTable* __restrict__ pt,
                                                    DevParams P, sift_kp* __restrict__ recs,
                                                    const unsigned* __restrict__ n_p,
                                                    unsigned cap,
                                                    float* __restrict__ desc_f32) {
    __shared__ double sh[4][128];
    __shared__ double sinv[4];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const unsigned n = min(*n_p, cap);
    for (unsigned k = blockIdx.x * 4 + wv; k < n; k += gridDim.x * 4) {
        const double* hdr = reinterpret_cast<const double*>(&recs[k]);
        const double kx = hdr[0], ky = hdr[1];
        const int o = reinterpret_cast<const int*>(hdr)[4];
        const int layer = reinterpret_cast<const int*>(hdr)[5];
        const double ksize = hdr[3], pori = hdr[4];
        const double* img = pt->lvl[o][layer];
        const int W = pt->w[o], H = pt->h[o];
        const double inv = P.double_image ? (1.0 / pow2i(o - 1)) : (1.0 / pow2i(o));
        const int x = (int)(kx * inv);
        const int y = (int)(ky * inv);
        const double size = ksize * inv;
        const double bins_per_rad = kDescBins / kTwoPi;
        const double ca = cos(pori), sa = sin(pori);
        const double hw = P.desc_scale_factor * size;
        const double denom = 0.5 * kDescW * kDescW;
        const double rr = round(hw * 0.5 * sqrt(2.0) * (kDescW + 1.0) + 0.5);
        const double diag = sqrt((double)(W * W + H * H));
        const int radius = (int)((diag < rr) ? diag : rr);  // std::min(rr, diag)
        sh[wv][lane] = 0.0;
        sh[wv][lane + 64] = 0.0;
        wave_sync();
        const int side = 2 * radius + 1;
        const int ns = side * side;
        for (int s = lane; s < ns; s += 64) {
            const int row = s / side - radius;
            const int col = s % side - radius;
            const double row_rot = (col * sa + row * ca) / hw;
            const double col_rot = (col * ca - row * sa) / hw;
            const double rb = row_rot + kDescW / 2 - 0.5;
            const double cb = col_rot + kDescW / 2 - 0.5;
            if (!(rb > -1.0 && rb < kDescW && cb > -1.0 && cb < kDescW)) continue;
            const int ny = row + y, nx = col + x;
            if (!(nx > 0 && nx < (W - 1) && ny > 0 && ny < (H - 1))) continue;
            const size_t r0 = (size_t)ny * W;
            const double dx = img[r0 + nx + 1] - img[r0 + nx - 1];
            const double dy = img[r0 - W + nx] - img[r0 + W + nx];
            const double mag = sqrt(dx * dx + dy * dy);
            double ang = atan2(dy, dx);
            ang -= pori;
            ang = fmod(fmod(ang, kTwoPi) + kTwoPi, kTwoPi);
            const double ob = ang * bins_per_rad;
            const double wgt = exp(-(row_rot * row_rot + col_rot * col_rot) / denom);
            const double m = mag * wgt;
            const int br = (int)floor(rb), bc = (int)floor(cb), bo = (int)floor(ob);
            const double fr = rb - br, fc = cb - bc, fo = ob - bo;
#pragma unroll
            for (int r = 0; r <= 1; ++r) {
                const int ri = br + r;
                if (ri < 0 || ri >= kDescW) continue;
                const double vr = m * ((r == 0) ? 1.0 - fr : fr);
#pragma unroll
                for (int c = 0; c <= 1; ++c) {
                    const int ci = bc + c;
                    if (ci < 0 || ci >= kDescW) continue;
                    const double vc = vr * ((c == 0) ? 1.0 - fc : fc);
#pragma unroll
                    for (int q = 0; q <= 1; ++q) {
                        const int oi = (bo + q) % kDescBins;
                        atomicAdd(&sh[wv][ri * 32 + ci * 8 + oi], vc * ((q == 0) ? 1.0 - fo : fo));
                    }
                }
            }
        }
        wave_sync();
        if (lane == 0) {
            double* hv = sh[wv];
            double norm = 0.0;
            for (int i = 0; i < 128; ++i) norm += hv[i] * hv[i];
            norm = sqrt(norm);
            double ninv = 1.0 / norm;
            norm = 0.0;
            for (int i = 0; i < 128; ++i) {
                double v = hv[i] * ninv;
                if (v > kMagThr) v = kMagThr;
                hv[i] = v;
                norm += v * v;
            }
            norm = sqrt(norm);
            sinv[wv] = 1.0 / norm;
        }
        wave_sync();
        const double ninv = sinv[wv];
        uint8_t* d = recs[k].desc;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = lane + 64 * h;
            const double hv = sh[wv][i];
            const double q = floor(kIntFactor * hv * ninv);
            int val = (q == q) ? (int)q : 0;  // NaN -> 0 (Appendix A.17)
            val = val < 0 ? 0 : (val > 255 ? 255 : val);
            d[i] = (uint8_t)val;
            if (desc_f32) desc_f32[(size_t)k * 128 + i] = (float)(hv * ninv);
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
template <int R>
static hipError_t launch_blur_r(const double* src, double* dst, int W, int H, int rows,
                                const BlurTaps& taps, double* dec, int Wd, int Hd,
                                hipStream_t s) {
    dim3 grid((W + 63) / 64, ((H + rows - 1) / rows + 3) / 4);
    if (dec)
        hipLaunchKernelGGL((k_blur<R, true>), grid, dim3(256), 0, s, src, dst, W, H, rows,
                           taps, dec, Wd, Hd);
    else
        hipLaunchKernelGGL((k_blur<R, false>), grid, dim3(256), 0, s, src, dst, W, H, rows,
                           taps, dec, Wd, Hd);
    return hipGetLastError();
}

using BlurFn = hipError_t (*)(const double*, double*, int, int, int, const BlurTaps&,
                              double*, int, int, hipStream_t);

template <int... Rs>
struct BlurTable {
    static constexpr BlurFn fns[sizeof...(Rs)] = {&launch_blur_r<Rs>...};
};
template <int... Rs>
constexpr BlurFn BlurTable<Rs...>::fns[sizeof...(Rs)];

using BlurAll = BlurTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
                          19, 20, 21, 22, 23, 24>;
static_assert(kMaxTemplR == 24, "BlurAll must cover 1..kMaxTemplR");

int blur_rows_for(int W, int H, int R) {
    // enough wavefronts to fill 256 CUs several times over, but strips tall
    // enough that the 2R-row priming stays a modest fraction
    const int nsx = (W + 63) / 64;
    long want = 4096;
    int rows = (int)((long)H * nsx / want);
    const int min_rows = 2 * R + 12 > 32 ? 2 * R + 12 : 32;
    if (rows < min_rows) rows = min_rows;
    if (rows > H) rows = H;
    if (rows < 1) rows = 1;
    return rows;
}

hipError_t launch_blur(const double* src, double* dst, int W, int H, const BlurTaps& taps,
                       double* dec, int Wd, int Hd, double* tmp, hipStream_t s) {
    const int R = taps.R;
    if (R >= 1 && R <= kMaxTemplR) {
        const int rows = blur_rows_for(W, H, R);
        return BlurAll::fns[R - 1](src, dst, W, H, rows, taps, dec, Wd, Hd, s);
    }
    // wide kernels (or R == 0): generic two-pass path through `tmp`
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(k_blur_rows_any, grid, dim3(256), 0, s, src, tmp, W, H, taps);
    hipLaunchKernelGGL(k_blur_cols_any, grid, dim3(256), 0, s, tmp, dst, W, H, taps, dec,
                       Wd, Hd);
    return hipGetLastError();
}

hipError_t launch_prepare(const double* in, int w, int h, int c, int dbl, double* out,
                          int W0, int H0, hipStream_t s) {
    dim3 grid((W0 + 255) / 256, H0);
    hipLaunchKernelGGL(k_prepare, grid, dim3(256), 0, s, in, w, h, c, dbl, out, W0, H0);
    return hipGetLastError();
}

hipError_t launch_extrema(const PyrTable* d_pt, int o, int W, int H, int n_gauss,
                          int window_size, int thr, sift_extremum* out, unsigned* counter,
                          unsigned cap, hipStream_t s) {
    const int b = window_size / 2;
    if (b == 1) {
        const int nsx = (W + 63) / 64;
        int rows = (int)((long)(H - 2) * nsx / 4096);
        if (rows < 16) rows = 16;
        const int nstrips = (H - 2 + rows - 1) / rows;
        dim3 grid(nsx, (nstrips + 3) / 4);
        if (grid.y == 0) return hipSuccess;
        switch (n_gauss) {
#define SIFT_EXT_CASE(NL)                                                              \
    case NL:                                                                           \
        hipLaunchKernelGGL((k_extrema3<NL>), grid, dim3(256), 0, s, d_pt, o, thr, rows, \
                           out, counter, cap);                                         \
        return hipGetLastError();
            SIFT_EXT_CASE(4)
            SIFT_EXT_CASE(5)
            SIFT_EXT_CASE(6)
            SIFT_EXT_CASE(7)
            SIFT_EXT_CASE(8)
            SIFT_EXT_CASE(9)
            SIFT_EXT_CASE(10)
            SIFT_EXT_CASE(11)
#undef SIFT_EXT_CASE
            default:
                break;
        }
    }
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(k_extrema_any, grid, dim3(256), 0, s, d_pt, o, thr, b, n_gauss - 1, out,
                       counter, cap);
    return hipGetLastError();
}

hipError_t launch_refine(const PyrTable* d_pt, const DevParams& P,
                         const sift_extremum* cand, const unsigned* n_cand, unsigned cap_cand,
                         RawKp* out, unsigned* n_out, unsigned cap_out, hipStream_t s) {
    unsigned blocks = (cap_cand + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_refine, dim3(blocks), dim3(256), 0, s, d_pt, P, cand, n_cand,
                       cap_cand, out, n_out, cap_out);
    return hipGetLastError();
}

hipError_t launch_orient(const PyrTable* d_pt, const DevParams& P, const RawKp* raw,
                         const unsigned* n_raw, unsigned cap_raw, sift_kp* out,
                         double* out_off0, unsigned* n_out, unsigned cap_out,
                         hipStream_t s) {
    unsigned blocks = (cap_raw + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_orient, dim3(blocks), dim3(256), 0, s, d_pt, P, raw, n_raw, cap_raw,
                       out, out_off0, n_out, cap_out);
    return hipGetLastError();
}

hipError_t launch_descriptor(const PyrTable* d_pt, const DevParams& P, sift_kp* recs,
                             const unsigned* n, unsigned cap, float* desc_f32,
                             hipStream_t s) {
    unsigned blocks = (cap + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_descriptor, dim3(blocks), dim3(256), 0, s, d_pt, P, recs, n, cap,
                       desc_f32);
    return hipGetLastError();
}

}  // namespace sift_amd
