// sift_stitch.hip — the data-parallel parts of the stitching consumer
// (SURVEY §8(f) row 4): RANSAC homography scoring and panorama compositing
// on gfx950, behind include/sift_hip.h (sift_hip_ransac_*, sift_hip_warp_blend).
//
// The reference's consumer of detect + match is its stitching notebook
// (stitching/sift_stitch.ipynb, absent from the checkout,
// .MISSING_LARGE_BLOBS:3), fed by the datasets' stitch graphs
// (stitching/collection/Dataset/*/<name>-STITCH-GRAPH.txt). Nothing of its
// algorithm survives, so this is a standard homography stitcher on top of
// the reference's matcher (src/sift.cpp:783-815) and the parity of its
// kernels is pinned to oracle/sift_cpu.cpp's restatement (bit-exact scores,
// models and canvases), not to the reference.
//
// RANSAC: the point pairs are Hartley-normalised on the host (centroid to
// the origin, mean distance sqrt(2)); hypothesis h is scored by ONE
// wavefront: every lane draws the same 4 distinct pairs from a splitmix64
// stream seeded by (seed, h), solves the same 8x8 DLT system (wave-uniform,
// ~300 FP64 ops), then the lanes sweep the pairs 64 at a time and count
// inliers with a ballot. The best model is refitted on the host by least
// squares over its inliers. Compositing: one thread per canvas pixel walks
// the images in index order (inverse homography, clamped bilinear sample,
// feather weight). Built with -ffp-contract=off like the rest of the
// library, so the device and the oracle evaluate identical IEEE sequences.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "sift_types.h"

namespace {

constexpr int kMaxPickTries = 32;  // redraws per sample index before giving up
constexpr double kSingular = 1e-9;  // |pivot| below this (normalised coordinates): no model

__host__ __device__ inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// 4 distinct indices in [0, n) for hypothesis h; false when the stream keeps
// repeating (only possible for tiny n)
__host__ __device__ inline bool draw_sample(uint64_t seed, uint32_t h, uint32_t n, uint32_t* idx) {
    uint64_t st = seed ^ ((uint64_t)h * 0xD1B54A32D192ED03ull);
    for (int k = 0; k < 4; ++k) {
        bool ok = false;
        for (int t = 0; t < kMaxPickTries && !ok; ++t) {
            const uint32_t v = (uint32_t)(splitmix64(st) % n);
            ok = true;
            for (int j = 0; j < k; ++j) ok = ok && idx[j] != v;
            idx[k] = v;
        }
        if (!ok) return false;
    }
    return true;
}

// Solve M (8 x 9 augmented, row-major) in place by Gaussian elimination
// with partial pivoting (first maximum on ties); h[0..7]. False if a pivot
// is below kSingular.
__host__ __device__ inline bool solve8(double* M, double* h) {
    for (int c = 0; c < 8; ++c) {
        int piv = c;
        double best = fabs(M[c * 9 + c]);
        for (int r = c + 1; r < 8; ++r) {
            const double a = fabs(M[r * 9 + c]);
            if (a > best) {
                best = a;
                piv = r;
            }
        }
        if (!(best >= kSingular)) return false;
        if (piv != c)
            for (int k = 0; k < 9; ++k) {
                const double t = M[c * 9 + k];
                M[c * 9 + k] = M[piv * 9 + k];
                M[piv * 9 + k] = t;
            }
        for (int r = c + 1; r < 8; ++r) {
            const double f = M[r * 9 + c] / M[c * 9 + c];
            for (int k = c; k < 9; ++k) M[r * 9 + k] -= f * M[c * 9 + k];
        }
    }
    for (int r = 7; r >= 0; --r) {
        double acc = 0.0;
        for (int k = r + 1; k < 8; ++k) acc += M[r * 9 + k] * h[k];
        h[r] = (M[r * 9 + 8] - acc) / M[r * 9 + r];
    }
    return true;
}

// The two DLT rows of pair (x, y) -> (u, v) with h33 = 1:
// [x y 1 0 0 0 -ux -uy | u] and [0 0 0 x y 1 -vx -vy | v]
__host__ __device__ inline void dlt_rows(double x, double y, double u, double v, double* r0,
                                         double* r1) {
    r0[0] = x, r0[1] = y, r0[2] = 1.0, r0[3] = 0.0, r0[4] = 0.0, r0[5] = 0.0;
    r0[6] = -(u * x), r0[7] = -(u * y), r0[8] = u;
    r1[0] = 0.0, r1[1] = 0.0, r1[2] = 0.0, r1[3] = x, r1[4] = y, r1[5] = 1.0;
    r1[6] = -(v * x), r1[7] = -(v * y), r1[8] = v;
}

// squared reprojection error of (x, y) -> (u, v) under h (h33 = 1)
__host__ __device__ inline double reproj2(const double* h, double x, double y, double u,
                                          double v) {
    const double w = (h[6] * x + h[7] * y) + 1.0;
    const double px = ((h[0] * x + h[1] * y) + h[2]) / w;
    const double py = ((h[3] * x + h[4] * y) + h[5]) / w;
    const double dx = px - u, dy = py - v;
    return dx * dx + dy * dy;
}

// src/dst: n normalised pairs, (x, y) interleaved. One wavefront per
// hypothesis, four per workgroup.
__global__ __launch_bounds__(256) void k_ransac_score(const double* __restrict__ src,
                                                      const double* __restrict__ dst, uint32_t n,
                                                      uint32_t n_hyp, uint64_t seed, double thr2,
                                                      int* __restrict__ scores) {
    const int lane = threadIdx.x & 63;
    const uint32_t hyp = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (hyp >= n_hyp) return;  // whole wave
    uint32_t idx[4];
    double h[8];
    bool ok = draw_sample(seed, hyp, n, idx);
    if (ok) {
        double M[72];
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = idx[k];
            dlt_rows(src[2 * i], src[2 * i + 1], dst[2 * i], dst[2 * i + 1], M + 18 * k,
                     M + 18 * k + 9);
        }
        ok = solve8(M, h);
    }
    if (!ok) {
        if (lane == 0) scores[hyp] = -1;
        return;
    }
    int count = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        bool in = false;
        if (i < n) in = reproj2(h, src[2 * i], src[2 * i + 1], dst[2 * i], dst[2 * i + 1]) < thr2;
        count += __popcll(__ballot(in));
    }
    if (lane == 0) scores[hyp] = count;
}

// One thread per canvas pixel; images (HWC bytes) at img + off[i].
struct WarpImage {
    double Hinv[9];
    unsigned long long off;
    int w, h;
};

__global__ __launch_bounds__(256) void k_warp_blend(const unsigned char* __restrict__ img,
                                                    const WarpImage* __restrict__ ims, int n_img,
                                                    int c, int out_w, int out_h,
                                                    unsigned char* __restrict__ out) {
    const int X = blockIdx.x * 16 + (threadIdx.x & 15);
    const int Y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (X >= out_w || Y >= out_h) return;
    const double Xd = X, Yd = Y;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double wsum = 0.0;
    for (int i = 0; i < n_img; ++i) {
        const WarpImage& im = ims[i];
        const double* A = im.Hinv;
        const double wh = (A[6] * Xd + A[7] * Yd) + A[8];
        if (!(wh > 0.0)) continue;
        const double x = ((A[0] * Xd + A[1] * Yd) + A[2]) / wh;
        const double y = ((A[3] * Xd + A[4] * Yd) + A[5]) / wh;
        const int w = im.w, hh = im.h;
        if (!(x >= 0.0 && x <= w - 1.0 && y >= 0.0 && y <= hh - 1.0)) continue;
        const int x0 = (int)floor(x), y0 = (int)floor(y);
        const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, hh - 1);
        const double fx = x - x0, fy = y - y0;
        const double wt = fmin(fmin(x + 1.0, w - x), fmin(y + 1.0, hh - y));
        const unsigned char* p = img + im.off;
        for (int ch = 0; ch < c; ++ch) {
            const double p00 = p[((size_t)y0 * w + x0) * c + ch];
            const double p10 = p[((size_t)y0 * w + x1) * c + ch];
            const double p01 = p[((size_t)y1 * w + x0) * c + ch];
            const double p11 = p[((size_t)y1 * w + x1) * c + ch];
            const double v = (p00 * (1.0 - fx) + p10 * fx) * (1.0 - fy) +
                             (p01 * (1.0 - fx) + p11 * fx) * fy;
            acc[ch] += wt * v;
        }
        wsum += wt;
    }
    unsigned char* o = out + ((size_t)Y * out_w + X) * c;
    for (int ch = 0; ch < c; ++ch) {
        double v = wsum > 0.0 ? floor(acc[ch] / wsum + 0.5) : 0.0;
        v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
        o[ch] = (unsigned char)v;
    }
}

// Hartley normalisation of n points (x, y interleaved): centroid, then the
// scale making the mean distance sqrt(2); sequential sums in index order.
struct Norm {
    double cx, cy, s;
};

Norm normalise(const double* p, size_t n, double* out) {
    double sx = 0.0, sy = 0.0;
    for (size_t i = 0; i < n; ++i) {
        sx += p[2 * i];
        sy += p[2 * i + 1];
    }
    Norm t;
    t.cx = sx / (double)n;
    t.cy = sy / (double)n;
    double sd = 0.0;
    for (size_t i = 0; i < n; ++i) {
        const double dx = p[2 * i] - t.cx, dy = p[2 * i + 1] - t.cy;
        sd += std::sqrt(dx * dx + dy * dy);
    }
    const double md = sd / (double)n;
    t.s = md > 0.0 ? std::sqrt(2.0) / md : 1.0;
    for (size_t i = 0; i < n; ++i) {
        out[2 * i] = (p[2 * i] - t.cx) * t.s;
        out[2 * i + 1] = (p[2 * i + 1] - t.cy) * t.s;
    }
    return t;
}

// least-squares refit over the inliers (normal equations A^T A h = A^T b,
// accumulated in pair order); false if singular
bool refit(const double* src, const double* dst, const unsigned char* in, size_t n, double* h) {
    double M[72];
    std::memset(M, 0, sizeof M);
    for (size_t i = 0; i < n; ++i) {
        if (!in[i]) continue;
        double r[2][9];
        dlt_rows(src[2 * i], src[2 * i + 1], dst[2 * i], dst[2 * i + 1], r[0], r[1]);
        for (int q = 0; q < 2; ++q)
            for (int a = 0; a < 8; ++a)
                for (int b = 0; b < 9; ++b) M[a * 9 + b] += r[q][a] * r[q][b];
    }
    double hn[8];
    if (!solve8(M, hn)) return false;
    std::memcpy(h, hn, sizeof hn);
    return true;
}

size_t mark_inliers(const double* src, const double* dst, size_t n, const double* h, double thr2,
                    unsigned char* in) {
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
        in[i] = reproj2(h, src[2 * i], src[2 * i + 1], dst[2 * i], dst[2 * i + 1]) < thr2;
        k += in[i];
    }
    return k;
}

struct DevScratch {  // per-call device buffers (the consumer is not a hot loop)
    void* p = nullptr;
    ~DevScratch() {
        if (p) (void)hipFree(p);
    }
};

int check_params(const sift_ransac_params* p, size_t n) {
    if (!p || n < 4 || n > (size_t)UINT32_MAX / 2) return SIFT_ERR_ARG;
    if (p->n_hyp < 1 || p->n_hyp > (1 << 20) || !(p->threshold > 0.0) || p->refine_iters < 0)
        return SIFT_ERR_ARG;
    return SIFT_OK;
}

// normalised pairs -> device, one scoring launch, scores back
int score_all(hipStream_t s, const double* ns, const double* nd, size_t n,
              const sift_ransac_params* p, double thr2, int* scores) {
    const size_t pts = 2 * n * sizeof(double);
    const size_t need = 2 * pts + (size_t)p->n_hyp * sizeof(int);
    DevScratch buf;
    if (hipMalloc(&buf.p, need) != hipSuccess) return SIFT_ERR_NOMEM;
    double* d_src = static_cast<double*>(buf.p);
    double* d_dst = d_src + 2 * n;
    int* d_sc = reinterpret_cast<int*>(d_dst + 2 * n);
    if (hipMemcpyAsync(d_src, ns, pts, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_dst, nd, pts, hipMemcpyHostToDevice, s) != hipSuccess)
        return SIFT_ERR_HIP;
    hipLaunchKernelGGL(k_ransac_score, dim3((p->n_hyp + 3) / 4), dim3(256), 0, s, d_src, d_dst,
                       (uint32_t)n, (uint32_t)p->n_hyp, p->seed, thr2, d_sc);
    if (hipGetLastError() != hipSuccess) return SIFT_ERR_HIP;
    if (hipMemcpyAsync(scores, d_sc, (size_t)p->n_hyp * sizeof(int), hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return SIFT_ERR_HIP;
    return SIFT_OK;
}

struct Prepared {
    std::vector<double> ns, nd;
    Norm ts, td;
    double thr2;
};

Prepared prepare(const double* src, const double* dst, size_t n, const sift_ransac_params* p) {
    Prepared q;
    q.ns.resize(2 * n);
    q.nd.resize(2 * n);
    q.ts = normalise(src, n, q.ns.data());
    q.td = normalise(dst, n, q.nd.data());
    // the pixel threshold in normalised destination units
    const double t = p->threshold * q.td.s;
    q.thr2 = t * t;
    return q;
}

}  // namespace

extern "C" {

void sift_ransac_params_default(sift_ransac_params* p) {
    if (!p) return;
    p->n_hyp = 4096;
    p->refine_iters = 2;
    p->threshold = 3.0;
    p->seed = 0x5EEDull;
}

hipStream_t sift_ctx_stream_internal(sift_ctx* ctx);

int sift_hip_ransac_scores(sift_ctx* ctx, const double* src_xy, const double* dst_xy, size_t n,
                           const sift_ransac_params* p, int* scores) {
    if (!ctx || !src_xy || !dst_xy || !scores) return SIFT_ERR_ARG;
    int st = check_params(p, n);
    if (st != SIFT_OK) return st;
    Prepared q = prepare(src_xy, dst_xy, n, p);
    return score_all(sift_ctx_stream_internal(ctx), q.ns.data(), q.nd.data(), n, p, q.thr2,
                     scores);
}

int sift_hip_ransac_homography(sift_ctx* ctx, const double* src_xy, const double* dst_xy,
                               size_t n, const sift_ransac_params* p, double* H,
                               unsigned char* inliers, size_t* n_inliers) {
    if (!ctx || !src_xy || !dst_xy || !H || !n_inliers) return SIFT_ERR_ARG;
    int st = check_params(p, n);
    if (st != SIFT_OK) return st;
    Prepared q = prepare(src_xy, dst_xy, n, p);
    std::vector<int> scores(p->n_hyp);
    st = score_all(sift_ctx_stream_internal(ctx), q.ns.data(), q.nd.data(), n, p, q.thr2,
                   scores.data());
    if (st != SIFT_OK) return st;
    int best = -1, best_n = 0;
    for (int k = 0; k < p->n_hyp; ++k)
        if (scores[k] > best_n) best_n = scores[k], best = k;
    const double ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    std::vector<unsigned char> in(n, 0);
    *n_inliers = 0;
    if (best < 0) {
        std::memcpy(H, ident, sizeof ident);
        if (inliers) std::memset(inliers, 0, n);
        return SIFT_OK;
    }
    // the winning model again on the host (same sampler and solve)
    double h[8];
    {
        uint32_t idx[4];
        double M[72];
        draw_sample(p->seed, (uint32_t)best, (uint32_t)n, idx);
        for (int k = 0; k < 4; ++k)
            dlt_rows(q.ns[2 * idx[k]], q.ns[2 * idx[k] + 1], q.nd[2 * idx[k]],
                     q.nd[2 * idx[k] + 1], M + 18 * k, M + 18 * k + 9);
        solve8(M, h);
    }
    size_t k_in = mark_inliers(q.ns.data(), q.nd.data(), n, h, q.thr2, in.data());
    for (int it = 0; it < p->refine_iters && k_in >= 4; ++it) {
        double hr[8];
        if (!refit(q.ns.data(), q.nd.data(), in.data(), n, hr)) break;
        std::memcpy(h, hr, sizeof hr);
        k_in = mark_inliers(q.ns.data(), q.nd.data(), n, h, q.thr2, in.data());
    }
    // H = Td^-1 * Hn * Ts, scaled to H[8] = 1
    const double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    const double Ts[9] = {q.ts.s, 0, -q.ts.s * q.ts.cx, 0, q.ts.s, -q.ts.s * q.ts.cy, 0, 0, 1};
    const double Tdi[9] = {1.0 / q.td.s, 0, q.td.cx, 0, 1.0 / q.td.s, q.td.cy, 0, 0, 1};
    double A[9], B[9];
    for (int r = 0; r < 3; ++r)
        for (int c2 = 0; c2 < 3; ++c2) {
            A[r * 3 + c2] = 0.0;
            for (int k = 0; k < 3; ++k) A[r * 3 + c2] += Hn[r * 3 + k] * Ts[k * 3 + c2];
        }
    for (int r = 0; r < 3; ++r)
        for (int c2 = 0; c2 < 3; ++c2) {
            B[r * 3 + c2] = 0.0;
            for (int k = 0; k < 3; ++k) B[r * 3 + c2] += Tdi[r * 3 + k] * A[k * 3 + c2];
        }
    for (int k = 0; k < 9; ++k) H[k] = B[k] / B[8];
    *n_inliers = k_in;
    if (inliers) std::memcpy(inliers, in.data(), n);
    return SIFT_OK;
}

int sift_hip_warp_blend(sift_ctx* ctx, const unsigned char* const* images, const int* w,
                        const int* h, int c, int n_images, const double* Hinv, int out_w,
                        int out_h, unsigned char* out) {
    if (!ctx || !images || !w || !h || !Hinv || !out || n_images < 1 || c < 1 || c > 4 ||
        out_w < 1 || out_h < 1 || (size_t)out_w * out_h > ((size_t)1 << 30))
        return SIFT_ERR_ARG;
    std::vector<WarpImage> ims(n_images);
    size_t total = 0;
    for (int i = 0; i < n_images; ++i) {
        if (!images[i] || w[i] < 1 || h[i] < 1) return SIFT_ERR_ARG;
        std::memcpy(ims[i].Hinv, Hinv + 9 * i, 9 * sizeof(double));
        ims[i].off = total;
        ims[i].w = w[i];
        ims[i].h = h[i];
        total += (size_t)w[i] * h[i] * c;
    }
    const size_t out_bytes = (size_t)out_w * out_h * c;
    const size_t meta = sizeof(WarpImage) * n_images;
    DevScratch buf;
    if (hipMalloc(&buf.p, total + out_bytes + meta + 16) != hipSuccess) return SIFT_ERR_NOMEM;
    unsigned char* d_img = static_cast<unsigned char*>(buf.p);
    unsigned char* d_out = d_img + total;
    WarpImage* d_ims = reinterpret_cast<WarpImage*>(
        (reinterpret_cast<uintptr_t>(d_out + out_bytes) + 15) & ~(uintptr_t)15);
    hipStream_t s = sift_ctx_stream_internal(ctx);
    for (int i = 0; i < n_images; ++i)
        if (hipMemcpyAsync(d_img + ims[i].off, images[i], (size_t)w[i] * h[i] * c,
                           hipMemcpyHostToDevice, s) != hipSuccess)
            return SIFT_ERR_HIP;
    if (hipMemcpyAsync(d_ims, ims.data(), meta, hipMemcpyHostToDevice, s) != hipSuccess)
        return SIFT_ERR_HIP;
    hipLaunchKernelGGL(k_warp_blend, dim3((out_w + 15) / 16, (out_h + 15) / 16), dim3(256), 0, s,
                       d_img, d_ims, n_images, c, out_w, out_h, d_out);
    if (hipGetLastError() != hipSuccess) return SIFT_ERR_HIP;
    if (hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return SIFT_ERR_HIP;
    return SIFT_OK;
}

}  // extern "C"
