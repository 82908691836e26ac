// oracle/sift_cpu.cpp — TEST INFRASTRUCTURE ONLY (the checker, never the
// product). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load liboracle_sift.so.
//
// A from-scratch scalar restatement of the reference SIFT pipeline
// (ahmedhassayoune/sift-project, src/sift.cpp:7-776 and src/image.cpp:8-238)
// with every floating-point expression evaluated in the reference's order and
// no FMA contraction (build with -ffp-contract=off), so that its outputs are
// bit-identical to the compiled reference. Parity of this restatement is
// PINNED by tests/test_oracle.py against the golden vectors in tests/golden/,
// which were produced by the reference itself compiled from
// /root/reference/src (oracle/Makefile, oracle/ref_harness.cpp,
// tests/golden/make_goldens.py).
//
// Unlike the reference it keeps every stage's output (pyramid, extrema,
// refined, oriented, final) so the HIP path can be checked stage by stage.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/sift_hip.h"

namespace {

constexpr double kTwoPi = 6.283185307179586;  // M_PI2, sift.hh:5
constexpr int kMaxSteps = 5;                  // MAX_CONVERGENCE_STEPS, sift.hh:7
constexpr double kConvThr = 0.5;              // CONVERGENCE_THR, sift.hh:8
constexpr int kSmoothIters = 2;               // ORI_SMOOTH_ITERATIONS, sift.hh:9
constexpr int kHistW = 4;                     // DESC_HIST_WIDTH, sift.hh:10
constexpr int kHistBins = 8;                  // DESC_HIST_BINS, sift.hh:11
constexpr double kMagThr = 0.2;               // DESC_MAGNITUDE_THR, sift.hh:12
constexpr double kIntFactor = 512.0;          // INT_DESCR_FCTR, sift.hh:13

// One single-channel plane, row-major (image_io.cpp:81-92 with channels=1).
struct Plane {
    int w = 0, h = 0;
    std::vector<double> v;
    Plane() = default;
    Plane(int w_, int h_) : w(w_), h(h_), v((size_t)w_ * h_) {}
    double at(int x, int y) const { return v[(size_t)y * w + x]; }
    double& at(int x, int y) { return v[(size_t)y * w + x]; }
};

// ---- image ops (image.cpp) ------------------------------------------------

// convert_to_grayscale, image.cpp:8-24: 0.2126 r + 0.7152 g + 0.0722 b,
// evaluated left to right.
Plane gray_of(const double* hwc, int w, int h, int c) {
    Plane out(w, h);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const double* p = hwc + i * c;
        out.v[i] = 0.2126 * p[0] + 0.7152 * p[1] + 0.0722 * p[2];
    }
    return out;
}

// resize_inter_bilinear(img, 2, 2), image.cpp:62-88.
Plane upsample2(const Plane& in) {
    Plane out(in.w * 2, in.h * 2);
    for (int oy = 0; oy < out.h; ++oy) {
        const double fy = oy / 2.0;
        const int y0 = (int)fy;
        const int y1 = std::min(y0 + 1, in.h - 1);
        const double dy = fy - y0;
        for (int ox = 0; ox < out.w; ++ox) {
            const double fx = ox / 2.0;
            const int x0 = (int)fx;
            const int x1 = std::min(x0 + 1, in.w - 1);
            const double dx = fx - x0;
            const double top = in.at(x0, y0) * (1 - dx) + in.at(x1, y0) * dx;
            const double bot = in.at(x0, y1) * (1 - dx) + in.at(x1, y1) * dx;
            out.at(ox, oy) = top * (1 - dy) + bot * dy;
        }
    }
    return out;
}

// resize_inter_nearest, image.cpp:41-55 (throws if w or h < 2).
bool decimate2(const Plane& in, Plane& out) {
    if (in.w < 2 || in.h < 2) return false;
    out = Plane(in.w / 2, in.h / 2);
    for (int y = 0; y < out.h; ++y)
        for (int x = 0; x < out.w; ++x) out.at(x, y) = in.at(2 * x, 2 * y);
    return true;
}

// Half-kernel of apply_gaussian_blur_fast, image.cpp:226-235:
// ks = ceil(3 sigma) + 1 taps, k[i] = exp(-i*i / (2 sigma^2)) * coef, where
// -i*i is an int product and coef = 1/(sqrt(2 pi) sigma) (it cancels in the
// normalisation but is kept for bit parity).
struct HalfKernel {
    std::vector<double> k;
    double sum_w = 0.0;  // k0 + sum 2 k[u], accumulated in the reference order
};

HalfKernel half_kernel(double sigma) {
    HalfKernel hk;
    const int ks = (int)std::ceil(3 * sigma) + 1;
    const double denom = 2 * sigma * sigma;
    const double coef = 1 / (std::sqrt(2 * M_PI) * sigma);
    hk.k.resize(ks);
    for (int i = 0; i < ks; ++i) hk.k[i] = std::exp(-i * i / denom) * coef;
    // apply_double_convolution_1d, image.cpp:171-185: the running sum_w is the
    // same sequence for every pixel, so it is a per-kernel constant.
    double s = hk.k[0];
    for (int u = 1; u < ks; ++u) s += 2.0 * hk.k[u];
    hk.sum_w = s;
    return hk;
}

// apply_double_convolution_1d, image.cpp:156-214: replicate-border separable
// convolution, horizontal pass into an f64 temporary, then vertical pass.
Plane blur(const Plane& in, double sigma) {
    const HalfKernel hk = half_kernel(sigma);
    const int ks = (int)hk.k.size();
    Plane tmp(in.w, in.h), out(in.w, in.h);
    for (int y = 0; y < in.h; ++y) {
        for (int x = 0; x < in.w; ++x) {
            double acc = in.at(x, y) * hk.k[0];
            for (int u = 1; u < ks; ++u) {
                const int xr = std::min(x + u, in.w - 1);
                const int xl = std::max(x - u, 0);
                acc += hk.k[u] * (in.at(xr, y) + in.at(xl, y));
            }
            tmp.at(x, y) = acc / hk.sum_w;
        }
    }
    for (int y = 0; y < in.h; ++y) {
        for (int x = 0; x < in.w; ++x) {
            double acc = tmp.at(x, y) * hk.k[0];
            for (int u = 1; u < ks; ++u) {
                const int yd = std::min(y + u, in.h - 1);
                const int yu = std::max(y - u, 0);
                acc += hk.k[u] * (tmp.at(x, yd) + tmp.at(x, yu));
            }
            out.at(x, y) = acc / hk.sum_w;
        }
    }
    return out;
}

// ---- SIFT stages (sift.cpp) -----------------------------------------------

struct Run {
    sift_params p{};
    int octaves = 0;
    int n_gauss = 0;  // intervals + 3  (sift.cpp:144)
    int n_dog = 0;    // intervals + 2  (sift.cpp:212)
    std::vector<double> sigmas;
    std::vector<std::vector<Plane>> gauss;  // [octave][level]
    std::vector<std::vector<Plane>> dog;    // [octave][layer]
    std::vector<sift_extremum> extrema;
    std::vector<sift_kp> refined;
    std::vector<double> refined_off0;
    std::vector<sift_kp> oriented;
    std::vector<sift_kp> final_kps;
    std::vector<float> desc_f32;
    double t[8] = {0};  // init, pyramid, dog, extrema, refine, orient, clean, desc
};

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
}

// compute_gaussian_kernels, sift.cpp:143-155.
std::vector<double> level_sigmas(double sigma, int intervals) {
    std::vector<double> s(intervals + 3);
    s[0] = sigma;
    const double k = std::pow(2.0, 1.0 / intervals);
    for (int i = 1; i < (int)s.size(); ++i) {
        const double prev = (std::pow(k, i - 1)) * sigma;
        s[i] = prev * std::sqrt(k * k - 1);
    }
    return s;
}

// detect_octave_extrema + is_extremum, sift.cpp:227-291. Scan order: x outer,
// y, z inner; an extremum is non-strict (ties count), which equals
// "v == max of the cube or v == min of the cube" since v is in the cube.
void scan_extrema(Run& R, int o, int threshold) {
    const std::vector<Plane>& D = R.dog[o];
    const int W = D[0].w, H = D[0].h, depth = (int)D.size();
    const int b = R.p.window_size / 2;
    for (int x = b; x < W - b; ++x) {
        for (int y = b; y < H - b; ++y) {
            for (int z = b; z < depth - b; ++z) {
                const double v = D[z].at(x, y);
                if (std::abs(v) <= threshold) continue;
                bool is_max = true, is_min = true;
                for (int dx = -b; dx <= b && (is_max || is_min); ++dx)
                    for (int dy = -b; dy <= b; ++dy)
                        for (int dz = -b; dz <= b; ++dz) {
                            const double n = D[z + dz].at(x + dx, y + dy);
                            if (v < n) is_max = false;
                            if (v > n) is_min = false;
                        }
                if (is_max || is_min) R.extrema.push_back({x, y, z, o});
            }
        }
    }
}

// compute_keypoints + get_pixel_cube/compute_gradient/compute_hessian/
// fit_quadratic, sift.cpp:32-106, 330-436.
void refine_all(Run& R) {
    const sift_params& P = R.p;
    const int b = P.window_size / 2;
    for (const sift_extremum& e : R.extrema) {
        const std::vector<Plane>& D = R.dog[e.octave];
        const int depth = (int)D.size(), W = D[0].w, H = D[0].h;
        double x = e.x, y = e.y;
        int layer = e.z;
        double off[3] = {0, 0, 0};
        int step;
        for (step = 0; step < kMaxSteps; ++step) {
            // cube[dz][dx][dy], each DoG value / 255.0 (sift.cpp:35-41)
            double c[3][3][3];
            for (int dz = -1; dz <= 1; ++dz)
                for (int dx = -1; dx <= 1; ++dx)
                    for (int dy = -1; dy <= 1; ++dy)
                        c[dz + 1][dx + 1][dy + 1] =
                            D[layer + dz].at((int)x + dx, (int)y + dy) / 255.0;
            const double g0 = 0.5 * (c[2][1][1] - c[0][1][1]);
            const double g1 = 0.5 * (c[1][2][1] - c[1][0][1]);
            const double g2 = 0.5 * (c[1][1][2] - c[1][1][0]);
            const double h00 = c[0][1][1] - 2 * c[1][1][1] + c[2][1][1];
            const double h11 = c[1][0][1] - 2 * c[1][1][1] + c[1][2][1];
            const double h22 = c[1][1][0] - 2 * c[1][1][1] + c[1][1][2];
            const double h01 = 0.25 * (c[2][2][1] - c[2][0][1] - c[0][2][1] + c[0][0][1]);
            const double h02 = 0.25 * (c[2][1][2] - c[2][1][0] - c[0][1][2] + c[0][1][0]);
            const double h12 = 0.25 * (c[1][0][0] - c[1][2][0] - c[1][0][2] + c[1][2][2]);
            // symmetric: h10=h01, h20=h02, h21=h12 (sift.cpp:69-77)
            const double det = h00 * h11 * h22 + 2 * (h01 * h12 * h02) -
                               h02 * h11 * h02 - h00 * h12 * h12 -
                               h01 * h01 * h22;
            const double i00 = (h11 * h22 - h12 * h12) / det;
            const double i01 = (h02 * h12 - h01 * h22) / det;
            const double i02 = (h01 * h12 - h02 * h11) / det;
            const double i11 = (h00 * h22 - h02 * h02) / det;
            const double i12 = (h02 * h01 - h00 * h12) / det;
            const double i22 = (h00 * h11 - h01 * h01) / det;
            off[0] = -i00 * g0 - i01 * g1 - i02 * g2;
            off[1] = -i01 * g0 - i11 * g1 - i12 * g2;
            off[2] = -i02 * g0 - i12 * g1 - i22 * g2;

            const double m = std::max(std::abs(off[0]),
                                      std::max(std::abs(off[1]), std::abs(off[2])));
            if (m < kConvThr) {
                const double dot = g0 * off[0] + g1 * off[1] + g2 * off[2];
                const double val = c[1][1][1] + 0.5 * dot;
                if (!((std::abs(val) * P.intervals) >= P.contrast_threshold)) {
                    step = kMaxSteps;
                    break;
                }
                const double tr = h11 + h22;
                const double dt = h11 * h22 - h12 * h12;
                if (tr <= 0) {  // sift.cpp:385-388
                    step = kMaxSteps;
                    break;
                }
                const double er = P.eigen_ratio;
                if ((tr * tr * er) >= ((er + 1) * (er + 1) * dt)) step = kMaxSteps;
                break;
            }
            layer += std::round(off[0]);  // int += double (sift.cpp:401)
            x += std::round(off[1]);
            y += std::round(off[2]);
            if (x < b || x >= (W - b) || y < b || y >= (H - b) || layer < b ||
                layer >= (depth - b)) {
                step = kMaxSteps;
                break;
            }
        }
        if (step >= kMaxSteps) continue;
        const double scale = std::pow(2, e.octave);
        sift_kp kp;
        std::memset(&kp, 0, sizeof kp);
        kp.octave = e.octave;
        kp.layer = layer;
        kp.x = scale * (x + off[1]);
        kp.y = scale * (y + off[2]);
        kp.size = P.init_sigma * scale *
                  std::pow(2, (static_cast<double>(layer) + off[0]) / P.intervals);
        kp.pori = 0.0;
        R.refined.push_back(kp);
        R.refined_off0.push_back(off[0]);
    }
}

// compute_orientations, sift.cpp:447-533.
void orient_all(Run& R) {
    const sift_params& P = R.p;
    const int nb = (int)P.num_bins;  // double -> int narrowing (sift.cpp:450)
    std::vector<double> hist(nb);
    for (const sift_kp& kp : R.refined) {
        const int o = kp.octave;
        const double inv = 1.0 / std::pow(2, o);
        const int x = std::round(kp.x * inv);
        const int y = std::round(kp.y * inv);
        const double size = kp.size * inv;
        const double scale = P.ori_sigma_factor * size;
        const int radius = std::round(3.0 * scale);
        const double denom = 2.0 * scale * scale;
        const Plane& img = R.gauss[o][kp.layer];
        std::fill(hist.begin(), hist.end(), 0.0);
        for (int i = -radius; i <= radius; ++i) {
            if (x + i - 1 < 0 || x + i + 1 >= img.w) continue;
            for (int j = -radius; j <= radius; ++j) {
                if (y + j - 1 < 0 || y + j + 1 >= img.h) continue;
                const double dx = img.at(x + i + 1, y + j) - img.at(x + i - 1, y + j);
                const double dy = img.at(x + i, y + j - 1) - img.at(x + i, y + j + 1);
                const double mag = std::sqrt(dx * dx + dy * dy);
                const double ang = std::atan2(dy, dx);
                const double w = std::exp(-(i * i + j * j) / denom);
                int bin = std::round(nb * (ang + M_PI) / kTwoPi);
                bin = (bin < nb) ? bin : 0;
                hist[bin] += w * mag;
            }
        }
        // in-place circular smoothing: h[i-1] is already smoothed (and h[0]
        // for i = nb-1) — Gauss-Seidel-like, sift.cpp:496-504.
        for (int it = 0; it < kSmoothIters; ++it)
            for (int i = 0; i < nb; ++i)
                hist[i] = 0.25 * hist[(i - 1 + nb) % nb] + 0.5 * hist[i] +
                          0.25 * hist[(i + 1) % nb];
        const double peak = *std::max_element(hist.begin(), hist.end());
        for (int i = 0; i < nb; ++i) {
            const double h0 = hist[(i - 1 + nb) % nb];
            const double h1 = hist[i];
            const double h2 = hist[(i + 1) % nb];
            if (h1 > h0 && h1 > h2 && h1 > (P.peak_ratio * peak)) {
                double fi = i + 0.5 * (h0 - h2) / (h0 - 2 * h1 + h2);
                fi = std::fmod(fi + nb, nb);
                double ori = kTwoPi * fi / nb;
                ori = std::fmod(ori + kTwoPi, kTwoPi);
                sift_kp k2 = kp;
                k2.pori = ori;
                if (P.double_image_size) {
                    k2.x /= 2;
                    k2.y /= 2;
                    k2.size /= 2;
                }
                R.oriented.push_back(k2);
            }
        }
    }
}

// Keypoint::operator< / operator== (sift.hh:25-41) and clean_keypoints
// (sift.cpp:20-24).
bool kp_less(const sift_kp& a, const sift_kp& b) {
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.pori != b.pori) return a.pori < b.pori;
    return a.octave > b.octave;
}
bool kp_equal(const sift_kp& a, const sift_kp& b) {
    return a.x == b.x && a.y == b.y && a.size == b.size && a.pori == b.pori;
}

// compute_descriptors + update_histogram + convert_hist_to_desc,
// sift.cpp:541-682.
void describe_all(Run& R) {
    const sift_params& P = R.p;
    R.desc_f32.assign(R.final_kps.size() * 128, 0.0f);
    for (size_t n = 0; n < R.final_kps.size(); ++n) {
        sift_kp& kp = R.final_kps[n];
        const Plane& img = R.gauss[kp.octave][kp.layer];
        const double inv = P.double_image_size ? (1.0 / std::pow(2, kp.octave - 1))
                                               : (1.0 / std::pow(2, kp.octave));
        const int x = kp.x * inv;  // truncation, sift.cpp:623-624
        const int y = kp.y * inv;
        const double size = kp.size * inv;
        const double bins_per_rad = kHistBins / kTwoPi;
        const double ca = std::cos(kp.pori), sa = std::sin(kp.pori);
        double hist[kHistW][kHistW][kHistBins];
        std::memset(hist, 0, sizeof hist);
        const double hw = P.desc_scale_factor * size;
        const double denom = 0.5 * kHistW * kHistW;
        const double rr = std::round(hw * 0.5 * std::sqrt(2.0) * (kHistW + 1.0) + 0.5);
        const int radius = std::min(rr, std::sqrt(img.w * img.w + img.h * img.h));
        for (int row = -radius; row <= radius; ++row) {
            for (int col = -radius; col <= radius; ++col) {
                const double row_rot = (col * sa + row * ca) / hw;
                const double col_rot = (col * ca - row * sa) / hw;
                const double rb = row_rot + kHistW / 2 - 0.5;
                const double cb = col_rot + kHistW / 2 - 0.5;
                if (!(rb > -1.0 && rb < kHistW && cb > -1.0 && cb < kHistW)) continue;
                const int ny = row + y, nx = col + x;
                if (!(nx > 0 && nx < (img.w - 1) && ny > 0 && ny < (img.h - 1))) continue;
                const double dx = img.at(nx + 1, ny) - img.at(nx - 1, ny);
                const double dy = img.at(nx, ny - 1) - img.at(nx, ny + 1);
                const double mag = std::sqrt(dx * dx + dy * dy);
                double ang = std::atan2(dy, dx);
                ang -= kp.pori;
                ang = std::fmod(std::fmod(ang, kTwoPi) + kTwoPi, kTwoPi);
                const double ob = ang * bins_per_rad;
                const double w = std::exp(-(row_rot * row_rot + col_rot * col_rot) / denom);
                const double m = mag * w;
                // trilinear split (update_histogram, sift.cpp:541-571)
                const int br = std::floor(rb), bc = std::floor(cb), bo = std::floor(ob);
                const double fr = rb - br, fc = cb - bc, fo = ob - bo;
                for (int r = 0; r <= 1; ++r) {
                    const int ri = br + r;
                    if (ri < 0 || ri >= kHistW) continue;
                    const double vr = m * ((r == 0) ? 1.0 - fr : fr);
                    for (int c = 0; c <= 1; ++c) {
                        const int ci = bc + c;
                        if (ci < 0 || ci >= kHistW) continue;
                        const double vc = vr * ((c == 0) ? 1.0 - fc : fc);
                        for (int q = 0; q <= 1; ++q) {
                            const int oi = (bo + q) % kHistBins;
                            hist[ri][ci][oi] += vc * ((q == 0) ? 1.0 - fo : fo);
                        }
                    }
                }
            }
        }
        // convert_hist_to_desc, sift.cpp:576-603.
        double* hv = &hist[0][0][0];
        double norm = 0.0;
        for (int i = 0; i < 128; ++i) norm += hv[i] * hv[i];
        norm = std::sqrt(norm);
        double ninv = 1.0 / norm;
        norm = 0.0;
        for (int i = 0; i < 128; ++i) {
            hv[i] *= ninv;
            if (hv[i] > kMagThr) hv[i] = kMagThr;
            norm += hv[i] * hv[i];
        }
        norm = std::sqrt(norm);
        ninv = 1.0 / norm;
        for (int i = 0; i < 128; ++i) {
            const double q = std::floor(kIntFactor * hv[i] * ninv);
            // NaN (all-zero histogram, Appendix A.17): the reference's
            // (int)NaN is INT_MIN on x86, min(.,255) keeps it and the uint8
            // cast yields 0 — made explicit here.
            int val = (q == q) ? (int)q : 0;
            if (val < 0) val = 0;
            kp.desc[i] = (uint8_t)std::min(val, 255);
            R.desc_f32[n * 128 + i] = (float)(hv[i] * ninv);
        }
    }
}

int run_pipeline(Run& R, const double* hwc, int w, int h, int c) {
    const sift_params& P = R.p;
    if (hwc == nullptr || w <= 0 || h <= 0) return SIFT_ERR_ARG;
    if (c != 1 && c != 3) return SIFT_ERR_CHANNELS;
    if (P.intervals < 1 || P.window_size < 1 || (int)P.num_bins < 1)
        return SIFT_ERR_PARAM;

    auto t0 = Clock::now();
    // compute_initial_image, sift.cpp:113-126
    Plane base;
    if (c != 1) {
        base = gray_of(hwc, w, h, c);
    } else {
        base = Plane(w, h);
        std::memcpy(base.v.data(), hwc, sizeof(double) * w * h);
    }
    if (P.double_image_size) base = upsample2(base);
    if (P.init_sigma * P.init_sigma - 1 <= 0) return SIFT_ERR_PARAM;
    base = blur(base, std::sqrt(P.init_sigma * P.init_sigma - 1));
    auto t1 = Clock::now();

    // compute_octaves_count, sift.cpp:132-137 (integer division by 3)
    const int q = std::min(base.w, base.h) / 3;
    if (q == 0) return SIFT_ERR_TOO_SMALL;
    R.octaves = std::floor(std::log2(q));
    if (P.max_octaves > 0 && R.octaves > P.max_octaves) R.octaves = P.max_octaves;
    if (R.octaves < 1) return SIFT_ERR_TOO_SMALL;
    R.sigmas = level_sigmas(P.init_sigma, P.intervals);
    R.n_gauss = P.intervals + 3;
    R.n_dog = P.intervals + 2;

    // compute_gaussian_images, sift.cpp:181-202
    R.gauss.assign(R.octaves, {});
    Plane cur = std::move(base);
    for (int o = 0; o < R.octaves; ++o) {
        std::vector<Plane>& L = R.gauss[o];
        L.resize(R.n_gauss);
        L[0] = cur;
        for (int i = 1; i < R.n_gauss; ++i) L[i] = blur(L[i - 1], R.sigmas[i]);
        if (!decimate2(L[R.n_gauss - 3], cur)) return SIFT_ERR_TOO_SMALL;
    }
    auto t2 = Clock::now();

    // compute_dog_images, sift.cpp:209-225
    R.dog.assign(R.octaves, {});
    for (int o = 0; o < R.octaves; ++o) {
        R.dog[o].resize(R.n_dog);
        for (int i = 0; i < R.n_dog; ++i) {
            const Plane& a = R.gauss[o][i + 1];
            const Plane& b = R.gauss[o][i];
            Plane d(a.w, a.h);
            for (size_t k = 0; k < d.v.size(); ++k) d.v[k] = a.v[k] - b.v[k];
            R.dog[o][i] = std::move(d);
        }
    }
    auto t3 = Clock::now();

    // detect_extrema, sift.cpp:300-319: the double threshold is passed into
    // an int parameter (sift.cpp:266).
    const int thr = (int)std::floor(0.5 * P.contrast_threshold /
                                    static_cast<double>(P.intervals) * 255.0);
    for (int o = 0; o < R.octaves; ++o) scan_extrema(R, o, thr);
    auto t4 = Clock::now();

    refine_all(R);
    auto t5 = Clock::now();
    orient_all(R);
    auto t6 = Clock::now();

    R.final_kps = R.oriented;
    std::sort(R.final_kps.begin(), R.final_kps.end(), kp_less);
    R.final_kps.erase(std::unique(R.final_kps.begin(), R.final_kps.end(), kp_equal),
                      R.final_kps.end());
    auto t7 = Clock::now();
    describe_all(R);
    auto t8 = Clock::now();

    R.t[0] = secs(t0, t1);
    R.t[1] = secs(t1, t2);
    R.t[2] = secs(t2, t3);
    R.t[3] = secs(t3, t4);
    R.t[4] = secs(t4, t5);
    R.t[5] = secs(t5, t6);
    R.t[6] = secs(t6, t7);
    R.t[7] = secs(t7, t8);
    return SIFT_OK;
}

}  // namespace

extern "C" {

void sift_cpu_params_default(sift_params* p);

void* sift_cpu_run(const double* hwc, int w, int h, int c, const sift_params* p,
                   int* status) {
    Run* R = new Run();
    if (p) {
        R->p = *p;
    } else {
        sift_cpu_params_default(&R->p);
    }
    const int st = run_pipeline(*R, hwc, w, h, c);
    if (status) *status = st;
    if (st != SIFT_OK) {
        delete R;
        return nullptr;
    }
    return R;
}

void sift_cpu_release(void* run) { delete static_cast<Run*>(run); }

int sift_cpu_octaves(void* run) { return static_cast<Run*>(run)->octaves; }
int sift_cpu_levels(void* run) { return static_cast<Run*>(run)->n_gauss; }

int sift_cpu_level(void* run, int o, int l, const double** data, int* w, int* h) {
    Run* R = static_cast<Run*>(run);
    if (o < 0 || o >= R->octaves || l < 0 || l >= R->n_gauss) return SIFT_ERR_ARG;
    const Plane& P = R->gauss[o][l];
    *data = P.v.data();
    *w = P.w;
    *h = P.h;
    return SIFT_OK;
}

size_t sift_cpu_extrema(void* run, const sift_extremum** out) {
    Run* R = static_cast<Run*>(run);
    *out = R->extrema.data();
    return R->extrema.size();
}

size_t sift_cpu_refined(void* run, const sift_kp** out, const double** off0) {
    Run* R = static_cast<Run*>(run);
    *out = R->refined.data();
    if (off0) *off0 = R->refined_off0.data();
    return R->refined.size();
}

size_t sift_cpu_oriented(void* run, const sift_kp** out) {
    Run* R = static_cast<Run*>(run);
    *out = R->oriented.data();
    return R->oriented.size();
}

size_t sift_cpu_final(void* run, const sift_kp** out, const float** desc_f32) {
    Run* R = static_cast<Run*>(run);
    *out = R->final_kps.data();
    if (desc_f32) *desc_f32 = R->desc_f32.data();
    return R->final_kps.size();
}

void sift_cpu_times(void* run, double* t8) {
    Run* R = static_cast<Run*>(run);
    for (int i = 0; i < 8; ++i) t8[i] = R->t[i];
}

// match_keypoints (reference sift.cpp:783-815) with euclid_dist
// (sift.cpp:688-695), same scan and update order: out_j[i] = index into k2 of
// the match of k1[i], or -1; out_d[i] = its best distance. Returns the match
// count. n2 == 0 gives no matches (the reference would read keypoints2[0]
// there when ratio > 1).
size_t sift_cpu_match(const sift_kp* k1, size_t n1, const sift_kp* k2, size_t n2, double ratio,
                      int* out_j, double* out_d) {
    size_t m = 0;
    for (size_t i = 0; i < n1; ++i) {
        double best = std::numeric_limits<double>::max();
        double second = std::numeric_limits<double>::max();
        size_t best_j = 0;
        for (size_t j = 0; j < n2; ++j) {
            double sum = 0.0;
            for (int t = 0; t < 128; ++t) {
                const int diff = (int)k1[i].desc[t] - (int)k2[j].desc[t];
                sum += diff * diff;
            }
            const double dist = std::sqrt(sum);
            if (dist < best) {
                second = best;
                best = dist;
                best_j = j;
            } else if (dist < second) {
                second = dist;
            }
        }
        const bool ok = n2 > 0 && best < ratio * second;
        out_j[i] = ok ? (int)best_j : -1;
        out_d[i] = best;
        m += ok;
    }
    return m;
}

// Same defaults as the product library (reference sift.hh:65-71); defined
// here too so the oracle library is self-contained.
void sift_cpu_params_default(sift_params* p) {
    std::memset(p, 0, sizeof *p);
    p->double_image_size = 1;
    p->intervals = 3;
    p->window_size = 3;
    p->max_octaves = 0;
    p->init_sigma = 1.6;
    p->contrast_threshold = 0.04;
    p->eigen_ratio = 10.0;
    p->num_bins = 36;
    p->peak_ratio = 0.8;
    p->ori_sigma_factor = 1.5;
    p->desc_scale_factor = 3.0;
    p->write_keypoints_png = 0;
}

}  // extern "C"
