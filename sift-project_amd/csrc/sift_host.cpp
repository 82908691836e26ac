// sift_host.cpp — glibc-exact host math of the pipeline (see sift_host.h).
// Built with g++ -ffp-contract=off, never with hipcc/clang.
#include "sift_host.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

namespace sift_amd {

namespace {

// apply_gaussian_blur_fast kernel construction (image.cpp:226-235) and the
// running sum_w of apply_double_convolution_1d (image.cpp:171-185), which is
// the same sequence for every pixel and therefore a per-kernel constant.
bool make_taps(double sigma, BlurTaps* t) {
    const double ks_d = std::ceil(3 * sigma);
    if (!(ks_d >= 0) || ks_d + 1 > kMaxTaps) return false;
    const int ks = (int)ks_d + 1;
    std::memset(t, 0, sizeof *t);
    const double exp_denom = 2 * sigma * sigma;
    const double coef = 1 / (std::sqrt(2 * M_PI) * sigma);
    for (int i = 0; i < ks; ++i) t->k[i] = std::exp(-i * i / exp_denom) * coef;
    double s = t->k[0];
    for (int u = 1; u < ks; ++u) s += 2.0 * t->k[u];
    t->sum_w = s;
    // RN(1/sum_w): the kernels divide by sum_w with Markstein's correction
    // (q = a*inv; r = fma(-q, sum_w, a); q + r*inv), correctly rounded
    t->inv = 1.0 / s;
    t->R = ks - 1;
    return true;
}

}  // namespace

int host_plan(const sift_params* p, int w, int h, int c, Geometry* g, BlurTaps* taps_init,
              BlurTaps* taps, DevParams* dp) {
    if (w <= 0 || h <= 0) return SIFT_ERR_ARG;
    if (c != 1 && c != 3) return SIFT_ERR_CHANNELS;
    if (p->intervals < 1 || p->intervals + 3 > kMaxLevels) return SIFT_ERR_PARAM;
    if (p->window_size < 2 || p->window_size / 2 > 3) return SIFT_ERR_PARAM;
    const int nb = (int)p->num_bins;
    if (nb < 1 || nb > kMaxBins) return SIFT_ERR_PARAM;
    if (!(p->init_sigma * p->init_sigma - 1 > 0)) return SIFT_ERR_PARAM;
    if (p->max_octaves < 0) return SIFT_ERR_PARAM;

    const int W0 = p->double_image_size ? 2 * w : w;
    const int H0 = p->double_image_size ? 2 * h : h;
    // compute_octaves_count (sift.cpp:132-137): integer division by 3
    const int q = std::min(W0, H0) / 3;
    if (q == 0) return SIFT_ERR_TOO_SMALL;
    int octaves = std::floor(std::log2(q));
    if (p->max_octaves > 0 && octaves > p->max_octaves) octaves = p->max_octaves;
    if (octaves < 1 || octaves > kMaxOctaves) return SIFT_ERR_TOO_SMALL;
    *g = Geometry();
    g->octaves = octaves;
    g->n_gauss = p->intervals + 3;
    int Wo = W0, Ho = H0;
    size_t off = 0;
    for (int o = 0; o < octaves; ++o) {
        // the reference decimates after every octave and throws below 2x2
        // (image.cpp:42-44, sift.cpp:195)
        if (Wo < 2 || Ho < 2) return SIFT_ERR_TOO_SMALL;
        g->W[o] = Wo;
        g->H[o] = Ho;
        g->sum_px += (size_t)Wo * Ho;
        for (int l = 0; l < g->n_gauss; ++l) {
            g->offs[o][l] = off;
            off += (size_t)Wo * Ho;
        }
        Wo /= 2;
        Ho /= 2;
    }
    g->total = off;

    // compute_gaussian_kernels (sift.cpp:143-155)
    std::vector<double> sig(g->n_gauss);
    sig[0] = p->init_sigma;
    const double k = std::pow(2.0, 1.0 / p->intervals);
    for (int i = 1; i < g->n_gauss; ++i) {
        const double prev = (std::pow(k, i - 1)) * p->init_sigma;
        sig[i] = prev * std::sqrt(k * k - 1);
    }
    // compute_initial_image's blur sigma (sift.cpp:124)
    if (!make_taps(std::sqrt(p->init_sigma * p->init_sigma - 1), taps_init))
        return SIFT_ERR_PARAM;
    for (int i = 1; i < g->n_gauss; ++i)
        if (!make_taps(sig[i], &taps[i])) return SIFT_ERR_PARAM;

    dp->intervals = p->intervals;
    dp->window_size = p->window_size;
    dp->num_bins = nb;
    dp->double_image = p->double_image_size ? 1 : 0;
    // detect_extrema: the double threshold is passed into an int parameter
    // (sift.cpp:266, 305-307)
    dp->threshold = (int)std::floor(0.5 * p->contrast_threshold /
                                    static_cast<double>(p->intervals) * 255.0);
    dp->n_dog = p->intervals + 2;
    dp->n_gauss = g->n_gauss;
    dp->octaves = octaves;
    dp->init_sigma = p->init_sigma;
    dp->contrast_threshold = p->contrast_threshold;
    dp->eigen_ratio = p->eigen_ratio;
    dp->peak_ratio = p->peak_ratio;
    dp->ori_sigma_factor = p->ori_sigma_factor;
    dp->desc_scale_factor = p->desc_scale_factor;
    return SIFT_OK;
}

namespace {

// image, then Keypoint::operator< (sift.hh:31-41): x asc, y asc, size desc,
// pori asc, octave desc
bool key_less(const FinalizeKey& a, const FinalizeKey& b) {
    if (a.img != b.img) return a.img < b.img;
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.pori != b.pori) return a.pori < b.pori;
    return a.octave > b.octave;
}

}  // namespace

void host_sort_run(const sift_kp* recs, const RecSide* side, unsigned b, unsigned e,
                   FinalizeKey* out, FinalizeWorkspace* ws) {
    // Sort a compact key array (48 B per record) by (image, Keypoint::
    // operator<). x >= 0 for every keypoint, and bucket(x) = x / x_max * B
    // is monotone non-decreasing under round-to-nearest, so a stable pass
    // over the buckets (image-major, then x) followed by a comparator sort
    // inside each (tiny) bucket yields exactly the order std::sort with the
    // full comparator would, in O(n + buckets).
    using Key = FinalizeKey;
    const unsigned n = e - b;
    std::vector<Key>& keys = ws->keys;
    keys.resize(n);
    double x_max = 0.0;
    int img_max = 0;
    for (unsigned i = 0; i < n; ++i) {
        const sift_kp& r = recs[b + i];
        const int im = side[b + i].img;
        keys[i] = {r.x, r.y, r.size, r.pori, r.octave, im, b + i};
        x_max = std::max(x_max, r.x);
        img_max = std::max(img_max, im);
    }
    const size_t n_img = (size_t)img_max + 1;
    const size_t B = std::max<size_t>(1, std::min<size_t>(n, (size_t)1 << 20) / n_img);
    std::vector<unsigned>& start = ws->start;
    start.assign(n_img * B + 1, 0);
    auto bucket = [&](const Key& k) -> size_t {
        size_t xb = 0;
        if (x_max > 0.0) {
            const double f = k.x / x_max * (double)B;
            xb = f >= (double)(B - 1) ? B - 1 : (f <= 0.0 ? 0 : (size_t)f);
        }
        return (size_t)k.img * B + xb;
    };
    for (unsigned i = 0; i < n; ++i) ++start[bucket(keys[i]) + 1];
    for (size_t q = 0; q < n_img * B; ++q) start[q + 1] += start[q];
    {
        std::vector<unsigned>& fill = ws->fill;
        fill.assign(start.begin(), start.end() - 1);
        for (unsigned i = 0; i < n; ++i) out[fill[bucket(keys[i])]++] = keys[i];
    }
    for (size_t q = 0; q < n_img * B; ++q) {
        Key* lo = out + start[q];
        Key* hi = out + start[q + 1];
        if (hi - lo > 1) std::sort(lo, hi, key_less);
    }
}

size_t host_merge_unique(FinalizeKey* keys, const std::vector<unsigned>& run_start,
                         unsigned* keep, size_t* per_img, FinalizeWorkspace* ws) {
    // pairwise merges of the sorted runs [run_start[i], run_start[i+1])
    std::vector<unsigned> bounds(run_start);
    const unsigned n = bounds.empty() ? 0 : bounds.back();
    std::vector<FinalizeKey>& tmp = ws->sorted;
    tmp.resize(n);
    FinalizeKey* src = keys;
    FinalizeKey* dst = tmp.data();
    while (bounds.size() > 2) {
        std::vector<unsigned> nb;
        nb.push_back(0);
        size_t i = 0;
        for (; i + 2 < bounds.size(); i += 2) {
            std::merge(src + bounds[i], src + bounds[i + 1], src + bounds[i + 1],
                       src + bounds[i + 2], dst + bounds[i], key_less);
            nb.push_back(bounds[i + 2]);
        }
        if (i + 1 < bounds.size()) {  // odd run out: carried over
            std::copy(src + bounds[i], src + bounds[i + 1], dst + bounds[i]);
            nb.push_back(bounds[i + 1]);
        }
        bounds.swap(nb);
        std::swap(src, dst);
    }
    size_t m = 0;
    const FinalizeKey* last = nullptr;
    for (unsigned i = 0; i < n; ++i) {
        const FinalizeKey& k = src[i];
        // std::unique compares with the last kept element (Keypoint::
        // operator==, sift.hh:25-27: x, y, size, pori), within one image
        if (last && last->img == k.img && last->x == k.x && last->y == k.y &&
            last->size == k.size && last->pori == k.pori)
            continue;
        keep[m++] = k.idx;
        if (per_img) ++per_img[k.img];
        last = &k;
    }
    return m;
}

size_t host_finalize(const sift_params* p, sift_kp* recs, const RecSide* side, unsigned n,
                     unsigned* keep, size_t* per_img, FinalizeWorkspace* ws) {
    ws->all.resize(n);
    host_sort_run(recs, side, 0, n, ws->all.data(), ws);
    return host_merge_unique(ws->all.data(), {0u, n}, keep, per_img, ws);
}

}  // namespace sift_amd
