// sift_api.cpp — the C++ drop-in for the reference's src/sift.cpp.
//
// Implements the four functions declared in include/sift.hh (reference
// sift.hh:65-81). detect_keypoints_and_descriptors forwards to the HIP
// pipeline through the C-ABI (include/sift_hip.h) and rethrows failures as
// std::runtime_error; the rest are host-side helpers kept for the
// reference's CLI (main.cpp:14-18). Image's own members (stb I/O, drawing)
// come from the reference's image_io.cpp / image.cpp, which stay in the
// consumer's build.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "sift.hh"
#include "sift_hip.h"

static_assert(sizeof(Keypoint) == sizeof(sift_kp), "Keypoint must match sift_kp");
static_assert(std::is_standard_layout<Keypoint>::value, "Keypoint must be standard layout");
static_assert(offsetof(Keypoint, desc) == offsetof(sift_kp, desc), "desc offset");
static_assert(offsetof(Keypoint, pori) == offsetof(sift_kp, pori), "pori offset");

namespace {

struct CtxHolder {
    sift_ctx* ctx = nullptr;
    ~CtxHolder() {
        if (ctx) sift_hip_destroy(ctx);
    }
};

// One context per host thread (a context owns one HIP stream).
sift_ctx* thread_context() {
    thread_local CtxHolder holder;
    if (!holder.ctx) {
        const char* dev = std::getenv("SIFT_AMD_DEVICE");
        const int st = sift_hip_create(dev ? std::atoi(dev) : 0, &holder.ctx);
        if (st != SIFT_OK)
            throw std::runtime_error(std::string("sift_hip_create: ") + sift_hip_strerror(st));
    }
    return holder.ctx;
}

bool env_flag(const char* name, bool dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    return !(v[0] == '0' && v[1] == '\0');
}

}  // namespace

std::vector<Keypoint> detect_keypoints_and_descriptors(
    const Image& img, const bool double_image_size, const double init_sigma,
    const int intervals, const int window_size, const double contrast_threshold,
    const double eigen_ratio, const double num_bins, const double peak_ratio,
    const double ori_sigma_factor, const double desc_scale_factor) {
    if (img.channels != 1 && img.channels != 3)
        throw std::runtime_error("detect_keypoints_and_descriptors: channels must be 1 or 3");
    sift_params p;
    sift_params_default(&p);
    p.double_image_size = double_image_size ? 1 : 0;
    p.init_sigma = init_sigma;
    p.intervals = intervals;
    p.window_size = window_size;
    p.contrast_threshold = contrast_threshold;
    p.eigen_ratio = eigen_ratio;
    p.num_bins = num_bins;
    p.peak_ratio = peak_ratio;
    p.ori_sigma_factor = ori_sigma_factor;
    p.desc_scale_factor = desc_scale_factor;

    // one job: the Image buffer goes up through pinned staging (as bytes when
    // it holds stb-decoded integers), and the sorted records are copied once,
    // straight into the returned vector
    sift_ctx* ctx = thread_context();
    const void* src = img.data.data();
    int ticket = 0;
    size_t n = 0;
    int st = sift_hip_submit(ctx, &src, 1, SIFT_INPUT_F64_HOST, img.width, img.height,
                             img.channels, &p, 0, &ticket);
    if (st == SIFT_OK) st = sift_hip_wait(ctx, ticket, nullptr, &n);
    std::vector<Keypoint> out;
    if (st == SIFT_OK) {
        out.resize(n);
        st = sift_hip_fetch(ctx, ticket, reinterpret_cast<sift_kp*>(out.data()), nullptr);
    }
    if (st != SIFT_OK)
        throw std::runtime_error(std::string("detect_keypoints_and_descriptors: ") +
                                 sift_hip_strerror(st));

    // the reference writes keypoints.png on every call (sift.cpp:765-768)
    if (env_flag("SIFT_AMD_KEYPOINTS_PNG", true)) {
        Image canvas(img);
        draw_keypoints(canvas, out, intervals + 3);
        canvas.save("keypoints.png");
    }
    return out;
}

// 2-NN ratio test (reference sift.cpp:688-695, 783-815) on the GPU matcher
// (sift_hip_match, csrc/sift_match.hip): same matches, same order, same
// distances; KeypointMatch copies the records as the reference does.
std::vector<KeypointMatch> match_keypoints(const std::vector<Keypoint>& keypoints1,
                                           const std::vector<Keypoint>& keypoints2,
                                           double ratio_threshold) {
    std::vector<KeypointMatch> matches;
    sift_match_pair* pairs = nullptr;
    size_t n = 0;
    const int st = sift_hip_match(
        thread_context(), reinterpret_cast<const sift_kp*>(keypoints1.data()), keypoints1.size(),
        reinterpret_cast<const sift_kp*>(keypoints2.data()), keypoints2.size(), ratio_threshold,
        &pairs, &n);
    if (st != SIFT_OK)
        throw std::runtime_error(std::string("match_keypoints: ") + sift_hip_strerror(st));
    std::unique_ptr<sift_match_pair, void (*)(void*)> guard(pairs, sift_hip_free);
    matches.reserve(n);
    for (size_t k = 0; k < n; ++k)
        matches.emplace_back(keypoints1[pairs[k].i1], keypoints2[pairs[k].i2], pairs[k].distance);
    return matches;
}

// Circle + orientation tick per keypoint, radius growing with the layer
// (reference sift.cpp:821-844).
void draw_keypoints(Image& img, const std::vector<Keypoint>& keypoints, double scales_count) {
    static const int palette[] = {RED, GREEN, BLUE, YELLOW, MAGENTA, CYAN, BLACK};
    const double r_max = 110, r_min = 5;
    for (const Keypoint& kp : keypoints) {
        const int cx = kp.x, cy = kp.y;
        const int radius = r_min * std::exp(kp.layer / (scales_count - 1) * std::log(r_max / r_min));
        const int color = palette[kp.layer % 7];
        img.draw_circle(cx, cy, radius, color);
        const int ex = cx + radius * std::cos(kp.pori);
        const int ey = cy + radius * std::sin(kp.pori);
        img.draw_line(cx, cy, ex, ey, color);
    }
}

// Side-by-side canvas with one line per match, saved as matches.png
// (reference sift.cpp:850-876).
void draw_matches(const Image& a, const Image& b, std::vector<KeypointMatch> matches) {
    Image canvas(a.width + b.width, std::max(a.height, b.height), 3);
    auto blit = [&](const Image& src, int x_off) {
        for (int x = 0; x < src.width; ++x)
            for (int y = 0; y < src.height; ++y) {
                canvas.set_pixel(x_off + x, y, R, src.get_pixel(x, y, R));
                canvas.set_pixel(x_off + x, y, G, src.get_pixel(x, y, src.channels == 3 ? G : R));
                canvas.set_pixel(x_off + x, y, B, src.get_pixel(x, y, src.channels == 3 ? B : R));
            }
    };
    blit(a, 0);
    blit(b, a.width);
    for (const KeypointMatch& m : matches)
        canvas.draw_line(m.kp1.x, m.kp1.y, a.width + m.kp2.x, m.kp2.y);
    canvas.save("matches.png");
}
