// sift.hh — public API of the MI355X SIFT extractor; drop-in for
// ahmedhassayoune/sift-project src/sift.hh (same macros, same Keypoint and
// KeypointMatch types, same four functions with the same defaults), so the
// reference's main.cpp and stitching flow build unchanged against
// libsift_amd.so.
#pragma once

#include <cstdint>
#include <ostream>
#include <vector>

#include "image.hh"

// algorithm constants (reference sift.hh:5-13)
#define M_PI2 6.283185307179586
#define MAX_CONVERGENCE_STEPS 5
#define CONVERGENCE_THR 0.5
#define ORI_SMOOTH_ITERATIONS 2
#define DESC_HIST_WIDTH 4
#define DESC_HIST_BINS 8
#define DESC_MAGNITUDE_THR 0.2
#define INT_DESCR_FCTR 512.0

// One keypoint (reference sift.hh:15-53). Standard layout, 168 bytes,
// identical to sift_kp of the C-ABI (include/sift_hip.h).
struct Keypoint {
    double x;           // input-image x
    double y;           // input-image y
    int octave;
    int layer;          // DoG layer, also the Gaussian level described
    double size;
    double pori;        // principal orientation, radians in [0, 2 pi)
    uint8_t desc[128];  // 4x4x8 gradient histogram, quantised

    // equality ignores octave and layer (reference sift.hh:25-27)
    bool operator==(const Keypoint& o) const {
        return x == o.x && y == o.y && size == o.size && pori == o.pori;
    }
    bool operator!=(const Keypoint& o) const { return !(*this == o); }
    // x asc, y asc, size desc, pori asc, octave desc (reference sift.hh:31-41)
    bool operator<(const Keypoint& o) const {
        if (x != o.x) return x < o.x;
        if (y != o.y) return y < o.y;
        if (size != o.size) return size > o.size;
        if (pori != o.pori) return pori < o.pori;
        return octave > o.octave;
    }
    bool operator>(const Keypoint& o) const { return o < *this; }
    bool operator<=(const Keypoint& o) const { return !(o < *this); }
    bool operator>=(const Keypoint& o) const { return !(*this < o); }

    friend std::ostream& operator<<(std::ostream& os, const Keypoint& kp) {
        return os << "Keypoint: x=" << kp.x << ", y=" << kp.y << ", octave=" << kp.octave
                  << ", size=" << kp.size << ", layer=" << kp.layer
                  << ", porientation=" << kp.pori;
    }
};

struct KeypointMatch {
    Keypoint kp1;
    Keypoint kp2;
    double distance;

    KeypointMatch(const Keypoint& a, const Keypoint& b, double d)
        : kp1(a), kp2(b), distance(d) {}
};

// Detect and describe (reference sift.hh:65-71). Runs on the HIP device
// selected by $SIFT_AMD_DEVICE (default 0). Like the reference it writes
// keypoints.png in the working directory unless $SIFT_AMD_KEYPOINTS_PNG=0.
// Throws std::runtime_error on failure.
std::vector<Keypoint> detect_keypoints_and_descriptors(
    const Image& img, const bool double_image_size = true, const double init_sigma = 1.6,
    const int intervals = 3, const int window_size = 3,
    const double contrast_threshold = 0.04, const double eigen_ratio = 10.0,
    const double num_bins = 36, const double peak_ratio = 0.8,
    const double ori_sigma_factor = 1.5, const double desc_scale_factor = 3.0);

// Brute-force 2-NN ratio-test matcher (reference sift.hh:73-75).
std::vector<KeypointMatch> match_keypoints(const std::vector<Keypoint>& keypoints1,
                                           const std::vector<Keypoint>& keypoints2,
                                           double ratio_threshold = 0.75);

void draw_keypoints(Image& img, const std::vector<Keypoint>& keypoints, double scales_count);

void draw_matches(const Image& a, const Image& b, std::vector<KeypointMatch> matches);
