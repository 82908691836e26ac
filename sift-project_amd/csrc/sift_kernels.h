// sift_kernels.h — device-side types and launch entry points shared by the
// kernels (sift_kernels.hip) and the C-ABI host layer (sift_ctx.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/sift_hip.h"

namespace sift_amd {

// Algorithm constants of the reference (sift.hh:5-13).
constexpr int kMaxSteps = 5;        // MAX_CONVERGENCE_STEPS
constexpr double kConvThr = 0.5;    // CONVERGENCE_THR
constexpr int kSmoothIters = 2;     // ORI_SMOOTH_ITERATIONS
constexpr int kDescW = 4;           // DESC_HIST_WIDTH
constexpr int kDescBins = 8;        // DESC_HIST_BINS
constexpr double kMagThr = 0.2;     // DESC_MAGNITUDE_THR
constexpr double kIntFactor = 512.0;  // INT_DESCR_FCTR

constexpr int kMaxOctaves = 16;   // floor(log2(min/3)) < 16 for any int image
constexpr int kMaxLevels = 12;    // intervals + 3 with intervals <= 9
constexpr int kMaxTemplR = 24;    // widest register-window blur kernel
constexpr int kMaxTaps = 64;      // generic path: kernels up to 64 taps
constexpr int kMaxBins = 256;     // orientation bins supported

// Half kernel of apply_gaussian_blur_fast (image.cpp:226-235) plus its
// normalising sum (image.cpp:171-185), computed on the host with glibc.
struct BlurTaps {
    double k[kMaxTaps];
    double sum_w;
    int R;  // taps k[0..R], R = ks-1
    int pad;
};

// Device-resident table of pyramid level planes.
struct PyrTable {
    double* lvl[kMaxOctaves][kMaxLevels];
    int w[kMaxOctaves];
    int h[kMaxOctaves];
};

// Scalar parameters of detect_keypoints_and_descriptors as the kernels need
// them (sift.hh:65-71, threshold per sift.cpp:305-307).
struct DevParams {
    int intervals;
    int window_size;
    int num_bins;
    int double_image;
    int threshold;
    int n_dog;
    int n_gauss;
    int octaves;
    double init_sigma;
    double contrast_threshold;
    double eigen_ratio;
    double peak_ratio;
    double ori_sigma_factor;
    double desc_scale_factor;
};

// Refined keypoint before orientation (sift.cpp:419-430) plus the scale
// offset, which the host needs to recompute size with glibc pow.
struct RawKp {
    double x, y, size, off0;
    int octave, layer;
};

int blur_rows_for(int W, int H, int R);

hipError_t launch_prepare(const double* in, int w, int h, int c, int dbl, double* out,
                          int W0, int H0, hipStream_t s);
hipError_t launch_blur(const double* src, double* dst, int W, int H, const BlurTaps& taps,
                       double* dec, int Wd, int Hd, double* tmp, hipStream_t s);
hipError_t launch_extrema(const PyrTable* d_pt, int o, int W, int H, int n_gauss,
                          int window_size, int thr, sift_extremum* out, unsigned* counter,
                          unsigned cap, hipStream_t s);
hipError_t launch_refine(const PyrTable* d_pt, const DevParams& P,
                         const sift_extremum* cand, const unsigned* n_cand, unsigned cap_cand,
                         RawKp* out, unsigned* n_out, unsigned cap_out, hipStream_t s);
hipError_t launch_orient(const PyrTable* d_pt, const DevParams& P, const RawKp* raw,
                         const unsigned* n_raw, unsigned cap_raw, sift_kp* out,
                         double* out_off0, unsigned* n_out, unsigned cap_out,
                         hipStream_t s);
hipError_t launch_descriptor(const PyrTable* d_pt, const DevParams& P, sift_kp* recs,
                             const unsigned* n, unsigned cap, float* desc_f32,
                             hipStream_t s);

}  // namespace sift_amd
