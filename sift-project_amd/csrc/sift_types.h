// sift_types.h — plain-C++ types shared by the HIP kernels, the HIP host
// layer and the g++-compiled reference-math layer (sift_host.cpp). No HIP
// headers here, so sift_host.cpp can be built by the same compiler family as
// the reference (g++), which matters for glibc-exact host math.
#pragma once

#include <cstddef>
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

// k_descriptor_split: replicas of the 4x4x8 f64 histogram per wave (power
// of two <= 16) and the waves per SIMD it is compiled for (= workgroups of
// 4 waves per CU; the host sizes a chip-filling grid from it). 4: 128 VGPRs
// with 6 spilled outside the sample loop, 4 x 39 KB of LDS per CU; against
// 3 (149 VGPRs): alone 156 -> 152.5 us per 1080p image, the driver's
// command -1.7 % (r05_v)
#ifndef SIFT_DSPLIT_REPS
#define SIFT_DSPLIT_REPS 8
#endif
#ifndef SIFT_DSPLIT_OCC
#define SIFT_DSPLIT_OCC (SIFT_DSPLIT_REPS >= 16 ? 2 : 4)
#endif
constexpr int kMaxOctaves = 16;   // floor(log2(min/3)) < 16 for any int image
constexpr int kOctBits = 4;       // sift_extremum.octave = o | image << kOctBits
constexpr int kMaxImages = 16;    // images of one job (one batched launch each)
constexpr int kMaxLevels = 12;    // intervals + 3 with intervals <= 9
constexpr int kMaxTemplR = 16;    // widest register-window blur kernel (the
                                  // NW-unrolled body stops unrolling past 16)
constexpr int kMaxTaps = 64;      // generic path: kernels up to 64 taps
constexpr int kMaxBins = 256;     // orientation bins supported
// octaves of at most this many pixels run LDS-resident: level + temporary +
// quarter-size next base + every level's staged taps (kMaxLevels x
// kLdsTapStride doubles: k[0..kMaxTemplR], sum_w, 1/sum_w) =
// (2.25 * 8960 + 228) * 8 B = 163,104 B of the 163,840 B LDS
constexpr int kLdsOctavePx = 8960;
constexpr int kLdsTapStride = kMaxTemplR + 3;
// ... by default only octaves of at most this many pixels run there (1080p:
// 60x33 and smaller; 120x67 as per-level tile launches on several CUs:
// -2.5 % pipelined, 76 -> 23 + 48 us alone, round 4)
constexpr int kLdsOctaveMaxPx = 2100;
constexpr size_t kLdsOctaveBytes =
    (2 * (size_t)kLdsOctavePx + kLdsOctavePx / 4 + (size_t)kMaxLevels * kLdsTapStride) *
    sizeof(double);
// planes live in LDS with an odd row stride (W | 1 doubles: lane-per-row
// accesses spread over the banks); an octave fits when its level and the
// next octave's base do
inline constexpr bool lds_octave_fits(int W, int H) {
    return (size_t)(W | 1) * H <= (size_t)kLdsOctavePx &&
           (size_t)((W / 2) | 1) * (H / 2) <= (size_t)kLdsOctavePx / 4;
}

// Half kernel of apply_gaussian_blur_fast (image.cpp:226-235) plus its
// normalising sum (image.cpp:171-185), computed on the host with glibc.
// Age priority of a job's kernels (SIFT_AGE_PRIO): the kernel raises its
// waves' issue priority by how close its job is to the oldest in flight,
// rank = ticket - 1 - *done (done: jobs of the context completed so far)
struct JobPrio {
    const unsigned* done;  // nullptr: off
    int ticket;
    int pad;
};

struct BlurTaps {
    double k[kMaxTaps];
    double sum_w;
    double inv;  // RN(1 / sum_w), for the correctly rounded division
    int R;  // taps k[0..R], R = ks-1
    int pad;
    JobPrio jp;
};

// What k_blur stages rows from: a W x H plane (p, with w = W), or the input
// image (p = HWC doubles of w x h x c) for the fused initial blur. Image b of
// a batched launch (blockIdx.z) reads p + b * bstride.
struct BlurSource {
    const double* p;
    size_t bstride;
    int w, h, c;
};

// Device-resident table of pyramid level planes of image 0 of a job; image b
// has the same layout img_stride doubles further (one arena per job).
struct PyrTable {
    double* lvl[kMaxOctaves][kMaxLevels];
    int w[kMaxOctaves];
    int h[kMaxOctaves];
    size_t img_stride;
    int n_img;
    int n_oct;
    JobPrio jp;
};

// Octaves in flight (k_octaves_flow): the levels of consecutive small
// octaves in ONE launch, 64 x 32 tiles as k_blur_tile, each tile started as
// soon as the rows it reads exist. Group i = one (octave, level >= 1) of every
// image: tasks [first, next group's first), ordered (band, image, tile);
// band counters at ctr[cnt + image * nby + band] count its finished tiles.
// dep: the group whose plane it reads (-1: written before the launch);
// dep_dec: that plane is the decimated one (2x the rows).
constexpr int kFlowMaxGroups = 48;
constexpr int kFlowMaxR = 12;  // radii the flow kernel instantiates
struct FlowGroup {
    int o, l, W, H, nbx, nby;
    int first, cnt;
    int dep, dep_dec, dec;
};
struct FlowGrid {
    int n_groups, total, n_img;
    int err;  // ctr word set when a dependency wait gave up (never expected)
    FlowGroup g[kFlowMaxGroups];
};

// Streaming extrema tasks: centre columns per wavefront strip (64 lanes
// minus the two halo lanes); centre rows per task are chosen per octave.
constexpr int kExtSpan = 62;

// Flattened tile grid of one extrema launch over a set of octaves: entry i
// (octave oct[i]) owns blocks [first_tile[i], first_tile[i+1]), tiles_x[i]
// tiles of 64 centre columns per band of 16 centre rows; blockIdx.y = image.
// (k_extrema_stream: "tiles" are tasks, tiles_x = strips of kExtSpan columns,
// each task seg[i] centre rows of one strip.)
struct ExtremaGrid {
    int n;
    int oct[kMaxOctaves];
    int tiles_x[kMaxOctaves];
    int seg[kMaxOctaves];  // k_extrema_stream: centre rows per task
    int first_tile[kMaxOctaves + 1];
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
// offset, which the host needs to recompute size with glibc pow, and the
// image of the job it belongs to.
struct RawKp {
    double x, y, size, off0;
    int octave, layer;
    int img, pad;
};

// Per-record side data next to the 168-B records: the scale offset (host
// size with glibc pow) and the image of the job.
struct RecSide {
    double off0;
    int img, pad;
};

// One final record for the device-side gather (sift_hip_fetch_device):
// its index in the job's device record array and its glibc-exact size.
struct GatherItem {
    double size;
    unsigned src;
    unsigned pad;
};

// Where k_descriptor also writes each finished record (mapped, coherent
// pinned host memory), so the host can finalise a keypoint batch while the
// device works on the next: rec/side index = record index (< cap), cnt =
// this launch's [begin, end) record range followed by the lane's live
// counters (candidates, refined keypoints, records) read from `live`, so the
// host has a job's counters when its last chains complete (no copy back).
constexpr int kExportCntWords = 5;
struct ExportSink {
    sift_kp* rec;
    RecSide* side;
    unsigned* cnt;
    unsigned cap;
    const unsigned* live;  // the lane's counters (with cnt)
};

}  // namespace sift_amd
