// sift_host.h — host-side reference math of the pipeline (sift_host.cpp).
//
// Everything here is computed with glibc libm in the reference's expression
// order and must be compiled with g++ (like the reference, Makefile:2,5):
// clang/LLVM rewrites pow(2.0, x) into exp2(x) even without fast-math, and
// glibc's exp2 and pow disagree in the last bit for rare arguments.
#pragma once

#include <cstddef>
#include <functional>
#include <vector>

#include "sift_types.h"

namespace sift_amd {

struct Geometry {
    int octaves = 0;
    int n_gauss = 0;
    int W[kMaxOctaves] = {0};
    int H[kMaxOctaves] = {0};
    size_t offs[kMaxOctaves][kMaxLevels] = {{0}};
    size_t total = 0;   // doubles in the pyramid
    size_t sum_px = 0;  // sum over octaves of W*H
};

// Octave geometry (sift.cpp:132-137, image.cpp:41-45), level sigmas
// (sift.cpp:143-155), blur taps (image.cpp:226-235), extremum threshold
// (sift.cpp:305-307) and parameter validation.
int host_plan(const sift_params* p, int w, int h, int c, Geometry* g, BlurTaps* taps_init,
              BlurTaps* taps, DevParams* dp);

// clean_keypoints (sift.cpp:20-24) in pieces, so a detect can sort the
// records of each keypoint batch while the device still works on the next:
// host_sort_run sorts the keys of records [b, e) into out[0, e-b) by image,
// then Keypoint::operator< (sift.hh:31-41); host_merge_unique merges
// consecutive sorted runs of `keys` (boundaries run_start, last = total) and
// applies std::unique (sift.hh:25-27) within each image, writing the kept
// record indices to keep[] (image-major) and counting them per image.
struct FinalizeKey {
    double x, y, size, pori;
    int octave;
    int img;
    unsigned idx;
};
struct FinalizeWorkspace {  // reused across calls
    std::vector<FinalizeKey> keys, sorted, all;
    std::vector<unsigned> start, fill;
};
void host_sort_run(const sift_kp* recs, const RecSide* side, unsigned b, unsigned e,
                   FinalizeKey* out, FinalizeWorkspace* ws);
size_t host_merge_unique(FinalizeKey* keys, const std::vector<unsigned>& run_start,
                         unsigned* keep, size_t* per_img, FinalizeWorkspace* ws);
// all of it over records [0, n): one run, merge/unique (the records carry
// the device's glibc-exact size, sift_pow2.h)
size_t host_finalize(const sift_params* p, sift_kp* recs, const RecSide* side, unsigned n,
                     unsigned* keep, size_t* per_img, FinalizeWorkspace* ws);

// Parallel host pass of the u8 upload path: dst[i] = (uint8_t)src[i] for
// every i when each src[i] is exactly an integer 0..255 (+0.0 only), which
// is what an stb-decoded Image holds (image_io.cpp:20-35); returns false
// (dst unspecified) otherwise.
bool host_pack_u8(const double* src, size_t n, uint8_t* dst);
// copies n doubles (host pool); false when any of them is NaN or infinite
bool host_copy_finite(const double* src, size_t n, double* dst);

// fn(t) for t in [0, n_tasks) on the same persistent host threads (the
// caller included); returns when all are done
void host_parallel(unsigned n_tasks, const std::function<void(unsigned)>& fn);

}  // namespace sift_amd
