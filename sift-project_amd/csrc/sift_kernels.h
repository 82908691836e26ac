// sift_kernels.h — device-side types and launch entry points shared by the
// kernels (sift_kernels.hip) and the C-ABI host layer (sift_ctx.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "sift_types.h"

namespace sift_amd {

struct BlurShape {
    int cols;  // adjacent columns per lane (strip width 64*cols)
    int rows;  // output rows per wavefront strip
};
BlurShape blur_shape_for(int W, int H, int R);
hipError_t prepare_kernel_attributes();

// Batched launches: n_img images of one job, image b's planes `bs` doubles
// after image 0's (src, dst and dec alike), blockIdx.z = image.
hipError_t launch_u8_to_f64(const uint8_t* in, double* out, size_t n, hipStream_t s);
// zero a job's counters and set its age rank in its device tables
hipError_t launch_job_begin(PyrTable* pt, const JobPrio& jp, unsigned* ctr, int n_ctr,
                            unsigned* ctr2, int n_ctr2, hipStream_t s);
hipError_t launch_prepare(const double* in, size_t in_bs, int w, int h, int c, int dbl,
                          double* out, size_t out_bs, int W0, int H0, int n_img, hipStream_t s);
// e0/e1: optional HIP events timestamped by the dispatch itself (profiling);
// tmp: n_img * W * H doubles for kernels wider than kMaxTemplR
// planes of at most tile_max_px pixels use the LDS-tile kernel (k_blur_tile),
// planes of >= 4 Mpx the pair walk (k_blur_pair), the others the strip walk
// (k_blur)
hipError_t launch_blur(const double* src, size_t src_bs, double* dst, size_t bs, int n_img, int W,
                       int H, const BlurTaps& taps, double* dec, int Wd, int Hd, double* tmp,
                       hipStream_t s, hipEvent_t e0, hipEvent_t e1, size_t tile_max_px);
// Initial blur fused with gray/bilinear-x2 staging from the input images
// (image b at in + b * in_bs). Returns false (nothing launched) when the
// fused path does not apply.
bool launch_blur_initial_fused(const double* in, size_t in_bs, int w, int h, int c, int dbl,
                               double* dst, size_t bs, int n_img, int W0, int H0,
                               const BlurTaps& taps, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                               hipError_t* err);
// every octave in [o_first, o_last] of every image (one workgroup per image;
// octave o_first is W_first x H_first and must satisfy lds_octave_fits)
struct LdsShape {
    int cap, dcap;  // doubles of the level regions and of the next-base region
    size_t bytes;   // dynamic LDS of the launch
};
LdsShape lds_shape(int W_first, int H_first, bool has_next, int n_gauss);
hipError_t launch_octaves_lds(const PyrTable* d_pt, int o_first, int o_last, int n_gauss,
                              const BlurTaps* d_taps, int n_img, int W_first, int H_first,
                              hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// levels [l_first, l_last] of one octave in one launch, tiled with
// recomputed halos (k_octave_fused; the base is level l_first - 1);
// plan_octave_fused returns false when a tile's regions do not fit in LDS or
// a radius is outside 1..12. radii[l]: level l's taps.
constexpr size_t kFusedMaxBytes = 160 * 1024;
struct FusedOctave {
    int o, n_gauss, W, H, Wd, Hd, dec_level;  // dec_level -1: no decimation in the group
    int l_first, l_last;                      // levels of the launch
    int tw, th, ntx, nty;                     // tile core, tiles across / down
    int R[kMaxLevels];                        // radius of level l
    int halo[kMaxLevels];                     // R[l+1] + ... + R[l_last]
    int capS, capT, threads;                  // LDS doubles: level region, temporary
    size_t bytes;                             // dynamic LDS of the launch
};
bool plan_octave_fused(int o, int n_gauss, int l_first, int l_last, int W, int H, int Wd, int Hd,
                       const int* radii, int tile, int threads, FusedOctave* f);
hipError_t launch_octave_fused(const PyrTable* d_pt, const FusedOctave& f, const BlurTaps* d_taps,
                               int n_img, hipStream_t s, hipEvent_t e0, hipEvent_t e1);
// the levels of the octaves of `fg` (all images) in one launch of `wgs`
// persistent workgroups; ctr: fg's counters, word 0 the task ticket, all
// zero before the launch (k_job_begin)
hipError_t launch_octaves_flow(const PyrTable* d_pt, const FlowGrid& fg, const BlurTaps* d_taps,
                               unsigned* ctr, int wgs, hipStream_t s, hipEvent_t e0,
                               hipEvent_t e1);
// snap (optional): the last workgroup writes the lane counter snapshot
// (candidate end, raw / record begins) for the keypoint chain; snap[3] must
// be zero before the launch.
// window_size 3: eg tasks = strips x segments per octave
hipError_t launch_extrema_stream(const PyrTable* d_pt, const ExtremaGrid& eg, int n_img,
                                 int n_gauss, int thr, sift_extremum* out, unsigned* counter,
                                 unsigned cap, unsigned* snap, hipStream_t s, hipEvent_t e0,
                                 hipEvent_t e1);
hipError_t launch_extrema_any(const PyrTable* d_pt, int o, int W, int H, int n_img, int n_gauss,
                              int window_size, int thr, sift_extremum* out, unsigned* counter,
                              unsigned cap, hipStream_t s);
// Keypoint stages process the index range [*begin, *end) of their input
// list (device counters), so a detect can run them in batches.
// snap[w] = ctr[w] for w in [w0, w1)
// the context's completed-job counter += 1 (SIFT_AGE_PRIO)
hipError_t launch_job_done(unsigned* done, hipStream_t s);
hipError_t launch_snapshot(const unsigned* ctr, unsigned* snap, hipStream_t s, int w0 = 0,
                           int w1 = 4);
hipError_t launch_refine(const PyrTable* d_pt, const DevParams& P, const sift_extremum* cand,
                         const unsigned* cand_begin, const unsigned* n_cand, unsigned cap_cand,
                         RawKp* out, unsigned* n_out, unsigned cap_out, unsigned* snap0,
                         hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// orientation of raw keypoints [*raw_begin, *n_raw) -> records appended at
// n_rec; descriptors of records [*rec_begin, *n_rec). `work`: two zeroed
// device words per launch (work counter, done counter); ex.cnt receives the
// descriptor launch's record range.
hipError_t launch_orient(const PyrTable* d_pt, const DevParams& P, const RawKp* raw,
                         const unsigned* raw_begin, const unsigned* n_raw, unsigned cap_raw,
                         sift_kp* recs, RecSide* rec_side, unsigned* n_rec, unsigned cap_rec,
                         unsigned* work, unsigned wgs, bool static_walk, hipStream_t s,
                         hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_descriptor(const PyrTable* d_pt, const DevParams& P, sift_kp* recs,
                             const RecSide* rec_side, const unsigned* rec_begin,
                             const unsigned* n_rec, unsigned cap_rec, float* desc_f32,
                             unsigned* work, const ExportSink& ex, unsigned wgs,
                             hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// out[i] = recs[items[i].src] with size = items[i].size (final records on the device)
hipError_t launch_gather_records(const sift_kp* recs, const GatherItem* items, unsigned n,
                                 sift_kp* out, unsigned long long* checksum,
                                 unsigned long long* acc, unsigned* done, hipStream_t s);
hipError_t launch_verify_slots(const void* slots, int n_slots, size_t slot_bytes, int hdr_rows,
                               int count_word, int sum_word, int n_sums, size_t cap_rows,
                               unsigned long long* bad, unsigned long long* scratch,
                               hipStream_t s);

// Matcher (sift_match.hip): records -> shifted descriptor rows + norms
// (n_pad a multiple of 32, rows [n, n_pad) padding), then the 2-NN ratio test
// of queries [0, n1) against the n2_pad reference rows: out_j[i] = index of
// the match or -1, out_d[i] = best distance.
hipError_t launch_match_prep(const sift_kp* d_kps, unsigned n, unsigned n_pad, uint8_t* rows,
                             int* q, hipStream_t s);
hipError_t launch_match2nn(const uint8_t* qrows, const int* qq, unsigned n1, unsigned n1_pad,
                           const uint8_t* rrows, const int* rq, unsigned n2_pad, double ratio,
                           int* out_j, double* out_d, hipStream_t s);

}  // namespace sift_amd
