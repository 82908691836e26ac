// sift_ctx.hip — C-ABI boundary (include/sift_hip.h) and host orchestration
// of the MI355X SIFT pipeline.
//
// Replaces the body of detect_keypoints_and_descriptors (reference
// src/sift.cpp:712-776). Host work is limited to what the reference computes
// with glibc and that feeds bit-exact outputs: the octave count
// (sift.cpp:132-137), the level sigmas (sift.cpp:143-155), the blur taps
// (image.cpp:226-235), the final keypoint size (std::pow, sift.cpp:427-429)
// and clean_keypoints (std::sort + std::unique, sift.cpp:20-24). Everything
// per-pixel and per-keypoint runs in the HIP kernels of sift_kernels.hip.
//
// Jobs. A job is 1..kMaxImages images of one shape and one parameter set
// (the reference function is pure per image, sift.cpp:712-776, so images
// are independent); every kernel of a job covers all its images in one
// launch (blockIdx.z / .y = image), so a batch of 8 1080p images costs the
// launches of one. A context owns kSlots job slots, each with its own
// pyramid arena, keypoint arrays, counters, staging and export buffers, so
// job k+1 can be enqueued (submit) before job k is finalised on the host
// (wait / fetch): the device runs job k+1's pyramid while the host sorts job
// k's records. Completion is tracked with per-slot events only — no stream
// synchronisation on the pipelined path.
//
// Streams. HIP gives a process four hardware queues by default and streams
// beyond that share a queue and serialise, so the context's first four
// streams are two pairs: a pyramid stream (high priority) and a keypoint
// stream (low priority) each. What a job runs on depends on what is in flight
// when it is submitted (sift_ctx::pool): alone (synchronous use) it takes
// all four (octaves alternate between both pyramid streams and keypoint
// batches between both keypoint streams); next to one other job, the pair
// that job left free (two jobs never wait on each other; with shared streams
// the pyramid chains of consecutive jobs serialised and set the step time);
// next to two or more, one free stream of its own, so four single-image jobs
// in flight keep four chains on four queues (measured 0.68 vs 0.75 ms per
// 1080p image at two in flight; BASELINE config 2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <new>
#include <vector>

#include "sift_host.h"
#include "sift_kernels.h"

using namespace sift_amd;

namespace {

using clk = std::chrono::steady_clock;

constexpr unsigned kKpWgsMax = 512;               // keypoint workgroups per launch, at most
// k_orient_wave with nothing beside it: every resident slot (4 workgroups
// per CU); against 512: alone 50.7 -> 46.0 us per 1080p image, configs 3 / 5
// orientation -16 / -18 % (r05_w, r05_final)
constexpr unsigned kOriWgsAlone = 1024;
constexpr unsigned kDescWgsAlone = 256u * SIFT_DSPLIT_OCC;  // k_descriptor_split: every resident slot
constexpr size_t kTileMaxPx = (size_t)1 << 21;    // planes up to this size: LDS-tile blur

// Keypoint lanes: batches go round-robin over kLanes streams, each lane with
// its own region of every keypoint array and its own counters, so the chains
// of consecutive batches run concurrently (within a lane they are serial and
// the snapshot ranges below stay contiguous). Two lanes: streams C, D. Four
// lanes (a job alone; SIFT_LANES=4): C, D, then B once the octaves with a
// batch of their own have their tail levels there, and A for the final
// batch right behind the small octaves, so no chain waits for another.
#ifndef SIFT_LANES
#define SIFT_LANES 4
#endif
constexpr int kLanes = SIFT_LANES;
static_assert(kLanes == 2 || kLanes == 4, "keypoint lanes: 2 or 4");
constexpr int kSlots = SIFT_MAX_INFLIGHT;
constexpr int kPairs = 2;
// device counter block of a slot: [4L..4L+3] live counters of lane L
// (candidates, refined, records), [8..11] zeros, then per keypoint batch g a
// 4-word snapshot (the batch's candidate end, written by its refine launch,
// and its raw / record begins, written by its extrema launch; lane-local),
// then four words per chain: work counters of orientation and descriptor
constexpr int kCtrZeros = 4 * kLanes;
constexpr int kCtrSnap = kCtrZeros + 4;
constexpr int kCtrWork = kCtrSnap + 4 * (kMaxOctaves + 1);
// then the record gather's checksum scratch: 64-bit accumulator + done count
constexpr int kCtrGather = kCtrWork + 4 * (kMaxOctaves + 2);
constexpr int kCtrWords = kCtrGather + 4;
// largest per-lane capacities (the kernels index with 32-bit unsigned)
constexpr size_t kMaxCand = (size_t)1 << 28;
constexpr int kPipeHint = 16;  // submits a pipelining hint lasts
constexpr size_t kMaxRec = (size_t)1 << 29;

template <class T>
struct Pinned {  // grow-only pinned host buffer (fast async copies, no staging)
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (p && cap >= n) return SIFT_OK;
        release();
        const size_t want = n < 1024 ? 1024 : n + n / 4;
        if (hipHostMalloc(&p, want * sizeof(T)) != hipSuccess) {
            p = nullptr;
            return SIFT_ERR_NOMEM;
        }
        cap = want;
        return SIFT_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Grow-only mapped, coherent pinned host buffer: kernels write it directly
// (visible to the host once the writing kernel has completed).
template <class T>
struct Mapped {
    T* h = nullptr;
    T* d = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (h && cap >= n) return SIFT_OK;
        release();
        n = n < 1024 ? 1024 : n + n / 4;
        if (hipHostMalloc(&h, n * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
            h = nullptr;
            return SIFT_ERR_NOMEM;
        }
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) {
            release();
            return SIFT_ERR_HIP;
        }
        cap = n;
        return SIFT_OK;
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = d = nullptr;
        cap = 0;
    }
};

template <class T>
struct DevBuf {  // grow-only device buffer (contents not preserved)
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (p && cap >= n) return SIFT_OK;
        release();
        if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
            p = nullptr;
            return SIFT_ERR_NOMEM;
        }
        cap = n;
        return SIFT_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Stage {
    PyrTable pt;
    BlurTaps taps[kMaxLevels];
};

struct EventPair {
    hipEvent_t a, b;
    double bytes;
    int row;  // profile table row (SIFT_PROF_*)
};

enum SlotState { kFree = 0, kSubmitted = 1, kFinalized = 2 };

// Everything one job owns; reused (grow-only) by later jobs in this slot.
struct Slot {
    int state = kFree;
    int ticket = -1;
    // the job
    int n_img = 0, w = 0, h = 0, c = 0;
    bool want_df = false;
    sift_params p{};
    Geometry g;
    DevParams dp{};
    BlurTaps taps_init{};
    BlurTaps taps[kMaxLevels]{};
    // device buffers
    DevBuf<double> in;       // staged input images (doubles), contiguous
    DevBuf<uint8_t> in8;     // staged input bytes (u8 upload path)
    DevBuf<double> pyr;      // n_img pyramids of g.total doubles
    DevBuf<double> tmp;      // generic wide-kernel blur temporaries
    DevBuf<sift_extremum> cand;
    DevBuf<RawKp> raw;
    DevBuf<sift_kp> ori;
    DevBuf<RecSide> side;
    DevBuf<float> df32;
    size_t cap_cand = 0, cap_raw = 0, cap_ori = 0;  // per lane
    unsigned* d_ctr = nullptr;
    unsigned* h_ctr = nullptr;  // pinned, live counters of every lane
    Stage* h_stage = nullptr;
    Stage* d_stage = nullptr;
    // what d_stage holds, age ranks zeroed (valid once uploaded): a job with
    // the same tables only sets its rank (k_job_begin)
    Stage stage_dev{};
    bool stage_valid = false;
    PyrTable h_pt{};
    Pinned<uint8_t> h_up;  // pinned upload staging
    // records exported by k_descriptor per keypoint chain (mapped pinned)
    Mapped<sift_kp> exp_rec;
    Mapped<RecSide> exp_side;
    Mapped<unsigned> exp_cnt;  // [begin, end) per chain
    DevBuf<unsigned> flow_ctr;  // k_octaves_flow ticket / error / band counters
    size_t exp_lane = 0;
    std::vector<hipEvent_t> chain_ev, sync_ev, ev_pool;
    std::vector<int> chain_lane;
    int n_chains = 0, ev_i = 0;
    size_t ev_used = 0;
    unsigned uses = 0;  // mask of sift_ctx::pool streams this job runs on
    hipEvent_t done_ev = nullptr;  // lane counters on the host
    hipEvent_t pyr0_ev = nullptr;  // octave 0 of this job's pyramid built (pyramid token)
    // streams of the current job: A, B pyramid (even / odd octaves), C, D
    // keypoint lanes 0 / 1 (A == B and C == D when the job runs alone on its
    // slot's pair)
    hipStream_t sA = nullptr, sB = nullptr, sC = nullptr, sD = nullptr;
    int lanes = kLanes;
    std::vector<EventPair> pending;
    // finalize
    bool exported = true;
    unsigned n_lane[kLanes] = {};
    unsigned lane_n[3][kLanes] = {};
    size_t host_base[kLanes] = {};
    const sift_kp* rec_src = nullptr;
    std::vector<unsigned> keep, run_start;
    std::vector<size_t> img_count;
    size_t n_final = 0;
    unsigned n_keys = 0;
    FinalizeWorkspace fin_ws;
    Pinned<sift_kp> h_ori;
    Pinned<RecSide> h_side;
    Pinned<float> h_df32;
    // fetch_device: (record index, size) per final record, read by the gather
    // kernel straight from mapped host memory (no copy launch)
    Mapped<GatherItem> h_gather;
    // an asynchronous device fetch still reading this slot's records:
    // completed before the slot is reused (sift_hip_fetch_device_async)
    hipEvent_t gather_ev = nullptr;
    bool gather_pending = false;
    bool job_done_enqueued = false;  // this job's k_job_done is on a stream
    sift_counts counts{};
    clk::time_point t_submit;
    double t_host[6] = {0, 0, 0, 0, 0, 0};  // [5]: blocked on device events in finalize
};

}  // namespace

struct sift_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // = pyr_stream[0]: the public stream (matcher)
    // persistent workgroups of orientation / descriptor per launch, per
    // image of the job (capped at kKpWgsMax). Fewer than the chip could
    // hold, deliberately: the keypoint kernels are gather-latency-bound, and
    // in the pipelined steady state their resident waves take register file
    // and memory bandwidth from the other jobs' blurs (round 3, interleaved
    // A/B on 1080p, single-image jobs four in flight: 192 per image 0.521
    // ms, 256 0.527, 512 0.548; 8-image jobs 0.503 ms per image at 512 in
    // all vs 0.537 at 1024). Round 4 with the f64 split descriptor (one
    // record per workgroup) and dynamic claims on every item: 128 / 256
    // measured -1.1 % against 192 / 384; once each workgroup's first item
    // was static and the extrema / orientation flushes per workgroup, 192 /
    // 384 came back ahead: -2.3 % over 6 interleaved runs of the driver's
    // command (profiles/r04_ab r04_ee; 512 descriptor workgroups +0.7 %,
    // 96 orientation +1.5 %). Jobs alone: x1.5, or the whole chip for a
    // launch with nothing beside it (enqueue_chain).
    unsigned kp_wgs = 192;
    unsigned desc_wgs = 384;  // k_descriptor_split: ONE record per workgroup
    // octaves of >= 2^this pixels (x images) get their own keypoint batch; the
    // rest form one final batch after the LDS octaves. A single-image job
    // sharing the chip (one stream, lanes = 1) uses 2^22: a 1080p job has two
    // batches (octave 0, the rest), 5 % faster pipelined than four (2^18).
    // Jobs alone on all four streams and multi-image jobs keep 2^18: the
    // batches overlap the smaller octaves' pyramid (2^22 raised the
    // synchronous latency from 0.90 to 1.25 ms and 8-image jobs by 4 %;
    // profiles/r02_ab/r02ap, r02as). SIFT_BATCH_PX_LOG2 (tests).
    int batch_px_log2 = 22;
    int batch_px_log2_alone = 18;
    // octaves of at most this many pixels (and within the LDS, lds_octave_fits)
    // run LDS-resident in the one-workgroup k_octaves_lds (SIFT_LDS_PX, tests:
    // both). A single-image job sharing the chip takes every octave that
    // fits (1080p: from octave 5, 120x67, on): five fewer launches in its
    // chain, -1.2 % on the driver's bench (profiles/r04_ab r04_ff); jobs
    // alone keep octave 5 on tile launches over the chip (kernel-alone
    // octave 5: 23 us over five launches vs ~29 us of the one-CU kernel,
    // which then takes 76 instead of 47 us; synchronous latency)
    size_t lds_max_px = kLdsOctaveMaxPx;
    size_t lds_max_px_shared = kLdsOctavePx;
    // octaves of the final batch up to this many pixels per image, above the
    // LDS octaves, in flight in one k_octaves_flow launch of flow_wgs
    // workgroups (SIFT_FLOW=1; SIFT_FLOW_PX, SIFT_FLOW_WGS). Off by default:
    // bit-exact, but a tile's dependent latency (~5 us: sc1 staging, two LDS
    // passes at one wave per SIMD, write-through drain, counter hand-off) is
    // no shorter than a dependent launch, and levels depend on levels.
    // Measured (r06_s6/s7): 1080p octaves 3-5 80 vs 78.5 us back to back,
    // octaves 2-5 alone 137.6 vs 99 us, synchronous latency 0.769 vs 0.753
    // ms, the driver's command 0.560 vs 0.539 ms per step.
    bool flow = false;
    size_t flow_max_px = (size_t)1 << 19;
    int flow_wgs = 128;
    // octaves of at most fuse_max_px pixels (and above the LDS octaves): two
    // k_octave_fused launches each (chain levels, tail levels) instead of one
    // per level; tiles of 32 x 32 from fuse_t32_px pixels on, 16 x 16 below
    // (SIFT_FUSE=1, SIFT_FUSE_PX, SIFT_FUSE_T32_PX). Bit-exact, off by
    // default. Alone per 1080p image (r06_fuse2, r06_fuse3): octaves 4 / 5
    // 20.5 / 20.4 us against 23.7 / 22.6 as per-level launches, the pyramid
    // 395 vs 403 us (octave 2, 960 x 540, loses: 46.5 vs 27.6 us); but its
    // 1024-thread, 58 KB workgroups hold CUs the concurrent keypoint chains
    // need: synchronous latency 0.795 vs 0.763 ms, the driver's command
    // 0.552 vs 0.542 ms per step, config 5 10.22 vs 9.67 ms per image.
    bool fuse = false;
    size_t fuse_max_px = (size_t)1 << 17;
    size_t fuse_t32_px = 0;
    bool serial = false;  // SIFT_SERIAL=1: every kernel on one stream (profiling)
    // Kernels raise their waves' issue priority by their job's age rank
    // (JobPrio; -1.3 % on the driver's bench command, round 3); d_done
    // counts the context's completed jobs (k_job_done at the end of every
    // job)
    unsigned* d_done = nullptr;
    unsigned prio_seq = 0;  // jobs whose k_job_done was enqueued (JobPrio.ticket)
    DevBuf<unsigned long long> verify_acc;  // sift_hip_verify_slots: per-slot sum + count
    hipEvent_t verify_ev = nullptr;         // the last verify_slots call's end
    bool verify_used = false;
    // Streams of a job (submit_impl): a caller seen pipelining (pipe_hint:
    // a job submitted next to another in the last kPipeHint submits) gets one
    // stream per job, the pair streams first, even when its pipeline is
    // momentarily empty, so the next jobs of a burst do not share the first
    // job's hardware queues; a job alone takes all four pair streams, next
    // to one other job a free pair. HIP pools hardware queues per stream
    // priority (high: -1; normal: 0, shared with every default stream of the
    // process, torch's included). Round 3 on the driver's bench command (20
    // steps, four in flight; profiles/r03_i): this policy 0.586-0.593 ms per
    // step; the round-2 policy (one stream per job only while others are in
    // flight) 0.582-0.640; normal-priority streams first 0.72 (the pool is
    // shared with torch); four equal high-priority streams 0.72-0.77 (the
    // jobs in flight progress and finish together, the host refills in
    // bursts). Launch graphs per slot cut the host's enqueue from 0.12 to
    // 0.03 ms per job but ran the step 2 % slower (profiles/r03_j): removed.
    int pipe_hint = 0;
    long ext_waves = 512;   // extrema tasks per octave (extrema_grid)
    int ext_seg_max = 32;   // centre rows per extrema task, at most
    // Pyramid token: a job's pyramid waits for the previous
    // job's octave 0 (an event). In the steady state of a pipeline it is long
    // built; a burst of jobs submitted together (a pipeline filling) would
    // otherwise run their HBM-bound octave-0 blurs side by side and then
    // their latency-bound keypoint chains side by side, instead of the
    // staggered mix of the steady state, and the first job of the burst
    // finishes late.
    // (round 4: the token after the previous job's octave-0 keypoints or
    // after its whole pyramid measured +15 % / +35 %, profiles/r04_ab r04_k)
    bool pyr_chain = true;
    // (round 4: SIFT_LEAD_ALONE, the first job of a burst on all four pair
    // streams, finished it at 1.23 instead of 1.8 ms but queued the next
    // three behind it: +2.7 % on the driver's bench, removed)
    int pyr_last = -1;  // slot of the last job that recorded its token
    // records per lane per octave-0 pixel, the largest any finalised job of
    // this context had: a slot's first job sizes its mapped export buffers
    // from it (otherwise a cold slot's first job overflows the default size
    // and falls back to the bulk download + a full host sort: 12-17 ms on an
    // 8K image, the first two jobs of every config-5 leg in round 4)
    double exp_px_hint = 0.0;
    // all records of a job per octave-0 pixel, the largest seen: a one-lane
    // (pipelined) job puts every record in its lane, so its buffers are sized
    // from this (sized from the lane hint, a job alone's largest lane, they
    // overflowed into the bulk path on each slot's first pipelined job)
    double exp_px_total = 0.0;
    Slot slots[kSlots];
    // two stream pairs, one per hardware queue each (HIP's default is four
    // queues per process): pair k = pyramid (high priority) + keypoint chains
    // (low priority)
    hipStream_t pyr_stream[kPairs] = {};
    hipStream_t kp_stream[kPairs] = {};
    // Stream pool: pyr0, pyr1, kp0, kp1, then kSlots - 4 more streams. A job
    // takes what the jobs in flight leave free (Slot::uses): all four pair
    // streams when it runs alone, a whole free pair next to one other job,
    // ONE free stream of its own when two or more are in flight (then up to
    // kSlots chains share the chip, each on its own hardware queue while
    // queues last: HIP's default is four per process, GPU_MAX_HW_QUEUES)
    hipStream_t pool[kSlots] = {};
    int next_ticket = 1;
    int last = -1;  // slot of the last finalised job (introspection)

    // profiling: per-row kernel time / algorithmic bytes / launches
    // (rows: pyramid launches per octave, extrema launches; SIFT_PROF_*)
    bool profiling = false;
    double prof_ms[SIFT_PROF_ROWS] = {};
    int64_t prof_launches[SIFT_PROF_ROWS] = {};
    double prof_bytes[SIFT_PROF_ROWS] = {};

    // matcher: one device arena (inputs, shifted rows, norms, results) and
    // pinned result staging
    unsigned char* d_mbuf = nullptr;
    size_t mbuf_cap = 0;
    Pinned<int> h_mj;
    Pinned<double> h_md;
};

namespace {

// SIFT_DEBUG=1: report the failing HIP call on stderr
bool debug_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SIFT_DEBUG");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

// a keypoint batch of a job alone waits only on the tail stream (B), whose
// join with A already orders the octave's chain levels (0: both streams)
#ifndef SIFT_TAIL_JOIN_ONLY
#define SIFT_TAIL_JOIN_ONLY 1
#endif

#define SIFT_HIP_TRY(expr)                                                            \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            if (debug_enabled())                                                        \
                std::fprintf(stderr, "sift_hip: %s:%d: %s: %s\n", __FILE__, __LINE__, #expr, \
                             hipGetErrorString(e_));                                   \
            return SIFT_ERR_HIP;                                                        \
        }                                                                               \
    } while (0)

hipEvent_t pool_event(Slot& s) {  // timing events (profiling)
    if (s.ev_used == s.ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        s.ev_pool.push_back(e);
    }
    return s.ev_pool[s.ev_used++];
}

hipEvent_t sync_event(Slot& s) {  // untimed cross-stream events
    while ((int)s.sync_ev.size() <= s.ev_i) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        s.sync_ev.push_back(e);
    }
    return s.sync_ev[s.ev_i++];
}

// Profiling events for one pyramid launch: timestamps recorded by the
// dispatch packet itself (hipExtLaunchKernel), so timing adds no gaps.
int prof_events(sift_ctx* ctx, Slot& s, hipEvent_t* e0, hipEvent_t* e1, double bytes, int row) {
    *e0 = *e1 = nullptr;
    if (!ctx->profiling) return SIFT_OK;
    *e0 = pool_event(s);
    *e1 = pool_event(s);
    if (!*e0 || !*e1) return SIFT_ERR_HIP;
    s.pending.push_back({*e0, *e1, bytes, row});
    return SIFT_OK;
}

// task table of one k_extrema_stream launch over octaves [o_begin, o_end):
// strips of kExtSpan centre columns x segments of centre rows
ExtremaGrid extrema_grid(const Geometry& g, int o_begin, int o_end, int n_img, long waves,
                         int seg_max) {
    ExtremaGrid eg;
    std::memset(&eg, 0, sizeof eg);
    for (int o = o_begin; o < o_end; ++o) {
        const int i = eg.n++;
        const int tx = g.W[o] > 2 ? (g.W[o] - 2 + kExtSpan - 1) / kExtSpan : 0;
        // segments for ~ext_waves waves per octave over the job, at least 4
        // rows (2 priming rows per segment), at most ext_seg_max. Round 4
        // (1080p): 512 waves / 32 rows: extrema alone 176 -> 135 us per image
        // (octave 1 in 32-row instead of 8-row tasks), the driver's 20-step
        // bench -3.5 %; 4096 / 64 was round 3's (3072 / 6144 / 12288 within
        // 1 % there); 256 / 128 and 128 / 256 slower (too few waves)
        const long rows = (long)tx * std::max(g.H[o] - 2, 0) * n_img / waves;
        const int ch = (int)std::min<long>(seg_max, std::max<long>(4, rows));
        const int ty = g.H[o] > 2 ? (g.H[o] - 2 + ch - 1) / ch : 0;
        eg.oct[i] = o;
        eg.tiles_x[i] = tx > 0 ? tx : 1;
        eg.seg[i] = ch;
        eg.first_tile[i + 1] = eg.first_tile[i] + tx * ty;
    }
    return eg;
}

hipError_t launch_extrema_set(const PyrTable* d_pt, const Geometry& g, int o_begin, int o_end,
                              int n_img, long waves, int seg_max, int thr, sift_extremum* cand, unsigned* counter,
                              unsigned cap, unsigned* snap, hipStream_t s, hipEvent_t e0,
                              hipEvent_t e1) {
    const ExtremaGrid eg = extrema_grid(g, o_begin, o_end, n_img, waves, seg_max);
    return launch_extrema_stream(d_pt, eg, n_img, g.n_gauss, thr, cand, counter, cap, snap, s, e0,
                                 e1);
}

// keypoint-array capacities of a slot (per lane), all size_t and bounded so
// that the kernels' 32-bit indices and the df32 product never wrap
int ensure_kp_arrays(Slot& s, size_t cand, size_t raw, size_t ori) {
    if (cand > kMaxCand || raw > kMaxCand || ori > kMaxRec) return SIFT_ERR_NOMEM;
    if (s.cand.ensure(cand * kLanes) != SIFT_OK) return SIFT_ERR_NOMEM;
    if (s.raw.ensure(raw * kLanes) != SIFT_OK) return SIFT_ERR_NOMEM;
    if (s.ori.ensure(ori * kLanes) != SIFT_OK) return SIFT_ERR_NOMEM;
    if (s.side.ensure(ori * kLanes) != SIFT_OK) return SIFT_ERR_NOMEM;
    if (s.want_df && s.df32.ensure(ori * kLanes * 128) != SIFT_OK) return SIFT_ERR_NOMEM;
    s.cap_cand = cand;
    s.cap_raw = raw;
    s.cap_ori = ori;
    return SIFT_OK;
}

// After a failure with work already enqueued: let every stream drain before
// the slot's buffers can be touched again, then free the slot.
void abandon(sift_ctx* ctx, Slot& s) {
    for (int k = 0; k < kPairs; ++k) {
        (void)hipStreamSynchronize(ctx->pyr_stream[k]);
        (void)hipStreamSynchronize(ctx->kp_stream[k]);
    }
    for (int k = 2 * kPairs; k < kSlots; ++k)
        if (ctx->pool[k]) (void)hipStreamSynchronize(ctx->pool[k]);
    s.pending.clear();
    s.gather_pending = false;  // every stream drained: no gather still reads the slot
    s.state = kFree;
    s.ticket = -1;
}

// One keypoint chain: extrema over octaves [o_begin, o_end) -> refine ->
// orientation -> descriptor, on lane `lane`'s arrays and live counters, on
// stream sx. `begin` (the snapshot: raw / record begins written by the
// extrema launch, candidate end by the refine launch) holds this chain's
// candidate end and its raw / record begins;
// candidates start at cand_begin (the lane's previous chain's snapshot);
// nullptr: the live counters (overflow re-run).
struct ChainSpec {
    int lane, o_begin, o_end;
    const unsigned* cand_begin;
    unsigned* begin;
    hipStream_t sx;
    unsigned* work;  // orientation / descriptor work counters (work, work + 2)
    ExportSink ex;
};

int enqueue_chain(sift_ctx* ctx, Slot& s, const ChainSpec& c) {
    const Geometry& g = s.g;
    const DevParams& dp = s.dp;
    const int n_img = s.n_img, L = c.lane, o_begin = c.o_begin, o_end = c.o_end;
    const PyrTable* d_pt = &s.d_stage->pt;
    const unsigned* zeros = s.d_ctr + kCtrZeros;
    const unsigned cap_cand = (unsigned)s.cap_cand, cap_raw = (unsigned)s.cap_raw,
                   cap_ori = (unsigned)s.cap_ori;
    hipStream_t sx = c.sx;
    unsigned* const begin = c.begin;
    const unsigned* const cand_begin = c.cand_begin;
    unsigned* const work = c.work;
    unsigned* live = s.d_ctr + 4 * L;
    sift_extremum* cand = s.cand.p + (size_t)L * s.cap_cand;
    RawKp* raw = s.raw.p + (size_t)L * s.cap_raw;
    sift_kp* recs = s.ori.p + (size_t)L * s.cap_ori;
    RecSide* side = s.side.p + (size_t)L * s.cap_ori;
    float* df32 = s.want_df ? s.df32.p + (size_t)L * s.cap_ori * 128 : nullptr;
    if (s.p.window_size / 2 == 1) {
        // algorithmic bytes: every Gaussian level read once per pixel
        double xb = 0.0;
        for (int o = o_begin; o < o_end; ++o) xb += 8.0 * g.n_gauss * (double)g.W[o] * g.H[o];
        hipEvent_t e0, e1;
        if (prof_events(ctx, s, &e0, &e1, xb * n_img, SIFT_PROF_EXTREMA) != SIFT_OK)
            return SIFT_ERR_HIP;
        SIFT_HIP_TRY(launch_extrema_set(d_pt, g, o_begin, o_end, n_img, ctx->ext_waves,
                                        ctx->ext_seg_max, dp.threshold, cand,
                                        live + 0, cap_cand, begin, sx, e0, e1));
    } else {
        for (int o = o_begin; o < o_end; ++o)
            SIFT_HIP_TRY(launch_extrema_any(d_pt, o, g.W[o], g.H[o], n_img, g.n_gauss,
                                            s.p.window_size, dp.threshold, cand, live + 0,
                                            cap_cand, sx));
        if (begin) SIFT_HIP_TRY(launch_snapshot(live, begin, sx, 0, 3));
    }
    const unsigned* b = begin ? begin : zeros;
    // persistent grid of this chain: kp_wgs / desc_wgs per image while other
    // jobs share the chip. Nothing else runs beside the last chain of a job
    // alone on the chip (two keypoint lanes, after its whole pyramid) or a
    // chain of a serialised context: those fill the chip (kKpWgsMax
    // orientation workgroups, kDescWgsAlone one-record descriptor
    // workgroups = every resident slot). The other chains of a job alone
    // overlap its own smaller octaves' blurs and take the shared grid (1.5x
    // of 192 / 384 delayed the small octaves behind them: synchronous latency
    // 0.86 vs 0.82-0.84 ms, profiles/r04_final/summary_lat.txt)
    const bool alone = ctx->serial || (s.lanes > 1 && o_end == g.octaves);
    const unsigned ori_wgs =
        alone ? kOriWgsAlone : std::min(kKpWgsMax, ctx->kp_wgs * (unsigned)n_img);
    const unsigned desc_wgs =
        alone ? kDescWgsAlone : std::min(kKpWgsMax, ctx->desc_wgs * (unsigned)n_img);
    hipEvent_t r0, r1, q0, q1, d0, d1;  // profiling events of the keypoint stages
    if (prof_events(ctx, s, &r0, &r1, 0.0, SIFT_PROF_REFINE) != SIFT_OK ||
        prof_events(ctx, s, &q0, &q1, 0.0, SIFT_PROF_ORIENT) != SIFT_OK ||
        prof_events(ctx, s, &d0, &d1, 0.0, SIFT_PROF_DESC) != SIFT_OK)
        return SIFT_ERR_HIP;
    // candidates [cand_begin, live[0]); the refine launch records that end in
    // the chain's snapshot (begin[0]) for the lane's next chain
    SIFT_HIP_TRY(launch_refine(d_pt, dp, cand, cand_begin, live + 0, cap_cand, raw, live + 1,
                               cap_raw, begin, sx, r0, r1));
    SIFT_HIP_TRY(launch_orient(d_pt, dp, raw, b + 1, live + 1, cap_raw, recs, side, live + 2,
                               cap_ori, work, ori_wgs, alone, sx, q0, q1));
    SIFT_HIP_TRY(launch_descriptor(d_pt, dp, recs, side, b + 2, live + 2, cap_ori, df32,
                                   work + 2, c.ex, desc_wgs, sx, d0, d1));
    return SIFT_OK;
}

// ---------------------------------------------------------------------------
// enqueue one job on slot s (everything up to the counter read-back)
// ---------------------------------------------------------------------------

// The mapped export buffers (records written by the descriptor kernel
// straight into host memory) are an optimisation: a job whose records do
// not fit takes one bulk download instead. So their size is capped, and a
// failed allocation falls back to the minimum, then to no buffer at all,
// rather than failing the job (the hint is the context-wide largest
// records-per-pixel seen, which one dense image can make large).
// Lanes split the buffer evenly among the lanes the job uses (s.lanes: one
// for a pipelined job, kLanes for a job alone), so a pipelined job's single
// lane gets all of it (sizing by kLanes doubled the pinned allocations and
// their growth inside the timed jobs of config 5 when kLanes went to 4:
// 9.97 -> 11.1 ms per image, r06_bigab).
constexpr size_t kExportMaxRecs = (size_t)1 << 22;  // every lane: 704 MB + sides
void grow_export(Slot& s, double want, size_t min_want) {
    const size_t w = (size_t)std::min<double>(want, (double)kExportMaxRecs);
    const size_t m = std::min(min_want, kExportMaxRecs);
    const size_t lanes = (size_t)std::max(1, s.lanes);
    if (s.exp_rec.cap >= std::max(w, m) && s.exp_side.cap >= s.exp_rec.cap) {
        s.exp_lane = s.exp_rec.cap / lanes;
        return;
    }
    for (size_t n : {std::max(w, m), m}) {
        if (s.exp_rec.ensure(n) == SIFT_OK && s.exp_side.ensure(s.exp_rec.cap) == SIFT_OK) {
            s.exp_lane = s.exp_rec.cap / lanes;
            return;
        }
        s.exp_rec.release();
        s.exp_side.release();
    }
    s.exp_lane = 0;
}

int enqueue_job(sift_ctx* ctx, Slot& s, const void* const* images, int kind) {
    const auto t0 = clk::now();
    s.t_submit = t0;
    const Geometry& g = s.g;
    const int n_img = s.n_img;
    const sift_params* p = &s.p;
    s.ev_i = 0;
    s.ev_used = 0;
    s.pending.clear();
    s.n_chains = 0;
    s.chain_lane.clear();
    int st;
    hipStream_t sA = s.sA, sB = s.sB, sC = s.sC, sD = s.sD;

    // ---- input images -> device (contiguous, image b at src + b * in_bs)
    const size_t ne = (size_t)s.w * s.h * s.c;
    const double* src = nullptr;
    const size_t in_bs = ne;
    if (kind == SIFT_INPUT_F64_DEVICE && n_img == 1) {
        src = static_cast<const double*>(images[0]);
    } else {
        if ((st = s.in.ensure(ne * n_img)) != SIFT_OK) return st;
        src = s.in.p;
        if (kind == SIFT_INPUT_F64_DEVICE) {
            for (int b = 0; b < n_img; ++b)
                SIFT_HIP_TRY(hipMemcpyAsync(s.in.p + b * ne, images[b], ne * sizeof(double),
                                            hipMemcpyDeviceToDevice, sA));
        } else if (kind == SIFT_INPUT_U8_DEVICE) {
            for (int b = 0; b < n_img; ++b)
                SIFT_HIP_TRY(launch_u8_to_f64(static_cast<const uint8_t*>(images[b]),
                                              s.in.p + b * ne, ne, sA));
        } else {
            // host images through pinned staging: bytes when every value is an
            // integer 0..255 (stb-decoded images always are; exact on the
            // device), doubles otherwise
            bool as_u8 = true;
            if ((st = s.h_up.ensure(ne * n_img * sizeof(double))) != SIFT_OK) return st;
            if (kind == SIFT_INPUT_U8_HOST) {
                for (int b = 0; b < n_img; ++b)
                    std::memcpy(s.h_up.p + b * ne, images[b], ne);
            } else {
                for (int b = 0; b < n_img && as_u8; ++b)
                    as_u8 = host_pack_u8(static_cast<const double*>(images[b]), ne,
                                         s.h_up.p + b * ne);
                // other doubles go up as they are, and must be finite: the
                // extrema scan is built without NaN semantics (Makefile
                // EXT_FLAGS) and the reference's image loader never produces
                // NaN / Inf (image_io.cpp:20-35)
                if (!as_u8)
                    for (int b = 0; b < n_img; ++b)
                        if (!host_copy_finite(static_cast<const double*>(images[b]), ne,
                                              reinterpret_cast<double*>(s.h_up.p) + b * ne))
                            return SIFT_ERR_ARG;
            }
            if (as_u8) {
                if ((st = s.in8.ensure(ne * n_img)) != SIFT_OK) return st;
                SIFT_HIP_TRY(hipMemcpyAsync(s.in8.p, s.h_up.p, ne * n_img,
                                            hipMemcpyHostToDevice, sA));
                SIFT_HIP_TRY(launch_u8_to_f64(s.in8.p, s.in.p, ne * n_img, sA));
            } else {
                SIFT_HIP_TRY(hipMemcpyAsync(s.in.p, s.h_up.p, ne * n_img * sizeof(double),
                                            hipMemcpyHostToDevice, sA));
            }
        }
    }

    // ---- pyramid tables
    const size_t stride = g.total;  // doubles per image pyramid
    if ((st = s.pyr.ensure(stride * n_img)) != SIFT_OK) return st;
    std::memset(&s.h_pt, 0, sizeof s.h_pt);
    for (int o = 0; o < g.octaves; ++o) {
        s.h_pt.w[o] = g.W[o];
        s.h_pt.h[o] = g.H[o];
        for (int l = 0; l < g.n_gauss; ++l) s.h_pt.lvl[o][l] = s.pyr.p + g.offs[o][l];
    }
    s.h_pt.img_stride = stride;
    s.h_pt.n_img = n_img;
    s.h_pt.n_oct = g.octaves;
    s.h_pt.jp = s.taps_init.jp;
    // the tables' device copy is uploaded only when they change (geometry,
    // parameters, buffers); the age rank is set by k_job_begin below. The
    // slot's previous job has been fetched, so its copy out of h_stage has
    // completed and the staging can be rewritten.
    {
        Stage cur;
        std::memset(&cur, 0, sizeof cur);  // padding included: compared bytewise
        cur.pt = s.h_pt;
        for (int l = 0; l < g.n_gauss; ++l) cur.taps[l] = s.taps[l];
        cur.pt.jp = JobPrio{};
        for (int l = 0; l < g.n_gauss; ++l) cur.taps[l].jp = JobPrio{};
        if (!s.stage_valid || std::memcmp(&cur, &s.stage_dev, sizeof cur) != 0) {
            s.stage_valid = false;
            std::memcpy(s.h_stage, &cur, sizeof cur);
            SIFT_HIP_TRY(
                hipMemcpyAsync(s.d_stage, s.h_stage, sizeof(Stage), hipMemcpyHostToDevice, sA));
            s.stage_dev = cur;
            s.stage_valid = true;
        }
    }
    const PyrTable* d_pt = &s.d_stage->pt;

    // wide kernels (R > kMaxTemplR) go through a temporary: one per pyramid
    // stream parity (octaves o and o+1 overlap)
    bool wide = s.taps_init.R > kMaxTemplR || s.taps_init.R < 1;
    for (int l = 1; l < g.n_gauss; ++l) wide |= s.taps[l].R > kMaxTemplR || s.taps[l].R < 1;
    const size_t tmp_half = (size_t)g.W[0] * g.H[0] * n_img;
    if (wide && (st = s.tmp.ensure(2 * tmp_half)) != SIFT_OK) return st;

    // capacities for the variable-size stages; grown and re-run on overflow
    const size_t want_cand =
        std::min<size_t>(std::max<size_t>(g.sum_px * n_img / 32, 65536), kMaxCand);
    if ((st = ensure_kp_arrays(s, std::max(s.cap_cand, want_cand),
                               std::max(s.cap_raw, want_cand),
                               std::max(s.cap_ori, 2 * want_cand))) != SIFT_OK)
        return st;

    const int lanes = s.lanes;
    hipStream_t lane_stream[4] = {sC, sD, sB, sA};
    const int dec_level = g.n_gauss - 3;  // = intervals (sift.cpp:195-196)
    // octaves from o_small on are small enough to run LDS-resident in one
    // launch (k_octaves_lds); the larger ones get one k_blur launch per level
    int o_small = g.octaves;
    const size_t lds_px = (s.lanes == 1 && n_img == 1 && !ctx->serial) ? ctx->lds_max_px_shared
                                                                        : ctx->lds_max_px;
    for (int o = 0; o < g.octaves; ++o)
        if (lds_octave_fits(g.W[o], g.H[o]) && (size_t)(g.W[o] | 1) * g.H[o] <= lds_px) {
            o_small = o;
            break;
        }
    // Keypoint batches: each large octave (>= batch_px pixels over the job's
    // images) is its own batch as soon as its levels exist; the smaller ones,
    // whose keypoint work is too small to amortise a chain of launches, form
    // one final batch. The final batch starts no later than o_small: octaves
    // built by k_octaves_lds have no per-octave batch of their own.
    const size_t batch_px = (size_t)1 << ((s.lanes > 1 || n_img > 1) ? ctx->batch_px_log2_alone
                                                                  : ctx->batch_px_log2);
    int o_merge = g.octaves;  // first octave of the final batch
    for (int o = 0; o < g.octaves; ++o)
        if ((size_t)g.W[o] * g.H[o] * n_img < batch_px) {
            o_merge = o;
            break;
        }
    o_merge = std::min(o_merge, o_small);
    // octaves [o_flow, o_small): in flight in one k_octaves_flow launch (the
    // final batch's octaves above the LDS ones, at most flow_max_px pixels)
    int o_flow = o_small;
    FlowGrid fg;
    std::memset(&fg, 0, sizeof fg);
    int flow_words = 0;
    if (ctx->flow) {
        for (int o = o_merge; o < o_small; ++o)
            if ((size_t)g.W[o] * g.H[o] <= ctx->flow_max_px) {
                o_flow = o;
                break;
            }
        bool ok = o_flow < o_small && (o_small - o_flow) * (g.n_gauss - 1) <= kFlowMaxGroups;
        for (int l = 1; ok && l < g.n_gauss; ++l) ok = s.taps[l].R >= 1 && s.taps[l].R <= kFlowMaxR;
        if (ok) {
            fg.n_img = n_img;
            fg.err = 1;
            flow_words = 2;  // ticket, error flag
            for (int o = o_flow; o < o_small; ++o)
                for (int l = 1; l < g.n_gauss; ++l) {
                    FlowGroup& G = fg.g[fg.n_groups];
                    G.o = o;
                    G.l = l;
                    G.W = g.W[o];
                    G.H = g.H[o];
                    G.nbx = (G.W + 63) / 64;
                    G.nby = (G.H + 31) / 32;
                    G.first = fg.total;
                    fg.total += G.nby * n_img * G.nbx;
                    G.cnt = flow_words;
                    flow_words += n_img * G.nby;
                    G.dep = l >= 2 ? fg.n_groups - 1
                                   : (o > o_flow ? (o - 1 - o_flow) * (g.n_gauss - 1) + dec_level - 1
                                                 : -1);
                    G.dep_dec = l == 1 && o > o_flow;
                    G.dec = l == dec_level && o + 1 < g.octaves;
                    ++fg.n_groups;
                }
            if ((st = s.flow_ctr.ensure(flow_words)) != SIFT_OK) return st;
        } else {
            o_flow = o_small;
        }
    }
    // octaves [o_fuse, o_small): two k_octave_fused launches each (levels
    // 1 .. intervals, the decimation chain, and the two tail levels; tiles
    // with recomputed halos), from the first octave of at most fuse_max_px
    // pixels whose tiles, and those of every smaller octave, fit in LDS
    int o_fuse = o_small;
    FusedOctave fchain[kMaxOctaves], ftail[kMaxOctaves];
    if (ctx->fuse && o_flow == o_small) {
        int radii[kMaxLevels] = {};
        for (int l = 1; l < g.n_gauss; ++l) radii[l] = s.taps[l].R;
        for (int o = o_small - 1; o >= 1; --o) {
            const size_t px = (size_t)g.W[o] * g.H[o];
            const int tile = px >= ctx->fuse_t32_px ? 32 : 16;
            const int thr = tile >= 32 ? 1024 : 256;
            const int Wd = o + 1 < g.octaves ? g.W[o + 1] : 0;
            const int Hd = o + 1 < g.octaves ? g.H[o + 1] : 0;
            if (px > ctx->fuse_max_px ||
                !plan_octave_fused(o, g.n_gauss, 1, dec_level, g.W[o], g.H[o], Wd, Hd, radii, tile,
                                   thr, &fchain[o]) ||
                !plan_octave_fused(o, g.n_gauss, dec_level + 1, g.n_gauss - 1, g.W[o], g.H[o], Wd,
                                   Hd, radii, tile, thr, &ftail[o]))
                break;
            o_fuse = o;
        }
    }
    SIFT_HIP_TRY(launch_job_begin(&s.d_stage->pt, s.h_pt.jp, s.d_ctr, kCtrWords,
                                  flow_words ? s.flow_ctr.p : nullptr, flow_words, sA));

    auto blur = [&](hipStream_t so, int o, int l, const double* bsrc, size_t src_bs,
                    const BlurTaps& t, bool dec) -> int {
        const int W = g.W[o], H = g.H[o];
        const int Wd = dec ? g.W[o + 1] : 0, Hd = dec ? g.H[o + 1] : 0;
        hipEvent_t e0, e1;
        const double bytes =
            n_img * (16.0 * (double)W * (double)H + (dec ? 8.0 * (double)Wd * Hd : 0.0));
        if (prof_events(ctx, s, &e0, &e1, bytes, SIFT_PROF_PYRAMID + o) != SIFT_OK)
            return SIFT_ERR_HIP;
        double* dst = s.h_pt.lvl[o][l];
        double* decp = dec ? s.h_pt.lvl[o + 1][0] : nullptr;
        double* tmp = wide ? s.tmp.p + (o & 1) * tmp_half : nullptr;
        SIFT_HIP_TRY(launch_blur(bsrc, src_bs, dst, stride, n_img, W, H, t, decp, Wd, Hd, tmp, so,
                                 e0, e1, kTileMaxPx));
        return SIFT_OK;
    };

    // ---- pyramid token: this job's pyramid starts once the previous job's
    // octave 0 is built (sift_ctx::pyr_chain)
    if (ctx->pyr_chain && ctx->pyr_last >= 0 && ctx->pyr_last != (int)(&s - ctx->slots) &&
        ctx->slots[ctx->pyr_last].state == kSubmitted)
        SIFT_HIP_TRY(hipStreamWaitEvent(sA, ctx->slots[ctx->pyr_last].pyr0_ev, 0));

    // ---- Gaussian pyramid (compute_initial_image + compute_gaussian_images)
    const int W0 = g.W[0], H0 = g.H[0];
    {
        hipEvent_t e0, e1;
        // the fused initial blur's real I/O: the input image read once (8 B
        // per value) and G[0][0] written once (not 16 B per
        // output pixel)
        const double init_bytes =
            n_img * (8.0 * (double)s.w * (double)s.h * s.c + 8.0 * (double)W0 * H0);
        if (prof_events(ctx, s, &e0, &e1, init_bytes, SIFT_PROF_PYRAMID) != SIFT_OK)
            return SIFT_ERR_HIP;
        hipError_t err = hipSuccess;
        const bool fused = launch_blur_initial_fused(src, in_bs, s.w, s.h, s.c,
                                                     p->double_image_size ? 1 : 0,
                                                     s.h_pt.lvl[0][0], stride, n_img, W0, H0,
                                                     s.taps_init, sA, e0, e1, &err);
        if (fused) {
            SIFT_HIP_TRY(err);
        } else {
            if (ctx->profiling) s.pending.pop_back();
            const double* base_src = src;
            size_t base_bs = in_bs;
            if (s.c != 1 || p->double_image_size) {
                // gray (+ bilinear x2) into level 1's storage; level 1 is
                // written by the first octave blur, after G[0][0] exists
                double* scratch = s.h_pt.lvl[0][1];
                SIFT_HIP_TRY(launch_prepare(src, in_bs, s.w, s.h, s.c,
                                            p->double_image_size ? 1 : 0, scratch, stride, W0,
                                            H0, n_img, sA));
                base_src = scratch;
                base_bs = stride;
            }
            if ((st = blur(sA, 0, 0, base_src, base_bs, s.taps_init, false)) != SIFT_OK)
                return st;
        }
    }
    const unsigned* zeros = s.d_ctr + kCtrZeros;
    auto snap = [&](int gb) { return s.d_ctr + kCtrSnap + 4 * gb; };
    // records of every chain also go to the mapped export buffers, sized from
    // the largest record count seen so far (a larger one falls back to one
    // bulk download at the end, and grows them for the next call)
    const double exp_hint =
        (lanes == 1 ? ctx->exp_px_total : ctx->exp_px_hint * lanes) * 1.5 * (double)W0 *
        (double)H0 * n_img;
    grow_export(s, std::max<double>(exp_hint, (double)s.exp_rec.cap), (size_t)8192 * n_img * lanes);
    if ((st = s.exp_cnt.ensure(kExportCntWords * (kMaxOctaves + 2))) != SIFT_OK) return st;
    // poison: a range no launch published reads as "not exported"
    std::fill(s.exp_cnt.h, s.exp_cnt.h + s.exp_cnt.cap, 0xFFFFFFFFu);
    // lane L exports its records (lane-local index i) to exp_rec[L * exp_lane + i]
    // (exp_lane = cap / lanes, set by grow_export; 0: no buffer, bulk path)

    auto run_chain = [&](int L, int o_begin, int o_end, const unsigned* cand_begin,
                         unsigned* begin, hipStream_t sx) -> int {
        const int ci = s.n_chains++;
        s.chain_lane.push_back(L);
        while ((int)s.chain_ev.size() <= ci) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return SIFT_ERR_HIP;
            s.chain_ev.push_back(e);
        }
        const ChainSpec c{L, o_begin, o_end, cand_begin, begin, sx,
                          s.d_ctr + kCtrWork + 4 * ci,
                          ExportSink{s.exp_rec.d + (size_t)L * s.exp_lane,
                                     s.exp_side.d + (size_t)L * s.exp_lane,
                                     s.exp_cnt.d + kExportCntWords * ci, (unsigned)s.exp_lane,
                                     s.d_ctr + 4 * L}};
        if ((st = enqueue_chain(ctx, s, c)) != SIFT_OK) return st;
        SIFT_HIP_TRY(hipEventRecord(s.chain_ev[ci], c.sx));
        return SIFT_OK;
    };
    int n_batches = 0;
    int lane_last[4] = {-1, -1, -1, -1};  // the lane's previous batch
    int lane_rr = 0;
    // batch gb: octaves [o_begin, o_end), whose levels were enqueued on
    // `sps`. Lanes round-robin; with four lanes the per-octave batches take
    // lanes 0-2 (C, D, B) and the final batch lane 3 (A, free once the
    // pyramid is done), so no per-octave chain delays the pyramid on A.
    auto batch = [&](int o_begin, int o_end, std::initializer_list<hipStream_t> sps) -> int {
        const int gb = n_batches++;
        const bool final_batch = o_end == g.octaves;
        int L;
        if (lanes > 2 && final_batch) {
            L = 3;
        } else {
            L = lane_rr % (lanes > 2 ? 3 : lanes);
            ++lane_rr;
        }
        const int prev = lane_last[L];
        lane_last[L] = gb;
        const hipStream_t sx = lane_stream[L];
        for (hipStream_t sp : sps) {
            if (sp == sx) continue;  // same stream: already ordered
            hipEvent_t pyr_done = sync_event(s);
            if (!pyr_done) return SIFT_ERR_HIP;
            SIFT_HIP_TRY(hipEventRecord(pyr_done, sp));
            SIFT_HIP_TRY(hipStreamWaitEvent(sx, pyr_done, 0));
        }
        return run_chain(L, o_begin, o_end, prev < 0 ? zeros : snap(prev), snap(gb), sx);
    };
    // Two pyramid streams (a job alone): the decimation chain on A — levels
    // 1 .. intervals of every octave, octave o+1 needs only level
    // `intervals` of octave o (sift.cpp:195-196) — and each octave's two
    // tail levels on B after an event on A, so the chain never queues behind
    // a tail (round 4 alternated whole octaves between A and B: octave 2
    // waited on A behind octave 0's R = 8 / 10 levels, ~80 us on 1080p,
    // and every octave switch paid a cross-stream join on the chain).
    // One stream (a pipelined job): in order.
    const bool two_pyr = sA != sB;
    // with four lanes the batch of octave 2 runs on B: the tail levels of the
    // octaves of the final batch then go on A, so they never queue behind it
    const int o_tail_end = kLanes > 2 ? o_merge : o_small;
    for (int o = 0; o < o_small; ++o) {
        if (o == o_flow) {  // octaves [o_flow, o_small) on A, one launch
            double bytes = 0.0;
            for (int q = o_flow; q < o_small; ++q) {
                bytes += 16.0 * (g.n_gauss - 1) * (double)g.W[q] * (double)g.H[q];
                if (q + 1 < g.octaves) bytes += 8.0 * (double)g.W[q + 1] * (double)g.H[q + 1];
            }
            hipEvent_t e0, e1;
            if (prof_events(ctx, s, &e0, &e1, bytes * n_img, SIFT_PROF_PYRAMID + o_flow) !=
                SIFT_OK)
                return SIFT_ERR_HIP;
            SIFT_HIP_TRY(launch_octaves_flow(d_pt, fg, s.d_stage->taps, s.flow_ctr.p,
                                             ctx->flow_wgs, sA, e0, e1));
        }
        if (o >= o_fuse) {  // the chain group on A, the tail group as the tail levels
            for (const FusedOctave* fo : {&fchain[o], &ftail[o]}) {
                const bool tail = fo == &ftail[o] && two_pyr && o < o_tail_end;
                if (tail) {
                    hipEvent_t chain_ev = sync_event(s);
                    if (!chain_ev) return SIFT_ERR_HIP;
                    SIFT_HIP_TRY(hipEventRecord(chain_ev, sA));
                    SIFT_HIP_TRY(hipStreamWaitEvent(sB, chain_ev, 0));
                }
                double bytes =
                    16.0 * (fo->l_last - fo->l_first + 1) * (double)g.W[o] * (double)g.H[o];
                if (fo->dec_level >= 0) bytes += 8.0 * (double)fo->Wd * (double)fo->Hd;
                hipEvent_t e0, e1;
                if (prof_events(ctx, s, &e0, &e1, bytes * n_img, SIFT_PROF_PYRAMID + o) != SIFT_OK)
                    return SIFT_ERR_HIP;
                SIFT_HIP_TRY(launch_octave_fused(d_pt, *fo, s.d_stage->taps, n_img,
                                                 tail ? sB : sA, e0, e1));
            }
        }
        for (int l = 1; o < o_flow && o < o_fuse && l < g.n_gauss; ++l) {
            const bool tail = two_pyr && l > dec_level && o < o_tail_end;
            hipStream_t so = tail ? sB : sA;
            if (tail && l == dec_level + 1) {
                hipEvent_t chain_ev = sync_event(s);
                if (!chain_ev) return SIFT_ERR_HIP;
                SIFT_HIP_TRY(hipEventRecord(chain_ev, sA));
                SIFT_HIP_TRY(hipStreamWaitEvent(sB, chain_ev, 0));
            }
            const bool dec = (l == dec_level) && (o + 1 < g.octaves);
            if ((st = blur(so, o, l, s.h_pt.lvl[o][l - 1], stride, s.taps[l], dec)) != SIFT_OK)
                return st;
        }
        if (o == 0 && ctx->pyr_chain) {
            SIFT_HIP_TRY(hipEventRecord(s.pyr0_ev, two_pyr && o < o_flow ? sB : sA));
            ctx->pyr_last = (int)(&s - ctx->slots);
        }
        // two pyramid streams: B joined A before the octave's tail levels, so
        // an event after them on B covers the whole octave; one join, not two
        if (o < o_merge && (st = (two_pyr && SIFT_TAIL_JOIN_ONLY) ? batch(o, o + 1, {sB})
                                                                   : batch(o, o + 1, {sA, sB})))
            return st;
    }
    if (o_small < g.octaves) {  // on the chain stream, after the last decimation
        hipStream_t so = sA;
        double bytes = 0.0;
        for (int o = o_small; o < g.octaves; ++o) {
            bytes += 16.0 * (g.n_gauss - 1) * (double)g.W[o] * (double)g.H[o];
            if (o + 1 < g.octaves) bytes += 8.0 * (double)g.W[o + 1] * (double)g.H[o + 1];
        }
        hipEvent_t e0, e1;
        if (prof_events(ctx, s, &e0, &e1, bytes * n_img, SIFT_PROF_PYRAMID + o_small) != SIFT_OK)
            return SIFT_ERR_HIP;
        SIFT_HIP_TRY(launch_octaves_lds(d_pt, o_small, g.octaves - 1, g.n_gauss, s.d_stage->taps,
                                        n_img, g.W[o_small], g.H[o_small], so, e0, e1));
    }
    // (the final batch of a job alone on stream A right behind k_octaves_lds,
    // saving the lane stream's wait: synchronous latency +1.2 %, r05_s)
    // (four lanes: the final batch's octaves were built on A alone; B holds
    // the octave-2 chain, which it must not wait for)
    if (o_merge < g.octaves &&
        (st = (kLanes > 2 && two_pyr) ? batch(o_merge, g.octaves, {sA})
                                      : batch(o_merge, g.octaves, {sA, sB})) !=
            SIFT_OK)
        return st;
    // the other lane streams join C for the age counter (k_job_done): the
    // job's last device work. The host does not wait for it: each lane's last
    // descriptor launch publishes the lane's counters with its record range
    // (ExportSink), so the job is complete on the host once its chains' events
    // are.
    for (hipStream_t sj : {sD, sB, sA}) {
        if (sj == sC || (kLanes == 2 && sj != sD)) continue;
        if (sj == sB && sB == sD) continue;
        hipEvent_t jd = sync_event(s);
        if (!jd) return SIFT_ERR_HIP;
        SIFT_HIP_TRY(hipEventRecord(jd, sj));
        SIFT_HIP_TRY(hipStreamWaitEvent(sC, jd, 0));
    }
    if (s.taps_init.jp.done) {
        SIFT_HIP_TRY(launch_job_done(ctx->d_done, sC));
        s.job_done_enqueued = true;
    }
    SIFT_HIP_TRY(hipEventRecord(s.done_ev, sC));
    s.t_host[0] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    return SIFT_OK;
}

// ---------------------------------------------------------------------------
// finalise a submitted job on the host: per-chain sizes + sorted runs as the
// chains complete, overflow re-run, merge + unique per image
// ---------------------------------------------------------------------------
int finalize_job(sift_ctx* ctx, Slot& s) {
    const auto t0 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const Geometry& g = s.g;
    const sift_params* p = &s.p;
    int st;
    hipStream_t sC = s.sC;
    s.exported = s.exp_lane > 0;  // no export buffer: the bulk path
    s.n_keys = 0;
    s.run_start.clear();
    s.fin_ws.all.resize(s.exp_rec.cap);
    double blocked = 0.0;  // host time spent waiting for the device
    auto sync_ev = [&](hipEvent_t e) -> hipError_t {
        const auto a = clk::now();
        const hipError_t r = hipEventSynchronize(e);
        blocked += ms(a, clk::now());
        return r;
    };
    for (int ci = 0; ci < s.n_chains; ++ci) {
        SIFT_HIP_TRY(sync_ev(s.chain_ev[ci]));
        const unsigned* cnt = s.exp_cnt.h + kExportCntWords * ci;
        const unsigned b = cnt[0], e = cnt[1];
        if (e > s.exp_lane || b > e) {
            s.exported = false;
            break;
        }
        const size_t base = (size_t)s.chain_lane[ci] * s.exp_lane;
        s.run_start.push_back(s.n_keys);
        host_sort_run(s.exp_rec.h, s.exp_side.h, (unsigned)(base + b), (unsigned)(base + e),
                      s.fin_ws.all.data() + s.n_keys, &s.fin_ws);
        s.n_keys += e - b;
    }
    s.run_start.push_back(s.n_keys);

    // ---- the counters; re-run every candidate stage on overflow. Every
    // chain has completed when its records were all exported: each lane's
    // counters are those its last chain published. Otherwise (export
    // overflow) they are copied back once the job's device work is done.
    bool published = s.exported && s.n_chains > 0;
    if (published) {
        std::fill(s.h_ctr, s.h_ctr + 4 * kLanes, 0u);
        for (int ci = 0; ci < s.n_chains; ++ci) {
            const unsigned* cnt = s.exp_cnt.h + kExportCntWords * ci;
            unsigned* h = s.h_ctr + 4 * s.chain_lane[ci];
            h[0] = cnt[2];
            h[1] = cnt[3];
            h[2] = cnt[4];
        }
    }
    clk::time_point t_wait;
    for (int attempt = 0;; ++attempt) {
        if (attempt > 0) {
            // the pyramid is complete: every octave again, on C.
            // Later jobs may be queued on the streams; they use other slots'
            // buffers, and the re-run simply queues behind them.
            s.exported = false;
            SIFT_HIP_TRY(hipMemsetAsync(s.d_ctr, 0, kCtrWords * sizeof(unsigned), sC));
            s.n_chains = 0;
            s.chain_lane.clear();
            // every octave again as one chain on lane 0 (a keypoint's
            // records do not depend on its chain); no export
            {
                unsigned* begin = s.d_ctr + kCtrSnap;
                const ChainSpec c{0, 0, g.octaves, s.d_ctr + kCtrZeros, begin, sC,
                                  s.d_ctr + kCtrWork,
                                  ExportSink{s.exp_rec.d, s.exp_side.d, nullptr, 0, nullptr}};
                s.n_chains = 1;
                s.chain_lane.push_back(0);
                if ((st = enqueue_chain(ctx, s, c)) != SIFT_OK) return st;
            }
        }
        if (attempt > 0 || !published) {
            SIFT_HIP_TRY(hipMemcpyAsync(s.h_ctr, s.d_ctr, 4 * kLanes * sizeof(unsigned),
                                        hipMemcpyDeviceToHost, sC));
            SIFT_HIP_TRY(hipEventRecord(s.done_ev, sC));
            SIFT_HIP_TRY(sync_ev(s.done_ev));
        }
        t_wait = clk::now();
        size_t nc = 0, nr = 0, no = 0;  // largest per-lane counts
        for (int L = 0; L < kLanes; ++L) {
            nc = std::max<size_t>(nc, s.h_ctr[4 * L]);
            nr = std::max<size_t>(nr, s.h_ctr[4 * L + 1]);
            no = std::max<size_t>(no, s.h_ctr[4 * L + 2]);
        }
        if (nc <= s.cap_cand && nr <= s.cap_raw && no <= s.cap_ori) break;
        if (attempt >= 3) return SIFT_ERR_NOMEM;
        // grow every stage that overflowed (refine/orient counts are lower
        // bounds when an upstream stage overflowed, so grow generously);
        // ensure_kp_arrays rejects capacities the kernels cannot index
        const size_t nc2 = std::max(s.cap_cand, nc) * 2;
        const size_t nr2 = std::max(std::max(s.cap_raw, nr) * 2, nc2);
        const size_t no2 = std::max(std::max(s.cap_ori, no) * 2, 2 * nr2);
        if ((st = ensure_kp_arrays(s, nc2, nr2, no2)) != SIFT_OK) return st;
    }

    unsigned n_ori = 0;
    for (int L = 0; L < kLanes; ++L) {
        s.n_lane[L] = s.h_ctr[4 * L + 2];
        s.lane_n[0][L] = s.h_ctr[4 * L];
        s.lane_n[1][L] = s.h_ctr[4 * L + 1];
        s.lane_n[2][L] = s.n_lane[L];
        n_ori += s.n_lane[L];
    }
    if (s.exported && s.n_keys != n_ori) s.exported = false;
    ctx->exp_px_hint = std::max(ctx->exp_px_hint,
                                (double)*std::max_element(s.n_lane, s.n_lane + kLanes) /
                                    ((double)g.W[0] * (double)g.H[0] * s.n_img));
    ctx->exp_px_total =
        std::max(ctx->exp_px_total, (double)n_ori / ((double)g.W[0] * (double)g.H[0] * s.n_img));
    s.rec_src = s.exp_rec.h;
    // host position of lane L's record i: exported, L * exp_lane + i; after a
    // bulk download, the lanes are concatenated
    const RecSide* side_src = s.exp_side.h;
    for (int L = 0, acc = 0; L < kLanes; acc += s.n_lane[L], ++L)
        s.host_base[L] = s.exported ? (size_t)L * s.exp_lane : (size_t)acc;
    const bool bulk = !s.exported;
    if (bulk) {  // bulk download of every record
        if ((st = s.h_ori.ensure(n_ori)) != SIFT_OK) return st;
        if ((st = s.h_side.ensure(n_ori)) != SIFT_OK) return st;
        for (int L = 0; L < kLanes; ++L) {
            if (!s.n_lane[L]) continue;
            SIFT_HIP_TRY(hipMemcpyAsync(s.h_ori.p + s.host_base[L], s.ori.p + (size_t)L * s.cap_ori,
                                        s.n_lane[L] * sizeof(sift_kp), hipMemcpyDeviceToHost, sC));
            SIFT_HIP_TRY(hipMemcpyAsync(s.h_side.p + s.host_base[L],
                                        s.side.p + (size_t)L * s.cap_ori,
                                        s.n_lane[L] * sizeof(RecSide), hipMemcpyDeviceToHost, sC));
        }
        s.rec_src = s.h_ori.p;
        side_src = s.h_side.p;
    }
    if (s.want_df) {
        const size_t span = s.exported ? s.exp_rec.cap : (size_t)n_ori;
        if ((st = s.h_df32.ensure(std::max<size_t>(span, 1) * 128)) != SIFT_OK) return st;
        for (int L = 0; L < kLanes; ++L)
            if (s.n_lane[L])
                SIFT_HIP_TRY(hipMemcpyAsync(s.h_df32.p + s.host_base[L] * 128,
                                            s.df32.p + (size_t)L * s.cap_ori * 128,
                                            (size_t)s.n_lane[L] * 128 * sizeof(float),
                                            hipMemcpyDeviceToHost, sC));
    }
    if (bulk || s.want_df) {
        SIFT_HIP_TRY(hipEventRecord(s.done_ev, sC));
        SIFT_HIP_TRY(sync_ev(s.done_ev));
    }
    const auto t_copy = clk::now();

    {  // events of a job submitted with profiling on (bench.py samples jobs)
        for (const EventPair& e : s.pending) {
            float ems = 0.f;
            SIFT_HIP_TRY(hipEventElapsedTime(&ems, e.a, e.b));
            ctx->prof_ms[e.row] += ems;
            ctx->prof_bytes[e.row] += e.bytes;
            ctx->prof_launches[e.row] += 1;
        }
    }
    s.pending.clear();

    // clean_keypoints per image: merge the sorted runs and unique (or all of
    // it, after a bulk download), in the g++-built layer
    s.keep.resize(std::max<unsigned>(n_ori, 1));
    s.img_count.assign(s.n_img, 0);
    if (s.exported) {
        s.n_final = host_merge_unique(s.fin_ws.all.data(), s.run_start, s.keep.data(),
                                      s.img_count.data(), &s.fin_ws);
    } else {
        s.n_final = host_finalize(p, s.h_ori.p, side_src, n_ori, s.keep.data(),
                                  s.img_count.data(), &s.fin_ws);
        // the next job in this slot exports this many records per lane
        const unsigned lane_max = *std::max_element(s.n_lane, s.n_lane + kLanes);
        if (lane_max > s.exp_lane)
            grow_export(s, ((double)lane_max + lane_max / 2) * s.lanes,
                        (size_t)8192 * s.n_img * s.lanes);
    }
    const auto t_fin = clk::now();
    s.t_host[1] = ms(t0, t_wait);
    s.t_host[2] = ms(t_wait, t_copy);
    s.t_host[3] = ms(t_copy, t_fin);
    s.t_host[5] = blocked;

    s.counts.extrema = s.counts.refined = 0;
    for (int L = 0; L < kLanes; ++L) {
        s.counts.extrema += s.lane_n[0][L];
        s.counts.refined += s.lane_n[1][L];
    }
    s.counts.oriented = n_ori;
    s.counts.final_n = (int64_t)s.n_final;
    s.counts.octaves = g.octaves;
    s.counts.levels_per_octave = g.n_gauss;
    s.counts.octave0_w = g.W[0];
    s.counts.octave0_h = g.H[0];
    s.state = kFinalized;
    ctx->last = (int)(&s - ctx->slots);
    return SIFT_OK;
}

Slot* slot_of(sift_ctx* ctx, int ticket) {
    for (Slot& s : ctx->slots)
        if (s.state != kFree && s.ticket == ticket) return &s;
    return nullptr;
}

int submit_impl(sift_ctx* ctx, const void* const* images, int n_images, int kind, int w, int h,
                int c, const sift_params* p, int want_df, int* ticket) {
    if (!ctx || !images || !ticket || n_images < 1 || n_images > SIFT_MAX_BATCH) return SIFT_ERR_ARG;
    if (kind < SIFT_INPUT_F64_HOST || kind > SIFT_INPUT_U8_DEVICE) return SIFT_ERR_ARG;
    for (int b = 0; b < n_images; ++b)
        if (!images[b]) return SIFT_ERR_ARG;
    if (w <= 0 || h <= 0) return SIFT_ERR_ARG;
    if (c != 1 && c != 3) return SIFT_ERR_CHANNELS;
    sift_params def;
    if (!p) {
        sift_params_default(&def);
        p = &def;
    }
    // the lowest free slot that is not the introspected one (the last
    // finalised job, sift_hip_copy_level & co.), else that one: a stream of
    // jobs with d in flight cycles through d + 1 slots, whose grow-only
    // buffers are then all warm (a rotation over every slot met cold,
    // allocating slots for the first kSlots jobs)
    Slot* sp = nullptr;
    for (int k = 0; k < kSlots; ++k) {
        Slot& s = ctx->slots[k];
        if (s.state == kFree && k != ctx->last) {
            sp = &s;
            break;
        }
    }
    if (!sp && ctx->last >= 0 && ctx->slots[ctx->last].state == kFree) sp = &ctx->slots[ctx->last];
    if (!sp) return SIFT_ERR_STATE;  // SIFT_MAX_INFLIGHT jobs already in flight
    Slot& s = *sp;
    // an async device fetch may still read this slot's records: the new
    // job's streams wait for it on the device (below), not the host. The
    // flag is cleared only once those waits are enqueued, so a submit that
    // fails before them leaves it for the next one.
    const bool gather_wait = s.gather_pending;
    int st = host_plan(p, w, h, c, &s.g, &s.taps_init, s.taps, &s.dp);
    if (st != SIFT_OK) return st;
    // age rank (JobPrio): jobs are numbered by prio_seq, which advances only
    // when a job's k_job_done was enqueued (the job will count in d_done);
    // both counters wrap together modulo 2^32
    const JobPrio jp{ctx->d_done,
                     (int)(ctx->prio_seq + 1u), 0};
    s.taps_init.jp = jp;
    for (BlurTaps& t : s.taps) t.jp = jp;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->last == (int)(&s - ctx->slots)) ctx->last = -1;  // its buffers get reused
    s.n_img = n_images;
    s.w = w;
    s.h = h;
    s.c = c;
    s.p = *p;
    s.want_df = want_df != 0;
    s.ticket = ctx->next_ticket++;
    if (ctx->next_ticket <= 0) ctx->next_ticket = 1;
    {
        int others = 0;
        unsigned used = 0;
        for (const Slot& o : ctx->slots)
            if (&o != &s && o.state == kSubmitted) {
                ++others;
                used |= o.uses;
            }
        hipStream_t* q = ctx->pool;  // pyr0, pyr1, kp0, kp1, ...
        // a caller that keeps jobs in flight (pipe_hint: one submitted next
        // to another in the last kPipeHint submits) gets one stream per job,
        // the pair streams first, even when its pipeline is momentarily
        // empty, so the next jobs of a burst find their hardware queues free;
        // a job alone takes all four pair streams (see sift_ctx::pipe_hint)
        const bool hinted = ctx->pipe_hint > 0;
        if (others > 0) ctx->pipe_hint = kPipeHint;
        else if (ctx->pipe_hint > 0) --ctx->pipe_hint;
        if (others > 0 || hinted) {
            int k = 0;
            while (k + 1 < kSlots && (used >> k & 1u)) ++k;
            s.sA = s.sB = s.sC = s.sD = q[k];
            s.lanes = 1;
            s.uses = 1u << k;
        } else {
            s.sA = q[0], s.sB = q[1], s.sC = q[2], s.sD = q[3];
            s.lanes = kLanes;
            s.uses = 0xFu;
        }
        if (ctx->serial) {  // profiling: one stream, no overlap (kernel costs alone)
            s.sA = s.sB = s.sC = s.sD = q[0];
            s.lanes = 1;
        }
    }
    if (gather_wait) {
        const hipStream_t js[4] = {s.sA, s.sB, s.sC, s.sD};
        for (int i = 0; i < 4; ++i) {
            bool dup = false;
            for (int j = 0; j < i; ++j) dup |= js[j] == js[i];
            if (!dup && hipStreamWaitEvent(js[i], s.gather_ev, 0) != hipSuccess) {
                s.state = kFree;
                s.ticket = -1;
                return SIFT_ERR_HIP;
            }
        }
        s.gather_pending = false;
    }
    s.state = kSubmitted;
    s.job_done_enqueued = false;
    st = enqueue_job(ctx, s, images, kind);
    if (s.job_done_enqueued) ++ctx->prio_seq;
    if (st != SIFT_OK) {
        abandon(ctx, s);
        return st;
    }
    *ticket = s.ticket;
    return SIFT_OK;
}

int wait_impl(sift_ctx* ctx, Slot& s) {
    if (s.state == kFinalized) return SIFT_OK;
    (void)hipSetDevice(ctx->device);
    const int st = finalize_job(ctx, s);
    if (st != SIFT_OK) abandon(ctx, s);
    return st;
}

// kept records of a finalised job, image-major, into caller storage
void gather(Slot& s, sift_kp* out, float* df) {
    const auto t0 = clk::now();
    // record i's host row: exported -> lane-local index already offset by
    // host_base at export time (keep holds host positions); bulk -> concatenated
    // large outputs (config 5: 166 k records = 28 MB, much of it first
    // touches of the caller's fresh pages) on the host pool's threads; the
    // caller takes pieces too, so small outputs (1080p: ~6 k records, ~25 us
    // alone) finish no later than on one thread
    constexpr size_t kPiece = 512;
    const size_t n = s.n_final;
    const unsigned pieces = (unsigned)((n + kPiece - 1) / kPiece);
    auto copy = [&](unsigned t) {
        const size_t b = (size_t)t * kPiece, e = std::min(n, b + kPiece);
        if (out)
            for (size_t i = b; i < e; ++i) out[i] = s.rec_src[s.keep[i]];
        if (df && s.want_df)
            for (size_t i = b; i < e; ++i)
                std::memcpy(df + i * 128, s.h_df32.p + (size_t)s.keep[i] * 128,
                            128 * sizeof(float));
    };
    if (pieces > 1) host_parallel(pieces, copy);
    else
        for (unsigned t = 0; t < pieces; ++t) copy(t);
    s.t_host[4] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

// final records of a finalised job into device memory, enqueued on the
// slot's keypoint stream; `consumer` (optional) is ordered after the gather
// by an event, so the caller's stream can use d_out with no host wait. The
// slot's buffers stay in use until gather_ev, which the streams of the slot's next
// job wait for on the device (submit_impl).
int gather_device(Slot& s, sift_kp* d_out, hipStream_t consumer, unsigned long long* checksum) {
    const size_t n = s.n_final;
    int st;
    if (n == 0 && checksum) SIFT_HIP_TRY(hipMemsetAsync(checksum, 0, sizeof *checksum, s.sC));
    if (n > 0) {
        if ((st = s.h_gather.ensure(n)) != SIFT_OK) return st;
        for (size_t i = 0; i < n; ++i) {
            const unsigned pos = s.keep[i];  // host position of the record
            int L;
            size_t j;
            if (s.exported) {
                L = (int)(pos / s.exp_lane);
                j = pos - (size_t)L * s.exp_lane;
            } else {
                L = pos < s.n_lane[0] ? 0 : 1;
                j = pos - (L ? s.n_lane[0] : 0);
            }
            s.h_gather.h[i] = GatherItem{s.rec_src[pos].size, (unsigned)(L * s.cap_ori + j), 0};
        }
        // the checksum scratch words were zeroed with the job's counters
        SIFT_HIP_TRY(launch_gather_records(
            s.ori.p, s.h_gather.d, (unsigned)n, d_out, checksum,
            reinterpret_cast<unsigned long long*>(s.d_ctr + kCtrGather), s.d_ctr + kCtrGather + 2,
            s.sC));
    }
    if (!s.gather_ev)
        SIFT_HIP_TRY(hipEventCreateWithFlags(&s.gather_ev, hipEventDisableTiming));
    SIFT_HIP_TRY(hipEventRecord(s.gather_ev, s.sC));
    s.gather_pending = true;
    if (consumer && consumer != s.sC) SIFT_HIP_TRY(hipStreamWaitEvent(consumer, s.gather_ev, 0));
    return SIFT_OK;
}

}  // namespace

extern "C" {

void sift_params_default(sift_params* p) {
    if (!p) return;
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

int sift_hip_create(int device, sift_ctx** out) {
    if (!out) return SIFT_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SIFT_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return SIFT_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return SIFT_ERR_HIP;
    sift_ctx* ctx = new (std::nothrow) sift_ctx();
    if (!ctx) return SIFT_ERR_NOMEM;
    ctx->device = device;
    int prio_lo = 0, prio_hi = 0;  // numerically lower = higher priority
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
    if (const char* e = std::getenv("SIFT_BATCH_PX_LOG2")) {
        const int v = std::atoi(e);
        if (v >= 0 && v <= 40) ctx->batch_px_log2 = ctx->batch_px_log2_alone = v;
    }
    if (const char* e = std::getenv("SIFT_SERIAL")) ctx->serial = std::atoi(e) != 0;
    if (const char* e = std::getenv("SIFT_FLOW")) ctx->flow = std::atoi(e) != 0;
    if (const char* e = std::getenv("SIFT_FLOW_PX")) ctx->flow_max_px = (size_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SIFT_FLOW_WGS")) ctx->flow_wgs = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("SIFT_FUSE")) ctx->fuse = std::atoi(e) != 0;
    if (const char* e = std::getenv("SIFT_FUSE_PX")) ctx->fuse_max_px = (size_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SIFT_FUSE_T32_PX"))
        ctx->fuse_t32_px = (size_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SIFT_LDS_PX"))
        ctx->lds_max_px = ctx->lds_max_px_shared = (size_t)std::max(0, std::atoi(e));
    bool ok = prepare_kernel_attributes() == hipSuccess;
    ok = ok && hipMalloc(&ctx->d_done, sizeof(unsigned)) == hipSuccess &&
         hipMemset(ctx->d_done, 0, sizeof(unsigned)) == hipSuccess;
    for (int k = 0; k < kPairs; ++k)
        ok = ok &&
             hipStreamCreateWithPriority(&ctx->pyr_stream[k], hipStreamNonBlocking, prio_hi) ==
                 hipSuccess &&
             hipStreamCreateWithPriority(&ctx->kp_stream[k], hipStreamNonBlocking, prio_lo) ==
                 hipSuccess;
    ctx->stream = ctx->pyr_stream[0];
    ctx->pool[0] = ctx->pyr_stream[0];
    ctx->pool[1] = ctx->pyr_stream[1];
    ctx->pool[2] = ctx->kp_stream[0];
    ctx->pool[3] = ctx->kp_stream[1];
    for (int k = 2 * kPairs; k < kSlots; ++k)
        ok = ok && hipStreamCreateWithFlags(&ctx->pool[k], hipStreamNonBlocking) == hipSuccess;
    for (Slot& s : ctx->slots) {
        ok = ok && hipMalloc(&s.d_ctr, kCtrWords * sizeof(unsigned)) == hipSuccess &&
             hipHostMalloc(&s.h_ctr, 4 * kLanes * sizeof(unsigned)) == hipSuccess &&
             hipHostMalloc(&s.h_stage, sizeof(Stage)) == hipSuccess &&
             hipMalloc(&s.d_stage, sizeof(Stage)) == hipSuccess &&
             hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.pyr0_ev, hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) {
        sift_hip_destroy(ctx);
        return SIFT_ERR_HIP;
    }
    *out = ctx;
    return SIFT_OK;
}

int sift_hip_destroy(sift_ctx* ctx) {
    if (!ctx) return SIFT_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    for (int k = 0; k < kPairs; ++k) {
        if (ctx->pyr_stream[k]) (void)hipStreamSynchronize(ctx->pyr_stream[k]);
        if (ctx->kp_stream[k]) (void)hipStreamSynchronize(ctx->kp_stream[k]);
    }
    for (int k = 2 * kPairs; k < kSlots; ++k)
        if (ctx->pool[k]) (void)hipStreamSynchronize(ctx->pool[k]);
    for (Slot& s : ctx->slots) {
        s.in.release();
        s.in8.release();
        s.flow_ctr.release();
        s.pyr.release();
        s.tmp.release();
        s.cand.release();
        s.raw.release();
        s.ori.release();
        s.side.release();
        s.df32.release();
        if (s.d_ctr) (void)hipFree(s.d_ctr);
        if (s.d_stage) (void)hipFree(s.d_stage);
        if (s.h_ctr) (void)hipHostFree(s.h_ctr);
        if (s.h_stage) (void)hipHostFree(s.h_stage);
        s.h_up.release();
        s.exp_rec.release();
        s.exp_side.release();
        s.exp_cnt.release();
        s.h_ori.release();
        s.h_side.release();
        s.h_df32.release();
        s.h_gather.release();
        if (s.gather_ev) (void)hipEventDestroy(s.gather_ev);
        for (hipEvent_t e : s.chain_ev) (void)hipEventDestroy(e);
        for (hipEvent_t e : s.sync_ev) (void)hipEventDestroy(e);
        for (hipEvent_t e : s.ev_pool) (void)hipEventDestroy(e);
        if (s.done_ev) (void)hipEventDestroy(s.done_ev);
        if (s.pyr0_ev) (void)hipEventDestroy(s.pyr0_ev);
    }
    if (ctx->d_mbuf) (void)hipFree(ctx->d_mbuf);
    ctx->h_mj.release();
    ctx->h_md.release();
    for (int k = 0; k < kPairs; ++k) {
        if (ctx->pyr_stream[k]) (void)hipStreamDestroy(ctx->pyr_stream[k]);
        if (ctx->kp_stream[k]) (void)hipStreamDestroy(ctx->kp_stream[k]);
    }
    for (int k = 2 * kPairs; k < kSlots; ++k)
        if (ctx->pool[k]) (void)hipStreamDestroy(ctx->pool[k]);
    if (ctx->verify_ev) {
        (void)hipEventSynchronize(ctx->verify_ev);
        (void)hipEventDestroy(ctx->verify_ev);
    }
    ctx->verify_acc.release();
    if (ctx->d_done) (void)hipFree(ctx->d_done);
    delete ctx;
    return SIFT_OK;
}

int sift_hip_submit(sift_ctx* ctx, const void* const* images, int n_images, int input_kind,
                    int w, int h, int c, const sift_params* p, int want_desc_f32, int* ticket) {
    return submit_impl(ctx, images, n_images, input_kind, w, h, c, p, want_desc_f32, ticket);
}

int sift_hip_wait(sift_ctx* ctx, int ticket, size_t* counts, size_t* total) {
    if (!ctx) return SIFT_ERR_ARG;
    Slot* s = slot_of(ctx, ticket);
    if (!s) return SIFT_ERR_STATE;
    const int st = wait_impl(ctx, *s);
    if (st != SIFT_OK) return st;
    if (counts)
        for (int b = 0; b < s->n_img; ++b) counts[b] = s->img_count[b];
    if (total) *total = s->n_final;
    return SIFT_OK;
}

int sift_hip_fetch(sift_ctx* ctx, int ticket, sift_kp* out, float* desc_f32) {
    if (!ctx) return SIFT_ERR_ARG;
    Slot* s = slot_of(ctx, ticket);
    if (!s) return SIFT_ERR_STATE;
    int st = wait_impl(ctx, *s);
    if (st != SIFT_OK) return st;
    gather(*s, out, desc_f32);
    s->state = kFree;
    s->ticket = -1;
    return SIFT_OK;
}

int sift_hip_fetch_device(sift_ctx* ctx, int ticket, void* d_out, size_t cap) {
    if (!ctx || (!d_out && cap)) return SIFT_ERR_ARG;
    Slot* s = slot_of(ctx, ticket);
    if (!s) return SIFT_ERR_STATE;
    int st = wait_impl(ctx, *s);
    if (st != SIFT_OK) return st;
    if (cap < s->n_final) return SIFT_ERR_ARG;  // the job stays fetchable
    (void)hipSetDevice(ctx->device);
    st = gather_device(*s, static_cast<sift_kp*>(d_out), nullptr, nullptr);
    if (st == SIFT_OK && hipEventSynchronize(s->gather_ev) != hipSuccess) st = SIFT_ERR_HIP;
    if (st != SIFT_OK) {  // as fetch_device_async: drain and release the job
        abandon(ctx, *s);
        return st;
    }
    s->gather_pending = false;
    s->state = kFree;
    s->ticket = -1;
    return SIFT_OK;
}

int sift_hip_fetch_device_async(sift_ctx* ctx, int ticket, void* d_out, size_t cap,
                                void* stream, uint64_t* d_checksum) {
    if (!ctx || (!d_out && cap)) return SIFT_ERR_ARG;
    Slot* s = slot_of(ctx, ticket);
    if (!s) return SIFT_ERR_STATE;
    int st = wait_impl(ctx, *s);
    if (st != SIFT_OK) return st;
    if (cap < s->n_final) return SIFT_ERR_ARG;  // the job stays fetchable
    (void)hipSetDevice(ctx->device);
    st = gather_device(*s, static_cast<sift_kp*>(d_out), static_cast<hipStream_t>(stream),
                       reinterpret_cast<unsigned long long*>(d_checksum));
    if (st != SIFT_OK) {  // nothing usable was enqueued past this point: drain
        abandon(ctx, *s);
        return st;
    }
    s->state = kFree;
    s->ticket = -1;
    return SIFT_OK;
}

int sift_hip_verify_slots(sift_ctx* ctx, const void* d_slots, int n_slots, size_t slot_bytes,
                          int hdr_rows, int count_word, int sum_word, int n_sum_words,
                          size_t cap_rows, uint64_t* d_bad, void* stream) {
    if (!ctx || !d_bad || (n_slots > 0 && !d_slots) || n_slots < 0 || hdr_rows < 0 ||
        count_word < 0 || sum_word < 0 || n_sum_words < 1 || slot_bytes % 8 ||
        (size_t)(count_word + 1) * 8 > slot_bytes ||
        (size_t)(sum_word + n_sum_words) * 8 > slot_bytes ||
        ((size_t)hdr_rows + cap_rows) * sizeof(sift_kp) > slot_bytes)
        return SIFT_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // every call shares the context's accumulator scratch: calls are chained
    // on the device (each waits for the previous one's event, whatever its
    // stream), and the scratch is regrown only after the last call finished
    if (!ctx->verify_ev)
        SIFT_HIP_TRY(hipEventCreateWithFlags(&ctx->verify_ev, hipEventDisableTiming));
    // scratch: (accumulator, done count) per slot, left zeroed by every call
    const size_t need = 2 * (size_t)std::max(n_slots, 1);
    if (ctx->verify_acc.cap < need && ctx->verify_used)
        SIFT_HIP_TRY(hipEventSynchronize(ctx->verify_ev));
    const bool fresh = !ctx->verify_acc.p || ctx->verify_acc.cap < need;
    if (ctx->verify_acc.ensure(need) != SIFT_OK) return SIFT_ERR_NOMEM;
    if (ctx->verify_used) SIFT_HIP_TRY(hipStreamWaitEvent(st, ctx->verify_ev, 0));
    if (fresh)
        SIFT_HIP_TRY(hipMemsetAsync(ctx->verify_acc.p, 0,
                                    ctx->verify_acc.cap * sizeof(unsigned long long), st));
    SIFT_HIP_TRY(launch_verify_slots(d_slots, n_slots, slot_bytes, hdr_rows, count_word, sum_word,
                                     n_sum_words, cap_rows,
                                     reinterpret_cast<unsigned long long*>(d_bad),
                                     ctx->verify_acc.p, st));
    SIFT_HIP_TRY(hipEventRecord(ctx->verify_ev, st));
    ctx->verify_used = true;
    return SIFT_OK;
}

int sift_hip_detect_batch(sift_ctx* ctx, const void* const* images, int n_images,
                          int input_kind, int w, int h, int c, const sift_params* p,
                          sift_kp** out_kps, size_t* counts, float** out_desc_f32) {
    if (!out_kps || !counts) return SIFT_ERR_ARG;
    *out_kps = nullptr;
    if (out_desc_f32) *out_desc_f32 = nullptr;
    int ticket = 0;
    int st = submit_impl(ctx, images, n_images, input_kind, w, h, c, p, out_desc_f32 != nullptr,
                         &ticket);
    if (st != SIFT_OK) return st;
    size_t n = 0;
    if ((st = sift_hip_wait(ctx, ticket, counts, &n)) != SIFT_OK) return st;
    sift_kp* kps = (sift_kp*)std::malloc(std::max<size_t>(n, 1) * sizeof(sift_kp));
    float* df = out_desc_f32 ? (float*)std::malloc(std::max<size_t>(n, 1) * 128 * sizeof(float))
                             : nullptr;
    if (!kps || (out_desc_f32 && !df)) {
        std::free(kps);
        std::free(df);
        (void)sift_hip_fetch(ctx, ticket, nullptr, nullptr);
        return SIFT_ERR_NOMEM;
    }
    st = sift_hip_fetch(ctx, ticket, kps, df);
    *out_kps = kps;
    if (out_desc_f32) *out_desc_f32 = df;
    return st;
}

int sift_hip_detect(sift_ctx* ctx, const double* hwc, int w, int h, int c,
                    const sift_params* p, sift_kp** out_kps, size_t* out_n,
                    float** out_desc_f32) {
    if (!ctx || !hwc || !out_kps || !out_n) return SIFT_ERR_ARG;
    const void* img = hwc;
    return sift_hip_detect_batch(ctx, &img, 1, SIFT_INPUT_F64_HOST, w, h, c, p, out_kps, out_n,
                                 out_desc_f32);
}

int sift_hip_detect_device(sift_ctx* ctx, const double* d_hwc, int w, int h, int c,
                           const sift_params* p, sift_kp** out_kps, size_t* out_n,
                           float** out_desc_f32) {
    if (!ctx || !d_hwc || !out_kps || !out_n) return SIFT_ERR_ARG;
    const void* img = d_hwc;
    return sift_hip_detect_batch(ctx, &img, 1, SIFT_INPUT_F64_DEVICE, w, h, c, p, out_kps, out_n,
                                 out_desc_f32);
}

namespace {

// sift_hip_match / sift_hip_match_device (sift_match.hip does the work): both
// record lists -> shifted rows + norms, one 2-NN launch, per-query results
// back to the host, compacted in query order.
static int match_impl(sift_ctx* ctx, const sift_kp* k1, size_t n1, const sift_kp* k2, size_t n2,
                      bool on_device, double ratio, sift_match_pair** out, size_t* n_out) {
    if (!ctx || !out || !n_out) return SIFT_ERR_ARG;
    *out = nullptr;
    *n_out = 0;
    if ((n1 && !k1) || (n2 && !k2)) return SIFT_ERR_ARG;
    if (n1 > (1u << 28) || n2 > (1u << 28)) return SIFT_ERR_ARG;
    if (n1 == 0 || n2 == 0) return SIFT_OK;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    const size_t n1p = (n1 + 31) & ~(size_t)31, n2p = (n2 + 31) & ~(size_t)31;
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_k1 = 0;
    const size_t o_k2 = o_k1 + (on_device ? 0 : up(n1 * sizeof(sift_kp)));
    const size_t o_r1 = o_k2 + (on_device ? 0 : up(n2 * sizeof(sift_kp)));
    const size_t o_r2 = o_r1 + up(n1p * 128);
    const size_t o_q1 = o_r2 + up(n2p * 128);
    const size_t o_q2 = o_q1 + up(n1p * sizeof(int));
    const size_t o_j = o_q2 + up(n2p * sizeof(int));
    const size_t o_d = o_j + up(n1 * sizeof(int));
    const size_t need = o_d + up(n1 * sizeof(double));
    if (ctx->mbuf_cap < need) {
        if (ctx->d_mbuf) (void)hipFree(ctx->d_mbuf);
        ctx->d_mbuf = nullptr;
        ctx->mbuf_cap = 0;
        if (hipMalloc(&ctx->d_mbuf, need) != hipSuccess) return SIFT_ERR_NOMEM;
        ctx->mbuf_cap = need;
    }
    int st;
    if ((st = ctx->h_mj.ensure(n1)) != SIFT_OK || (st = ctx->h_md.ensure(n1)) != SIFT_OK)
        return st;
    unsigned char* b = ctx->d_mbuf;
    hipStream_t s = ctx->stream;
    const sift_kp* d1 = k1;
    const sift_kp* d2 = k2;
    if (!on_device) {
        SIFT_HIP_TRY(hipMemcpyAsync(b + o_k1, k1, n1 * sizeof(sift_kp), hipMemcpyHostToDevice, s));
        SIFT_HIP_TRY(hipMemcpyAsync(b + o_k2, k2, n2 * sizeof(sift_kp), hipMemcpyHostToDevice, s));
        d1 = reinterpret_cast<const sift_kp*>(b + o_k1);
        d2 = reinterpret_cast<const sift_kp*>(b + o_k2);
    }
    uint8_t* r1 = b + o_r1;
    uint8_t* r2 = b + o_r2;
    int* q1 = reinterpret_cast<int*>(b + o_q1);
    int* q2 = reinterpret_cast<int*>(b + o_q2);
    int* dj = reinterpret_cast<int*>(b + o_j);
    double* dd = reinterpret_cast<double*>(b + o_d);
    SIFT_HIP_TRY(launch_match_prep(d1, (unsigned)n1, (unsigned)n1p, r1, q1, s));
    SIFT_HIP_TRY(launch_match_prep(d2, (unsigned)n2, (unsigned)n2p, r2, q2, s));
    SIFT_HIP_TRY(launch_match2nn(r1, q1, (unsigned)n1, (unsigned)n1p, r2, q2, (unsigned)n2p,
                                 ratio, dj, dd, s));
    SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_mj.p, dj, n1 * sizeof(int), hipMemcpyDeviceToHost, s));
    SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_md.p, dd, n1 * sizeof(double), hipMemcpyDeviceToHost, s));
    SIFT_HIP_TRY(hipStreamSynchronize(s));
    size_t m = 0;
    for (size_t i = 0; i < n1; ++i) m += ctx->h_mj.p[i] >= 0;
    if (m == 0) return SIFT_OK;
    sift_match_pair* res = static_cast<sift_match_pair*>(std::malloc(m * sizeof(sift_match_pair)));
    if (!res) return SIFT_ERR_NOMEM;
    size_t k = 0;
    for (size_t i = 0; i < n1; ++i) {
        const int j = ctx->h_mj.p[i];
        if (j < 0) continue;
        res[k].i1 = (uint32_t)i;
        res[k].i2 = (uint32_t)j;
        res[k].distance = ctx->h_md.p[i];
        ++k;
    }
    *out = res;
    *n_out = m;
    return SIFT_OK;
}

}  // namespace

int sift_hip_match(sift_ctx* ctx, const sift_kp* kps1, size_t n1, const sift_kp* kps2,
                   size_t n2, double ratio_threshold, sift_match_pair** out, size_t* n_out) {
    return match_impl(ctx, kps1, n1, kps2, n2, false, ratio_threshold, out, n_out);
}

int sift_hip_match_device(sift_ctx* ctx, const sift_kp* d_kps1, size_t n1,
                          const sift_kp* d_kps2, size_t n2, double ratio_threshold,
                          sift_match_pair** out, size_t* n_out) {
    return match_impl(ctx, d_kps1, n1, d_kps2, n2, true, ratio_threshold, out, n_out);
}

void sift_hip_free(void* p) { std::free(p); }

const char* sift_hip_strerror(int status) {
    switch (status) {
        case SIFT_OK: return "ok";
        case SIFT_ERR_ARG: return "invalid argument";
        case SIFT_ERR_CHANNELS: return "unsupported channel count (1 or 3)";
        case SIFT_ERR_TOO_SMALL: return "image too small for the octave pyramid";
        case SIFT_ERR_HIP: return "HIP runtime error";
        case SIFT_ERR_NOMEM: return "out of memory";
        case SIFT_ERR_NO_DEVICE: return "no such HIP device";
        case SIFT_ERR_PARAM: return "parameter outside the supported range";
        case SIFT_ERR_STATE: return "invalid call order (no such job / no previous detect / too many jobs in flight)";
        case SIFT_ERR_NO_COMM: return "RCCL unavailable or a collective failed";
        case SIFT_ERR_PEER: return "another rank of the collective failed";
        default: return "unknown error";
    }
}

namespace {
Slot* last_slot(sift_ctx* ctx) {
    if (!ctx || ctx->last < 0) return nullptr;
    return &ctx->slots[ctx->last];
}
}  // namespace

int sift_hip_last_counts(sift_ctx* ctx, sift_counts* out) {
    if (!ctx || !out) return SIFT_ERR_ARG;
    Slot* s = last_slot(ctx);
    if (!s) return SIFT_ERR_STATE;
    *out = s->counts;
    return SIFT_OK;
}

int sift_hip_copy_level(sift_ctx* ctx, int octave, int level, double* host_out,
                        size_t cap_elems, int* w_out, int* h_out) {
    if (!ctx || !host_out) return SIFT_ERR_ARG;
    Slot* s = last_slot(ctx);
    if (!s) return SIFT_ERR_STATE;
    if (octave < 0 || octave >= s->counts.octaves || level < 0 ||
        level >= s->counts.levels_per_octave)
        return SIFT_ERR_ARG;
    const int W = s->h_pt.w[octave], H = s->h_pt.h[octave];
    if (cap_elems < (size_t)W * H) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    SIFT_HIP_TRY(hipMemcpyAsync(host_out, s->h_pt.lvl[octave][level],
                                (size_t)W * H * sizeof(double), hipMemcpyDeviceToHost, s->sA));
    SIFT_HIP_TRY(hipStreamSynchronize(s->sA));
    if (w_out) *w_out = W;
    if (h_out) *h_out = H;
    return SIFT_OK;
}

int sift_hip_copy_extrema(sift_ctx* ctx, sift_extremum* host_out, size_t cap, size_t* n_out) {
    if (!ctx || !n_out) return SIFT_ERR_ARG;
    Slot* s = last_slot(ctx);
    if (!s) return SIFT_ERR_STATE;
    const size_t n = (size_t)s->counts.extrema;
    *n_out = n;
    if (!host_out) return SIFT_OK;
    if (cap < n) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    for (int L = 0, off = 0; L < kLanes; off += s->lane_n[0][L], ++L)
        if (s->lane_n[0][L])
            SIFT_HIP_TRY(hipMemcpyAsync(host_out + off, s->cand.p + (size_t)L * s->cap_cand,
                                        s->lane_n[0][L] * sizeof(sift_extremum),
                                        hipMemcpyDeviceToHost, s->sA));
    SIFT_HIP_TRY(hipStreamSynchronize(s->sA));
    return SIFT_OK;
}

int sift_hip_copy_records_device(sift_ctx* ctx, void* d_dst, size_t cap, size_t* n_out) {
    if (!ctx || !n_out) return SIFT_ERR_ARG;
    Slot* s = last_slot(ctx);
    if (!s) return SIFT_ERR_STATE;
    const size_t n = (size_t)s->counts.oriented;
    *n_out = n;
    if (!d_dst) return SIFT_OK;
    if (cap < n) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    for (int L = 0, off = 0; L < kLanes; off += s->lane_n[2][L], ++L)
        if (s->lane_n[2][L])
            SIFT_HIP_TRY(hipMemcpyAsync(static_cast<sift_kp*>(d_dst) + off,
                                        s->ori.p + (size_t)L * s->cap_ori,
                                        s->lane_n[2][L] * sizeof(sift_kp),
                                        hipMemcpyDeviceToDevice, s->sA));
    SIFT_HIP_TRY(hipStreamSynchronize(s->sA));
    return SIFT_OK;
}

int sift_hip_last_timing(sift_ctx* ctx, double* ms, int n) {
    if (!ctx || !ms || n < 0) return SIFT_ERR_ARG;
    Slot* s = last_slot(ctx);
    if (!s) return SIFT_ERR_STATE;
    for (int i = 0; i < n && i < 6; ++i) ms[i] = s->t_host[i];
    return SIFT_OK;
}

void* sift_hip_stream(sift_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int sift_hip_set_profiling(sift_ctx* ctx, int enable) {
    if (!ctx) return SIFT_ERR_ARG;
    ctx->profiling = enable != 0;
    return SIFT_OK;
}

int sift_hip_profile_table(sift_ctx* ctx, double* ms, double* bytes, int64_t* launches,
                           int reset) {
    if (!ctx) return SIFT_ERR_ARG;
    for (int r = 0; r < SIFT_PROF_ROWS; ++r) {
        if (ms) ms[r] = ctx->prof_ms[r];
        if (bytes) bytes[r] = ctx->prof_bytes[r];
        if (launches) launches[r] = ctx->prof_launches[r];
        if (reset) {
            ctx->prof_ms[r] = 0.0;
            ctx->prof_bytes[r] = 0.0;
            ctx->prof_launches[r] = 0;
        }
    }
    return SIFT_OK;
}

int sift_hip_blur_profile(sift_ctx* ctx, double* ms, int64_t* launches, double* bytes,
                          int reset) {
    if (!ctx) return SIFT_ERR_ARG;
    double m = 0.0, b = 0.0;
    int64_t n = 0;
    for (int r = SIFT_PROF_PYRAMID; r < SIFT_PROF_PYRAMID + 16; ++r) {
        m += ctx->prof_ms[r];
        b += ctx->prof_bytes[r];
        n += ctx->prof_launches[r];
    }
    if (ms) *ms = m;
    if (launches) *launches = n;
    if (bytes) *bytes = b;
    if (reset)
        for (int r = SIFT_PROF_PYRAMID; r < SIFT_PROF_PYRAMID + 16; ++r) {
            ctx->prof_ms[r] = 0.0;
            ctx->prof_bytes[r] = 0.0;
            ctx->prof_launches[r] = 0;
        }
    return SIFT_OK;
}

}  // extern "C"

// the context's public stream, on its device (sift_stitch.hip)
extern "C" hipStream_t sift_ctx_stream_internal(sift_ctx* ctx) {
    (void)hipSetDevice(ctx->device);
    return ctx->stream;
}
