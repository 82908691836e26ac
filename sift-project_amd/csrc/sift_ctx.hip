// sift_ctx.hip — C-ABI boundary (include/sift_hip.h) and host orchestration
// of the MI355X SIFT pipeline.
//
// Replaces the body of detect_keypoints_and_descriptors (reference
// src/sift.cpp:712-776). Host work is limited to what the reference computes
// with glibc and that feeds bit-exact outputs: the octave count
// (sift.cpp:132-137), the level sigmas (sift.cpp:143-155), the blur taps
// (image.cpp:226-235), the final keypoint size (std::pow, sift.cpp:427-429)
// and clean_keypoints (std::sort + std::unique, sift.cpp:20-24). Everything
// per-pixel and per-keypoint runs in the HIP kernels of sift_kernels.hip,
// enqueued on three streams with no host synchronisation until the counters are
// read back at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <new>
#include <vector>

#include "sift_host.h"
#include "sift_kernels.h"

using namespace sift_amd;

namespace {

// Keypoint lanes: batches alternate between two streams (C, D), each with
// its own region of every keypoint array and its own counters, so the chains
// of consecutive batches run concurrently (within a lane they are serial and
// the snapshot ranges below stay contiguous).
constexpr int kLanes = 2;
// device counter block: [4L..4L+3] live counters of lane L (candidates,
// refined, records), [8..11] zeros, then per keypoint batch g a 4-word
// snapshot taken after its extrema (the batch's candidate end and its raw /
// record begins, lane-local), then four words per chain: work and done
// counters of orientation and descriptor
constexpr int kCtrZeros = 4 * kLanes;
constexpr int kCtrSnap = kCtrZeros + 4;
constexpr int kCtrWork = kCtrSnap + 4 * (kMaxOctaves + 1);
constexpr int kCtrWords = kCtrWork + 4 * (kMaxOctaves + 2);

template <class T>
struct Pinned {  // grow-only pinned host buffer (fast async D2H, no staging)
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (p && cap >= n) return SIFT_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = n < 1024 ? 1024 : n + n / 4;
        if (hipHostMalloc(&p, want * sizeof(T)) != hipSuccess) return SIFT_ERR_NOMEM;
        cap = want;
        return SIFT_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Stage {
    PyrTable pt;
    BlurTaps taps[kMaxLevels];
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

struct EventPair {
    hipEvent_t a, b;
    double bytes;
};

}  // namespace

struct sift_ctx {
    int device = 0;
    hipStream_t stream = nullptr;   // A: pyramid
    hipStream_t stream2 = nullptr;  // B: odd octaves of the pyramid
    hipStream_t stream3 = nullptr;  // C: extrema, refine, orientation, descriptor
    hipStream_t stream4 = nullptr;  // D: keypoint chains of odd batches (lane 1)
    // persistent workgroups of orientation / descriptor per launch: 512 (two
    // per CU; with two keypoint lanes in flight this leaves room for the
    // small octaves' blurs); measured best of 256/384/512/768/1024
    unsigned kp_wgs = 512;
    int batch_px_log2 = 18;         // octaves of >= 2^this pixels get their own batch
    std::vector<hipEvent_t> sync_ev;

    double* d_in = nullptr;
    size_t in_cap = 0;  // elements
    double* d_pyr = nullptr;
    size_t pyr_cap = 0;
    double* d_tmp = nullptr;
    size_t tmp_cap = 0;

    sift_extremum* d_cand = nullptr;
    RawKp* d_raw = nullptr;
    sift_kp* d_ori = nullptr;
    double* d_off0 = nullptr;
    float* d_df32 = nullptr;
    // capacities per lane (each array holds kLanes regions of that size)
    unsigned cap_cand = 0, cap_raw = 0, cap_ori = 0, cap_off0 = 0, cap_df32 = 0;
    int lanes = kLanes;  // 1: every batch on C (SIFT_KP_LANES=1, for A/B)
    unsigned lane_n[3][kLanes] = {};  // last detect: candidates, refined, records per lane
    unsigned* d_ctr = nullptr;
    unsigned* h_ctr = nullptr;  // pinned, live counters of every lane
    PyrTable h_pt{};
    // per-call tables: pinned host staging -> one async copy -> device
    Stage* h_stage = nullptr;
    Stage* d_stage = nullptr;
    PyrTable* d_pt = nullptr;     // &d_stage->pt
    BlurTaps* d_taps = nullptr;   // d_stage->taps

    // last detect
    bool have_run = false;
    sift_counts counts{};
    sift_params last_p{};

    // profiling
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<EventPair> pending;
    double prof_ms = 0.0;
    int64_t prof_launches = 0;
    double prof_bytes = 0.0;

    // records exported by k_descriptor per keypoint batch (mapped pinned)
    Mapped<sift_kp> exp_rec;
    Mapped<double> exp_off0;
    Mapped<unsigned> exp_cnt;  // [begin, end) per chain
    std::vector<hipEvent_t> chain_ev;
    std::vector<unsigned> run_start;

    // matcher: one device arena (inputs, shifted rows, norms, results) and
    // pinned result staging
    unsigned char* d_mbuf = nullptr;
    size_t mbuf_cap = 0;
    Pinned<int> h_mj;
    Pinned<double> h_md;

    // host staging (pinned)
    Pinned<sift_kp> h_ori;
    Pinned<double> h_off0;
    Pinned<float> h_df32;
    std::vector<unsigned> keep;
    FinalizeWorkspace fin_ws;

    // host-side phase wall times of the last detect (ms): enqueue, wait for
    // the device pipeline, records download, finalize (size + sort/unique),
    // output assembly
    double t_host[5] = {0, 0, 0, 0, 0};
};

namespace {

#define SIFT_HIP_TRY(expr)                          \
    do {                                            \
        hipError_t e_ = (expr);                     \
        if (e_ != hipSuccess) return SIFT_ERR_HIP;  \
    } while (0)

int ensure(double** p, size_t* cap, size_t need) {
    if (*cap >= need) return SIFT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, need * sizeof(double)) != hipSuccess) return SIFT_ERR_NOMEM;
    *cap = need;
    return SIFT_OK;
}

template <class T>
int ensure_t(T** p, unsigned* cap, unsigned need) {
    if (*cap >= need && *p) return SIFT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, (size_t)need * sizeof(T)) != hipSuccess) return SIFT_ERR_NOMEM;
    *cap = need;
    return SIFT_OK;
}

// kLanes regions of `need` elements each; *cap = per-lane capacity
template <class T>
int ensure_lanes(T** p, unsigned* cap, unsigned need) {
    if (*cap >= need && *p) return SIFT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, (size_t)need * kLanes * sizeof(T)) != hipSuccess) return SIFT_ERR_NOMEM;
    *cap = need;
    return SIFT_OK;
}

hipEvent_t next_event(sift_ctx* ctx) {
    if (ctx->ev_used == ctx->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ctx->ev_pool.push_back(e);
    }
    return ctx->ev_pool[ctx->ev_used++];
}

// Profiling events for one pyramid launch: timestamps recorded by the
// dispatch packet itself (hipExtLaunchKernel), so timing adds no gaps.
int prof_events(sift_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1, double bytes) {
    *e0 = *e1 = nullptr;
    if (!ctx->profiling) return SIFT_OK;
    *e0 = next_event(ctx);
    *e1 = next_event(ctx);
    if (!*e0 || !*e1) return SIFT_ERR_HIP;
    ctx->pending.push_back({*e0, *e1, bytes});
    return SIFT_OK;
}

int blur_launch(sift_ctx* ctx, hipStream_t s, const double* src, double* dst, int W, int H,
                const BlurTaps& t, double* dec, int Wd, int Hd) {
    if (t.R > kMaxTemplR || t.R < 1) {
        if (ensure(&ctx->d_tmp, &ctx->tmp_cap, (size_t)W * H) != SIFT_OK) return SIFT_ERR_NOMEM;
    }
    hipEvent_t e0, e1;
    const double bytes = 16.0 * (double)W * (double)H + (dec ? 8.0 * (double)Wd * Hd : 0.0);
    if (prof_events(ctx, &e0, &e1, bytes) != SIFT_OK) return SIFT_ERR_HIP;
    SIFT_HIP_TRY(launch_blur(src, dst, W, H, t, dec, Wd, Hd, ctx->d_tmp, s, e0, e1));
    return SIFT_OK;
}

hipEvent_t sync_event(sift_ctx* ctx, int i) {  // untimed cross-stream events
    while ((int)ctx->sync_ev.size() <= i) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        ctx->sync_ev.push_back(e);
    }
    return ctx->sync_ev[i];
}

ExtremaGrid extrema_grid(const Geometry& g, int o_begin, int o_end) {
    ExtremaGrid eg;
    std::memset(&eg, 0, sizeof eg);
    for (int o = o_begin; o < o_end; ++o) {
        const int i = eg.n++;
        const int tx = g.W[o] > 2 ? (g.W[o] - 2 + 63) / 64 : 0;
        const int ty = g.H[o] > 2 ? (g.H[o] - 2 + 15) / 16 : 0;
        eg.oct[i] = o;
        eg.tiles_x[i] = tx > 0 ? tx : 1;
        eg.first_tile[i + 1] = eg.first_tile[i] + tx * ty;
    }
    return eg;
}

int detect_impl(sift_ctx* ctx, const double* d_img, int w, int h, int c,
                const sift_params* p, sift_kp** out_kps, size_t* out_n,
                float** out_desc_f32) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    Geometry g;
    BlurTaps taps_init;
    std::vector<BlurTaps> taps(kMaxLevels);
    DevParams dp;
    int st = host_plan(p, w, h, c, &g, &taps_init, taps.data(), &dp);
    if (st != SIFT_OK) return st;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    ctx->have_run = false;
    ctx->ev_used = 0;
    ctx->pending.clear();

    if ((st = ensure(&ctx->d_pyr, &ctx->pyr_cap, g.total)) != SIFT_OK) return st;
    std::memset(&ctx->h_pt, 0, sizeof ctx->h_pt);
    for (int o = 0; o < g.octaves; ++o) {
        ctx->h_pt.w[o] = g.W[o];
        ctx->h_pt.h[o] = g.H[o];
        for (int l = 0; l < g.n_gauss; ++l) ctx->h_pt.lvl[o][l] = ctx->d_pyr + g.offs[o][l];
    }
    // the previous call's copy out of h_stage has completed (every detect
    // ends with a stream synchronisation), so the staging can be rewritten
    ctx->h_stage->pt = ctx->h_pt;
    for (int l = 0; l < g.n_gauss; ++l) ctx->h_stage->taps[l] = taps[l];
    SIFT_HIP_TRY(hipMemcpyAsync(ctx->d_stage, ctx->h_stage, sizeof(Stage),
                                hipMemcpyHostToDevice, ctx->stream));

    // capacities for the variable-size stages; grown and re-run on overflow
    unsigned want_cand = (unsigned)std::min<size_t>(std::max<size_t>(g.sum_px / 32, 65536),
                                                   (size_t)1 << 28);
    if ((st = ensure_lanes(&ctx->d_cand, &ctx->cap_cand, want_cand)) != SIFT_OK) return st;
    if ((st = ensure_lanes(&ctx->d_raw, &ctx->cap_raw, ctx->cap_cand)) != SIFT_OK) return st;
    if ((st = ensure_lanes(&ctx->d_ori, &ctx->cap_ori, 2 * ctx->cap_raw)) != SIFT_OK) return st;
    if ((st = ensure_lanes(&ctx->d_off0, &ctx->cap_off0, ctx->cap_ori)) != SIFT_OK) return st;
    if (out_desc_f32 &&
        (st = ensure_lanes(&ctx->d_df32, &ctx->cap_df32, ctx->cap_ori * 128u)) != SIFT_OK)
        return st;

    // Three streams (HIP's default is four hardware queues per process, and
    // streams beyond that share a queue and serialise): A (ctx->stream) and
    // B (ctx->stream2) build the pyramid, even and odd octaves, at high
    // priority; C (ctx->stream3) runs, per octave batch as soon as its levels
    // exist, the extrema then refine -> orientation -> descriptor. The
    // keypoint work of octave 0 overlaps the pyramid of the smaller octaves,
    // which is latency-bound and leaves most of the chip idle.
    hipStream_t sA = ctx->stream, sB = ctx->stream2, sC = ctx->stream3, sD = ctx->stream4;
    const int lanes = ctx->lanes;
    hipStream_t lane_stream[kLanes] = {sC, sD};
    int ev_i = 0;

    SIFT_HIP_TRY(hipMemsetAsync(ctx->d_ctr, 0, kCtrWords * sizeof(unsigned), sA));
    // ---- Gaussian pyramid (compute_initial_image + compute_gaussian_images)
    const int W0 = g.W[0], H0 = g.H[0];
    double* G00 = ctx->h_pt.lvl[0][0];
    {
        hipEvent_t e0, e1;
        if (prof_events(ctx, &e0, &e1, 16.0 * (double)W0 * H0) != SIFT_OK) return SIFT_ERR_HIP;
        hipError_t err = hipSuccess;
        const bool fused = launch_blur_initial_fused(d_img, w, h, c, p->double_image_size ? 1 : 0,
                                                     G00, W0, H0, taps_init, sA, e0, e1, &err);
        if (fused) {
            SIFT_HIP_TRY(err);
        } else {
            if (ctx->profiling) ctx->pending.pop_back();
            const double* base_src = d_img;
            if (c != 1 || p->double_image_size) {
                // gray (+ bilinear x2) into level 1's storage; level 1 is
                // written by the first octave blur, after G[0][0] exists
                double* scratch = ctx->h_pt.lvl[0][1];
                SIFT_HIP_TRY(launch_prepare(d_img, w, h, c, p->double_image_size ? 1 : 0,
                                            scratch, W0, H0, sA));
                base_src = scratch;
            }
            if ((st = blur_launch(ctx, sA, base_src, G00, W0, H0, taps_init, nullptr, 0, 0)) !=
                SIFT_OK)
                return st;
        }
    }
    const int dec_level = g.n_gauss - 3;  // = intervals (sift.cpp:195-196)
    // octaves from o_small on are small enough to run LDS-resident in one
    // launch (k_octaves_lds); the larger ones get one k_blur launch per level
    int o_small = g.octaves;
    for (int o = 0; o < g.octaves; ++o)
        if ((size_t)g.W[o] * g.H[o] <= (size_t)kLdsOctavePx) {
            o_small = o;
            break;
        }
    const bool tiles = p->window_size / 2 == 1;
    // Keypoint batches on stream C: each large octave (>= batch_px pixels) is
    // its own batch as soon as its levels exist; the smaller ones, whose
    // keypoint work is too small to amortise a chain of launches, form one
    // final batch. A batch: extrema, a counter snapshot (its candidate end,
    // raw / record begins), refine, orientation, descriptor.
    const size_t batch_px = (size_t)1 << ctx->batch_px_log2;
    int o_merge = g.octaves;  // first octave of the final batch
    for (int o = 0; o < g.octaves; ++o)
        if ((size_t)g.W[o] * g.H[o] < batch_px) {
            o_merge = o;
            break;
        }
    const unsigned* zeros = ctx->d_ctr + kCtrZeros;
    auto snap = [&](int g) { return ctx->d_ctr + kCtrSnap + 4 * g; };
    auto launch_extrema_range = [&](int o_begin, int o_end, int L) -> int {
        hipStream_t sx = lane_stream[L];
        sift_extremum* cand = ctx->d_cand + (size_t)L * ctx->cap_cand;
        unsigned* live = ctx->d_ctr + 4 * L;
        if (tiles) {
            const ExtremaGrid eg = extrema_grid(g, o_begin, o_end);
            SIFT_HIP_TRY(launch_extrema_tiles(ctx->d_pt, eg, g.n_gauss, dp.threshold, cand,
                                              live + 0, ctx->cap_cand, sx));
        } else {
            for (int o = o_begin; o < o_end; ++o)
                SIFT_HIP_TRY(launch_extrema_any(ctx->d_pt, o, g.W[o], g.H[o], g.n_gauss,
                                                p->window_size, dp.threshold, cand, live + 0,
                                                ctx->cap_cand, sx));
        }
        return SIFT_OK;
    };
    // records of every chain also go to the mapped export buffers, sized from
    // the largest record count seen so far (a larger one falls back to one
    // bulk download at the end, and grows them for the next call)
    if ((st = ctx->exp_rec.ensure(std::max<size_t>(ctx->exp_rec.cap, 16384 * kLanes))) !=
            SIFT_OK ||
        (st = ctx->exp_off0.ensure(ctx->exp_rec.cap)) != SIFT_OK ||
        (st = ctx->exp_cnt.ensure(2 * (kMaxOctaves + 2))) != SIFT_OK)
        return st;
    // poison: a range no launch published reads as "not exported"
    std::fill(ctx->exp_cnt.h, ctx->exp_cnt.h + ctx->exp_cnt.cap, 0xFFFFFFFFu);
    // lane L exports its records (lane-local index i) to exp_rec[L * exp_lane + i]
    const unsigned exp_lane = (unsigned)(ctx->exp_rec.cap / kLanes);
    int n_chains = 0;
    std::vector<int> chain_lane;
    // extrema over [o_begin, o_end) then refine -> orientation -> descriptor,
    // on lane L. `begin` (a counter snapshot taken right after the extrema)
    // holds this batch's candidate end and its raw / record begins; candidates
    // start at cand_begin (the lane's previous batch's snapshot). The re-run
    // passes nullptr (lane 0, live counters).
    auto run_chain = [&](int L, int o_begin, int o_end, const unsigned* cand_begin,
                         unsigned* begin) -> int {
        const int ci = n_chains++;
        chain_lane.push_back(L);
        hipStream_t sx = lane_stream[L];
        unsigned* live = ctx->d_ctr + 4 * L;
        sift_extremum* cand = ctx->d_cand + (size_t)L * ctx->cap_cand;
        RawKp* raw = ctx->d_raw + (size_t)L * ctx->cap_raw;
        sift_kp* recs = ctx->d_ori + (size_t)L * ctx->cap_ori;
        double* off0 = ctx->d_off0 + (size_t)L * ctx->cap_ori;
        float* df32 = out_desc_f32 ? ctx->d_df32 + (size_t)L * ctx->cap_ori * 128 : nullptr;
        unsigned* work = ctx->d_ctr + kCtrWork + 4 * ci;
        while ((int)ctx->chain_ev.size() <= ci) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return SIFT_ERR_HIP;
            ctx->chain_ev.push_back(e);
        }
        const ExportSink ex{ctx->exp_rec.d + (size_t)L * exp_lane,
                            ctx->exp_off0.d + (size_t)L * exp_lane, ctx->exp_cnt.d + 2 * ci,
                            exp_lane};
        int st2 = launch_extrema_range(o_begin, o_end, L);
        if (st2 != SIFT_OK) return st2;
        if (begin) SIFT_HIP_TRY(launch_snapshot(live, begin, sx, 0, 4));
        const unsigned* b = begin ? begin : zeros;
        SIFT_HIP_TRY(launch_refine(ctx->d_pt, dp, cand, cand_begin, begin ? begin : live + 0,
                                   ctx->cap_cand, raw, live + 1, ctx->cap_raw, sx));
        SIFT_HIP_TRY(launch_orient(ctx->d_pt, dp, raw, b + 1, live + 1, ctx->cap_raw, recs, off0,
                                   live + 2, ctx->cap_ori, work, ctx->kp_wgs, sx));
        SIFT_HIP_TRY(launch_descriptor(ctx->d_pt, dp, recs, off0, b + 2, live + 2, ctx->cap_ori,
                                       df32, work + 2, ex, ctx->kp_wgs, sx));
        SIFT_HIP_TRY(hipEventRecord(ctx->chain_ev[ci], sx));
        return SIFT_OK;
    };
    int n_batches = 0;
    // batch g (lane g % lanes): octaves [o_begin, o_end), whose levels were
    // enqueued on `sps`
    auto batch = [&](int o_begin, int o_end, std::initializer_list<hipStream_t> sps) -> int {
        const int gb = n_batches++;
        const int L = gb % lanes;
        for (hipStream_t sp : sps) {
            hipEvent_t pyr_done = sync_event(ctx, ev_i++);
            if (!pyr_done) return SIFT_ERR_HIP;
            SIFT_HIP_TRY(hipEventRecord(pyr_done, sp));
            SIFT_HIP_TRY(hipStreamWaitEvent(lane_stream[L], pyr_done, 0));
        }
        return run_chain(L, o_begin, o_end, gb < lanes ? zeros : snap(gb - lanes), snap(gb));
    };
    // The pyramid alternates between two streams, octave o on pyr[o % 2]:
    // octave o+1 only needs the decimated level `intervals` of octave o, so it
    // starts as soon as that level exists and overlaps the last two levels of
    // octave o (the small octaves are latency-bound: two in flight at once).
    hipStream_t pyr[2] = {sA, sB};
    hipEvent_t base_ready = nullptr;  // next octave's base written (decimation)
    auto next_base_event = [&](hipStream_t so) -> int {
        base_ready = sync_event(ctx, ev_i++);
        if (!base_ready) return SIFT_ERR_HIP;
        SIFT_HIP_TRY(hipEventRecord(base_ready, so));
        return SIFT_OK;
    };
    for (int o = 0; o < o_small; ++o) {
        hipStream_t so = pyr[o & 1];
        if (o > 0) SIFT_HIP_TRY(hipStreamWaitEvent(so, base_ready, 0));
        for (int l = 1; l < g.n_gauss; ++l) {
            const bool dec = (l == dec_level) && (o + 1 < g.octaves);
            st = blur_launch(ctx, so, ctx->h_pt.lvl[o][l - 1], ctx->h_pt.lvl[o][l], g.W[o],
                             g.H[o], taps[l], dec ? ctx->h_pt.lvl[o + 1][0] : nullptr,
                             dec ? g.W[o + 1] : 0, dec ? g.H[o + 1] : 0);
            if (st != SIFT_OK) return st;
            if (dec && (st = next_base_event(so)) != SIFT_OK) return st;
        }
        if (o < o_merge && (st = batch(o, o + 1, {so})) != SIFT_OK) return st;
    }
    if (o_small < g.octaves) {
        hipStream_t so = pyr[o_small & 1];
        if (o_small > 0) SIFT_HIP_TRY(hipStreamWaitEvent(so, base_ready, 0));
        double bytes = 0.0;
        for (int o = o_small; o < g.octaves; ++o) {
            bytes += 16.0 * (g.n_gauss - 1) * (double)g.W[o] * (double)g.H[o];
            if (o + 1 < g.octaves) bytes += 8.0 * (double)g.W[o + 1] * (double)g.H[o + 1];
        }
        hipEvent_t e0, e1;
        if (prof_events(ctx, &e0, &e1, bytes) != SIFT_OK) return SIFT_ERR_HIP;
        SIFT_HIP_TRY(launch_octaves_lds(ctx->d_pt, o_small, g.octaves - 1, g.n_gauss,
                                        ctx->d_taps, so, e0, e1));
    }
    if (o_merge < g.octaves && (st = batch(o_merge, g.octaves, {sA, sB})) != SIFT_OK) return st;
    // stream B joins A (the ctx's public stream) before the call returns, and
    // lane D joins C (the counters are read back on C)
    {
        hipEvent_t j = sync_event(ctx, ev_i++);
        if (!j) return SIFT_ERR_HIP;
        SIFT_HIP_TRY(hipEventRecord(j, sB));
        SIFT_HIP_TRY(hipStreamWaitEvent(sA, j, 0));
        hipEvent_t jd = sync_event(ctx, ev_i++);
        if (!jd) return SIFT_ERR_HIP;
        SIFT_HIP_TRY(hipEventRecord(jd, sD));
        SIFT_HIP_TRY(hipStreamWaitEvent(sC, jd, 0));
    }

    // ---- finalise each batch on the host while the device runs the next:
    // sizes with glibc pow and a sorted run per batch, from the exported
    // records (sift.cpp:20-24, 427-429)
    SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_ctr, ctx->d_ctr, 4 * kLanes * sizeof(unsigned),
                                hipMemcpyDeviceToHost, sC));
    clk::time_point t_enq = clk::now(), t_wait;
    bool exported = true;
    unsigned n_keys = 0;
    ctx->run_start.clear();
    ctx->fin_ws.all.resize(ctx->exp_rec.cap);
    for (int ci = 0; ci < n_chains; ++ci) {
        SIFT_HIP_TRY(hipEventSynchronize(ctx->chain_ev[ci]));
        const unsigned b = ctx->exp_cnt.h[2 * ci], e = ctx->exp_cnt.h[2 * ci + 1];
        if (e > exp_lane || b > e) {
            exported = false;
            break;
        }
        const unsigned base = (unsigned)chain_lane[ci] * exp_lane;
        host_sizes(p, ctx->exp_rec.h, ctx->exp_off0.h, base + b, base + e);
        ctx->run_start.push_back(n_keys);
        host_sort_run(ctx->exp_rec.h, base + b, base + e, ctx->fin_ws.all.data() + n_keys,
                      &ctx->fin_ws);
        n_keys += e - b;
    }
    ctx->run_start.push_back(n_keys);

    // ---- the counters; re-run every candidate stage on overflow
    for (int attempt = 0;; ++attempt) {
        if (attempt > 0) {  // pyramid is complete; one batch over everything, on C
            exported = false;
            SIFT_HIP_TRY(hipMemsetAsync(ctx->d_ctr, 0, kCtrWords * sizeof(unsigned), sC));
            SIFT_HIP_TRY(hipStreamSynchronize(sC));
            n_chains = 0;
            chain_lane.clear();
            if ((st = run_chain(0, 0, g.octaves, zeros, nullptr)) != SIFT_OK) return st;
            SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_ctr, ctx->d_ctr, 4 * kLanes * sizeof(unsigned),
                                        hipMemcpyDeviceToHost, sC));
        }
        SIFT_HIP_TRY(hipStreamSynchronize(sC));
        t_wait = clk::now();
        unsigned nc = 0, nr = 0, no = 0;  // largest per-lane counts
        for (int L = 0; L < kLanes; ++L) {
            nc = std::max(nc, ctx->h_ctr[4 * L]);
            nr = std::max(nr, ctx->h_ctr[4 * L + 1]);
            no = std::max(no, ctx->h_ctr[4 * L + 2]);
        }
        if (nc <= ctx->cap_cand && nr <= ctx->cap_raw && no <= ctx->cap_ori) break;
        if (attempt >= 3) return SIFT_ERR_NOMEM;
        // grow every stage that overflowed (refine/orient counts are lower
        // bounds when an upstream stage overflowed, so grow generously)
        const unsigned nc2 = std::max(ctx->cap_cand, nc) * 2u;
        const unsigned nr2 = std::max(std::max(ctx->cap_raw, nr) * 2u, nc2);
        const unsigned no2 = std::max(std::max(ctx->cap_ori, no) * 2u, 2u * nr2);
        if ((st = ensure_lanes(&ctx->d_cand, &ctx->cap_cand, nc2)) != SIFT_OK) return st;
        if ((st = ensure_lanes(&ctx->d_raw, &ctx->cap_raw, nr2)) != SIFT_OK) return st;
        if ((st = ensure_lanes(&ctx->d_ori, &ctx->cap_ori, no2)) != SIFT_OK) return st;
        if ((st = ensure_lanes(&ctx->d_off0, &ctx->cap_off0, ctx->cap_ori)) != SIFT_OK) return st;
        if (out_desc_f32 &&
            (st = ensure_lanes(&ctx->d_df32, &ctx->cap_df32, ctx->cap_ori * 128u)) != SIFT_OK)
            return st;
    }

    unsigned n_lane[kLanes];  // records per lane
    unsigned n_ori = 0;
    for (int L = 0; L < kLanes; ++L) {
        n_lane[L] = ctx->h_ctr[4 * L + 2];
        ctx->lane_n[0][L] = ctx->h_ctr[4 * L];
        ctx->lane_n[1][L] = ctx->h_ctr[4 * L + 1];
        ctx->lane_n[2][L] = n_lane[L];
        n_ori += n_lane[L];
    }
    if (exported && n_keys != n_ori) exported = false;
    const sift_kp* rec_src = ctx->exp_rec.h;
    // host position of lane L's record i: exported, L * exp_lane + i; after a
    // bulk download, the lanes are concatenated
    size_t host_base[kLanes];
    for (int L = 0, acc = 0; L < kLanes; acc += n_lane[L], ++L)
        host_base[L] = exported ? (size_t)L * exp_lane : (size_t)acc;
    if (!exported) {  // bulk download of every record
        if ((st = ctx->h_ori.ensure(n_ori)) != SIFT_OK) return st;
        if ((st = ctx->h_off0.ensure(n_ori)) != SIFT_OK) return st;
        for (int L = 0; L < kLanes; ++L) {
            if (!n_lane[L]) continue;
            SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_ori.p + host_base[L],
                                        ctx->d_ori + (size_t)L * ctx->cap_ori,
                                        n_lane[L] * sizeof(sift_kp), hipMemcpyDeviceToHost, sC));
            SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_off0.p + host_base[L],
                                        ctx->d_off0 + (size_t)L * ctx->cap_ori,
                                        n_lane[L] * sizeof(double), hipMemcpyDeviceToHost, sC));
        }
        rec_src = ctx->h_ori.p;
    }
    if (out_desc_f32) {
        const size_t span = exported ? ctx->exp_rec.cap : (size_t)n_ori;
        if ((st = ctx->h_df32.ensure(std::max<size_t>(span, 1) * 128)) != SIFT_OK) return st;
        for (int L = 0; L < kLanes; ++L)
            if (n_lane[L])
                SIFT_HIP_TRY(hipMemcpyAsync(ctx->h_df32.p + host_base[L] * 128,
                                            ctx->d_df32 + (size_t)L * ctx->cap_ori * 128,
                                            (size_t)n_lane[L] * 128 * sizeof(float),
                                            hipMemcpyDeviceToHost, sC));
    }
    SIFT_HIP_TRY(hipStreamSynchronize(sC));
    const auto t_copy = clk::now();

    if (ctx->profiling) {
        for (const EventPair& e : ctx->pending) {
            float ems = 0.f;
            SIFT_HIP_TRY(hipEventElapsedTime(&ems, e.a, e.b));
            ctx->prof_ms += ems;
            ctx->prof_bytes += e.bytes;
            ctx->prof_launches += 1;
        }
        ctx->pending.clear();
    }

    // clean_keypoints: merge the sorted runs and unique (or all of it, after
    // a bulk download), in the g++-built layer
    ctx->keep.resize(std::max<unsigned>(n_ori, 1));
    size_t n;
    if (exported) {
        n = host_merge_unique(ctx->exp_rec.h, ctx->fin_ws.all.data(), ctx->run_start,
                              ctx->keep.data(), &ctx->fin_ws);
    } else {
        n = host_finalize(p, ctx->h_ori.p, ctx->h_off0.p, n_ori, ctx->keep.data(),
                          &ctx->fin_ws);
        // the next call exports this many records per lane
        const unsigned lane_max = std::max(n_lane[0], n_lane[1]);
        if (lane_max > exp_lane) {
            const size_t want = ((size_t)lane_max + lane_max / 2) * kLanes;
            if ((st = ctx->exp_rec.ensure(want)) != SIFT_OK ||
                (st = ctx->exp_off0.ensure(want)) != SIFT_OK)
                return st;
        }
    }
    const auto t_fin = clk::now();

    sift_kp* kps = (sift_kp*)std::malloc(std::max<size_t>(n, 1) * sizeof(sift_kp));
    if (!kps) return SIFT_ERR_NOMEM;
    for (size_t i = 0; i < n; ++i) kps[i] = rec_src[ctx->keep[i]];
    float* df = nullptr;
    if (out_desc_f32) {
        df = (float*)std::malloc(std::max<size_t>(n, 1) * 128 * sizeof(float));
        if (!df) {
            std::free(kps);
            return SIFT_ERR_NOMEM;
        }
        for (size_t i = 0; i < n; ++i)
            std::memcpy(df + i * 128, ctx->h_df32.p + (size_t)ctx->keep[i] * 128,
                        128 * sizeof(float));
    }
    const auto t_out = clk::now();
    ctx->t_host[0] = ms(t0, t_enq);
    ctx->t_host[1] = ms(t_enq, t_wait);
    ctx->t_host[2] = ms(t_wait, t_copy);
    ctx->t_host[3] = ms(t_copy, t_fin);
    ctx->t_host[4] = ms(t_fin, t_out);
    *out_kps = kps;
    *out_n = n;
    if (out_desc_f32) *out_desc_f32 = df;

    ctx->counts.extrema = (int64_t)ctx->lane_n[0][0] + ctx->lane_n[0][1];
    ctx->counts.refined = (int64_t)ctx->lane_n[1][0] + ctx->lane_n[1][1];
    ctx->counts.oriented = n_ori;
    ctx->counts.final_n = (int64_t)n;
    ctx->counts.octaves = g.octaves;
    ctx->counts.levels_per_octave = g.n_gauss;
    ctx->counts.octave0_w = g.W[0];
    ctx->counts.octave0_h = g.H[0];
    ctx->last_p = *p;
    ctx->have_run = true;
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
    if (const char* e = std::getenv("SIFT_KP_WGS")) ctx->kp_wgs = (unsigned)std::atoi(e);
    if (ctx->kp_wgs < 1) ctx->kp_wgs = 1;
    if (const char* e = std::getenv("SIFT_BATCH_PX_LOG2")) ctx->batch_px_log2 = std::atoi(e);
    if (const char* e = std::getenv("SIFT_KP_LANES")) ctx->lanes = std::atoi(e) == 1 ? 1 : kLanes;
    if (ctx->batch_px_log2 < 0 || ctx->batch_px_log2 > 40) ctx->batch_px_log2 = 18;
    if (hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stream3, hipStreamNonBlocking, prio_lo) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stream4, hipStreamNonBlocking, prio_lo) != hipSuccess ||
        hipMalloc(&ctx->d_ctr, kCtrWords * sizeof(unsigned)) != hipSuccess ||
        hipHostMalloc(&ctx->h_ctr, 4 * kLanes * sizeof(unsigned)) != hipSuccess ||
        hipHostMalloc(&ctx->h_stage, sizeof(Stage)) != hipSuccess ||
        hipMalloc(&ctx->d_stage, sizeof(Stage)) != hipSuccess ||
        prepare_kernel_attributes() != hipSuccess) {
        sift_hip_destroy(ctx);
        return SIFT_ERR_HIP;
    }
    ctx->d_pt = &ctx->d_stage->pt;
    ctx->d_taps = ctx->d_stage->taps;
    *out = ctx;
    return SIFT_OK;
}

int sift_hip_destroy(sift_ctx* ctx) {
    if (!ctx) return SIFT_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    if (ctx->stream3) (void)hipStreamSynchronize(ctx->stream3);
    if (ctx->stream4) (void)hipStreamSynchronize(ctx->stream4);
    void* bufs[] = {ctx->d_in, ctx->d_pyr, ctx->d_tmp, ctx->d_cand, ctx->d_raw,
                    ctx->d_ori, ctx->d_off0, ctx->d_df32, ctx->d_ctr, ctx->d_stage,
                    ctx->d_mbuf};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (ctx->h_ctr) (void)hipHostFree(ctx->h_ctr);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    ctx->h_ori.release();
    ctx->exp_rec.release();
    ctx->exp_off0.release();
    ctx->exp_cnt.release();
    for (hipEvent_t e : ctx->chain_ev) (void)hipEventDestroy(e);
    ctx->h_off0.release();
    ctx->h_df32.release();
    ctx->h_mj.release();
    ctx->h_md.release();
    for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->sync_ev) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    if (ctx->stream3) (void)hipStreamDestroy(ctx->stream3);
    if (ctx->stream4) (void)hipStreamDestroy(ctx->stream4);
    delete ctx;
    return SIFT_OK;
}

int sift_hip_detect(sift_ctx* ctx, const double* hwc, int w, int h, int c,
                    const sift_params* p, sift_kp** out_kps, size_t* out_n,
                    float** out_desc_f32) {
    if (!ctx || !hwc || !out_kps || !out_n) return SIFT_ERR_ARG;
    if (w <= 0 || h <= 0) return SIFT_ERR_ARG;
    if (c != 1 && c != 3) return SIFT_ERR_CHANNELS;
    sift_params def;
    if (!p) {
        sift_params_default(&def);
        p = &def;
    }
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    const size_t ne = (size_t)w * h * c;
    int st = ensure(&ctx->d_in, &ctx->in_cap, ne);
    if (st != SIFT_OK) return st;
    SIFT_HIP_TRY(hipMemcpyAsync(ctx->d_in, hwc, ne * sizeof(double), hipMemcpyHostToDevice,
                                ctx->stream));
    return detect_impl(ctx, ctx->d_in, w, h, c, p, out_kps, out_n, out_desc_f32);
}

int sift_hip_detect_device(sift_ctx* ctx, const double* d_hwc, int w, int h, int c,
                           const sift_params* p, sift_kp** out_kps, size_t* out_n,
                           float** out_desc_f32) {
    if (!ctx || !d_hwc || !out_kps || !out_n) return SIFT_ERR_ARG;
    sift_params def;
    if (!p) {
        sift_params_default(&def);
        p = &def;
    }
    return detect_impl(ctx, d_hwc, w, h, c, p, out_kps, out_n, out_desc_f32);
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
        case SIFT_ERR_STATE: return "no previous detect on this context";
        default: return "unknown error";
    }
}

int sift_hip_last_counts(sift_ctx* ctx, sift_counts* out) {
    if (!ctx || !out) return SIFT_ERR_ARG;
    if (!ctx->have_run) return SIFT_ERR_STATE;
    *out = ctx->counts;
    return SIFT_OK;
}

int sift_hip_copy_level(sift_ctx* ctx, int octave, int level, double* host_out,
                        size_t cap_elems, int* w_out, int* h_out) {
    if (!ctx || !host_out) return SIFT_ERR_ARG;
    if (!ctx->have_run) return SIFT_ERR_STATE;
    if (octave < 0 || octave >= ctx->counts.octaves || level < 0 ||
        level >= ctx->counts.levels_per_octave)
        return SIFT_ERR_ARG;
    const int W = ctx->h_pt.w[octave], H = ctx->h_pt.h[octave];
    if (cap_elems < (size_t)W * H) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    SIFT_HIP_TRY(hipMemcpyAsync(host_out, ctx->h_pt.lvl[octave][level],
                                (size_t)W * H * sizeof(double), hipMemcpyDeviceToHost,
                                ctx->stream));
    SIFT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (w_out) *w_out = W;
    if (h_out) *h_out = H;
    return SIFT_OK;
}

int sift_hip_copy_extrema(sift_ctx* ctx, sift_extremum* host_out, size_t cap, size_t* n_out) {
    if (!ctx || !n_out) return SIFT_ERR_ARG;
    if (!ctx->have_run) return SIFT_ERR_STATE;
    const size_t n = (size_t)ctx->counts.extrema;
    *n_out = n;
    if (!host_out) return SIFT_OK;
    if (cap < n) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    for (int L = 0, off = 0; L < kLanes; off += ctx->lane_n[0][L], ++L)
        if (ctx->lane_n[0][L])
            SIFT_HIP_TRY(hipMemcpyAsync(host_out + off, ctx->d_cand + (size_t)L * ctx->cap_cand,
                                        ctx->lane_n[0][L] * sizeof(sift_extremum),
                                        hipMemcpyDeviceToHost, ctx->stream));
    SIFT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SIFT_OK;
}

int sift_hip_copy_records_device(sift_ctx* ctx, void* d_dst, size_t cap, size_t* n_out) {
    if (!ctx || !n_out) return SIFT_ERR_ARG;
    if (!ctx->have_run) return SIFT_ERR_STATE;
    const size_t n = (size_t)ctx->counts.oriented;
    *n_out = n;
    if (!d_dst) return SIFT_OK;
    if (cap < n) return SIFT_ERR_ARG;
    SIFT_HIP_TRY(hipSetDevice(ctx->device));
    for (int L = 0, off = 0; L < kLanes; off += ctx->lane_n[2][L], ++L)
        if (ctx->lane_n[2][L])
            SIFT_HIP_TRY(hipMemcpyAsync(static_cast<sift_kp*>(d_dst) + off,
                                        ctx->d_ori + (size_t)L * ctx->cap_ori,
                                        ctx->lane_n[2][L] * sizeof(sift_kp),
                                        hipMemcpyDeviceToDevice, ctx->stream));
    SIFT_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SIFT_OK;
}

int sift_hip_last_timing(sift_ctx* ctx, double* ms, int n) {
    if (!ctx || !ms || n < 0) return SIFT_ERR_ARG;
    if (!ctx->have_run) return SIFT_ERR_STATE;
    for (int i = 0; i < n && i < 5; ++i) ms[i] = ctx->t_host[i];
    return SIFT_OK;
}

void* sift_hip_stream(sift_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int sift_hip_set_profiling(sift_ctx* ctx, int enable) {
    if (!ctx) return SIFT_ERR_ARG;
    ctx->profiling = enable != 0;
    return SIFT_OK;
}

int sift_hip_blur_profile(sift_ctx* ctx, double* ms, int64_t* launches, double* bytes,
                          int reset) {
    if (!ctx) return SIFT_ERR_ARG;
    if (ms) *ms = ctx->prof_ms;
    if (launches) *launches = ctx->prof_launches;
    if (bytes) *bytes = ctx->prof_bytes;
    if (reset) {
        ctx->prof_ms = 0.0;
        ctx->prof_launches = 0;
        ctx->prof_bytes = 0.0;
    }
    return SIFT_OK;
}

}  // extern "C"
