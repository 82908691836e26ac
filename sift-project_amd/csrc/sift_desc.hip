// sift_desc.hip — compute_descriptors + update_histogram +
// convert_hist_to_desc (reference src/sift.cpp:541-682) on gfx950.
//
// Default (desc_mode 0): k_descriptor_split<true>, every per-sample
// operation in f64 as the reference does it (sift.cpp:641-678), one record
// per 256-thread workgroup, its rows dealt to the four waves.
// desc_mode 1 / 2 keep the round-3 kernels with f32 sample math for A/B
// (k_descriptor_wave: one wave per record; k_descriptor_split<false>).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sift_device.h"
#include "sift_kernels.h"
#include "sift_math64.h"

// replicas of the 4x4x8 f64 histogram per wave (power of two <= 16) and the
// minimum workgroups per CU of k_descriptor_split
#ifndef SIFT_DSPLIT_REPS
#define SIFT_DSPLIT_REPS 16
#endif
#ifndef SIFT_DSPLIT_OCC
#define SIFT_DSPLIT_OCC (SIFT_DSPLIT_REPS >= 16 ? 2 : 4)
#endif

namespace sift_amd {

namespace {

// atan2 in f32 for the descriptor's sample math: octant reduction to
// a = min(|x|, |y|) / max(|x|, |y|) (v_rcp_f32, 1 ulp), atan(a) as
// a + a^3 p(a^2) with a degree-7 p fitted for minimum max error on [0, 1]
// (8.5e-8 rad in f32 arithmetic over 2e6 points), then the quadrant fix-up.
// About 20 VALU instructions against ~35 for atan2f; total error below
// 2e-7 rad, i.e. < 3e-7 of a descriptor orientation bin (contract: 1e-4 on
// the normalised floats). atan2(0, 0) = 0; signs of zeros as atan2f.
__device__ __forceinline__ float atan2_f32(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    const float t = a * a;
    float p = 0.0026222362648695707f;
    p = fmaf(p, t, -0.015132501721382141f);
    p = fmaf(p, t, 0.04112179949879646f);
    p = fmaf(p, t, -0.0736670047044754f);
    p = fmaf(p, t, 0.1057392954826355f);
    p = fmaf(p, t, -0.1418597400188446f);
    p = fmaf(p, t, 0.1999039649963379f);
    p = fmaf(p, t, -0.33332985639572144f);
    float th = fmaf(a * t, p, a);
    if (ay > ax) th = 1.57079637f - th;
    if (x < 0.0f) th = 3.14159274f - th;
    return copysignf(th, y);
}


// ---------------------------------------------------------------------------
// k_descriptor_wave (desc_mode 1, the default): one WAVEFRONT per record
// (sift.cpp:610-682), four independent waves per workgroup pulling records
// from the work counter; no workgroup barrier anywhere.
//
// Per-record cost was dominated by work every wave of the 256-thread
// version repeated (record setup with f64 sin/cos, the f64 row-interval
// solve with exact snapping, histogram zero/reduce/normalise): ~1150 VALU
// instructions per wave per record against ~1100 for the samples
// themselves (r02 SQ counters). Here a record's setup runs once, and:
//  * The sample set is enumerated as an f32 SUPERSET of the reference's
//    rotated box (row intervals widened by 0.01 column). No exact test is
//    needed: a sample's trilinear weights vanish continuously at the box
//    edges (row_bin -> -1 puts weight fr -> 0 on row 0 and the rest on the
//    skipped row -1; row_bin -> 4 puts 1 - fr -> 0 on row 3), so a sample
//    just outside contributes exactly nothing (its cells are skipped) and
//    one just inside contributes ~1e-7 of its magnitude — the same order as
//    the f32 sample math itself (contract: 1e-4 on the floats).
//  * Sample math as describe<1> (f32, f64 histograms); the integer bounds
//    (radius, image border) are exact.
//  * kDescWReps replica-interleaved f64 copies of the 4x4x8 histogram per
//    wave; the 128 bins are reduced two per lane (bins l and l + 64), the
//    two normalisation sums are in-wave reductions.
// A wave's LDS instructions execute in order, so zeroing -> accumulation
// -> reduction -> next record's zeroing needs only compiler ordering
// (wave_sync).
// ---------------------------------------------------------------------------
#ifndef SIFT_DESCW_REPS  // 16: conflict-free atomics; 4 / 8 measured equal on the bench
#define SIFT_DESCW_REPS 16
#endif
#ifndef SIFT_DESCW_OCC  // min workgroups per CU (16 replicas: 64 KB LDS each)
#define SIFT_DESCW_OCC (SIFT_DESCW_REPS >= 16 ? 2 : 5)
#endif
#ifndef SIFT_DESCW_WALK
#define SIFT_DESCW_WALK 0
#endif
#ifndef SIFT_DESCW_AHEAD
#define SIFT_DESCW_AHEAD 1
#endif
constexpr int kDescWReps = SIFT_DESCW_REPS;
static_assert(kDescWReps >= 1 && kDescWReps <= 16 && (kDescWReps & (kDescWReps - 1)) == 0,
              "replicas: a power of two <= 16");
// Replica-interleaved layout: bin i of replica r at hist[i * kDescWReps + r],
// r = lane % kDescWReps. ds_add_f64 serves 16 lanes per LDS cycle over 32
// banks (bank = dword address mod 32); a lane's bank pair is then
// 2 (i * kDescWReps + r) mod 32, so with 16 replicas every lane of a group
// owns its bank pair whatever bins the samples hit (conflict-free), with 8
// two lanes share a replica and collide only on bins of equal parity. (A
// replica-major layout, r * stride + i, leaves the bank to the bin: the
// atomics measured ~1 extra LDS cycle per LDS cycle, lane % 4 or % 16 alike.)
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ __launch_bounds__(256, SIFT_DESCW_OCC) void k_descriptor_wave(
    const PyrTable* __restrict__ pt, DevParams P, sift_kp* __restrict__ recs,
    const RecSide* __restrict__ rec_side, const unsigned* __restrict__ rec_begin,
    const unsigned* __restrict__ n_rec, unsigned cap_rec, float* __restrict__ desc_f32,
    unsigned* __restrict__ work, ExportSink ex) {
    __shared__ __attribute__((aligned(16))) double hist_all[4 * 128 * kDescWReps];
    set_job_prio(pt->jp, 0);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* const hist = hist_all + wv * 128 * kDescWReps;
    double* const rep = hist + (lane & (kDescWReps - 1));  // bin i at rep[i * kDescWReps]
    const unsigned n = min(*n_rec, cap_rec);
    const unsigned k0 = min(*rec_begin, n);
    // the launch's record range is fixed before it starts (orientation has
    // completed); the host reads it after the chain's completion event
    if (ex.cnt && blockIdx.x == 0 && threadIdx.x == 0) {
        ex.cnt[0] = k0;
        ex.cnt[1] = n;
    }
    constexpr float kHalfW = (float)(kDescW / 2 - 0.5);  // row_bin = row_rot + 1.5
    const float wscale = (float)(-1.4426950408889634 / (0.5 * kDescW * kDescW));
    for (;;) {
        unsigned claim = 0;
        if (lane == 0) claim = atomicAdd(work, 1u);
        const unsigned k = k0 + __builtin_amdgcn_readfirstlane(claim);
        if (k >= n) break;
        // ---- record setup (wave-uniform)
        const sift_kp& R = recs[k];
        const double kx = R.x, ky = R.y, ksize = R.size, pori = R.pori;
        const int o = R.octave, layer = R.layer;
        const RecSide rside = rec_side[k];
        gdouble* img = gbl(plane(pt, rside.img, o, layer));
        const int W = pt->w[o], H = pt->h[o];
        const double inv = P.double_image ? (1.0 / pow2i(o - 1)) : (1.0 / pow2i(o));
        const int x = (int)(kx * inv);
        const int y = (int)(ky * inv);
        const double hw = P.desc_scale_factor * (ksize * inv);
        const double rr = round(hw * 0.5 * sqrt(2.0) * (kDescW + 1.0) + 0.5);
        const double diag = sqrt((double)(W * W + H * H));
        const int radius = (int)((diag < rr) ? diag : rr);  // std::min(rr, diag)
        const int side = 2 * radius + 1;
        float saf, caf;
        sincosf((float)pori, &saf, &caf);
        const float ihwf = (float)(1.0 / hw);
        const float porif = (float)pori;
        // |row_rot| < 2.5 and |col_rot| < 2.5, in units of hw
        const float limf = (float)((0.5 * kDescW + 0.5) * hw);
        for (int i = lane; i < 64 * kDescWReps; i += 64)
            reinterpret_cast<double2*>(hist)[i] = make_double2(0.0, 0.0);
        wave_sync();
        // ---- rows in groups of 64 (lane = row), samples 64 at a time
        for (int g0 = 0; g0 < side; g0 += 64) {
            const int row = g0 + lane - radius;
            int lo = 0, len = 0;
            if (g0 + lane < side && row + y > 0 && row + y < H - 1) {
                const float fr = (float)row, ra = fr * caf, rs = fr * saf;
                float clo = (float)max(-radius, 1 - x), chi = (float)min(radius, W - 2 - x);
                // |c sa + r ca| < lim and |c ca - r sa| < lim, widened by 0.01
                // column (f32 rounding of the bounds is far below that)
                if (fabsf(saf) > 1e-6f) {
                    const float is = 1.0f / saf;
                    const float a1 = (-limf - ra) * is, a2 = (limf - ra) * is;
                    clo = fmaxf(clo, fminf(a1, a2) - 0.01f);
                    chi = fminf(chi, fmaxf(a1, a2) + 0.01f);
                } else if (!(fabsf(ra) < limf + 0.01f)) {
                    chi = clo - 1.0f;
                }
                if (fabsf(caf) > 1e-6f) {
                    const float ic = 1.0f / caf;
                    const float b1 = (-limf + rs) * ic, b2 = (limf + rs) * ic;
                    clo = fmaxf(clo, fminf(b1, b2) - 0.01f);
                    chi = fminf(chi, fmaxf(b1, b2) + 0.01f);
                } else if (!(fabsf(rs) < limf + 0.01f)) {
                    chi = clo - 1.0f;
                }
                lo = (int)ceilf(clo);
                const int hi = (int)floorf(chi);
                len = hi >= lo ? hi - lo + 1 : 0;
            }
            int pre = len;  // inclusive scan of the row lengths
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(pre, off);
                if (lane >= off) pre += t;
            }
            const int total = __builtin_amdgcn_readlane(pre, 63);
            // (row, col) of sample t0 + lane; false past the end. Its row r
            // is the number of rows whose inclusive prefix is <= t: a
            // branch-free binary search over the 64 prefixes (the scalar
            // walk over the rows a block touches cost ~20 SALU per block)
#if SIFT_DESCW_WALK
            int cur = 0;  // A/B: the scalar walk
#endif
            auto locate = [&](int t0, int& srow, int& scol) -> bool {
                const int t = t0 + lane;
#if SIFT_DESCW_WALK
                int r = cur, nxt = cur;
                for (int q = cur; q < 64; ++q) {
                    const int pq = __builtin_amdgcn_readlane(pre, q);
                    if (pq > t0 + 63) break;
                    r += (pq <= t) ? 1 : 0;
                    nxt = q + 1;
                }
                cur = nxt;
#else
                int r = 0;
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1)
                    if (__shfl(pre, r + step - 1) <= t) r += step;
#endif
                const int lo_r = __shfl(lo, r);
                const int ex_r = __shfl(pre, r) - __shfl(len, r);
                srow = g0 + r - radius;
                scol = lo_r + (t - ex_r);
                return t < total;
            };
            // gradient loads issued unconditionally (see describe's fetch)
            auto fetch = [&](bool ok, int srow, int scol, double* v) {
                const size_t r0 = ok ? (size_t)(srow + y) * W + scol + x : (size_t)W + 1;
                v[0] = img[r0 + 1];
                v[1] = img[r0 - 1];
                v[2] = img[r0 - W];
                v[3] = img[r0 + W];
            };
            // kAhead blocks of 64 samples whose gradient loads are in flight
            // while the current block is processed
            constexpr int kAhead = SIFT_DESCW_AHEAD;
            int srow = 0, scol = 0, qrow[kAhead], qcol[kAhead];
            bool qok[kAhead];
            double cv[4] = {0.0, 0.0, 0.0, 0.0}, qv[kAhead][4];
            bool cok = total > 0 && locate(0, srow, scol);
            fetch(cok, srow, scol, cv);
#pragma unroll
            for (int a = 0; a + 1 < kAhead; ++a) {
                qrow[a] = qcol[a] = 0;
                qok[a] = 64 * (a + 1) < total && locate(64 * (a + 1), qrow[a], qcol[a]);
                fetch(qok[a], qrow[a], qcol[a], qv[a]);
            }
            for (int t0 = 0; t0 < total; t0 += 64) {
                {
                    int& nrow = qrow[kAhead - 1];
                    int& ncol = qcol[kAhead - 1];
                    nrow = ncol = 0;
                    qok[kAhead - 1] =
                        t0 + 64 * kAhead < total && locate(t0 + 64 * kAhead, nrow, ncol);
                    fetch(qok[kAhead - 1], nrow, ncol, qv[kAhead - 1]);
                }
                if (cok) {
                    const float fcol = (float)scol, frow = (float)srow;
                    const float row_rot = fmaf(fcol, saf, frow * caf) * ihwf;
                    const float col_rot = fmaf(fcol, caf, -(frow * saf)) * ihwf;
                    const float rb = row_rot + kHalfW;
                    const float cb = col_rot + kHalfW;
                    const float dx = (float)(cv[0] - cv[1]);
                    const float dy = (float)(cv[2] - cv[3]);
                    const float mag = __builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy));
                    const float ob = (atan2_f32(dy, dx) - porif) * (float)(kDescBins / kTwoPi);
                    const float wgt =
                        __builtin_amdgcn_exp2f(fmaf(row_rot, row_rot, col_rot * col_rot) * wscale);
                    const float m = mag * wgt;
                    const float fbr = floorf(rb), fbc = floorf(cb), fbo = floorf(ob);
                    const int br = (int)fbr, bc = (int)fbc, bo = (int)fbo;
                    const float fr = rb - fbr, fc = cb - fbc, fo = ob - fbo;
#pragma unroll
                    for (int rq = 0; rq <= 1; ++rq) {
                        const int ri = br + rq;
                        if ((unsigned)ri >= (unsigned)kDescW) continue;
                        const float vr = m * ((rq == 0) ? 1.0f - fr : fr);
#pragma unroll
                        for (int cq = 0; cq <= 1; ++cq) {
                            const int ci = bc + cq;
                            if ((unsigned)ci >= (unsigned)kDescW) continue;
                            const float vc = vr * ((cq == 0) ? 1.0f - fc : fc);
                            double* hb = &rep[(ri * 32 + ci * 8) * kDescWReps];
                            atomicAdd(&hb[(bo & 7) * kDescWReps], (double)(vc * (1.0f - fo)));
                            atomicAdd(&hb[((bo + 1) & 7) * kDescWReps], (double)(vc * fo));
                        }
                    }
                }
                srow = qrow[0];
                scol = qcol[0];
                cok = qok[0];
#pragma unroll
                for (int q = 0; q < 4; ++q) cv[q] = qv[0][q];
#pragma unroll
                for (int a = 0; a + 1 < kAhead; ++a) {
                    qrow[a] = qrow[a + 1];
                    qcol[a] = qcol[a + 1];
                    qok[a] = qok[a + 1];
#pragma unroll
                    for (int q = 0; q < 4; ++q) qv[a][q] = qv[a + 1][q];
                }
            }
        }
        wave_sync();
        // ---- reduce the replicas (bins lane, lane + 64), normalise, clamp,
        // renormalise, quantise (sift.cpp:576-603)
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int q = 0; q < kDescWReps; ++q) {
            // fixed order per bin, rotated by lane so the 16 lanes of a read
            // group start on different bank pairs
            const int r = (q + lane) & (kDescWReps - 1);
            v0 += hist[lane * kDescWReps + r];
            v1 += hist[(lane + 64) * kDescWReps + r];
        }
        const double ninv = 1.0 / sqrt(wave_sum_f64(v0 * v0 + v1 * v1));
        double c0 = v0 * ninv, c1 = v1 * ninv;
        if (c0 > kMagThr) c0 = kMagThr;
        if (c1 > kMagThr) c1 = kMagThr;
        const double inv2 = 1.0 / sqrt(wave_sum_f64(c0 * c0 + c1 * c1));
        auto quant = [&](double c) -> uint8_t {
            const double q = floor(kIntFactor * c * inv2);
            int val = (q == q) ? (int)q : 0;  // NaN -> 0 (Appendix A.17)
            return (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
        };
        const uint8_t u0 = quant(c0), u1 = quant(c1);
        recs[k].desc[lane] = u0;
        recs[k].desc[lane + 64] = u1;
        if (desc_f32) {
            desc_f32[(size_t)k * 128 + lane] = (float)(c0 * inv2);
            desc_f32[(size_t)k * 128 + lane + 64] = (float)(c1 * inv2);
        }
        if (k < ex.cap) {
            ex.rec[k].desc[lane] = u0;
            ex.rec[k].desc[lane + 64] = u1;
            if (lane == 0) {
                sift_kp& r = ex.rec[k];
                r.x = kx;
                r.y = ky;
                r.octave = o;
                r.layer = layer;
                r.size = ksize;
                r.pori = pori;
                ex.side[k] = rside;
            }
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// k_descriptor_split<F64> (desc_mode 0 with F64, the default): one record
// per 256-thread workgroup, from the work counter.
//  * The rows of the window are dealt round-robin to the four waves (row j
//    of the window to wave j % 4); each wave enumerates its rows' sample
//    intervals as k_descriptor_wave does (f32 superset of the rotated box,
//    wave scan, binary-search locate) and walks them 64 samples per step
//    with the next step's gradient loads in flight. A record takes a quarter
//    of a wavefront's serial walk (the synchronous latency's tail, DESIGN
//    §4), and the split depends only on the record, so its bytes do not
//    depend on how its job was batched.
//  * F64: the reference's per-sample expressions in f64 (sift.cpp:641-678):
//    row_rot / col_rot with the correctly rounded division by hist_width,
//    (row_rot + 2) - 0.5, the gradient, sqrt, atan2 - pori and the two
//    fmods (exact compare-and-subtract), exp of -(row_rot^2 + col_rot^2)/8,
//    the trilinear split. Samples of the f32 superset outside the box get
//    row_bin / col_bin <= -1 or >= 4 from these exact expressions: their
//    cells are all skipped, or take weight 0 (row_bin = -1 exactly), so the
//    contributing sample set is exactly the reference's. What differs from
//    the reference is the last bit of sqrt/atan2/exp/sin/cos (device math,
//    see above) and the histogram summation order; the normalised floats
//    agree to ~1e-15.
//  * Each wave adds into its own kSplitReps lane-interleaved f64 replicas
//    (ds_add_f64, conflict-free at 16); a wave reduces its replicas to two
//    bins per lane, and wave 0 sums the four waves' partials in wave order,
//    normalises, clamps, renormalises and quantises (sift.cpp:576-603).
//    Fixed order throughout: the bytes depend only on the record.
// ---------------------------------------------------------------------------
constexpr int kSplitReps = SIFT_DSPLIT_REPS;
static_assert(kSplitReps >= 1 && kSplitReps <= 16 && (kSplitReps & (kSplitReps - 1)) == 0,
              "replicas: a power of two <= 16");

template <bool F64>
__global__ __launch_bounds__(256, SIFT_DSPLIT_OCC) void k_descriptor_split(
    const PyrTable* __restrict__ pt, DevParams P, sift_kp* __restrict__ recs,
    const RecSide* __restrict__ rec_side, const unsigned* __restrict__ rec_begin,
    const unsigned* __restrict__ n_rec, unsigned cap_rec, float* __restrict__ desc_f32,
    unsigned* __restrict__ work, ExportSink ex) {
    __shared__ __attribute__((aligned(16))) double hist_all[4 * 128 * kSplitReps];
    __shared__ double2 atab[17];
    __shared__ unsigned next_k;
    set_job_prio(pt->jp, 0);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* const hist = hist_all + wv * 128 * kSplitReps;
    double* const rep = hist + (lane & (kSplitReps - 1));  // bin i at rep[i * kSplitReps]
    const unsigned n = min(*n_rec, cap_rec);
    const unsigned k0 = min(*rec_begin, n);
    // the launch's record range is fixed before it starts (orientation has
    // completed); the host reads it after the chain's completion event
    if (ex.cnt && blockIdx.x == 0 && threadIdx.x == 0) {
        ex.cnt[0] = k0;
        ex.cnt[1] = n;
    }
    if (threadIdx.x < 17) atab[threadIdx.x] = kAtanTab[threadIdx.x];
    if (threadIdx.x == 0) next_k = atomicAdd(work, 1u);
    __syncthreads();
    constexpr float kHalfW = (float)(kDescW / 2 - 0.5);
    const float wscale = (float)(-1.4426950408889634 / (0.5 * kDescW * kDescW));
    constexpr double kBinsPerRad = kDescBins / kTwoPi;  // sift.cpp:628
    for (;;) {
        const unsigned k = k0 + next_k;
        if (k >= n) break;
        // ---- record setup (wave-uniform, every wave)
        const sift_kp& R = recs[k];
        const double kx = R.x, ky = R.y, ksize = R.size, pori = R.pori;
        const int o = R.octave, layer = R.layer;
        const RecSide rside = rec_side[k];
        gdouble* img = gbl(plane(pt, rside.img, o, layer));
        const int W = pt->w[o], H = pt->h[o];
        const double inv = P.double_image ? (1.0 / pow2i(o - 1)) : (1.0 / pow2i(o));
        const int x = (int)(kx * inv);
        const int y = (int)(ky * inv);
        const double hw = P.desc_scale_factor * (ksize * inv);
        const double rr = round(hw * 0.5 * sqrt(2.0) * (kDescW + 1.0) + 0.5);
        const double diag = sqrt((double)(W * W + H * H));
        const int radius = (int)((diag < rr) ? diag : rr);  // std::min(rr, diag)
        const int side = 2 * radius + 1;
        const double ihw = 1.0 / hw;
        double sa = 0.0, ca = 1.0;
        if (F64) {
            sa = sin(pori);
            ca = cos(pori);
        }
        float saf, caf;
        if (F64) {
            saf = (float)sa;
            caf = (float)ca;
        } else {
            sincosf((float)pori, &saf, &caf);
        }
        const float ihwf = (float)ihw;
        const float porif = (float)pori;
        const float limf = (float)((0.5 * kDescW + 0.5) * hw);  // |rot| < 2.5 hw
        for (int i = lane; i < 64 * kSplitReps; i += 64)
            reinterpret_cast<double2*>(hist)[i] = make_double2(0.0, 0.0);
        wave_sync();
        // ---- this wave's rows j = wv + 4 i, 64 of them (lane = row) per group
        for (int g0 = wv; g0 < side; g0 += 4 * 64) {
            const int j = g0 + 4 * lane;
            const int row = j - radius;
            int lo = 0, len = 0;
            if (j < side && row + y > 0 && row + y < H - 1) {
                const float fr = (float)row, ra = fr * caf, rs = fr * saf;
                float clo = (float)max(-radius, 1 - x), chi = (float)min(radius, W - 2 - x);
                // |c sa + r ca| < lim and |c ca - r sa| < lim, widened by 0.01
                // column (f32 rounding of the bounds is far below that)
                if (fabsf(saf) > 1e-6f) {
                    const float is = 1.0f / saf;
                    const float a1 = (-limf - ra) * is, a2 = (limf - ra) * is;
                    clo = fmaxf(clo, fminf(a1, a2) - 0.01f);
                    chi = fminf(chi, fmaxf(a1, a2) + 0.01f);
                } else if (!(fabsf(ra) < limf + 0.01f)) {
                    chi = clo - 1.0f;
                }
                if (fabsf(caf) > 1e-6f) {
                    const float ic = 1.0f / caf;
                    const float b1 = (-limf + rs) * ic, b2 = (limf + rs) * ic;
                    clo = fmaxf(clo, fminf(b1, b2) - 0.01f);
                    chi = fminf(chi, fmaxf(b1, b2) + 0.01f);
                } else if (!(fabsf(rs) < limf + 0.01f)) {
                    chi = clo - 1.0f;
                }
                lo = (int)ceilf(clo);
                const int hi = (int)floorf(chi);
                len = hi >= lo ? hi - lo + 1 : 0;
            }
            int pre = len;  // inclusive scan of the row lengths
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(pre, off);
                if (lane >= off) pre += t;
            }
            const int total = __builtin_amdgcn_readlane(pre, 63);
            // (row, col) of sample t0 + lane: its row r is the number of rows
            // whose inclusive prefix is <= t (branch-free binary search)
            auto locate = [&](int t0, int& srow, int& scol) -> bool {
                const int t = t0 + lane;
                int r = 0;
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1)
                    if (__shfl(pre, r + step - 1) <= t) r += step;
                const int lo_r = __shfl(lo, r);
                const int ex_r = __shfl(pre, r) - __shfl(len, r);
                srow = g0 + 4 * r - radius;
                scol = lo_r + (t - ex_r);
                return t < total;
            };
            // gradient loads issued unconditionally (lanes past the end read
            // pixel (1, 1)) so the compiler can count them
            auto fetch = [&](bool ok, int srow, int scol, double* v) {
                const size_t r0 = ok ? (size_t)(srow + y) * W + scol + x : (size_t)W + 1;
                v[0] = img[r0 + 1];
                v[1] = img[r0 - 1];
                v[2] = img[r0 - W];
                v[3] = img[r0 + W];
            };
            int srow = 0, scol = 0, nrow = 0, ncol = 0;
            double cv[4], nv[4];
            bool cok = total > 0 && locate(0, srow, scol);
            fetch(cok, srow, scol, cv);
            for (int t0 = 0; t0 < total; t0 += 64) {
                // the next block's loads are in flight while this one is processed
                nrow = ncol = 0;
                const bool nok = t0 + 64 < total && locate(t0 + 64, nrow, ncol);
                fetch(nok, nrow, ncol, nv);
                if (F64 && cok) {
                    const double dcol = (double)scol, drow = (double)srow;
                    const double row_rot = div_sum_w(dcol * sa + drow * ca, hw, ihw);
                    const double col_rot = div_sum_w(dcol * ca - drow * sa, hw, ihw);
                    const double rb = row_rot + kDescW / 2 - 0.5;
                    const double cb = col_rot + kDescW / 2 - 0.5;
                    const double dx = cv[0] - cv[1];
                    const double dy = cv[2] - cv[3];
                    const double mag = sqrt_f64(dx * dx + dy * dy);
                    double ang = atan2_f64(dy, dx, atab) - pori;
                    // fmod(fmod(ang, 2pi) + 2pi, 2pi) with |ang| < 2 * 2pi:
                    // fmod(a, M) = a - trunc(a/M) M is exact here, so
                    // compare-and-subtract reproduces it bit for bit
                    if (ang >= kTwoPi) ang -= kTwoPi;
                    else if (ang <= -kTwoPi) ang += kTwoPi;
                    ang += kTwoPi;
                    if (ang >= kTwoPi) ang -= kTwoPi;
                    if (ang >= kTwoPi) ang -= kTwoPi;
                    const double ob = ang * kBinsPerRad;
                    const double wgt =
                        exp_f64(-(row_rot * row_rot + col_rot * col_rot) / (0.5 * kDescW * kDescW));
                    const double m = mag * wgt;
                    const double fbr = floor(rb), fbc = floor(cb), fbo = floor(ob);
                    const int br = (int)fbr, bc = (int)fbc, bo = (int)fbo;
                    const double fr = rb - fbr, fc = cb - fbc, fo = ob - fbo;
#pragma unroll
                    for (int rq = 0; rq <= 1; ++rq) {
                        const int ri = br + rq;
                        if ((unsigned)ri >= (unsigned)kDescW) continue;
                        const double vr = m * ((rq == 0) ? 1.0 - fr : fr);
#pragma unroll
                        for (int cq = 0; cq <= 1; ++cq) {
                            const int ci = bc + cq;
                            if ((unsigned)ci >= (unsigned)kDescW) continue;
                            const double vc = vr * ((cq == 0) ? 1.0 - fc : fc);
                            double* hb = &rep[(ri * 32 + ci * 8) * kSplitReps];
                            atomicAdd(&hb[(bo & 7) * kSplitReps], vc * (1.0 - fo));
                            atomicAdd(&hb[((bo + 1) & 7) * kSplitReps], vc * fo);
                        }
                    }
                } else if (!F64 && cok) {
                    const float fcol = (float)scol, frow = (float)srow;
                    const float row_rot = fmaf(fcol, saf, frow * caf) * ihwf;
                    const float col_rot = fmaf(fcol, caf, -(frow * saf)) * ihwf;
                    const float rb = row_rot + kHalfW;
                    const float cb = col_rot + kHalfW;
                    const float dx = (float)(cv[0] - cv[1]);
                    const float dy = (float)(cv[2] - cv[3]);
                    const float mag = __builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy));
                    const float ob = (atan2_f32(dy, dx) - porif) * (float)(kDescBins / kTwoPi);
                    const float wgt =
                        __builtin_amdgcn_exp2f(fmaf(row_rot, row_rot, col_rot * col_rot) * wscale);
                    const float m = mag * wgt;
                    const float fbr = floorf(rb), fbc = floorf(cb), fbo = floorf(ob);
                    const int br = (int)fbr, bc = (int)fbc, bo = (int)fbo;
                    const float fr = rb - fbr, fc = cb - fbc, fo = ob - fbo;
#pragma unroll
                    for (int rq = 0; rq <= 1; ++rq) {
                        const int ri = br + rq;
                        if ((unsigned)ri >= (unsigned)kDescW) continue;
                        const float vr = m * ((rq == 0) ? 1.0f - fr : fr);
#pragma unroll
                        for (int cq = 0; cq <= 1; ++cq) {
                            const int ci = bc + cq;
                            if ((unsigned)ci >= (unsigned)kDescW) continue;
                            const float vc = vr * ((cq == 0) ? 1.0f - fc : fc);
                            double* hb = &rep[(ri * 32 + ci * 8) * kSplitReps];
                            atomicAdd(&hb[(bo & 7) * kSplitReps], (double)(vc * (1.0f - fo)));
                            atomicAdd(&hb[((bo + 1) & 7) * kSplitReps], (double)(vc * fo));
                        }
                    }
                }
                srow = nrow;
                scol = ncol;
                cok = nok;
#pragma unroll
                for (int q = 0; q < 4; ++q) cv[q] = nv[q];
            }
        }
        wave_sync();
        // ---- this wave's replicas -> bins lane, lane + 64 (fixed order per
        // bin, rotated by lane so the 16 lanes of a read group start on
        // different bank pairs), parked at the front of its own region
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int q = 0; q < kSplitReps; ++q) {
            const int r = (q + lane) & (kSplitReps - 1);
            v0 += hist[lane * kSplitReps + r];
            v1 += hist[(lane + 64) * kSplitReps + r];
        }
        wave_sync();
        hist[lane] = v0;
        hist[lane + 64] = v1;
        __syncthreads();
        if (wv == 0) {
            // the four waves' partials in wave order; normalise, clamp,
            // renormalise, quantise (sift.cpp:576-603)
#pragma unroll
            for (int w = 1; w < 4; ++w) {
                v0 += hist_all[w * 128 * kSplitReps + lane];
                v1 += hist_all[w * 128 * kSplitReps + lane + 64];
            }
            const double ninv = 1.0 / sqrt(wave_sum_f64(v0 * v0 + v1 * v1));
            double c0 = v0 * ninv, c1 = v1 * ninv;
            if (c0 > kMagThr) c0 = kMagThr;
            if (c1 > kMagThr) c1 = kMagThr;
            const double inv2 = 1.0 / sqrt(wave_sum_f64(c0 * c0 + c1 * c1));
            auto quant = [&](double c) -> uint8_t {
                const double q = floor(kIntFactor * c * inv2);
                int val = (q == q) ? (int)q : 0;  // NaN -> 0 (Appendix A.17)
                return (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
            };
            const uint8_t u0 = quant(c0), u1 = quant(c1);
            recs[k].desc[lane] = u0;
            recs[k].desc[lane + 64] = u1;
            if (desc_f32) {
                desc_f32[(size_t)k * 128 + lane] = (float)(c0 * inv2);
                desc_f32[(size_t)k * 128 + lane + 64] = (float)(c1 * inv2);
            }
            if (k < ex.cap) {
                ex.rec[k].desc[lane] = u0;
                ex.rec[k].desc[lane + 64] = u1;
                if (lane == 0) {
                    sift_kp& r = ex.rec[k];
                    r.x = kx;
                    r.y = ky;
                    r.octave = o;
                    r.layer = layer;
                    r.size = ksize;
                    r.pori = pori;
                    ex.side[k] = rside;
                }
            }
        } else if (wv == 1 && lane == 0) {
            next_k = atomicAdd(work, 1u);  // the next record, while wave 0 finishes
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_descriptor(const PyrTable* d_pt, const DevParams& P, sift_kp* recs,
                             const RecSide* rec_side, const unsigned* rec_begin,
                             const unsigned* n_rec, unsigned cap_rec, float* desc_f32,
                             unsigned* work, const ExportSink& ex, unsigned wgs,
                             int mode, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    // persistent: workgroups pull records
    if (mode == 1) {  // four waves per workgroup, a record per wave (f32 sample math)
        const unsigned blocks = std::min<unsigned>(wgs, cap_rec > 0 ? (cap_rec + 3) / 4 : 1);
        return launch_timed(k_descriptor_wave, dim3(blocks), dim3(256), 0, s, e0, e1, d_pt, P,
                            recs, rec_side, rec_begin, n_rec, cap_rec, desc_f32, work, ex);
    }
    const unsigned blocks = std::min<unsigned>(wgs, cap_rec > 0 ? cap_rec : 1);
    auto kern = mode == 2 ? k_descriptor_split<false> : k_descriptor_split<true>;
    return launch_timed(kern, dim3(blocks), dim3(256), 0, s, e0, e1, d_pt, P, recs, rec_side,
                        rec_begin, n_rec, cap_rec, desc_f32, work, ex);
}

}  // namespace sift_amd
