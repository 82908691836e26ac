// sift_desc.hip — compute_descriptors + update_histogram +
// convert_hist_to_desc (reference src/sift.cpp:541-682) on gfx950.
//
// k_descriptor_split: one record per 256-thread workgroup, the window's
// rows dealt to its four waves; every per-sample operation in double, as the
// reference (sift.cpp:641-678), into f64 histograms.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sift_device.h"
#include "sift_kernels.h"
#include "sift_math64.h"

#ifndef SIFT_DESC_AHEAD  // steps of 64 samples whose gradient loads are in flight
#define SIFT_DESC_AHEAD 1
#endif
#ifndef SIFT_DESC_SWZ  // replica swizzle of the histogram bins (hist_slot)
#define SIFT_DESC_SWZ 0
#endif
#ifndef SIFT_DESC_PERM  // 1: lanes sharing a replica take samples 16 apart (sample_of_lane)
#define SIFT_DESC_PERM 0
#endif
// Doubles between consecutive bins of a replica (>= replicas). ds_add_f64
// serves a wave in four 16-lane groups, one LDS cycle each, 16 double slots
// (double index mod 16; tools/lds_atomic_probe.hip, r06_s2: consecutive
// doubles 4.0 cycles per instruction, stride 2 or 8 lanes per address 8.0).
// With 8 interleaved replicas (stride 8) the two lanes of a group that share
// a replica collide whenever their bins have the same parity; stride 9 maps
// bin i of replica r to slot 9i + r (mod 16), so they collide only for bins
// equal mod 16. Stride 9 keeps 4 workgroups per CU (39 KB of LDS); 10 and 11
// do not. Alone per 1080p image (r06_s5, two boxes): stride 8 133-154 us,
// 9 120-123 us, 10 / 11 149-151 us; synchronous latency -4 %; the driver's
// command +-0.6 %. Every histogram is bit-identical (hist_slot relocates).
#ifndef SIFT_DESC_BSTRIDE
#define SIFT_DESC_BSTRIDE 9
#endif
#ifndef SIFT_DESC_RMAJOR  // > 0: replica-major layout, replicas SIFT_DESC_RMAJOR + 128 doubles apart
#define SIFT_DESC_RMAJOR 0
#endif

namespace sift_amd {

namespace {

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// ---------------------------------------------------------------------------
// Per-record geometry (sift.cpp:616-639), wave-uniform.
// ---------------------------------------------------------------------------
struct DescRecord {
    double kx, ky, ksize, pori;
    int o, layer;
    RecSide side;
    const double* img;
    int W, H, x, y, radius;
    double hw, ihw, sa, ca;  // hist_width, 1 / hist_width, sin / cos of pori
    float saf, caf, limf;    // f32 copies for the window bounds
};

// sa / ca: the f64 sin / cos of pori, computed once per record by the
// kernel (sc)
__device__ __forceinline__ DescRecord load_record(const PyrTable* pt, const DevParams& P,
                                                  const sift_kp& R, const RecSide& side,
                                                  const double2* sc) {
    DescRecord d;
    d.kx = R.x;
    d.ky = R.y;
    d.ksize = R.size;
    d.pori = R.pori;
    d.o = R.octave;
    d.layer = R.layer;
    d.side = side;
    d.img = plane(pt, side.img, d.o, d.layer);
    d.W = pt->w[d.o];
    d.H = pt->h[d.o];
    const double inv = P.double_image ? (1.0 / pow2i(d.o - 1)) : (1.0 / pow2i(d.o));
    d.x = (int)(d.kx * inv);  // truncation (sift.cpp:620-624)
    d.y = (int)(d.ky * inv);
    d.hw = P.desc_scale_factor * (d.ksize * inv);
    const double rr = round(d.hw * 0.5 * sqrt(2.0) * (kDescW + 1.0) + 0.5);
    const double diag = sqrt((double)(d.W * d.W + d.H * d.H));
    d.radius = (int)((diag < rr) ? diag : rr);  // std::min(rr, diag)
    d.ihw = 1.0 / d.hw;
    d.sa = sc->x;
    d.ca = sc->y;
    d.saf = (float)d.sa;
    d.caf = (float)d.ca;
    d.limf = (float)((0.5 * kDescW + 0.5) * d.hw);  // |row_rot|, |col_rot| < 2.5 hw
    return d;
}

// LDS slot of bin i of replica r in a wave's NR lane-interleaved replicas.
// Unswizzled (bin i at i * NR + r) the lanes that share a replica map onto
// the same banks whenever their bins agree modulo 32 / NR, and neighbouring
// samples mostly differ only in their spatial cell (i = row_bin * 32 +
// col_bin * 8 + ori_bin): 45 % of the descriptor's LDS cycles were bank
// conflicts (round 5). XOR-ing the replica index with bits of the cell moves
// neighbouring cells to other banks. It only relocates the slot: the adds
// into a given (replica, bin) and their order are unchanged, so every
// histogram is bit-identical.
constexpr int kBinStride = SIFT_DESC_BSTRIDE;
static_assert(kBinStride >= SIFT_DSPLIT_REPS, "bin stride");

template <int NR>
__device__ __forceinline__ int hist_slot(int i, int r) {
    int f = 0;
    if (SIFT_DESC_SWZ == 1) f = i >> 2;                                // ori bit 2, col_bin
    if (SIFT_DESC_SWZ == 2) f = ((i >> 3) & 3) | (((i >> 5) & 1) << 2);  // col_bin, row_bin bit 0
    if (SIFT_DESC_SWZ == 3) f = i >> 1;
    if (SIFT_DESC_RMAJOR > 0) return (r ^ (f & (NR - 1))) * (128 + SIFT_DESC_RMAJOR) + i;
    return i * kBinStride + (r ^ (f & (NR - 1)));
}

// ---------------------------------------------------------------------------
// One sample (col, row) with gradient loads cv = I(x+1), I(x-1), I(y-1),
// I(y+1) into this lane's replica r of the wave's histograms `hist`
// (bin i at hist[hist_slot(i, r)]).
// The reference's expressions (sift.cpp:641-678): row_rot / col_rot
// with the correctly rounded division by hist_width, (row_rot + 2) - 0.5,
// sqrt, atan2 - pori and the two fmods (exact compare-and-subtract),
// exp(-(row_rot^2 + col_rot^2) / 8), the trilinear split of
// update_histogram (sift.cpp:541-571). Samples of the enumerated f32
// superset outside the box get row_bin / col_bin <= -1 or >= 4 from these
// exact expressions: their cells are all skipped, or take weight 0
// (row_bin = -1 exactly), so the contributing sample set is the reference's.
// ---------------------------------------------------------------------------
template <int NR>
__device__ __forceinline__ void add_sample_f64(double* hist, int r, int scol, int srow, const double* cv,
                                               const DescRecord& d, const double2* atab,
                                               const double* gtab) {
    constexpr double kBinsPerRad = kDescBins / kTwoPi;  // sift.cpp:628
    const double dcol = (double)scol, drow = (double)srow;
    const double row_rot = div_sum_w(dcol * d.sa + drow * d.ca, d.hw, d.ihw);
    const double col_rot = div_sum_w(dcol * d.ca - drow * d.sa, d.hw, d.ihw);
    const double rb = row_rot + kDescW / 2 - 0.5;
    const double cb = col_rot + kDescW / 2 - 0.5;
    const double dx = cv[0] - cv[1];
    const double dy = cv[2] - cv[3];
    const double mag = sqrt_f64(dx * dx + dy * dy);
    double ang = atan2_f64(dy, dx, atab) - d.pori;
    // fmod(fmod(ang, 2pi) + 2pi, 2pi): atan2 in [-pi, pi] and pori in
    // [0, 2pi) put ang in (-3pi, pi], so the inner fmod only adds 2pi when
    // ang <= -2pi and the outer one only subtracts 2pi once; both exact
    // (Sterbenz), so compare-and-add reproduces them bit for bit
    if (ang <= -kTwoPi) ang += kTwoPi;
    ang += kTwoPi;
    if (ang >= kTwoPi) ang -= kTwoPi;
    const double ob = ang * kBinsPerRad;
    // exp(-(row_rot^2 + col_rot^2) / 8): with the per-record table the
    // separable form G(row) G(col), G(i) = exp(-i^2 / (8 hw^2)) (rotation
    // keeps row_rot^2 + col_rot^2 = (row^2 + col^2) / hw^2; the two
    // evaluations differ by a few 1e-16 relative)
    const double wgt =
        gtab ? gtab[srow < 0 ? -srow : srow] * gtab[scol < 0 ? -scol : scol]
             : exp_f64(-(row_rot * row_rot + col_rot * col_rot) / (0.5 * kDescW * kDescW));
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
            const int cell = ri * 32 + ci * 8;
            atomicAdd(&hist[hist_slot<NR>(cell + (bo & 7), r)], vc * (1.0 - fo));
            atomicAdd(&hist[hist_slot<NR>(cell + ((bo + 1) & 7), r)], vc * fo);
        }
    }
}

// ---------------------------------------------------------------------------
// The samples of rows j0, j0 + dj, ... of the window (row j = row - radius),
// 64 rows per group (lane = row), walked 64 samples per step:
//  * each lane bounds its row's sample interval: an f32 SUPERSET of the
//    reference's rotated box (|col sa + row ca| < 2.5 hw and
//    |col ca - row sa| < 2.5 hw, widened by 0.01 column; f32 rounding of
//    the bounds is far below that) intersected exactly with the radius and
//    the image border (sift.cpp:634-656);
//  * a wave scan of the row lengths, then sample t0 + lane is located by a
//    branch-free binary search over the 64 inclusive prefixes;
//  * the next SIFT_DESC_AHEAD steps' four gradient loads per lane are in
//    flight while the current step's samples are processed (issued
//    unconditionally: lanes past the end read pixel (1, 1), so the compiler
//    can count them).
// ---------------------------------------------------------------------------
// Sample t0 + sample_of_lane(lane) of a step goes to lane `lane`. With
// SIFT_DESC_PERM the lanes that share a replica (lane & 7) within an LDS
// lane group take samples 16 apart instead of 8 (lane r + 8h + 32G <- sample
// r + 8G + 16h): the samples of one replica still go to the same replica
// (sample & 7 == lane & 7), but neighbouring samples, which mostly hit the
// same bin, no longer meet on one address inside one atomic instruction.
__device__ __forceinline__ int sample_of_lane(int lane) {
    if (!SIFT_DESC_PERM) return lane;
    return (lane & 7) | ((lane >> 5) << 3) | (((lane >> 3) & 3) << 4);
}

template <int NR>
__device__ __forceinline__ void desc_walk(const DescRecord& d, int j0, int dj, double* hist,
                                          const double2* atab, const double* gtab) {
    const int lane = threadIdx.x & 63;
    const int slane = sample_of_lane(lane);
    const int side = 2 * d.radius + 1;
    gdouble* img = gbl(d.img);
    const int W = d.W, H = d.H, x = d.x, y = d.y, radius = d.radius;
    for (int g0 = j0; g0 < side; g0 += 64 * dj) {
        const int j = g0 + dj * lane;
        const int row = j - radius;
        int lo = 0, len = 0;
        if (j < side && row + y > 0 && row + y < H - 1) {
            const float fr = (float)row, ra = fr * d.caf, rs = fr * d.saf;
            float clo = (float)max(-radius, 1 - x), chi = (float)min(radius, W - 2 - x);
            if (fabsf(d.saf) > 1e-6f) {
                const float is = 1.0f / d.saf;
                const float a1 = (-d.limf - ra) * is, a2 = (d.limf - ra) * is;
                clo = fmaxf(clo, fminf(a1, a2) - 0.01f);
                chi = fminf(chi, fmaxf(a1, a2) + 0.01f);
            } else if (!(fabsf(ra) < d.limf + 0.01f)) {
                chi = clo - 1.0f;
            }
            if (fabsf(d.caf) > 1e-6f) {
                const float ic = 1.0f / d.caf;
                const float b1 = (-d.limf + rs) * ic, b2 = (d.limf + rs) * ic;
                clo = fmaxf(clo, fminf(b1, b2) - 0.01f);
                chi = fminf(chi, fmaxf(b1, b2) + 0.01f);
            } else if (!(fabsf(rs) < d.limf + 0.01f)) {
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
        auto locate = [&](int t0, int& srow, int& scol) -> bool {
            const int t = t0 + slane;
            int r = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1)
                if (__shfl(pre, r + step - 1) <= t) r += step;
            const int lo_r = __shfl(lo, r);
            const int ex_r = __shfl(pre, r) - __shfl(len, r);
            srow = g0 + dj * r - radius;
            scol = lo_r + (t - ex_r);
            return t < total;
        };
        auto fetch = [&](bool ok, int srow, int scol, double* v) {
            const size_t r0 = ok ? (size_t)(srow + y) * W + scol + x : (size_t)W + 1;
            v[0] = img[r0 + 1];
            v[1] = img[r0 - 1];
            v[2] = img[r0 - W];
            v[3] = img[r0 + W];
        };
        // a ring of AHEAD + 1 steps: step t0 is processed while the loads
        // of the next AHEAD steps are in flight (slots are compile-time:
        // the queue shifts by register moves)
        constexpr int A = SIFT_DESC_AHEAD;
        int qrow[A + 1], qcol[A + 1];
        bool qok[A + 1];
        double qv[A + 1][4];
#pragma unroll
        for (int a = 0; a < A; ++a) {
            qrow[a] = qcol[a] = 0;
            qok[a] = 64 * a < total && locate(64 * a, qrow[a], qcol[a]);
            fetch(qok[a], qrow[a], qcol[a], qv[a]);
        }
        for (int t0 = 0; t0 < total; t0 += 64) {
            qrow[A] = qcol[A] = 0;
            qok[A] = t0 + 64 * A < total && locate(t0 + 64 * A, qrow[A], qcol[A]);
            fetch(qok[A], qrow[A], qcol[A], qv[A]);
            if (qok[0])
                add_sample_f64<NR>(hist, lane & (NR - 1), qcol[0], qrow[0], qv[0], d, atab, gtab);
#pragma unroll
            for (int a = 0; a < A; ++a) {
                qrow[a] = qrow[a + 1];
                qcol[a] = qcol[a + 1];
                qok[a] = qok[a + 1];
#pragma unroll
                for (int q = 0; q < 4; ++q) qv[a][q] = qv[a + 1][q];
            }
        }
    }
}

// This wave's NR replicas (bin i of replica r at hist[hist_slot(i, r)]) -> bins
// lane and lane + 64, in a fixed order per bin (rotated by lane so the 16
// lanes of a read group start on different bank pairs)
template <int NR>
__device__ __forceinline__ void reduce_replicas(const double* hist, double& v0, double& v1) {
    const int lane = threadIdx.x & 63;
    v0 = v1 = 0.0;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        const int r = (q + lane) & (NR - 1);
        v0 += hist[hist_slot<NR>(lane, r)];
        v1 += hist[hist_slot<NR>(lane + 64, r)];
    }
}

// convert_hist_to_desc (sift.cpp:576-603) of bins lane / lane + 64 of record
// k, by one wave: normalise, clamp at 0.2, renormalise, quantise; the record
// and its export copy are written
__device__ __forceinline__ void finish_record(double v0, double v1, const DescRecord& d,
                                              unsigned k, sift_kp* __restrict__ recs,
                                              float* __restrict__ desc_f32,
                                              const ExportSink& ex) {
    const int lane = threadIdx.x & 63;
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
            r.x = d.kx;
            r.y = d.ky;
            r.octave = d.o;
            r.layer = d.layer;
            r.size = d.ksize;
            r.pori = d.pori;
            ex.side[k] = d.side;
        }
    }
}

// ---------------------------------------------------------------------------
// k_descriptor_split: one record per 256-thread workgroup.
//  * Row j of the window goes to wave j % 4 (desc_walk with dj = 4), so a
//    record takes a quarter of a wavefront's serial walk, and the split
//    depends only on the record: its bytes do not depend on how its job
//    was batched.
//  * Each wave adds into its own kSplitReps lane-interleaved f64 replicas
//    (ds_add_f64; conflict-free at 16: a lane's bank pair is
//    2 (i * 16 + r) mod 32, its own whatever bin the sample hits); a wave
//    reduces its replicas to two bins per lane, wave 0 sums the four waves'
//    partials in wave order and finishes the record. Fixed order
//    throughout: the bytes depend only on the record.
//  * Workgroup b's first record is b; one lane of wave 1 claims the next
//    (work counter) and evaluates the f64 sin / cos of its orientation (once
//    per record) while wave 0 finishes the current one; two barriers per
//    record.
// ---------------------------------------------------------------------------
constexpr int kSplitReps = SIFT_DSPLIT_REPS;
// Gaussian weight table G(0..radius) of the current record: one exp per thread per record instead of one per sample; records
// with a larger radius evaluate exp per sample
constexpr int kGTab = 256;
// one wave's replicas: 128 bins (the last one padded to a full stride), even
constexpr int kHistWave = SIFT_DESC_RMAJOR > 0 ? (SIFT_DSPLIT_REPS * (128 + SIFT_DESC_RMAJOR) + 1) & ~1
                                               : (128 * kBinStride + 1) & ~1;
static_assert(kSplitReps >= 1 && kSplitReps <= 16 && (kSplitReps & (kSplitReps - 1)) == 0,
              "replicas: a power of two <= 16");

__global__ __launch_bounds__(256, SIFT_DSPLIT_OCC) void k_descriptor_split(
    const PyrTable* __restrict__ pt, DevParams P, sift_kp* __restrict__ recs,
    const RecSide* __restrict__ rec_side, const unsigned* __restrict__ rec_begin,
    const unsigned* __restrict__ n_rec, unsigned cap_rec, float* __restrict__ desc_f32,
    unsigned* __restrict__ work, ExportSink ex) {
    __shared__ __attribute__((aligned(16))) double hist_all[4 * kHistWave];
    __shared__ double2 atab[17];
    __shared__ unsigned next_k;
    __shared__ double2 next_sc;  // sin, cos of the next record's pori
    __shared__ double gtab[kGTab];
    set_job_prio(pt->jp, 0);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double* const hist = hist_all + wv * kHistWave;
    const unsigned n = min(*n_rec, cap_rec);
    const unsigned k0 = min(*rec_begin, n);
    // the launch's record range is fixed before it starts (orientation has
    // completed); the host reads it after the chain's completion event
    if (ex.cnt && blockIdx.x == 0 && threadIdx.x == 0) {
        ex.cnt[0] = k0;
        ex.cnt[1] = n;
        ex.cnt[2] = ex.live[0];  // the lane's final counters: extrema and
        ex.cnt[3] = ex.live[1];  // refine and orientation of this chain
        ex.cnt[4] = *n_rec;      // have completed (same stream)
    }
    if (threadIdx.x < 17) atab[threadIdx.x] = kAtanTab[threadIdx.x];
    // workgroup b's first record is b of the launch's range, the later ones
    // come from the work counter offset by the grid (every workgroup claiming
    // at once at the start serialised at one L2 channel, ~10 ns per atomic;
    // static striding throughout measured slower: no dynamic balance)
    auto prepare = [&](unsigned c) {
        next_k = c;
        if (k0 + c < n) {
            const double pr = recs[k0 + c].pori;
            next_sc = make_double2(sin(pr), cos(pr));
        }
    };
    if (threadIdx.x == 0) prepare(blockIdx.x);
    __syncthreads();
    for (;;) {
        const unsigned cur = next_k;
        const unsigned k = k0 + cur;
        if (k >= n) break;
        const double2 sc = next_sc;
        const DescRecord d = load_record(pt, P, recs[k], rec_side[k], &sc);
        const bool use_tab = d.radius < kGTab;
        if (use_tab && (int)threadIdx.x <= d.radius) {
            const double i = (double)threadIdx.x;
            gtab[threadIdx.x] = exp_f64(-(i * i) / (0.5 * kDescW * kDescW * d.hw * d.hw));
        }
        for (int i = lane; i < kHistWave / 2; i += 64)
            reinterpret_cast<double2*>(hist)[i] = make_double2(0.0, 0.0);
        __syncthreads();  // the table (uniform: every thread gets here)
        desc_walk<kSplitReps>(d, wv, 4, hist, atab, use_tab ? gtab : nullptr);
        wave_sync();
        double v0, v1;
        reduce_replicas<kSplitReps>(hist, v0, v1);
        wave_sync();
        hist[lane] = v0;  // this wave's partial, parked at the front of its region
        hist[lane + 64] = v1;
        __syncthreads();
        if (wv == 0) {
#pragma unroll
            for (int w = 1; w < 4; ++w) {  // the partials in wave order
                v0 += hist_all[w * kHistWave + lane];
                v1 += hist_all[w * kHistWave + lane + 64];
            }
            finish_record(v0, v1, d, k, recs, desc_f32, ex);
        } else if (wv == 1 && lane == 0) {
            prepare(gridDim.x + atomicAdd(work, 1u));
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_descriptor(const PyrTable* d_pt, const DevParams& P, sift_kp* recs,
                             const RecSide* rec_side, const unsigned* rec_begin,
                             const unsigned* n_rec, unsigned cap_rec, float* desc_f32,
                             unsigned* work, const ExportSink& ex, unsigned wgs, hipStream_t s,
                             hipEvent_t e0, hipEvent_t e1) {
    // persistent grid: workgroups pull records
    const unsigned blocks = std::min<unsigned>(wgs, cap_rec > 0 ? cap_rec : 1);
    return launch_timed(k_descriptor_split, dim3(blocks), dim3(256), 0, s, e0, e1, d_pt, P, recs,
                        rec_side, rec_begin, n_rec, cap_rec, desc_f32, work, ex);
}

}  // namespace sift_amd
