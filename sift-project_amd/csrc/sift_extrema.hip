// sift_extrema.hip — detect_octave_extrema (sift.cpp:227-291) on the GPU:
// k_extrema_stream (window_size 3, the default) and k_extrema_any (other
// windows). Their own translation unit because it is built with
// -fno-honor-nans (Makefile): the cube test's fmax / fmin then need no
// canonicalisation of their operands (gfx950 IEEE mode), which was a third
// of the kernel's VALU instructions (46 of ~75 v_max_f64 per row). Every
// value they compare is a difference of two finite pyramid levels; max and
// min are exact, so the candidates are the same.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "sift_device.h"
#include "sift_kernels.h"

#ifndef SIFT_EXT_PF
#define SIFT_EXT_PF 2  // k_extrema_stream: rows in flight
#endif

namespace sift_amd {

// ---------------------------------------------------------------------------
// Extrema: detect_octave_extrema + is_extremum (sift.cpp:227-291). A pixel is
// kept iff |D_z| > threshold (the int threshold of sift.cpp:266,279) and it
// is a NON-strict maximum or minimum of its (2b+1)^3 cube, i.e. v == max(cube)
// or v == min(cube): v is itself in the cube, so the centre comparison is
// vacuous (sift.cpp:241-246). DoG values are G_{l+1} - G_l computed on the fly.
// ---------------------------------------------------------------------------
// Chain snapshots (snap != nullptr): the extrema launch's first thread
// records the lane's raw / record begins at its start (the previous chain on
// the lane's stream has completed), k_refine's first thread records the
// candidate end (the extrema launch has completed). Round 3 took all three
// in the extrema launch's last workgroup, found by a done counter: one
// same-address atomic per workgroup (~1,000 per 1080p octave-0 launch).
// No memory fences in these kernels: __threadfence() on gfx950 is an L2
// writeback + invalidate of the XCD (one per workgroup tripled the extrema
// time and evicted the concurrent blurs' lines); the kernel boundary orders
// the writes for the next kernel.

// ---------------------------------------------------------------------------
// k_extrema_stream<NL>: the same test (sift.cpp:227-291, window_size 3) as a
// streaming scan. One wavefront per task = (octave, strip of 62 centre
// columns, segment of centre rows); lane l owns column x0 - 1 + l
// (lanes 0 and 63 are the halo). The wave walks the rows of its segment:
// per row every lane loads the NL Gaussian levels of its column (PF rows in
// flight), forms the NL-1 DoG values, gets its x-1 / x+1 neighbours with DPP
// wave shifts (no LDS), and keeps the 3-row window of horizontal max / min
// of every layer in registers (ring slots are compile-time: the row loop is
// unrolled by 3). Row y's centres are decided when row y+1 arrives; the
// cube of DoG layer z is layers z-1..z+1, rows y-1..y+1, columns x-1..x+1,
// and the test is the reference's non-strict one (v is in its own cube, so
// "no neighbour greater" == (v == max)). No LDS, no barrier until the end;
// 48 B read per pixel and (62 + 2) / 62 x (kExtSeg + 2) / kExtSeg reuse.
// Candidates: ballot per (row, layer) into a per-wave LDS buffer, one
// counter atomic per wave. The last workgroup takes the lane snapshot
// (see Chain snapshots above). (A tiled variant staging 66x18 DoG halo tiles in LDS
// was replaced by this scan in round 2 and removed in round 4.)
// ---------------------------------------------------------------------------
// (bound_ctrl: lane 0 / lane 63, whose neighbour is outside the wave, read
// 0 — they are halo lanes, never a centre — so no fill value has to be
// written into the destination first: one DPP move per 32-bit half, 20
// fewer moves per row)
__device__ __forceinline__ double dpp_from_left(double v) {  // lane i <- lane i-1
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_from_right(double v) {  // lane i <- lane i+1
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}

// level loads of the extrema scan: read once (SIFT_EXT_NT=1: non-temporal,
// so they do not displace the lines other jobs' blurs re-read from L2/MALL)
#ifndef SIFT_EXT_NT
#define SIFT_EXT_NT 0
#endif
__device__ __forceinline__ double ext_load(gdouble* p) {
    if (SIFT_EXT_NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int NL>
__global__ __launch_bounds__(256) void k_extrema_stream(const PyrTable* __restrict__ pt,
                                                        ExtremaGrid eg, int thr,
                                                        sift_extremum* __restrict__ out,
                                                        unsigned* __restrict__ counter,
                                                        unsigned cap, unsigned* snap) {
    set_job_prio(pt->jp, 0);
    constexpr int ND = NL - 1;   // DoG layers
    constexpr int NZ = ND - 2;   // layers with a full cube (z = 1 .. ND-2)
    constexpr int PF = SIFT_EXT_PF;  // rows in flight
    constexpr unsigned kCandBuf = 256;  // per-wave candidate buffer (LDS)
    __shared__ sift_extremum cbuf[4][kCandBuf];
    __shared__ unsigned wg_n[4], wg_base[4];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int task = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
    const int b = blockIdx.y;
    // the chain's raw / record begins: the lane's counters as the previous
    // chain on this stream left them (its candidate end is taken by k_refine)
    if (snap && blockIdx.x == 0 && b == 0 && threadIdx.x == 0) {
        snap[1] = counter[1];
        snap[2] = counter[2];
    }
    sift_extremum* cb = cbuf[wv];
    unsigned nbuf = 0;  // wave-uniform
    if (task < eg.first_tile[eg.n]) {
        int e = 0;
        while (e + 1 < eg.n && task >= eg.first_tile[e + 1]) ++e;
        const int o = eg.oct[e];
        const int t = task - eg.first_tile[e];
        const int strip = t % eg.tiles_x[e], seg = t / eg.tiles_x[e];
        const int W = pt->w[o], H = pt->h[o];
        const int xc0 = 1 + strip * kExtSpan;  // first centre column of the strip
        const int x = xc0 - 1 + lane;
        const int gx = min(x, W - 1);
        const bool centre_lane = lane >= 1 && lane <= kExtSpan && x <= W - 2;
        const int yc0 = 1 + seg * eg.seg[e];
        const int yc1 = min(yc0 + eg.seg[e], H - 1);  // centres [yc0, yc1)
        const int r0 = yc0 - 1, r1 = yc1;           // rows read, inclusive
        gdouble* lv[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) lv[l] = gbl(plane(pt, b, o, l)) + gx;
        const double dthr = (double)thr;
        const int otag = o | (b << kOctBits);
        // candidates collect in a per-wave LDS buffer; a full buffer goes out
        // with one counter atomic, the rest with ONE atomic per workgroup at
        // the end: a returning atomic per (row, layer) on the single global
        // counter serialised the whole launch on the small octaves, where
        // candidates are dense, and same-address atomics serialise at one
        // L2 channel (~10 ns each: one per wave was ~40 us of a 1080p
        // octave-0 launch's ~4200 waves)
        auto flush = [&]() {
            if (nbuf == 0) return;
            wave_sync();
            unsigned base = 0;
            if (lane == 0) base = atomicAdd(counter, nbuf);
            base = __shfl(base, 0);
            for (unsigned i = lane; i < nbuf; i += 64)
                if (base + i < cap) out[base + i] = cb[i];
            wave_sync();
            nbuf = 0;
        };
        double pf[PF][NL];
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const size_t ro = (size_t)min(r0 + p, r1) * W;
#pragma unroll
            for (int l = 0; l < NL; ++l) pf[p][l] = ext_load(&lv[l][ro]);
        }
        // two stored rows (y-1, y) of horizontal max / min and the DoG of
        // row y; row y+1's come in as the current row. Rows go in pairs, so
        // the stored slot (r & 1) and the prefetch slot are compile-time (no
        // register moves per row); 136 VGPRs instead of 154 for the three-row
        // window: alone 108.6 -> 107.0 us per 1080p image, the driver's
        // command -1 % (r05_aa; forced to 128 VGPRs for 4 waves per SIMD it
        // spills and takes 113.5)
        static_assert(2 % PF == 0 || PF == 1, "prefetch slots: PF divides the row pair");
        double hmx[2][ND], hmn[2][ND], dc[2][NZ];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int z = 0; z < ND; ++z) hmx[q][z] = hmn[q][z] = 0.0;
        for (int rb = r0; rb <= r1; rb += 2) {
#pragma unroll
            for (int sl = 0; sl < 2; ++sl) {
                const int r = rb + sl;
                const int sq = sl % PF;
                if (r <= r1) {
                    // row r: DoG, horizontal 3-max / 3-min per layer
                    double cmx[ND], cmn[ND], cd[NZ];
#pragma unroll
                    for (int z = 0; z < ND; ++z) {
                        const double d = pf[sq][z + 1] - pf[sq][z];
                        const double dl = dpp_from_left(d), dr = dpp_from_right(d);
                        cmx[z] = fmax(fmax(dl, d), dr);
                        cmn[z] = fmin(fmin(dl, d), dr);
                        if (z >= 1 && z <= NZ) cd[z - 1] = d;
                    }
                    {  // row r + PF into the slot just consumed
                        const size_t ro = (size_t)min(r + PF, r1) * W;
#pragma unroll
                        for (int l = 0; l < NL; ++l) pf[sq][l] = ext_load(&lv[l][ro]);
                    }
                    // centres of row y = r - 1: rows y-1 / y stored in slots
                    // sl / sl^1, row y+1 the current one
                    if (r >= r0 + 2) {
                        const int y = r - 1;
                        const int sy = sl ^ 1, sp = sl;  // unrolled: constants
                        // vertical 3-row max / min of every layer's horizontal
                        // ones, once per row; a layer's cube is then three of
                        // them (16 max + 16 min per row instead of 27 + 27
                        // inside the centre test)
                        double vmx[ND], vmn[ND];
#pragma unroll
                        for (int z = 0; z < ND; ++z) {
                            vmx[z] = fmax(fmax(hmx[sp][z], hmx[sy][z]), cmx[z]);
                            vmn[z] = fmin(fmin(hmn[sp][z], hmn[sy][z]), cmn[z]);
                        }
#pragma unroll
                        for (int z = 1; z <= NZ; ++z) {
                            const double v = dc[sy][z - 1];
                            const double mx = fmax(fmax(vmx[z - 1], vmx[z]), vmx[z + 1]);
                            const double mn = fmin(fmin(vmn[z - 1], vmn[z]), vmn[z + 1]);
                            // (bitwise: compares and mask ANDs, no
                            // exec-mask branches around them)
                            const bool cand =
                                centre_lane & (fabs(v) > dthr) & ((v == mx) | (v == mn));
                            const unsigned long long m = __ballot(cand);
                            if (m) {
                                const unsigned k = (unsigned)__popcll(m);
                                if (nbuf + k > kCandBuf) flush();
                                if (cand)
                                    cb[nbuf + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] =
                                        sift_extremum{x, y, z, otag};
                                nbuf += k;
                            }
                        }
                    }
                    // row r replaces row r - 2 in its slot
#pragma unroll
                    for (int z = 0; z < ND; ++z) {
                        hmx[sl][z] = cmx[z];
                        hmn[sl][z] = cmn[z];
                    }
#pragma unroll
                    for (int z = 0; z < NZ; ++z) dc[sl][z] = cd[z];
                }
            }
        }
    }
    // the workgroup's remaining candidates: one counter atomic
    if (lane == 0) wg_n[wv] = nbuf;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = wg_n[0] + wg_n[1] + wg_n[2] + wg_n[3];
        const unsigned base = t ? atomicAdd(counter, t) : 0u;
        wg_base[0] = base;
        wg_base[1] = base + wg_n[0];
        wg_base[2] = wg_base[1] + wg_n[1];
        wg_base[3] = wg_base[2] + wg_n[2];
    }
    __syncthreads();
    const unsigned base = wg_base[wv];
    for (unsigned i = lane; i < nbuf; i += 64)
        if (base + i < cap) out[base + i] = cb[i];
}

// Generic border b (window_size 4..7): one thread per (x, y), direct cube.
__global__ __launch_bounds__(256) void k_extrema_any(const PyrTable* __restrict__ pt, int o,
                                                     int thr, int b, int nd,
                                                     sift_extremum* __restrict__ out,
                                                     unsigned* __restrict__ counter,
                                                     unsigned cap) {
    const int W = pt->w[o], H = pt->h[o];
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    const int im = blockIdx.z;
    if (x < b || x >= W - b || y < b || y >= H - b) return;
    for (int z = b; z < nd - b; ++z) {
        const size_t c = (size_t)y * W + x;
        const double v = plane(pt, im, o, z + 1)[c] - plane(pt, im, o, z)[c];
        if (fabs(v) <= (double)thr) continue;
        bool mx = true, mn = true;
        for (int dz = -b; dz <= b; ++dz)
            for (int dy = -b; dy <= b; ++dy)
                for (int dx = -b; dx <= b; ++dx) {
                    const size_t q = (size_t)(y + dy) * W + (x + dx);
                    const double n = plane(pt, im, o, z + dz + 1)[q] - plane(pt, im, o, z + dz)[q];
                    if (v < n) mx = false;
                    if (v > n) mn = false;
                }
        if (mx || mn) {
            const unsigned idx = atomicAdd(counter, 1u);
            if (idx < cap) out[idx] = sift_extremum{x, y, z, o | (im << kOctBits)};
        }
    }
}


hipError_t launch_extrema_stream(const PyrTable* d_pt, const ExtremaGrid& eg, int n_img,
                                 int n_gauss, int thr, sift_extremum* out, unsigned* counter,
                                 unsigned cap, unsigned* snap, hipStream_t s, hipEvent_t e0,
                                 hipEvent_t e1) {
    const int tasks = eg.first_tile[eg.n];
    if (tasks == 0 || n_img == 0) {
        if (e0) (void)hipEventRecord(e0, s);
        if (e1) (void)hipEventRecord(e1, s);
        return snap ? launch_snapshot(counter, snap, s, 0, 3) : hipSuccess;
    }
    const dim3 grid((tasks + 3) / 4, n_img);
    switch (n_gauss) {
#define SIFT_EXT_CASE(NL)                                                                   \
    case NL:                                                                                \
        return launch_timed(k_extrema_stream<NL>, grid, dim3(256), 0, s, e0, e1, d_pt, eg,   \
                            thr, out, counter, cap, snap);
        SIFT_EXT_CASE(4)
        SIFT_EXT_CASE(5)
        SIFT_EXT_CASE(6)
        SIFT_EXT_CASE(7)
        SIFT_EXT_CASE(8)
        SIFT_EXT_CASE(9)
        SIFT_EXT_CASE(10)
        SIFT_EXT_CASE(11)
        SIFT_EXT_CASE(12)
#undef SIFT_EXT_CASE
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t launch_extrema_any(const PyrTable* d_pt, int o, int W, int H, int n_img, int n_gauss,
                              int window_size, int thr, sift_extremum* out, unsigned* counter,
                              unsigned cap, hipStream_t s) {
    const int b = window_size / 2;
    dim3 grid((W + 255) / 256, H, n_img);
    hipLaunchKernelGGL(k_extrema_any, grid, dim3(256), 0, s, d_pt, o, thr, b, n_gauss - 1, out,
                       counter, cap);
    return hipGetLastError();
}

}  // namespace sift_amd
