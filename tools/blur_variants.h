// blur_variants.h — candidate octave-0 blur kernels for tools/blur_lab.hip
// (test tooling; included after the library's sift_kernels.hip). Every
// variant evaluates apply_double_convolution_1d (reference image.cpp:156-214)
// with the library's per-output order: acc = v*k0, acc += k[u]*(v[+u]+v[-u]),
// Markstein-corrected division by sum_w, replicate borders by clamping.
#pragma once

namespace sift_amd {
namespace lab {

// ---------------------------------------------------------------------------
// k_blur_pc<R, C, DECIM>: producer / consumer wave pairs. A workgroup holds
// two pairs; a pair owns a strip of 64*C columns x `rows` output rows. The
// producer wave stages each source row in its LDS line (as k_blur) and writes
// the row pass into a 3-slot LDS ring; the consumer wave moves each row-pass
// row from the ring into its (2R+1)-deep register window and evaluates the
// column pass. One workgroup barrier per step keeps the pairs in lockstep.
// The two roles' loop-carried registers share one array (st: the producer's
// prefetched rows / the consumer's window), so a wave pays for one role.
// ---------------------------------------------------------------------------
template <int R, int C, bool DECIM>
__global__ __launch_bounds__(256) void k_blur_pc(const double* __restrict__ src, size_t src_bs,
                                                 double* __restrict__ dst, size_t bs, int W, int H,
                                                 int rows, BlurTaps taps,
                                                 double* __restrict__ dec, int Wd, int Hd) {
    constexpr int PF = 2;
    constexpr int SPAN = 64 * C;
    constexpr int NL = (SPAN + 2 * R + 63) / 64;
    constexpr int NW = 2 * R + 1;
    constexpr int NST = (PF * NL > C * NW) ? PF * NL : C * NW;
    __shared__ __attribute__((aligned(16))) double sline[2][64 * NL + 2];
    __shared__ __attribute__((aligned(16))) double ring[2][3 * SPAN];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pair = wv >> 1;
    const bool producer = (wv & 1) == 0;
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    src += bz * src_bs;
    dst += bz * bs;
    if (DECIM) dec += bz * bs;
    const int x0 = bx * SPAN;
    if (by * 2 * rows >= H) return;  // both pairs below the image
    const int y_begin = (by * 2 + pair) * rows;
    const int y_end = min(y_begin + rows, H);
    const int nsrc = rows + 2 * R;   // source rows of the walk
    const int nsteps = nsrc + 1;     // the consumer runs one step behind
    double* const sl = sline[pair];
    double* const rg = ring[pair];
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    int gx[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
    const int yy0 = y_begin - R;
    double st[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) st[i] = 0.0;
    if (producer) {
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            const int ry = clampi(yy0 + p, 0, H - 1);
#pragma unroll
            for (int q = 0; q < NL; ++q) st[p * NL + q] = src[(size_t)ry * W + gx[q]];
        }
    }
    const int xa = x0 + C * lane;
    int slot_w = 0;  // ring slot the producer writes this step (step % 3)
    for (int sb = 0; sb < nsteps; sb += NW) {
#pragma unroll
        for (int t = 0; t < NW; ++t) {
            const int s = sb + t;
            if (s < nsteps) {
                if (producer) {
                    if (s < nsrc) {
#pragma unroll
                        for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = st[q];
#pragma unroll
                        for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
                            for (int q = 0; q < NL; ++q) st[p * NL + q] = st[(p + 1) * NL + q];
                        const int ry = clampi(yy0 + s + PF, 0, H - 1);
#pragma unroll
                        for (int q = 0; q < NL; ++q)
                            st[(PF - 1) * NL + q] = src[(size_t)ry * W + gx[q]];
                        wave_sync();
                        double v[C + 2 * R];
                        if (C == 2) {
                            const double2* s2 = reinterpret_cast<const double2*>(sl + 2 * lane);
#pragma unroll
                            for (int q = 0; q < (C + 2 * R) / 2; ++q) {
                                const double2 x = s2[q];
                                v[2 * q] = x.x;
                                v[2 * q + 1] = x.y;
                            }
                        } else {
#pragma unroll
                            for (int q = 0; q < C + 2 * R; ++q) v[q] = sl[lane + q];
                        }
                        double* out = rg + slot_w * SPAN + C * lane;
#pragma unroll
                        for (int c = 0; c < C; ++c) {
                            double acc = v[c + R] * k[0];
#pragma unroll
                            for (int u = 1; u <= R; ++u) acc += k[u] * (v[c + R + u] + v[c + R - u]);
                            out[c] = div_sum_w(acc, sw, inv);
                        }
                        wave_sync();
                    }
                } else if (s >= 1) {
                    // source row s - 1 of the walk -> window slot (t - 1) mod NW
                    const int slot_r = slot_w == 0 ? 2 : slot_w - 1;
                    const double* in = rg + slot_r * SPAN + C * lane;
#pragma unroll
                    for (int c = 0; c < C; ++c) st[c * NW + (t + NW - 1) % NW] = in[c];
                    if (s - 1 >= 2 * R) {
                        const int y = y_begin + (s - 1) - 2 * R;
                        double o[C];
#pragma unroll
                        for (int c = 0; c < C; ++c) {
                            // centre: source row s - 1 - R -> slot (t - 1 - R) mod NW
                            double a = st[c * NW + (t + 2 * NW - 1 - R) % NW] * k[0];
#pragma unroll
                            for (int u = 1; u <= R; ++u)
                                a += k[u] * (st[c * NW + (t + 2 * NW - 1 - R + u) % NW] +
                                             st[c * NW + (t + 2 * NW - 1 - R - u) % NW]);
                            o[c] = div_sum_w(a, sw, inv);
                        }
                        if (y < y_end && xa < W) {
                            if (C == 2)
                                *reinterpret_cast<double2*>(dst + (size_t)y * W + xa) =
                                    make_double2(o[0], o[C - 1]);
                            else
                                dst[(size_t)y * W + xa] = o[0];
                            if (DECIM && !(y & 1) && (y >> 1) < Hd &&
                                (C == 2 || !(xa & 1)) && (xa >> 1) < Wd)
                                dec[(size_t)(y >> 1) * Wd + (xa >> 1)] = o[0];
                        }
                    }
                }
                slot_w = slot_w == 2 ? 0 : slot_w + 1;
                __syncthreads();
            }
        }
    }
}

template <int R, int C>
hipError_t launch_pc_r(const double* src, double* dst, int W, int H, int rows,
                       const BlurTaps& t, double* dec, int Wd, int Hd, hipStream_t s,
                       hipEvent_t e0, hipEvent_t e1) {
    const dim3 grid((W + 64 * C - 1) / (64 * C), ((H + rows - 1) / rows + 1) / 2, 1);
    if (dec)
        return launch_timed(k_blur_pc<R, C, true>, grid, dim3(256), 0, s, e0, e1, src, (size_t)0,
                            dst, (size_t)0, W, H, rows, t, dec, Wd, Hd);
    return launch_timed(k_blur_pc<R, C, false>, grid, dim3(256), 0, s, e0, e1, src, (size_t)0, dst,
                        (size_t)0, W, H, rows, t, dec, Wd, Hd);
}


// ---------------------------------------------------------------------------
// k_blur_ud<R, C, DECIM>: k_blur's strip walk with the priming shared. The
// two waves of a pair own the `rows` rows on either side of a boundary b and
// walk AWAY from it (wave 0 of the pair upward over [b - rows, b), wave 1
// downward over [b, b + rows)). Both need the row passes of source rows
// [b - R, b + R) before their first output: each evaluates the R rows on its
// own side, keeps them in its window and hands them to its partner through
// LDS (one workgroup barrier), so a wave evaluates R + rows row passes
// instead of 2R + rows. The column pass's pair sums are commutative, so the
// walk direction leaves every output bit-identical.
// Window positions in walk order: position p of the down wave is source row
// b - R + p, of the up wave b - 1 + R - p; positions [R, 2R) are a wave's
// own prologue rows, [0, R) its partner's (partner position R + j = my
// position R - 1 - j), position 2R + k is computed at walk step k.
// ---------------------------------------------------------------------------
template <int R, int C, bool DECIM>
__global__ __launch_bounds__(256) void k_blur_ud(const double* __restrict__ src, size_t src_bs,
                                                 double* __restrict__ dst, size_t bs, int W, int H,
                                                 int rows, BlurTaps taps,
                                                 double* __restrict__ dec, int Wd, int Hd) {
    constexpr int PF = 2;
    constexpr int NW = 2 * R + 2;
    constexpr int SPAN = 64 * C;
    constexpr int NL = (SPAN + 2 * R + 63) / 64;
    __shared__ __attribute__((aligned(16))) double sline[4][64 * NL + 2];
    __shared__ __attribute__((aligned(16))) double xch[4][R][SPAN];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool down = (wv & 1) != 0;
    int bx, by, bz;
    xcd_remap(bx, by, bz);
    src += bz * src_bs;
    dst += bz * bs;
    if (DECIM) dec += bz * bs;
    const int x0 = bx * SPAN;
    const int b = (by * 2 + (wv >> 1)) * 2 * rows + rows;  // the pair's boundary
    if ((by * 2) * 2 * rows >= H) return;  // the whole workgroup is below the image
    double* const sl = sline[wv];
    int gx[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) gx[q] = clampi(x0 - R + lane + 64 * q, 0, W - 1);
    double k[R + 1];
#pragma unroll
    for (int u = 0; u <= R; ++u) k[u] = taps.k[u];
    const double sw = taps.sum_w, inv = taps.inv;
    // source row of walk position p
    auto row_at = [&](int p) { return down ? b - R + p : b - 1 + R - p; };
    double win[C][NW];
    auto row_pass = [&](double* hn) {  // of the row staged in sl
        double v[C + 2 * R];
        if (C == 2) {
            const double2* s2 = reinterpret_cast<const double2*>(sl + 2 * lane);
#pragma unroll
            for (int q = 0; q < (C + 2 * R) / 2; ++q) {
                const double2 t = s2[q];
                v[2 * q] = t.x;
                v[2 * q + 1] = t.y;
            }
        } else {
#pragma unroll
            for (int q = 0; q < C + 2 * R; ++q) v[q] = sl[lane + q];
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double acc = v[c + R] * k[0];
#pragma unroll
            for (int u = 1; u <= R; ++u) acc += k[u] * (v[c + R + u] + v[c + R - u]);
            hn[c] = div_sum_w(acc, sw, inv);
        }
    };
    // ---- prologue: own rows (positions R .. 2R-1), staged one at a time
    {
        double nx[NL];
        {
            const int ry = clampi(row_at(R), 0, H - 1);
#pragma unroll
            for (int q = 0; q < NL; ++q) nx[q] = src[(size_t)ry * W + gx[q]];
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
#pragma unroll
            for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = nx[q];
            if (j + 1 < R) {
                const int ry = clampi(row_at(R + j + 1), 0, H - 1);
#pragma unroll
                for (int q = 0; q < NL; ++q) nx[q] = src[(size_t)ry * W + gx[q]];
            }
            wave_sync();
            double hn[C];
            row_pass(hn);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                win[c][R + j] = hn[c];
                xch[wv][j][C * lane + c] = hn[c];
            }
            wave_sync();
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) win[c][R - 1 - j] = xch[wv ^ 1][j][C * lane + c];
    // ---- walk: step k stages position 2R + k and evaluates the output at
    // position k - 1 + R (window positions k - 1 .. k - 1 + 2R)
    double pf[PF][NL];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int ry = clampi(row_at(2 * R + p), 0, H - 1);
#pragma unroll
        for (int q = 0; q < NL; ++q) pf[p][q] = src[(size_t)ry * W + gx[q]];
    }
    const int xa = x0 + C * lane;
    const int nsteps = rows + 1;
    for (int kb = 0; kb < nsteps; kb += NW) {
#pragma unroll
        for (int t = 0; t < NW; ++t) {
            const int kk = kb + t;
            if (kk < nsteps) {
#pragma unroll
                for (int q = 0; q < NL; ++q) sl[lane + 64 * q] = pf[0][q];
#pragma unroll
                for (int p = 0; p + 1 < PF; ++p)
#pragma unroll
                    for (int q = 0; q < NL; ++q) pf[p][q] = pf[p + 1][q];
                const int ry = clampi(row_at(2 * R + kk + PF), 0, H - 1);
#pragma unroll
                for (int q = 0; q < NL; ++q) pf[PF - 1][q] = src[(size_t)ry * W + gx[q]];
                wave_sync();
                double hn[C];
                row_pass(hn);
                if (kk >= 1) {
                    // centre position kk - 1 + R -> slot (2R + t - 1 - R) mod NW
                    const int y = down ? b + kk - 1 : b - kk;
                    double o[C];
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        double a = win[c][(t + R - 1 + NW) % NW] * k[0];
#pragma unroll
                        for (int u = 1; u <= R; ++u)
                            a += k[u] * (win[c][(t + R - 1 + u) % NW] +
                                         win[c][(t + R - 1 - u + 2 * NW) % NW]);
                        o[c] = div_sum_w(a, sw, inv);
                    }
                    if (y >= 0 && y < H && xa < W) {
                        if (C == 2)
                            *reinterpret_cast<double2*>(dst + (size_t)y * W + xa) =
                                make_double2(o[0], o[C - 1]);
                        else
                            dst[(size_t)y * W + xa] = o[0];
                        if (DECIM && !(y & 1) && (y >> 1) < Hd && (C == 2 || !(xa & 1)) &&
                            (xa >> 1) < Wd)
                            dec[(size_t)(y >> 1) * Wd + (xa >> 1)] = o[0];
                    }
                }
#pragma unroll
                for (int c = 0; c < C; ++c) win[c][(2 * R + t) % NW] = hn[c];
                wave_sync();
            }
        }
    }
}

template <int R, int C>
hipError_t launch_ud_r(const double* src, double* dst, int W, int H, int rows, const BlurTaps& t,
                       double* dec, int Wd, int Hd, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const dim3 grid((W + 64 * C - 1) / (64 * C), (H + 4 * rows - 1) / (4 * rows), 1);
    if (dec)
        return launch_timed(k_blur_ud<R, C, true>, grid, dim3(256), 0, s, e0, e1, src, (size_t)0,
                            dst, (size_t)0, W, H, rows, t, dec, Wd, Hd);
    return launch_timed(k_blur_ud<R, C, false>, grid, dim3(256), 0, s, e0, e1, src, (size_t)0, dst,
                        (size_t)0, W, H, rows, t, dec, Wd, Hd);
}

// the library's strip walk at an explicit shape (C columns per lane, rows)
template <int R, int C>
hipError_t launch_strip_r(const double* src, double* dst, int W, int H, int rows,
                          const BlurTaps& t, double* dec, int Wd, int Hd, hipStream_t s,
                          hipEvent_t e0, hipEvent_t e1) {
    const BlurSource bsrc{src, 0, W, H, 1};
    return launch_blur_r<R, C, kSrcPlane>(bsrc, dst, 0, 1, W, H, rows, t, dec, Wd, Hd, s, e0, e1);
}

// the library's pair walk (k_blur_pair) at an explicit shape
template <int R, int C>
hipError_t launch_pair_lab(const double* src, double* dst, int W, int H, int rows,
                           const BlurTaps& t, double* dec, int Wd, int Hd, hipStream_t s,
                           hipEvent_t e0, hipEvent_t e1) {
    return launch_pair_r<R, C>(src, 0, dst, 0, 1, W, H, rows, t, dec, Wd, Hd, s, e0, e1);
}

using VarFn = hipError_t (*)(const double*, double*, int, int, int, const BlurTaps&, double*, int,
                             int, hipStream_t, hipEvent_t, hipEvent_t);

// k_blur_pair_dma (the library's LDS-DMA pair walk) at an explicit shape and
// ring depth NB (env LAB_NB: 2, 4 or 8; default 4)
template <int R, int C, int NB>
hipError_t launch_pdma_lab(const double* src, double* dst, int W, int H, int rows,
                           const BlurTaps& t, double* dec, int Wd, int Hd, hipStream_t s,
                           hipEvent_t e0, hipEvent_t e1) {
    return launch_pair_dma_r<R, C, NB>(src, 0, dst, 0, 1, W, H, rows, t, dec, Wd, Hd, s, e0, e1);
}
template <int R, int C>
VarFn pick_pdma() {
    const char* e = std::getenv("LAB_NB");
    const int nb = e ? std::atoi(e) : 4;
    if (nb == 2) return &launch_pdma_lab<R, C, 2>;
    if (nb == 8) return &launch_pdma_lab<R, C, 8>;
    return &launch_pdma_lab<R, C, 4>;
}

// radii the lab instantiates (octave-0 levels of intervals 3 and 2)
#define LAB_RADII(X) X(4) X(5) X(6) X(7) X(8) X(10) X(14)

inline VarFn pick(const char* kind, int C, int R) {
#define LAB_CASE(RR)                                                                   \
    if (R == RR) {                                                                     \
        if (!std::strcmp(kind, "pc")) return C == 2 ? &launch_pc_r<RR, 2> : &launch_pc_r<RR, 1>; \
        if (!std::strcmp(kind, "ud")) return C == 2 ? &launch_ud_r<RR, 2> : &launch_ud_r<RR, 1>; \
        if (!std::strcmp(kind, "pair"))                                                \
            return C == 2 ? &launch_pair_lab<RR, 2> : &launch_pair_lab<RR, 1>;        \
        if (!std::strcmp(kind, "pdma"))                                                \
            return C == 2 ? pick_pdma<RR, 2>() : pick_pdma<RR, 1>();                   \
        if (!std::strcmp(kind, "strip"))                                               \
            return C == 2 ? &launch_strip_r<RR, 2> : &launch_strip_r<RR, 1>;          \
    }
    LAB_RADII(LAB_CASE)
#undef LAB_CASE
    return nullptr;
}

}  // namespace lab
}  // namespace sift_amd
