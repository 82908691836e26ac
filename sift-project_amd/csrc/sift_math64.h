// sift_math64.h — f64 sqrt / atan2 / exp for the descriptor's sample math
// (sift_desc.hip), shared with the GPU accuracy check
// (tools/math64_check.hip, tests/test_gpu_math64.py).
#pragma once

#include <hip/hip_runtime.h>

namespace sift_amd {

namespace {

// ---------------------------------------------------------------------------
// f64 sample math. The reference evaluates sqrt, atan2 and exp with glibc
// (sift.cpp:660-672); ROCm's ocml versions cost 22 / 105 / 42 VALU
// instructions per lane on gfx950 with their full-range handling. The
// descriptor's arguments have known ranges, so these do the same f64
// arithmetic without it:
//  * sqrt_f64: v_rsq_f64 + two Goldschmidt steps + two residual corrections
//    (the correctly rounded sequence LLVM emits for f64 sqrt, minus the
//    denormal scaling: s = dx^2 + dy^2 is 0 or far above 2^-767 here);
//  * atan2_f64: octant reduction to a = min/max in [0, 1], a table point
//    c = k/16 nearest a (picked from an f32 estimate), atan(a) = atan(c) +
//    atan(u) with u = (min - c max) / (max + c min), |u| <= 1/32 + 1e-7, one
//    Newton-refined f64 division and atan(u) through u^11 (next term < 1e-19
//    relative) added to atan(c) as a double-double; quadrant fix-ups with double-double pi/2 and pi. Error about
//    1 ulp, against glibc's correctly rounded-in-most-cases atan2;
//  * exp_f64: 2^k exp(r), k = rint(x log2 e), r by Cody-Waite (fdlibm's split
//    of ln 2), exp(r) by its Taylor series through r^13 (|r| <= 0.347, next
//    term < 5e-18 relative). The argument is -(row_rot^2 + col_rot^2)/8 in
//    [-1.6, 0].
// tests/test_gpu_math64.py checks all three against the device's own
// correctly rounded sqrt and ocml atan2 / exp on millions of arguments.
// ---------------------------------------------------------------------------
// atan(k/16), k = 0..16, as double-double pairs (hi = correctly rounded,
// lo = the remainder rounded; tools/gen_atan_table.py)
__constant__ double2 kAtanTab[17] = {
    {0x0.0p+0, 0x0.0p+0},
    {0x1.ff55bb72cfdeap-5, -0x1.c934d86d23f1dp-60},
    {0x1.fd5ba9aac2f6ep-4, -0x1.cd37686760c17p-59},
    {0x1.7b97b4bce5b02p-3, 0x1.347b0b4f881cap-58},
    {0x1.f5b75f92c80ddp-3, 0x1.8ab6e3cf7afbdp-57},
    {0x1.362773707ebccp-2, -0x1.963a544b672d8p-57},
    {0x1.6f61941e4def1p-2, -0x1.c63aae6f6e918p-56},
    {0x1.a64eec3cc23fdp-2, -0x1.24dec1b50b7ffp-56},
    {0x1.dac670561bb4fp-2, 0x1.a2b7f222f65e2p-56},
    {0x1.0657e94db30d0p-1, -0x1.d5b495f6349e6p-56},
    {0x1.1e00babdefeb4p-1, -0x1.928df287a668fp-58},
    {0x1.345f01cce37bbp-1, 0x1.1021137c71102p-55},
    {0x1.4978fa3269ee1p-1, 0x1.2419a87f2a458p-56},
    {0x1.5d58987169b18p-1, 0x1.0028e4bc5e7cap-57},
    {0x1.700a7c5784634p-1, -0x1.8c34d25aadef6p-56},
    {0x1.819d0b7158a4dp-1, -0x1.bf76229d3b917p-56},
    {0x1.921fb54442d18p-1, 0x1.1a62633145c07p-55},
};

__device__ __forceinline__ double sqrt_f64(double s) {
    const double y = __builtin_amdgcn_rsq(s);
    double g = s * y, h = 0.5 * y;
    const double r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, s);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, s);
    g = __builtin_fma(d, h, g);
    return s > 0.0 ? g : s;  // rsq(0) = inf
}

// atan2 for max(|x|, |y|) below the f32 normal range (never seen on image
// gradients, but kept correct): ocml's f64 atan2, out of line so the common
// path's registers do not pay for it
__device__ __noinline__ double atan2_tiny(double y, double x) { return atan2(y, x); }

// atan2(y, x); `tab` = kAtanTab staged in LDS
__device__ __forceinline__ double atan2_f64(double y, double x, const double2* tab) {
    const double ax = fabs(x), ay = fabs(y);
    const bool swap = ay > ax;
    const double mx = swap ? ay : ax, mn = swap ? ax : ay;
    // the table point comes from an f32 estimate of mn / mx: below FLT_MIN,
    // (float)mx flushes (inf / NaN estimate, kf = 16, |u| up to 1: outside
    // the series' range) and the f64 reciprocal below loses range too
    if (mx < 0x1p-120 && mx > 0.0) return atan2_tiny(y, x);
    const float af = (float)mn * __builtin_amdgcn_rcpf((float)mx);
    const float kf = __builtin_rintf(fminf(fmaxf(af * 16.0f, 0.0f), 16.0f));
    const double c = (double)kf * 0.0625;
    const double num = __builtin_fma(-c, mx, mn);
    const double den = __builtin_fma(c, mn, mx);
    double r = __builtin_amdgcn_rcp(den);
    double e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    double u = num * r;
    u = __builtin_fma(__builtin_fma(-den, u, num), r, u);
    const double t = u * u;
    double p = __builtin_fma(t, -1.0 / 11.0, 1.0 / 9.0);
    p = __builtin_fma(t, p, -1.0 / 7.0);
    p = __builtin_fma(t, p, 1.0 / 5.0);
    p = __builtin_fma(t, p, -1.0 / 3.0);
    const double2 ck = tab[(int)kf];
    double th = ck.x + (__builtin_fma(u * t, p, u) + ck.y);
    if (swap) th = (0x1.921fb54442d18p+0 - th) + 0x1.1a62633145c07p-54;  // pi/2 - th
    if (x < 0.0) th = (0x1.921fb54442d18p+1 - th) + 0x1.1a62633145c07p-53;  // pi - th
    if (!(mx > 0.0)) th = __builtin_signbit(x) ? 0x1.921fb54442d18p+1 : 0.0;
    return __builtin_copysign(th, y);
}

__device__ __forceinline__ double exp_f64(double x) {
    const double kf = __builtin_rint(x * 0x1.71547652b82fep+0);  // x / ln 2
    double r = __builtin_fma(-kf, 0x1.62e42feep-1, x);            // ln 2, high part
    r = __builtin_fma(-kf, 0x1.a39ef35793c76p-33, r);             // ln 2, low part
    double p = 1.0 / 6227020800.0;                                // 1/13!
    p = __builtin_fma(p, r, 1.0 / 479001600.0);
    p = __builtin_fma(p, r, 1.0 / 39916800.0);
    p = __builtin_fma(p, r, 1.0 / 3628800.0);
    p = __builtin_fma(p, r, 1.0 / 362880.0);
    p = __builtin_fma(p, r, 1.0 / 40320.0);
    p = __builtin_fma(p, r, 1.0 / 5040.0);
    p = __builtin_fma(p, r, 1.0 / 720.0);
    p = __builtin_fma(p, r, 1.0 / 120.0);
    p = __builtin_fma(p, r, 1.0 / 24.0);
    p = __builtin_fma(p, r, 1.0 / 6.0);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)kf);
}

}  // namespace

}  // namespace sift_amd
