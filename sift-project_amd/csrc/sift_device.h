// sift_device.h — device helpers shared by the kernel translation units
// (sift_kernels.hip: pyramid, extrema, refine, orientation; sift_desc.hip:
// descriptors). Internal to the library.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "sift_types.h"

#ifndef SIFT_AGE_BOOST0  // SIFT_AGE_PRIO: issue-priority boost of the oldest job in flight
#define SIFT_AGE_BOOST0 2
#endif
#ifndef SIFT_AGE_BOOST1  // ... and of the second oldest
#define SIFT_AGE_BOOST1 1
#endif

namespace sift_amd {

namespace {

constexpr double kTwoPi = 6.283185307179586;  // M_PI2 (sift.hh:5)
constexpr double kPi = 3.14159265358979323846;  // M_PI

// Compiler-level ordering for LDS traffic exchanged between the lanes of ONE
// wavefront (a wave's LDS instructions execute in order in hardware).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave issue priority of a kernel of job jp: `base` (the pyramid's static
// priority), raised by 2 for the oldest job in flight and by 1 for the next
// (rank from the context's completed-job counter, read once at start)
__device__ __forceinline__ void set_job_prio(const JobPrio& jp, int base) {
    int p = base;
    if (jp.done) {
        const int done = (int)__hip_atomic_load(jp.done, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        const int rank = (int)((unsigned)jp.ticket - 1u - (unsigned)done);  // mod 2^32
        p += rank <= 0 ? SIFT_AGE_BOOST0 : (rank == 1 ? SIFT_AGE_BOOST1 : 0);
    }
    switch (p < 3 ? p : 3) {
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 3: __builtin_amdgcn_s_setprio(3); break;
        default: break;
    }
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

// 2^e for small integer e, exact (the reference uses std::pow(2, int)).
__device__ __forceinline__ double pow2i(int e) { return ldexp(1.0, e); }

// Pyramid planes are device (global) memory; pointers read from the PyrTable
// are generic to the compiler, which would emit flat loads (counted in both
// vmcnt and lgkmcnt). Viewing them in address space 1 gives global loads.
typedef __attribute__((address_space(1))) const double gdouble;
__device__ __forceinline__ gdouble* gbl(const double* p) { return (gdouble*)p; }
// ... and for stores (a generic-pointer store is a FLAT store, counted in
// lgkmcnt too: every later LDS wait of the wave would also wait for it)
typedef __attribute__((address_space(1))) double gdouble_w;
__device__ __forceinline__ gdouble_w* gbl_w(double* p) { return (gdouble_w*)p; }

// lane l's value of a per-lane table (wave-uniform result, no memory access)
__device__ __forceinline__ int readlane_i32(int v, int l) {
    return __builtin_amdgcn_readlane(v, l);
}
template <class T>
__device__ __forceinline__ T* readlane_ptr(T* p, int l) {
    const unsigned long long u = reinterpret_cast<unsigned long long>(p);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}

// Plane of level l of octave o of image b of the job (one pyramid arena per
// image, identical layouts img_stride doubles apart).
__device__ __forceinline__ const double* plane(const PyrTable* pt, int b, int o, int l) {
    return pt->lvl[o][l] + (size_t)b * pt->img_stride;
}

// Correctly rounded a / s for the per-kernel constant s = sum_w, with
// inv = RN(1/s) from the host: q = RN(a*inv) is faithful and Markstein's
// correction q + (a - q*s)*inv (residual exact by FMA) rounds to RN(a/s) —
// the same final step as gfx950's own v_div_fmas sequence, without the
// v_rcp_f64 / Newton / scaling part. Checked against IEEE division on
// 2.5e12 random operands over every divisor the default pyramids use
// (tools/blur_lab.hip divcheck, 0 mismatches); the pyramid parity tests
// compare every level bit for bit.
__device__ __forceinline__ double div_sum_w(double a, double s, double inv) {
    const double q = a * inv;
    const double r = __builtin_fma(-q, s, a);
    return __builtin_fma(r, inv, q);
}

// atan2 in f32 (orientation bins, f32 descriptor math): octant reduction to
// a = min(|x|, |y|) / max(|x|, |y|) (v_rcp_f32, 1 ulp), atan(a) as
// a + a^3 p(a^2) with a degree-7 p fitted for minimum max error on [0, 1]
// (8.5e-8 rad in f32 arithmetic over 2e6 points), then the quadrant fix-up.
// About 20 VALU instructions against ~35 for atan2f; total error below
// 3.1e-7 rad with the f32 rounding of the inputs and of the result (checked
// against f64 atan2 on 4M gradients by tests/test_gpu_math64.py). That is
// < 4e-7 of a descriptor orientation bin and < 2e-6 of an orientation bin
// at 36 bins, far inside k_orient_wave's guard band (1e-4 of a bin). atan2(0, 0) = 0;
// signs of zeros as atan2f.
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

// Launch with optional HIP events whose start/stop timestamps ride on the
// dispatch packet itself (no extra barrier packets between kernels).
template <class K, class... Args>
static hipError_t launch_timed(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                               hipEvent_t e0, hipEvent_t e1, Args... args) {
    if (e0 && e1)
        hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, e0, e1, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    return hipGetLastError();
}

}  // namespace

}  // namespace sift_amd
