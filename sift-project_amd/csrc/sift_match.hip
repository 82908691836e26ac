// sift_match.hip — brute-force 2-NN ratio-test matcher on the GPU
// ("next" row 1).
//
// Reference: euclid_dist (src/sift.cpp:688-695) and match_keypoints
// (src/sift.cpp:783-815): for every keypoint of image 1, the two smallest
// Euclidean distances between its 128 u8 descriptor bytes and those of every
// keypoint of image 2; a match when best < ratio * second.
//
// Exactness. The reference sums (a_i - b_i)^2 in double: an integer below
// 2^23, so exact. The distances it compares are the correctly rounded square
// roots of those integers, a strictly increasing function on them
// (neighbouring roots below 2^23 differ by more than 1e-4), so comparing the
// integer sums S makes exactly the reference's decisions. Its scan order fixes
// the tie rules, which an order-free merge reproduces:
//   best   = smallest S, lowest index among equal S (strict '<' update);
//   second = second smallest S of the multiset (an S equal to best seen
//            later becomes second through the 'else if').
// The reported distance is sqrt((double)S) and the ratio test runs in double
// on it, with DBL_MAX for an absent second neighbour (n2 == 1) as in the
// reference.
//
// Arithmetic. S = |a|^2 + |b|^2 - 2 a.b with the dot products on the i8
// matrix cores (v_mfma_i32_32x32x32_i8). Bytes are stored shifted,
// a' = a - 128 (= a ^ 0x80 read as int8), so
//   a.b = a'.b' + 128 (sum a' + sum b') + 2^21,
//   S   = q(a) + q(b) - 2 a'.b',   q(v) = |v|^2 - 256 sum v' - 2^21,
// all exact in int32 (|q| < 2^23, |a'.b'| <= 2^21).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "sift_kernels.h"

namespace sift_amd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// q of a padding row (zero shifted bytes): its S is >= kAbsent for any query
constexpr int kPadQ = (1 << 30) + (1 << 25);
constexpr long long kAbsent = 1ll << 30;

struct Top2 {
    int b;  // smallest value
    int s;  // second smallest value of the multiset
    int i;  // index of the smallest (lowest among equal values)
};

__device__ __forceinline__ void top2_push(Top2& t, int v, int j) {
    if (v < t.b || (v == t.b && j < t.i)) {
        t.s = t.b;
        t.b = v;
        t.i = j;
    } else if (v < t.s) {
        t.s = v;
    }
}

// union of two disjoint partial scans
__device__ __forceinline__ Top2 top2_merge(Top2 x, Top2 y) {
    if (y.b < x.b || (y.b == x.b && y.i < x.i)) {
        const Top2 t = x;
        x = y;
        y = t;
    }
    x.s = min(x.s, y.b);
    return x;
}

// Records -> shifted descriptor rows [n_pad][128] and q; 16 threads per
// record, 8 bytes each. Rows [n, n_pad) are padding (zero bytes, kPadQ).
__global__ __launch_bounds__(256) void k_match_prep(const sift_kp* __restrict__ kps, unsigned n,
                                                    uint8_t* __restrict__ rows,
                                                    int* __restrict__ q) {
    const unsigned rec = blockIdx.x * 16 + (threadIdx.x >> 4);
    const int t = threadIdx.x & 15;
    uint2 v = make_uint2(0x80808080u, 0x80808080u);  // 128: shifted to 0
    if (rec < n) v = *reinterpret_cast<const uint2*>(kps[rec].desc + 8 * t);
    int s2 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int b = (int)(((k < 4 ? v.x : v.y) >> (8 * (k & 3))) & 255u);
        s2 += b * b;
        s1 += b - 128;
    }
    *reinterpret_cast<uint2*>(rows + (size_t)rec * 128 + 8 * t) =
        make_uint2(v.x ^ 0x80808080u, v.y ^ 0x80808080u);
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
        s2 += __shfl_xor(s2, off);
        s1 += __shfl_xor(s1, off);
    }
    if (t == 0) q[rec] = rec < n ? s2 - 256 * s1 - (1 << 21) : kPadQ;
}

// One workgroup per 32 queries (the MFMA's B columns, kept in registers);
// its four waves sweep 32-row tiles of image 2 (the A rows) round-robin.
// The 32x32 i32 result of a tile has the query on the lane (col = lane & 31)
// and 16 reference rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5) in registers,
// so each lane keeps a running top-2 for its query over its rows; lanes
// l and l ^ 32, then the four waves, are merged at the end.
__global__ __launch_bounds__(256) void k_match2nn(const uint8_t* __restrict__ qrows,
                                                  const int* __restrict__ qq, unsigned n1,
                                                  const uint8_t* __restrict__ rrows,
                                                  const int* __restrict__ rq, unsigned n2_pad,
                                                  double ratio, int* __restrict__ out_j,
                                                  double* __restrict__ out_d) {
    __shared__ Top2 part[4][32];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 31, h = lane >> 5;
    const unsigned q0 = blockIdx.x * 32;
    // B fragments: K-step s covers descriptor bytes [32s, 32s + 32); lane
    // (col, h) holds bytes 32s + 16h .. +15 of query q0 + col. A uses the same
    // byte assignment, so the sum over k is the full dot product whatever the
    // hardware's order inside a step.
    v4i bq[4];
    const v4i* qv = reinterpret_cast<const v4i*>(qrows + (size_t)(q0 + col) * 128);
#pragma unroll
    for (int s = 0; s < 4; ++s) bq[s] = qv[2 * s + h];
    Top2 t{INT_MAX, INT_MAX, INT_MAX};
    for (unsigned r0 = 32u * wv; r0 < n2_pad; r0 += 128u) {
        const v4i* rv = reinterpret_cast<const v4i*>(rrows + (size_t)(r0 + col) * 128);
        v4i a[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = rv[2 * s + h];
        v4i rqv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) rqv[g] = *reinterpret_cast<const v4i*>(rq + r0 + 8 * g + 4 * h);
        v16i acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; ++s)
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], bq[s], acc, 0, 0, 0);
        // S - q(query) for the 16 rows of this lane, in increasing row order
#pragma unroll
        for (int r = 0; r < 16; ++r)
            top2_push(t, rqv[r >> 2][r & 3] - 2 * acc[r],
                      (int)(r0 + (r & 3) + 8 * (r >> 2) + 4 * h));
    }
    Top2 o;
    o.b = __shfl_xor(t.b, 32);
    o.s = __shfl_xor(t.s, 32);
    o.i = __shfl_xor(t.i, 32);
    t = top2_merge(t, o);
    if (h == 0) part[wv][col] = t;
    __syncthreads();
    if (threadIdx.x < 32) {
        Top2 m = part[0][col];
#pragma unroll
        for (int w = 1; w < 4; ++w) m = top2_merge(m, part[w][col]);
        const unsigned qi = q0 + col;
        if (qi < n1) {
            const long long myq = qq[qi];
            const long long sb = myq + m.b, ss = myq + m.s;
            const double best = sqrt((double)sb);
            const double second = ss >= kAbsent ? DBL_MAX : sqrt((double)ss);
            out_j[qi] = best < ratio * second ? m.i : -1;
            out_d[qi] = best;
        }
    }
}

}  // namespace

hipError_t launch_match_prep(const sift_kp* d_kps, unsigned n, unsigned n_pad, uint8_t* rows,
                             int* q, hipStream_t s) {
    if (n_pad == 0 || n_pad % 32 != 0 || n > n_pad) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_match_prep, dim3(n_pad / 16), dim3(256), 0, s, d_kps, n, rows, q);
    return hipGetLastError();
}

hipError_t launch_match2nn(const uint8_t* qrows, const int* qq, unsigned n1, unsigned n1_pad,
                           const uint8_t* rrows, const int* rq, unsigned n2_pad, double ratio,
                           int* out_j, double* out_d, hipStream_t s) {
    if (n1_pad == 0 || n1_pad % 32 != 0 || n1 > n1_pad || n2_pad == 0 || n2_pad % 32 != 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_match2nn, dim3(n1_pad / 32), dim3(256), 0, s, qrows, qq, n1, rrows, rq,
                       n2_pad, ratio, out_j, out_d);
    return hipGetLastError();
}

}  // namespace sift_amd
