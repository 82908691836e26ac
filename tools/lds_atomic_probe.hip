// lds_atomic_probe.hip — what SQ_LDS_BANK_CONFLICT counts for the f64 LDS
// atomics of the descriptor histograms (csrc/sift_desc.hip add_sample_f64).
// Each kernel is one address pattern of ds_add_f64 over a wave's 1024-double
// region (no return value, as the descriptor's atomics); a ds_write_b64 /
// ds_read_b64 pair with distinct consecutive addresses is the reference. Run
// under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS
// and compare the kernels' conflict cycles per LDS instruction.
//
//   lds_atomic_probe      (prints the kernel names; the counters come from rocprofv3)
#include <hip/hip_runtime.h>

#include <cstdio>

namespace {

constexpr int kIters = 4096;

// lane -> double index of the pattern
template <int P>
__device__ __forceinline__ int slot(int lane, int it) {
    switch (P) {
        case 0: return lane;                       // distinct, consecutive
        case 1: return 8 * 5 + (lane & 7);         // 8 replicas, one bin: 8 lanes per address
        case 2: return 2 * lane;                   // stride 2 doubles
        case 3: return 0;                          // one address
        case 4: return 16 * (lane & 31);           // stride 16 doubles: one bank pair
        case 5: return 8 * ((lane >> 3) * 4) + (lane & 7);  // 8 replicas, bins 4 apart (same mod 4)
        case 6: return 8 * ((lane >> 3) * 1) + (lane & 7);  // 8 replicas, consecutive bins
        default: return 32 * (lane & 1) + (lane >> 1);      // distinct, two halves
    }
}

template <int P>
__global__ __launch_bounds__(256) void k_atomic(double* out) {
    __shared__ double h[4][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = lane; i < 1024; i += 64) h[wv][i] = 0.0;
    __syncthreads();
    double v = 1.0 + lane;
    for (int it = 0; it < kIters; ++it) {
        atomicAdd(&h[wv][slot<P>(lane, it)], v);
        v *= 0.999;
    }
    __syncthreads();
    if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = h[0][threadIdx.x];
}

__global__ __launch_bounds__(256) void k_write_read(double* out) {
    __shared__ double h[4][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double acc = 0.0;
    for (int it = 0; it < kIters; ++it) {
        h[wv][lane] = acc + it;
        __builtin_amdgcn_wave_barrier();
        acc += h[wv][(lane + 1) & 63];
        __builtin_amdgcn_wave_barrier();
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

}  // namespace

int main() {
    double* out = nullptr;
    if (hipMalloc(&out, 1024 * 256 * sizeof(double)) != hipSuccess) return 1;
    const dim3 grid(1024), block(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_atomic<0>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<1>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<2>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<3>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<4>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<5>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<6>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_atomic<7>, grid, block, 0, 0, out);
        hipLaunchKernelGGL(k_write_read, grid, block, 0, 0, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::printf("patterns: 0 distinct | 1 8 lanes/address | 2 stride 2 | 3 one address | "
                "4 one bank pair | 5 replicas x bins 4 apart | 6 replicas x consecutive bins | "
                "7 distinct halves | write_read\n");
    (void)hipFree(out);
    return 0;
}
