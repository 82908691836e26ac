// fp64_latency.hip — dependent-chain cycles of the FP64 VALU ops the blur
// chains use (acc += k*(a+b) under -ffp-contract=off: v_add_f64, v_mul_f64),
// one wave alone and several per SIMD, measured with s_memtime around
// unrolled chains. Test tooling only.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int CHAINS>
__global__ void k_chain(double* out, unsigned long long* cyc, double a, double b, int iters) {
    double acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = a + threadIdx.x + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) acc[c] = acc[c] * b + b;  // mul then add: 2 deps
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
void run(int waves_per_block, int blocks) {
    double* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, sizeof(double) * 64 * waves_per_block * blocks);
    (void)hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
    const int iters = 256;
    hipLaunchKernelGGL(k_chain<CHAINS>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc,
                       1.0, 0.999999, iters);
    hipLaunchKernelGGL(k_chain<CHAINS>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc,
                       1.0, 0.999999, iters);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const double ops = 2.0 * 16 * iters;  // dependent ops per chain
    std::printf("chains/wave %2d, waves/block %2d: %.2f cycles per dependent op of a chain, "
                "%.2f cycles per wave-instruction issued by the block\n",
                CHAINS, waves_per_block, c / ops, c / (ops * CHAINS * waves_per_block));
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    run<1>(1, 1);
    run<2>(1, 1);
    run<4>(1, 1);
    run<8>(1, 1);
    run<1>(4, 1);   // one wave per SIMD
    run<1>(8, 1);   // two per SIMD
    run<1>(16, 1);  // four per SIMD
    run<4>(4, 1);
    run<4>(8, 1);
    return 0;
}
