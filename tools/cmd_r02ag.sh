set -o pipefail
O=gpurun_out/r02ag
mkdir -p $O
L=sift-project_amd/alt
VARIANTS="base SIFT_HIP_LIB=$L/gen150/libsift_hip.so SIFT_HIP_LIB=$L/gen600/libsift_hip.so SIFT_HIP_LIB=$L/gen2100/libsift_hip.so" REPS=1 AB_OUT=r02ag/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_HIP_LIB=$L/gen600/libsift_hip.so SIFT_HIP_LIB=$L/gen2100/libsift_hip.so 2>&1 | tee $O/ab1.txt || exit 1
