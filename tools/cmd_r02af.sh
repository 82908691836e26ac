set -o pipefail
O=gpurun_out/r02af
mkdir -p $O
L=sift-project_amd/alt
VARIANTS="base SIFT_HIP_LIB=$L/gen600/libsift_hip.so SIFT_HIP_LIB=$L/genall/libsift_hip.so" REPS=1 AB_OUT=r02af/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
