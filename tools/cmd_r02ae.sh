set -o pipefail
O=gpurun_out/r02ae
mkdir -p $O
VARIANTS="base SIFT_LDS_PX=2100 SIFT_LDS_PX=600 SIFT_LDS_PX=150" REPS=1 AB_OUT=r02ae/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
