set -o pipefail
mkdir -p gpurun_out/r02n
SWEEP="base SIFT_BLUR_ROWS=48 SIFT_BLUR_ROWS=64 SIFT_BLUR_ROWS=96" REPS=2 SWEEP_OUT=r02n/sw1.txt tools/sweep.sh | grep mean || exit 1
SWEEP="base SIFT_BLUR_ROWS=64" REPS=1 SWEEP_OUT=r02n/sw8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean || exit 1
