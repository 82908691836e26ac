set -o pipefail
O=gpurun_out/r02ad
mkdir -p $O
VARIANTS="base SIFT_BLUR_COLS=1 SIFT_BLUR_ROWS=16 SIFT_BLUR_COLS=1,SIFT_BLUR_ROWS=16 SIFT_BLUR_ROWS=64" REPS=1 AB_OUT=r02ad/ab_alone.txt BENCH_ARGS="--steps 600 --warmup 20" tools/ab_alone.sh || exit 1
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_BLUR_COLS=1 SIFT_BLUR_ROWS=16 2>&1 | tee $O/ab1.txt || exit 1
