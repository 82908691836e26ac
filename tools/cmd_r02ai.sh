set -o pipefail
O=gpurun_out/r02ai
mkdir -p $O
VARIANTS="base SIFT_EXT_WAVES=3072 SIFT_EXT_WAVES=2048 SIFT_EXT_WAVES=1536" REPS=1 AB_OUT=r02ai/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_EXT_WAVES=3072 SIFT_EXT_WAVES=2048 2>&1 | tee $O/ab1.txt || exit 1
