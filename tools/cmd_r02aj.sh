set -o pipefail
O=gpurun_out/r02aj
mkdir -p $O
VARIANTS="SIFT_EXT_WAVES=1536 SIFT_EXT_WAVES=1024 SIFT_EXT_WAVES=768" REPS=1 AB_OUT=r02aj/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_EXT_WAVES=1536 SIFT_EXT_WAVES=1024 2>&1 | tee $O/ab1.txt || exit 1
