set -o pipefail
mkdir -p gpurun_out/r02j
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02j/t.log 2>&1 || { tail -30 gpurun_out/r02j/t.log; exit 1; }
tail -2 gpurun_out/r02j/t.log
SWEEP="base SIFT_JOB_DEPTH=4 SIFT_JOB_DEPTH=6 SIFT_JOB_DEPTH=4,GPU_MAX_HW_QUEUES=8 SIFT_JOB_DEPTH=8,GPU_MAX_HW_QUEUES=8" REPS=2 SWEEP_OUT=r02j/sw1.txt tools/sweep.sh | grep mean || exit 1
SWEEP="base SIFT_JOB_DEPTH=4" REPS=1 SWEEP_OUT=r02j/sw8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean || exit 1
