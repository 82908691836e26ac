set -o pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -v --timeout 120 --timeout-method thread -k "not slow" > gpurun_out/r02h/t.log 2>&1 || { tail -30 gpurun_out/r02h/t.log; exit 1; }
tail -2 gpurun_out/r02h/t.log
SWEEP="base SIFT_FUSED_PX_LOG2=0 SIFT_FUSED_PX_LOG2=22" REPS=2 SWEEP_OUT=r02h/sw1.txt tools/sweep.sh | grep mean || exit 1
SWEEP="base SIFT_FUSED_PX_LOG2=0" REPS=2 SWEEP_OUT=r02h/sw8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean || exit 1
SIFT_SERIAL=1 tools/gpu_prof.sh r02h_serial "--steps 60 --warmup 5 --sync" || exit 1
