set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/t3.log 2>&1; tail -2 gpurun_out/t3.log; grep -q "failed\|error" gpurun_out/t3.log && exit 1
SIFT_SERIAL=1 tools/gpu_prof.sh r02f "--steps 60 --warmup 5 --sync" || exit 1
SWEEP="base SIFT_EXTREMA_TILES=1" REPS=3 SWEEP_OUT=sw_ext.txt tools/sweep.sh | grep mean
SWEEP="base SIFT_EXTREMA_TILES=1" REPS=2 SWEEP_OUT=sw_ext8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean
