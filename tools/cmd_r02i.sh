set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not slow" > gpurun_out/r02i/t.log 2>&1 || { tail -30 gpurun_out/r02i/t.log; exit 1; }
tail -2 gpurun_out/r02i/t.log
SWEEP="base SIFT_LDS_PX=2100 SIFT_LDS_PX=600 SIFT_LDS_PX=0" REPS=2 SWEEP_OUT=r02i/sw1.txt tools/sweep.sh | grep mean || exit 1
SWEEP="base SIFT_LDS_PX=2100" REPS=2 SWEEP_OUT=r02i/sw8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean || exit 1
SIFT_SERIAL=1 tools/gpu_prof.sh r02i_serial "--steps 60 --warmup 5 --sync" || exit 1
