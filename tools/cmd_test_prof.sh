# GPU: parity suite (fast subset) then a serialized kernel profile (r02x)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/t_tp.log 2>&1; tail -2 gpurun_out/t_tp.log; grep -q "failed\|error" gpurun_out/t_tp.log && exit 1
SIFT_SERIAL=1 tools/gpu_prof.sh r02x "--steps 60 --warmup 5 --sync" || exit 1
SWEEP="base" REPS=3 SWEEP_OUT=sw_x.txt tools/sweep.sh | grep mean
