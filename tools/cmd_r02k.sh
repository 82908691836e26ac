set -o pipefail
mkdir -p gpurun_out/r02k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not slow" > gpurun_out/r02k/t.log 2>&1 || { tail -30 gpurun_out/r02k/t.log; exit 1; }
tail -2 gpurun_out/r02k/t.log
SWEEP="SIFT_JOB_DEPTH=2 SIFT_JOB_DEPTH=3 base SIFT_JOB_DEPTH=5 SIFT_JOB_DEPTH=6" REPS=2 SWEEP_OUT=r02k/sw1.txt tools/sweep.sh | grep mean || exit 1
