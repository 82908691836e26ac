set -o pipefail
mkdir -p gpurun_out/r02l
SWEEP="base GPU_MAX_HW_QUEUES=8 SIFT_JOB_DEPTH=6,GPU_MAX_HW_QUEUES=8 SIFT_JOB_DEPTH=8,GPU_MAX_HW_QUEUES=8" REPS=2 SWEEP_OUT=r02l/sw1.txt tools/sweep.sh | grep mean || exit 1
