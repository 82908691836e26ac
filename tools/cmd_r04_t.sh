#!/bin/bash
# static keypoint / record assignment (no work-counter atomics): parity,
# kernel-alone, 20-step bench against the previous build
set -o pipefail
mkdir -p gpurun_out/r04_t
P=sift-project_amd/alt/prev/libsift_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_t/pytest.log 2>&1 || { tail -30 gpurun_out/r04_t/pytest.log; exit 1; }
tail -1 gpurun_out/r04_t/pytest.log
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$P \
    > gpurun_out/r04_t/ka.txt 2>&1 || { tail -5 gpurun_out/r04_t/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_t/ka.txt
bash tools/bench_ab.sh r04_t/ab 4 base SIFT_HIP_LIB=$P || exit 1
