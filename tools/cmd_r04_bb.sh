#!/bin/bash
# chain snapshots without the extrema done counter: parity,
# kernel-alone, 20-step bench against the previous build
set -o pipefail
mkdir -p gpurun_out/r04_bb
P=sift-project_amd/alt/prev/libsift_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_bb/pytest.log 2>&1 || { tail -30 gpurun_out/r04_bb/pytest.log; exit 1; }
tail -1 gpurun_out/r04_bb/pytest.log
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$P \
    > gpurun_out/r04_bb/ka.txt 2>&1 || { tail -5 gpurun_out/r04_bb/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_bb/ka.txt
bash tools/bench_ab.sh r04_bb/ab 4 base SIFT_HIP_LIB=$P || exit 1
