#!/bin/bash
# claim counter groups (8 default) vs 1 / 4 / 16: parity, kernel-alone, 20-step bench
set -o pipefail
mkdir -p gpurun_out/r04_u
A=sift-project_amd/alt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_u/pytest.log 2>&1 || { tail -30 gpurun_out/r04_u/pytest.log; exit 1; }
tail -1 gpurun_out/r04_u/pytest.log
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$A/g1/libsift_hip.so \
    SIFT_HIP_LIB=$A/g4/libsift_hip.so SIFT_HIP_LIB=$A/g16/libsift_hip.so \
    > gpurun_out/r04_u/ka.txt 2>&1 || { tail -5 gpurun_out/r04_u/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_u/ka.txt
bash tools/bench_ab.sh r04_u/ab 4 base SIFT_HIP_LIB=$A/g1/libsift_hip.so SIFT_HIP_LIB=$A/g16/libsift_hip.so || exit 1
