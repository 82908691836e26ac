#!/bin/bash
# extrema scan v2 (pair-of-rows window, scalar-base loads, incremental cube
# test) at 3 and 4 waves/SIMD: parity on the goldens, kernel-alone, 20-step bench
set -o pipefail
mkdir -p gpurun_out/r04_w
A=sift-project_amd/alt
for v in v2 v2o4; do
  SIFT_HIP_LIB=$A/$v/libsift_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > gpurun_out/r04_w/pytest_$v.log 2>&1 || { tail -30 gpurun_out/r04_w/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r04_w/pytest_$v.log
done
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$A/v2/libsift_hip.so SIFT_HIP_LIB=$A/v2o4/libsift_hip.so \
    > gpurun_out/r04_w/ka.txt 2>&1 || { tail -5 gpurun_out/r04_w/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_w/ka.txt
bash tools/bench_ab.sh r04_w/ab 4 base SIFT_HIP_LIB=$A/v2/libsift_hip.so SIFT_HIP_LIB=$A/v2o4/libsift_hip.so || exit 1
