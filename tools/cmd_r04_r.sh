#!/bin/bash
# orientation: static striding vs first-static-then-claims
set -o pipefail
mkdir -p gpurun_out/r04_r
S=sift-project_amd/alt/oristatic/libsift_hip.so
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$S \
    > gpurun_out/r04_r/ka.txt 2>&1 || { tail -5 gpurun_out/r04_r/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_r/ka.txt
bash tools/bench_ab.sh r04_r/ab 5 base SIFT_HIP_LIB=$S || exit 1
