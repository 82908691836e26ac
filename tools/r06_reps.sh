#!/bin/bash
# round 6: descriptor with 4 histogram replicas per wave (bin stride 4 / 5) against 8 (stride 9, default; 8 for reference)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_reps
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L r4s4) $(L r4s5) $(L r8s8) base $(L r4s4) $(L r4s5) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L r4s5) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
