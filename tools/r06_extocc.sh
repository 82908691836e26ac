#!/bin/bash
# round 6: extrema resident workgroups per CU capped by dynamic LDS (pad48: 2 per CU = 2 waves per SIMD; pad32: 3, as the VGPRs allow)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_extocc
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L pad48) $(L pad32) base $(L pad48) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L pad48) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
bash tools/bench_ab.sh r06_extocc/ab 3 base $(L pad48) 2>&1 | tee $O/ab.txt
