#!/bin/bash
# round 6: descriptor occupancy x gradient prefetch depth (OCC 3 leaves 168 VGPRs: AHEAD 2 without spills)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_occ
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L o3a2) $(L o4a2) $(L o3a1) base $(L o3a2) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L o3a2) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
