#!/bin/bash
# round 6: descriptor bin stride 9 combined with the replica swizzles (SIFT_DESC_SWZ 1 / 2 / 3)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_swz9
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L s9w1) $(L s9w2) $(L s9w3) base $(L s9w1) $(L s9w2) $(L s9w3) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
