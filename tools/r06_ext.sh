#!/bin/bash
# round 6: extrema segment height (waves per octave-0 launch vs resident capacity: 136 VGPRs -> 3 waves per SIMD, 3072 resident)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_ext
mkdir -p $O
timeout -k 10 600 python3 tools/kernel_alone.py --n 100 base SIFT_EXT_SEG=46 SIFT_EXT_SEG=48 SIFT_EXT_SEG=64 SIFT_EXT_SEG=24 SIFT_EXT_SEG=40 base SIFT_EXT_SEG=46 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base SIFT_EXT_SEG=46 SIFT_EXT_SEG=64 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
bash tools/bench_ab.sh r06_ext/ab 3 base SIFT_EXT_SEG=46 SIFT_EXT_SEG=64 2>&1 | tee $O/ab.txt
