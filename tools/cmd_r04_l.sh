#!/bin/bash
# strip rows per radius for the octave-0 strip walk: kernel-alone + 20-step bench
set -o pipefail
mkdir -p gpurun_out/r04_l
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_BLUR_ROWS_R8=48 SIFT_BLUR_ROWS_R8=64 \
    SIFT_BLUR_ROWS_R8=24 SIFT_BLUR_ROWS_R6=48 SIFT_BLUR_ROWS_R8=64,SIFT_BLUR_ROWS_R6=48 \
    > gpurun_out/r04_l/ka.txt 2>&1 || { tail -5 gpurun_out/r04_l/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_l/ka.txt
bash tools/bench_ab.sh r04_l/ab 3 base SIFT_BLUR_ROWS_R8=48 SIFT_BLUR_ROWS_R8=64 || exit 1
