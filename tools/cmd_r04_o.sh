#!/bin/bash
# extrema task shape, round 2: 20-step bench + kernel-alone
set -o pipefail
mkdir -p gpurun_out/r04_o
bash tools/bench_ab.sh r04_o/ab 4 SIFT_EXT_WAVES=512 SIFT_EXT_WAVES=512,SIFT_EXT_SEGMAX=32 SIFT_EXT_WAVES=1024,SIFT_EXT_SEGMAX=32 SIFT_EXT_WAVES=256,SIFT_EXT_SEGMAX=32 || exit 1
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 SIFT_EXT_WAVES=512,SIFT_EXT_SEGMAX=32 SIFT_EXT_WAVES=256,SIFT_EXT_SEGMAX=32 \
    > gpurun_out/r04_o/ka.txt 2>&1 || { tail -5 gpurun_out/r04_o/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_o/ka.txt
