#!/bin/bash
# extrema waves per octave: kernel-alone + 20-step bench
set -o pipefail
mkdir -p gpurun_out/r04_m
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_EXT_WAVES=2048 SIFT_EXT_WAVES=1024 SIFT_EXT_WAVES=512 \
    > gpurun_out/r04_m/ka.txt 2>&1 || { tail -5 gpurun_out/r04_m/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_m/ka.txt
bash tools/bench_ab.sh r04_m/ab 4 base SIFT_EXT_WAVES=1024 SIFT_EXT_WAVES=512 || exit 1
