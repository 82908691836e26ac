#!/bin/bash
# extrema task shape (waves per octave, rows per task): kernel-alone + 20-step bench
set -o pipefail
mkdir -p gpurun_out/r04_n
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 SIFT_EXT_WAVES=512 SIFT_EXT_WAVES=256,SIFT_EXT_SEGMAX=128 \
    SIFT_EXT_WAVES=128,SIFT_EXT_SEGMAX=256 SIFT_EXT_WAVES=512,SIFT_EXT_SEGMAX=128 SIFT_EXT_WAVES=1024,SIFT_EXT_SEGMAX=32 \
    > gpurun_out/r04_n/ka.txt 2>&1 || { tail -5 gpurun_out/r04_n/ka.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_n/ka.txt
bash tools/bench_ab.sh r04_n/ab 4 SIFT_EXT_WAVES=512 SIFT_EXT_WAVES=256,SIFT_EXT_SEGMAX=128 SIFT_EXT_WAVES=128,SIFT_EXT_SEGMAX=256 || exit 1
