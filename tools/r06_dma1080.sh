#!/bin/bash
# round 6: the LDS-DMA pair walk on 1080p's octave 0 too (threshold 2^22 px): kernels alone, latency, the driver's command
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_dma1080
mkdir -p $O
A=$R/sift-project_amd/alt
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=$A/dma22/libsift_hip.so base SIFT_HIP_LIB=$A/dma22/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
bash tools/bench_ab.sh r06_dma1080/ab 4 base SIFT_HIP_LIB=$A/dma22/libsift_hip.so 2>&1 | tee $O/ab.txt
