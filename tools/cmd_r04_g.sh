#!/bin/bash
set -o pipefail
O=gpurun_out/r04_g2
mkdir -p $O
A=sift-project_amd/alt
timeout -k 10 300 python -u tools/kernel_alone.py --n 40 base SIFT_HIP_LIB=$A/epf3/libsift_hip.so \
    SIFT_HIP_LIB=$A/epf4/libsift_hip.so SIFT_KP_WGS=384 SIFT_KP_WGS=128 \
    > $O/alone.txt 2>&1 || { tail -20 $O/alone.txt; exit 1; }
grep -v amdgpu.ids $O/alone.txt
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_HIP_LIB=$A/epf3/libsift_hip.so \
    SIFT_HIP_LIB=$A/epf4/libsift_hip.so SIFT_KP_WGS=384 SIFT_KP_WGS=128 \
    > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
