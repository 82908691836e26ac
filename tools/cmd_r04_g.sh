#!/bin/bash
set -o pipefail
O=gpurun_out/r04_g
mkdir -p $O
A=sift-project_amd/alt
timeout -k 10 300 python -u tools/kernel_alone.py --n 40 base SIFT_HIP_LIB=$A/pf1/libsift_hip.so \
    SIFT_HIP_LIB=$A/pf4/libsift_hip.so SIFT_HIP_LIB=$A/rows16/libsift_hip.so SIFT_HIP_LIB=$A/c1/libsift_hip.so \
    > $O/alone.txt 2>&1 || { tail -20 $O/alone.txt; exit 1; }
grep -v amdgpu.ids $O/alone.txt
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_HIP_LIB=$A/pf1/libsift_hip.so \
    SIFT_HIP_LIB=$A/pf4/libsift_hip.so SIFT_HIP_LIB=$A/rows16/libsift_hip.so SIFT_HIP_LIB=$A/c1/libsift_hip.so \
    > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
