#!/bin/bash
set -o pipefail
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 900 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_KP_WGS=128 SIFT_KP_WGS=96 \
    SIFT_KP_WGS=64 SIFT_KP_WGS=128,SIFT_DESC_WGS=256 SIFT_KP_WGS=96,SIFT_DESC_WGS=256 \
    SIFT_KP_WGS=96,SIFT_DESC_WGS=192 SIFT_KP_WGS=64,SIFT_DESC_WGS=192 \
    > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
