#!/bin/bash
# round 6: descriptor shared grid 512 per image (and orientation 256) against the defaults, 5 rounds
set -o pipefail
bash tools/bench_ab.sh r06_wgs2/ab 5 base SIFT_DESC_WGS=512 SIFT_DESC_WGS=512,SIFT_KP_WGS=256 2>&1 | tee gpurun_out/r06_wgs2_ab.txt
