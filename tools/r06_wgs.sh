#!/bin/bash
# round 6: shared-grid keypoint workgroups per image (orientation 192, descriptor 384) on the driver's command
set -o pipefail
bash tools/bench_ab.sh r06_wgs/ab 3 base SIFT_KP_WGS=256 SIFT_KP_WGS=128 SIFT_DESC_WGS=512 SIFT_DESC_WGS=256 2>&1 | tee gpurun_out/r06_wgs_ab.txt
