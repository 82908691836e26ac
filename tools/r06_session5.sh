#!/bin/bash
# round 6: descriptor bin strides, four keypoint lanes (fixed counts): alone, parity, driver-command A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s5
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L bs9) $(L bs10) $(L bs11) $(L bs9p) $(L bs9s3) base $(L bs9) $(L bs10) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
SIFT_HIP_LIB=$A/lanes4/libsift_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lanes4.log 2>&1 || { tail -30 $O/pytest_lanes4.log; exit 1; }
tail -1 $O/pytest_lanes4.log
bash tools/bench_ab.sh r06_s5/ab 3 base $(L bs9) $(L bs10) $(L lanes4) 2>&1 | tee $O/ab.txt
