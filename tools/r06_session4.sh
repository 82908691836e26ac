#!/bin/bash
# round 6: descriptor stride / occupancy and four keypoint lanes: alone, latency, driver-command A/B, parity
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s4
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L bs9) $(L occ3) $(L bs9o3) $(L lanes4) base $(L lanes4) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
SIFT_HIP_LIB=$A/bs9/libsift_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_bs9.log 2>&1 || { tail -30 $O/pytest_bs9.log; exit 1; }
tail -1 $O/pytest_bs9.log
SIFT_HIP_LIB=$A/lanes4/libsift_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lanes4.log 2>&1 || { tail -30 $O/pytest_lanes4.log; exit 1; }
tail -1 $O/pytest_lanes4.log
bash tools/bench_ab.sh r06_s4/ab 3 base $(L bs9) $(L bs9o3) $(L lanes4) 2>&1 | tee $O/ab.txt
