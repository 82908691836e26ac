#!/bin/bash
# round 6: k_octaves_flow (small octaves in flight): parity first, then alone / latency / driver-command A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "flow" > $O/pytest_flow.log 2>&1 || { tail -40 $O/pytest_flow.log; exit 1; }
tail -3 $O/pytest_flow.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_FLOW=0 SIFT_FLOW_WGS=64 SIFT_FLOW_WGS=256 base SIFT_FLOW=0 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
bash tools/bench_ab.sh r06_s6/ab 3 base SIFT_FLOW=0 2>&1 | tee $O/ab.txt
