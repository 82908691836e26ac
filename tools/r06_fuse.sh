#!/bin/bash
# round 6: k_octave_fused (one launch per level group of a mid-sized octave) — parity first, then alone / latency / driver-command A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_fuse2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fused" > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -3 $O/pytest_fused.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_FUSE=1 SIFT_FUSE=1,SIFT_FUSE_T32_PX=4194304 SIFT_FUSE=1,SIFT_FUSE_PX=131072 SIFT_FUSE=1,SIFT_FUSE_T32_PX=0 base SIFT_FUSE=1 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
bash tools/bench_ab.sh r06_fuse2/ab 3 base SIFT_FUSE=1 SIFT_FUSE=1,SIFT_FUSE_PX=131072 2>&1 | tee $O/ab.txt
