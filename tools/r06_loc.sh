#!/bin/bash
# round 6: descriptor sample location by ballots + readlane (no ds_bpermute binary search) — parity, alone (1080p, 8K), A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_loc
mkdir -p $O
A=$R/sift-project_amd/alt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=$A/bsearch/libsift_hip.so base SIFT_HIP_LIB=$A/bsearch/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 4 base SIFT_HIP_LIB=$A/bsearch/libsift_hip.so base 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
bash tools/bench_ab.sh r06_loc/ab 3 base SIFT_HIP_LIB=$A/bsearch/libsift_hip.so 2>&1 | tee $O/ab.txt
