#!/bin/bash
# round 6: descriptor work counters in partitions (SIFT_DESC_PARTS) — parity, alone (1080p, 8K), A/B, big configs
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_parts
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L parts1) $(L parts16) base $(L parts1) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L parts1) $(L parts16) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
bash tools/bench_ab.sh r06_parts/ab 3 base $(L parts1) 2>&1 | tee $O/ab.txt
for v in base parts1; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib timeout -k 10 200 python3 tools/big_profile.py config5 --images 12 > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('config5 $v', round(d['ms_per_image'],3))"
done
