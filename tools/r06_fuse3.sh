#!/bin/bash
# round 6: fused octaves 3-5 (32 x 32 tiles) as the default — GPU suite, kernels alone, driver-command A/B, big configs
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_fuse3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_FUSE=0 base SIFT_FUSE=0 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
bash tools/bench_ab.sh r06_fuse3/ab 4 base SIFT_FUSE=0 2>&1 | tee $O/ab.txt
for v in base SIFT_FUSE=0; do
  for c in config5 config3; do
    env $([ $v != base ] && echo $v) timeout -k 10 200 python3 tools/big_profile.py $c --images 12 > $O/${c}_$v.json 2> $O/${c}_$v.err || { tail -5 $O/${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${c}_$v.json')); print('$c $v', round(d['ms_per_image'],3))"
  done
done
