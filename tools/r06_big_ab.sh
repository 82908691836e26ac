#!/bin/bash
# round 6: config 5 / config 3 pipelined legs per library variant (alternating)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_bigab
mkdir -p $O
A=$R/sift-project_amd/alt
for r in 1 2; do
  for v in base lanes2; do
    lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
    for c in config5 config3; do
      SIFT_HIP_LIB=$lib timeout -k 10 200 python3 tools/big_profile.py $c --images 12 > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || { tail -5 $O/${c}_${v}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${c}_${v}_$r.json')); print('$c $v $r', round(d['ms_per_image'],3))"
    done
  done
done
bash tools/bench_ab.sh r06_bigab/ab 3 base SIFT_HIP_LIB=$A/lanes2/libsift_hip.so
timeout -k 10 300 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=$A/lanes2/libsift_hip.so base SIFT_HIP_LIB=$A/lanes2/libsift_hip.so 2>&1 | grep -v amdgpu.ids
