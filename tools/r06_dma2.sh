#!/bin/bash
# round 6: LDS-DMA pair walk on planes >= 16.7 Mpx again (configs 3 / 5 only), now with 4 big jobs in flight and the export fix
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_dma2
mkdir -p $O
A=$R/sift-project_amd/alt
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base SIFT_HIP_LIB=$A/dma4/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config3 --n 3 base SIFT_HIP_LIB=$A/dma4/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone_c3.txt || exit 1
for r in 1 2; do
  for v in base dma4; do
    lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
    for c in config5 config3; do
      SIFT_HIP_LIB=$lib timeout -k 10 200 python3 tools/big_profile.py $c --images 12 > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || { tail -5 $O/${c}_${v}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${c}_${v}_$r.json')); print('$c $v $r', round(d['ms_per_image'],3))"
    done
  done
done
