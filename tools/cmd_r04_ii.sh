#!/bin/bash
# k_blur stores / line hand-off variants: parity of each variant library on the
# golden and stage-wise tests, then kernel-alone times and the 20-step bench
set -o pipefail
O=gpurun_out/r04_ii
mkdir -p $O
L=sift-project_amd/alt
for v in st sy; do
  SIFT_HIP_LIB=$L/$v/libsift_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 200 --timeout-method thread -k "reference_golden or stagewise or pyramid_paths or big_golden" \
      > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$L/st/libsift_hip.so \
    SIFT_HIP_LIB=$L/sy/libsift_hip.so base SIFT_HIP_LIB=$L/sy/libsift_hip.so \
    > $O/kernel_alone.txt 2> $O/kernel_alone.err || { tail -20 $O/kernel_alone.err; exit 1; }
cat $O/kernel_alone.txt
bash tools/bench_ab.sh r04_ii/ab 4 base SIFT_HIP_LIB=$L/st/libsift_hip.so SIFT_HIP_LIB=$L/sy/libsift_hip.so || exit 1
