#!/bin/bash
# k_blur prefetch depth after the guarded-store change (PF 2 default vs 3, 4):
# parity of the variant libraries, kernels alone, the 20-step bench
set -o pipefail
O=gpurun_out/r04_kk
mkdir -p $O
L=sift-project_amd/alt
for v in pf3 pf4; do
  SIFT_HIP_LIB=$L/$v/libsift_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 200 --timeout-method thread -k "reference_golden or stagewise or pyramid_paths" \
      > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/pytest_$v.log)"
done
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$L/pf3/libsift_hip.so \
    SIFT_HIP_LIB=$L/pf4/libsift_hip.so base SIFT_HIP_LIB=$L/pf3/libsift_hip.so SIFT_HIP_LIB=$L/pf4/libsift_hip.so \
    > $O/kernel_alone.txt 2> $O/kernel_alone.err || { tail -20 $O/kernel_alone.err; exit 1; }
grep -v amdgpu.ids $O/kernel_alone.txt
bash tools/bench_ab.sh r04_kk/ab 4 base SIFT_HIP_LIB=$L/pf3/libsift_hip.so SIFT_HIP_LIB=$L/pf4/libsift_hip.so || exit 1
