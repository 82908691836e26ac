#!/bin/bash
# k_octaves_lds with global-address-space plane pointers (global stores, not
# FLAT): parity of the variant library, kernels alone, the 20-step bench
set -o pipefail
O=gpurun_out/r04_jj
mkdir -p $O
L=sift-project_amd/alt
SIFT_HIP_LIB=$L/lg/libsift_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 200 --timeout-method thread -k "reference_golden or stagewise or pyramid_paths or big_golden" \
    > $O/pytest_lg.log 2>&1 || { tail -30 $O/pytest_lg.log; exit 1; }
echo "lg: $(tail -n 1 $O/pytest_lg.log)"
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=$L/lg/libsift_hip.so \
    base SIFT_HIP_LIB=$L/lg/libsift_hip.so > $O/kernel_alone.txt 2> $O/kernel_alone.err \
    || { tail -20 $O/kernel_alone.err; exit 1; }
grep -v amdgpu.ids $O/kernel_alone.txt
bash tools/bench_ab.sh r04_jj/ab 5 base SIFT_HIP_LIB=$L/lg/libsift_hip.so || exit 1
