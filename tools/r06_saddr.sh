#!/bin/bash
# round 6: extrema loads with scalar level bases + 32-bit vector offsets (126 instead of 136 VGPRs: 4 waves per SIMD) — parity, alone, A/B
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_saddr
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L extold) base $(L extold) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L extold) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config3 --n 3 base $(L extold) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c3.txt || exit 1
bash tools/bench_ab.sh r06_saddr/ab 4 base $(L extold) 2>&1 | tee $O/ab.txt
