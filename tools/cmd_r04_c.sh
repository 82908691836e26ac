#!/bin/bash
set -o pipefail
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "descriptor or deterministic or big or reference_golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/kernel_alone.py --n 40 base SIFT_DESC_WGS=512 SIFT_DESC_MODE=3 SIFT_DESC_MODE=1 \
    > $O/alone.txt 2>&1 || { tail -20 $O/alone.txt; exit 1; }
grep -v amdgpu.ids $O/alone.txt
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_DESC_WGS=512 SIFT_DESC_WGS=256 \
    SIFT_DESC_MODE=3 SIFT_DESC_MODE=1 SIFT_LDS_PX=9088 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
