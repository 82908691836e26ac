#!/bin/bash
# round-4 first GPU session: f64 math check, the whole GPU suite, descriptor A/B
set -o pipefail
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 120 tools/math64_check 4194304 > $O/math64.txt 2>&1 || { cat $O/math64.txt; exit 1; }
cat $O/math64.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_DESC_MODE=1 SIFT_DESC_MODE=2 \
    > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 4 --steps 100 --depth 1 base SIFT_DESC_MODE=1 \
    > $O/ab_sync.txt 2>&1 || { tail -20 $O/ab_sync.txt; exit 1; }
grep -v amdgpu.ids $O/ab_sync.txt
