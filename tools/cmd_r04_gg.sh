#!/bin/bash
# single-image shared jobs take octave 5 into k_octaves_lds: parity + 20-step bench
set -o pipefail
O=gpurun_out/r04_gg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/bench_ab.sh r04_gg/ab 5 base SIFT_LDS_PX_SHARED=2100 || exit 1
