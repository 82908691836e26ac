#!/bin/bash
set -o pipefail
O=gpurun_out/r04_f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/bench_ab.sh r04_f/ab20 5 base SIFT_PYR_CHAIN=0 || exit 1
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_PYR_CHAIN=0 \
    > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher \
    --no-alone --no-extra --no-big --step-log > $O/steplog.json 2> $O/steplog.err || { tail -20 $O/steplog.err; exit 1; }
grep -A30 "step log" $O/steplog.err | head -30
