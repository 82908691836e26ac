#!/bin/bash
# GPU session script (run from the repo root on the GPU box)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not slow" 2>&1 | tee gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | tee gpurun_out/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1 || exit 1
echo DONE
