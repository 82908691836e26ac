#!/bin/bash
# Round-2 GPU session: parity suite, bench, rocprofv3 kernel trace of the
# pipelined bench. Usage (repo root on the GPU box): tools/gpu_r02.sh <tag>
set -o pipefail
R=$(pwd)
T=${1:-r02}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not slow" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-extra --no-matcher > $R/$O/bench_prof.log 2>&1 || exit 1
echo DONE
