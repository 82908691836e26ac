#!/bin/bash
# round 6 final tree (export hint fix, 4 big jobs in flight): smoke, GPU suite, the driver's command x2, big legs
set -o pipefail
R=$(pwd)
O=gpurun_out/r06_final2
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$r.json')); print(json.dumps(d['summary']))"
done
