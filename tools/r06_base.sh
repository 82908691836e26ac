#!/bin/bash
# round 6 (session 2): state of the tree after the re-entry — smoke, GPU suite, driver bench, kernels alone
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_base
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['summary']))"
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_FLOW=1 base SIFT_FLOW=1 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt
