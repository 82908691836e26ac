#!/bin/bash
# round 6 final tree (LDS-DMA pair walk for planes >= 2^24 px): kernels alone, smoke, GPU suite,
# the driver's command twice, serial / pipelined rocprof, configs 3 / 5 traces
set -o pipefail
R=$(pwd)
O=gpurun_out/r06_final4
mkdir -p $O
timeout -k 10 400 python3 tools/kernel_alone.py --n 150 base 2>&1 | grep -v amdgpu.ids | tee $O/kalone.txt || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_session.sh r06_final4 test || exit 1
for r in 1 2; do
  timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$r.json')); print(json.dumps(d['summary']))"
done
bash tools/gpu_session.sh r06_final4 prof big || exit 1
