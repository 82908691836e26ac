#!/bin/bash
# round 6: the driver's command three times on one box (the big legs now run with the 1080p context closed)
set -o pipefail
R=$(pwd)
O=gpurun_out/${OUT:-r06_final3}
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$r.json')); print(json.dumps(d['summary']))"
done
