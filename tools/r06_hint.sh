#!/bin/bash
# round 6: export sizing from the total-records hint for one-lane jobs — GPU suite, driver bench, big legs
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_hint
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-alone --no-cpu-baseline --no-matcher > $O/b_$r.json 2> $O/b_$r.err || { tail -5 $O/b_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$r.json')); print('bench $r', round(d['ms_per_step'],4), [(c, round(d[c]['ms_per_image'],3), {k: round(v,3) for k,v in d[c]['host_phases_ms'].items() if k!='note'}) for c in ('config3','config5')])"
done
