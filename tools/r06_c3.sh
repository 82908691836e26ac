#!/bin/bash
# round 6: config 3 leg as the first GPU process of a call (job log), then bench's big legs twice
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_c3
mkdir -p $O
timeout -k 10 200 python3 tools/big_profile.py config3 --images 16 > $O/c3_first.json 2> $O/c3_first.err || { tail -5 $O/c3_first.err; exit 1; }
python3 - $O/c3_first.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("big_profile config3 first", round(d["ms_per_image"], 3))
for e in d["log"]:
    if "done_ms" in e:
        h = e["host"]
        print(f"  job {e['job']:2d} fetch {e['fetch_ms']:7.2f} done {e['done_ms']:7.2f} " + " ".join(f"{k} {v:.2f}" for k, v in h.items() if isinstance(v, (int, float))))
PY
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-alone --no-cpu-baseline --no-matcher > $O/b_$r.json 2> $O/b_$r.err || { tail -5 $O/b_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$r.json')); print('bench $r', round(d['ms_per_step'],4), [(c, round(d[c]['ms_per_image'],3), round(d[c]['host_phases_ms']['blocked'],2)) for c in ('config3','config5')])"
done
