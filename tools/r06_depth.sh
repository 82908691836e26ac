#!/bin/bash
# round 6: jobs in flight — the driver's command at depth 3 / 4 / 5 / 6; configs 3 / 5 at 2 / 3 / 4
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_depth
mkdir -p $O
bash tools/bench_ab.sh r06_depth/ab 3 base SIFT_JOB_DEPTH=3 SIFT_JOB_DEPTH=5 SIFT_JOB_DEPTH=6 2>&1 | tee $O/ab.txt
for c in config5 config3; do
  for d in 2 3 4; do
    timeout -k 10 200 python3 tools/big_profile.py $c --images 12 --depth $d > $O/${c}_d$d.json 2> $O/${c}_d$d.err || { tail -5 $O/${c}_d$d.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${c}_d$d.json')); print('$c depth $d', round(d['ms_per_image'],3))"
  done
done
