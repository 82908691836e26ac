#!/bin/bash
set -o pipefail
O=gpurun_out/r04_i
mkdir -p $O
bash tools/bench_ab.sh r04_i/ab20 5 base SIFT_LEAD_ALONE=1 || exit 1
for v in base SIFT_LEAD_ALONE=1; do
  envs=""; [ "$v" != base ] && envs=$v
  env $envs timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher \
    --no-alone --no-extra --no-big --step-log > $O/steplog_$v.json 2> $O/steplog_$v.err || { tail -20 $O/steplog_$v.err; exit 1; }
  echo $v; grep "done" $O/steplog_$v.err | awk '{print $3, $4}' | tr '\n' ' '; echo
done
