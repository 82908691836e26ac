#!/bin/bash
# A/B of the driver's bench command itself: each variant is a separate
# process (its own HIP queue mapping, like the driver's run), runs
# alternate variant by variant, `n` rounds; prints ms_per_step per run and
# the per-variant median. Variants: "base" or VAR=value[,VAR=value...]
# (SIFT_HIP_LIB=... selects an alternative library build).
#   tools/bench_ab.sh <out dir under gpurun_out> <rounds> VARIANT...
set -o pipefail
O=gpurun_out/${1:?out}
N=${2:?rounds}
shift 2
mkdir -p $O
for r in $(seq 1 $N); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=""
    [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    env $envs timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        --no-matcher --no-alone --no-big --no-extra > $O/v${i}_r$r.json 2> $O/v${i}_r$r.err \
        || { tail -5 $O/v${i}_r$r.err; exit 1; }
  done
done
python3 - "$O" "$N" "$@" <<'EOF'
import json, statistics, sys
o, n, vs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
base = None
for i, v in enumerate(vs, 1):
    ms = [json.load(open(f"{o}/v{i}_r{r}.json"))["ms_per_step"] for r in range(1, n + 1)]
    med = statistics.median(ms)
    base = base or med
    print(f"{v:60s} median {med:.4f} ms/step  ({med / base:.3f})  runs " +
          " ".join(f"{m:.3f}" for m in ms))
EOF
