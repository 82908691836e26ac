#!/bin/bash
# Bench sweep over tuning environments (run on the GPU box from the repo
# root). Each SWEEP entry is a comma-separated list of VAR=value settings
# ("base" = none), e.g. SIFT_KP_WGS (persistent workgroups of orientation /
# descriptor), SIFT_BATCH_PX_LOG2 (octaves of >= 2^b pixels get their own
# keypoint batch), SIFT_EXT_STREAM (extrema on a fourth stream),
# GPU_MAX_HW_QUEUES (HIP hardware queues per process, <= 32).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${SWEEP_OUT:-sweep.txt}
: > $out
SWEEP=${SWEEP:-"base SIFT_EXT_STREAM=1"}
for rep in $(seq ${REPS:-1}); do
for cfg in $SWEEP; do
    envs=()
    [ "$cfg" != base ] && IFS=, read -ra envs <<< "$cfg"
    line=$(env "${envs[@]}" timeout -k 10 120 python bench.py ${BENCH_ARGS:---steps 1000 --warmup 20} \
        --no-cpu-baseline --no-events --no-matcher --no-extra 2>/dev/null) || { echo "$cfg FAILED" >> $out; exit 1; }
    ms=$(python -c "import json,sys; d=json.loads(sys.argv[1]); print(round(d['ms_per_step'],4), round(d['value']))" "$line")
    echo "$cfg ms/kps=$ms" | tee -a $out
done
done
python - "$out" <<'PY'
import collections, sys
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    k, v = line.split(" ms/kps=")
    d[k].append(float(v.split()[0]))
for k, v in d.items():
    print(f"{k:60s} mean {sum(v)/len(v):.4f} ms  min {min(v):.4f}  n={len(v)}")
PY
