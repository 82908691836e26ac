#!/bin/bash
# A/B of build/env variants with the kernel-alone roofline: for each VARIANTS
# entry (comma-separated VAR=value list, "base" = none) run the bench with
# events and print the pipelined rate plus the alone pyramid / extrema rates.
set -o pipefail
out=gpurun_out/${AB_OUT:-ab_alone.txt}
mkdir -p "$(dirname $out)"
: > $out
for rep in $(seq ${REPS:-1}); do
for cfg in ${VARIANTS:-base}; do
    envs=()
    [ "$cfg" != base ] && IFS=, read -ra envs <<< "$cfg"
    line=$(env "${envs[@]}" timeout -k 10 150 python bench.py ${BENCH_ARGS:---steps 1000 --warmup 20} \
        --no-cpu-baseline --no-matcher --no-extra 2>/dev/null) || { echo "$cfg FAILED" | tee -a $out; exit 1; }
    python - "$cfg" "$line" <<'PY' | tee -a $out
import json, sys
d = json.loads(sys.argv[2]); a = d["roofline"]["alone"]; e = d["extrema_roofline"]["alone"]
o = " ".join(f"o{r['octave']}:{r['us_per_launch']:.1f}" for r in a["per_octave"])
print(f"{sys.argv[1]:40s} ms/img {d['ms_per_step']:.4f} kps {d['value']/1e6:.3f}M | alone pyr "
      f"{a['achieved']:.0f} GB/s frac {a['frac']:.3f} {a['us_per_image']:.0f} us/img [{o}] | ext "
      f"{e['achieved']:.0f} GB/s {e['us_per_image']:.0f} us/img | pipe frac {d['roofline']['frac']:.3f}")
PY
done
done
