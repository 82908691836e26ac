#!/bin/bash
# A/B timing of library variants within ONE GPU call (boxes differ by up to
# ~15 %, so variants are only comparable side by side): every tools/ab/*.so
# (or $LIBS) is loaded through SIFT_HIP_LIB by bench.py, interleaved REPS times.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab.txt
: > $out
LIBS=${LIBS:-$(ls tools/ab/*.so)}
for rep in $(seq ${REPS:-3}); do
    for lib in $LIBS; do
        line=$(SIFT_HIP_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py ${BENCH_ARGS:---steps 1000 --warmup 20} \
            --no-cpu-baseline --no-events --no-matcher --no-extra 2>/dev/null) || { echo "$lib FAILED" >> $out; exit 1; }
        ms=$(python -c "import json,sys; print(round(json.loads(sys.argv[1])['ms_per_step'],4))" "$line")
        echo "$lib $ms" | tee -a $out
    done
done
python - <<'PY'
import collections
d = collections.defaultdict(list)
for line in open("gpurun_out/ab.txt"):
    k, v = line.split()
    d[k].append(float(v))
for k, v in d.items():
    print(f"{k:32s} mean {sum(v)/len(v):.4f} ms  min {min(v):.4f}  n={len(v)}")
PY
