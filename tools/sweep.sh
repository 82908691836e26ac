#!/bin/bash
# Bench sweep over the keypoint-stream tuning knobs (run on the GPU box from
# the repo root): SIFT_C_CU_RESERVE (eighths of the CUs kept free of keypoint
# kernels) x SIFT_KP_WGS (persistent workgroups of orientation/descriptor) x
# SIFT_BATCH_PX_LOG2 (octaves of at least 2^b pixels get their own keypoint batch).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
SWEEP=${SWEEP:-"0:1024:20 1:1024:20 2:1024:20 0:512:20 0:768:20 1:768:20 0:1024:18 1:1024:18 1:768:18"}
for cfg in $SWEEP; do
    IFS=: read r w b <<< "$cfg"
    line=$(SIFT_C_CU_RESERVE=$r SIFT_KP_WGS=$w SIFT_BATCH_PX_LOG2=$b timeout -k 10 120 python bench.py --steps 40 --warmup 5 \
        --no-cpu-baseline --no-events 2>/dev/null) || { echo "reserve=$r wgs=$w batch=$b FAILED" >> $out; exit 1; }
    ms=$(python -c "import json,sys; d=json.loads(sys.argv[1]); print(round(d['ms_per_step'],4), round(d['value']))" "$line")
    echo "reserve=$r wgs=$w batch=$b ms/kps=$ms" | tee -a $out
done
