#!/bin/bash
# Lab session: blur design-space sweep + PMC counters on the keypoint kernels.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/lab
timeout -k 10 240 ./tools/blur_lab > gpurun_out/lab/blur_lab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/lab/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex 'k_descriptor|k_orient|k_extrema|k_refine|k_blur' --output-format csv -d $R/gpurun_out/lab/pmc1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/lab/pmc1.log 2>&1 || exit 1
echo LAB_DONE
