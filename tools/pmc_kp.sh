#!/bin/bash
# SQ counters of the pipeline kernels (separate passes, kernel-trace only),
# serialized pipeline so each kernel runs alone.
set -o pipefail
R=$(pwd)
T=${1:-pmc}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_descriptor|k_orient|k_refine|k_extrema|k_blur|k_octaves' --output-format csv -d $O/pass$i -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pass$i.log 2>&1 || { tail -5 $O/pass$i.log; exit 1; }
done
echo PMC_DONE
