#!/bin/bash
# FP64 VALU instruction counts of the pipeline kernels, each alone on the chip
# (SIFT_SERIAL=1, synchronous detects): one pass, 6 SQ counters, kernel-trace
# only; totals per detect via tools/sq_summary.py (5 timed + 2 warm-up = 7)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-pmc_fp64}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_descriptor|k_orient|k_refine|k_extrema|k_blur|k_octaves' --output-format csv -d $O/pass -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pass.log 2>&1 || { tail -5 $O/pass.log; exit 1; }
cd $R
python3 tools/sq_summary.py $(find $O/pass -name '*counter_collection.csv') --detects 7 > $O/fp64_summary.txt
cat $O/fp64_summary.txt
cp $(find $O/pass -name "*counter_collection.csv") $O/counters.csv && rm -rf $O/pass
