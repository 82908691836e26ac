#!/bin/bash
# kernel trace of the world-1 exchange bench: what device work the exchange adds
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04_y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/p -o run \
    -- python3 $R/bench.py --steps 200 --warmup 20 --exchange --no-extra --no-big --no-cpu-baseline \
    --no-matcher --no-alone > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R
ls $O/p
cp $O/p/run_kernel_stats.csv $O/kernel_stats_exch.csv 2>/dev/null
cp $O/p/run_memory_copy_stats.csv $O/copy_stats_exch.csv 2>/dev/null
rm -rf $O/p
