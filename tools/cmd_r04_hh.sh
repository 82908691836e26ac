#!/bin/bash
# host waits by polling hipEventQuery (SIFT_SPIN_WAIT=1) vs hipEventSynchronize:
# synchronous latency (kernel_alone) and the driver's 20-step bench
set -o pipefail
O=gpurun_out/r04_hh
mkdir -p $O
timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_SPIN_WAIT=1 base SIFT_SPIN_WAIT=1 \
    > $O/kernel_alone.txt 2> $O/kernel_alone.err || { tail -20 $O/kernel_alone.err; exit 1; }
cat $O/kernel_alone.txt
bash tools/bench_ab.sh r04_hh/ab 5 base SIFT_SPIN_WAIT=1 || exit 1
