#!/bin/bash
# PMC traffic session: calibrate FETCH_SIZE/WRITE_SIZE on a known 8-B/lane
# copy, then collect both counters (separate passes, kernel-trace only) on the
# bench run restricted to the pyramid kernels.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc/calib_$C -o run -- $R/tools/pmc_calib > $R/gpurun_out/pmc/calib_$C.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex 'k_blur|k_octaves_lds' --output-format csv -d $R/gpurun_out/pmc/bench_$C -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc/bench_$C.log 2>&1 || exit 1
done
echo PMC_DONE
