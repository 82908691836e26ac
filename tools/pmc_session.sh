#!/bin/bash
# PMC traffic session: calibrate FETCH_SIZE/WRITE_SIZE on a known 8-B/lane
# copy (tools/pmc_calib), then collect both counters (separate passes,
# kernel-trace only) on the default bench restricted to the pyramid
# (k_blur, k_blur_tile, k_octaves_lds) and extrema kernels.
# usage: tools/pmc_session.sh <out dir under gpurun_out>
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/calib_$C -o run -- $R/tools/pmc_calib > $O/calib_$C.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex 'k_blur|k_octaves_lds|k_extrema' --output-format csv -d $O/bench_$C -o run -- python3 $R/bench.py --steps 20 --warmup 2 --no-extra --no-cpu-baseline --no-matcher --no-alone --no-big > $O/bench_$C.log 2>&1 || exit 1
done
echo PMC_DONE
