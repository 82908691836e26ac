#!/bin/bash
# Round-2 closing GPU session: full parity suite, PMC traffic refresh
# (separate passes), bench, rocprofv3 kernel traces of the pipelined bench and
# of the serialised (kernel-alone) detect.
set -o pipefail
R=$(pwd)
O=gpurun_out/r02_final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "PMC traffic kept: profiles/traffic.json matches the kernel sources"
cp profiles/traffic.json $O/traffic.json
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-alone > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err || exit 1
SIFT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/ser -o run -- python3 $R/bench.py --sync --steps 200 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-alone > $R/$O/bench_ser.json 2> $R/$O/bench_ser.err || exit 1
cd $R && python tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/summary.txt && python tools/prof_summary.py $O/ser/run_kernel_trace.csv > $O/summary_serial.txt && echo DONE
