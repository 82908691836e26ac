# round 3: timeline of synchronous (latency) detects, kernels on their real streams
O=gpurun_out/${TL_OUT:-r03l}
mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/lat -o run -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 --no-events > $R/$O/bench_lat.json 2> $R/$O/bench_lat.err || { tail -20 $R/$O/bench_lat.err; exit 1; }
cd $R
head -1 $O/lat/run_kernel_trace.csv
python3 tools/prof_summary.py $O/lat/run_kernel_trace.csv > $O/summary_lat.txt && tail -45 $O/summary_lat.txt
