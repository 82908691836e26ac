set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser -o run -- python3 $R/bench.py --sync --steps 200 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/ser.json 2> $O/ser.err || { tail -5 $O/ser.err; exit 1; }
cat $O/ser/run_kernel_stats.csv | cut -d, -f1-5 | head -12
cd $R
SWEEP="base SIFT_KP_WGS=768" REPS=3 BENCH_ARGS="--steps 3000 --warmup 20" SWEEP_OUT=r02s/sw.txt tools/sweep.sh | grep mean || exit 1
