set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SWEEP="base SIFT_KP_WGS=768 SIFT_KP_WGS=1024 SIFT_FUSE_INITIAL=0" REPS=2 SWEEP_OUT=r02r/sw.txt tools/sweep.sh | grep mean || exit 1
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
SIFT_FUSE_INITIAL=$f SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser$f -o run -- python3 $R/bench.py --sync --steps 200 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/ser$f.json 2> $O/ser$f.err || { tail -5 $O/ser$f.err; exit 1; }
cat $O/ser$f/run_kernel_stats.csv | cut -d, -f1-5 | head -12
done
