set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=sift-project_amd/alt
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base SIFT_HIP_LIB=$L/prev/libsift_hip.so 2>&1 | tee $O/ab1.txt || exit 1
cd /tmp && export TMPDIR=/tmp
SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser -o run -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/ser.json 2> $O/ser.err || { tail -5 $O/ser.err; exit 1; }
cut -d, -f1-5 $O/ser/run_kernel_stats.csv | head -6
