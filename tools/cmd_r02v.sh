set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=sift-project_amd/alt
timeout -k 10 400 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base SIFT_HIP_LIB=$L/da2/libsift_hip.so SIFT_HIP_LIB=$L/da2o4/libsift_hip.so SIFT_EXT_WAVES=3072 SIFT_REFINE_WGS=128 2>&1 | tee $O/ab1.txt || exit 1
cd /tmp && export TMPDIR=/tmp
SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser -o run -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/ser.json 2> $O/ser.err || { tail -5 $O/ser.err; exit 1; }
cut -d, -f1-5 $O/ser/run_kernel_stats.csv | head -12
SIFT_HIP_LIB=$R/sift-project_amd/alt/da2/libsift_hip.so SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/serda2 -o run -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/serda2.json 2> $O/serda2.err || { tail -5 $O/serda2.err; exit 1; }
grep descriptor $O/serda2/run_kernel_stats.csv | cut -d, -f1-5
