set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02ah
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=sift-project_amd/alt
VARIANTS="base SIFT_HIP_LIB=$L/prev/libsift_hip.so SIFT_BLUR_ROWS=44" REPS=1 AB_OUT=r02ah/ab_alone.txt BENCH_ARGS="--steps 300 --warmup 20" tools/ab_alone.sh || exit 1
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_HIP_LIB=$L/prev/libsift_hip.so SIFT_BLUR_ROWS=44 2>&1 | tee $O/ab1.txt || exit 1
