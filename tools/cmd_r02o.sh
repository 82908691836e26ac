set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=sift-project_amd/alt
VARIANTS="base SIFT_DESC_F64=1 SIFT_HIP_LIB=$L/pf4/libsift_hip.so SIFT_HIP_LIB=$L/pf6/libsift_hip.so" REPS=2 AB_OUT=r02o/ab.txt tools/ab_alone.sh || exit 1
