set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=sift-project_amd/alt
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base SIFT_HIP_LIB=$L/noup/libsift_hip.so SIFT_FUSE_INITIAL=0 2>&1 | tee $O/ab1.txt || exit 1
