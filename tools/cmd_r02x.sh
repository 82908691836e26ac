set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02x
mkdir -p $O
L=sift-project_amd/alt
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base SIFT_HIP_LIB=$L/head/libsift_hip.so SIFT_HIP_LIB=$L/noext/libsift_hip.so SIFT_HIP_LIB=$L/noup/libsift_hip.so 2>&1 | tee $O/ab1.txt || exit 1
