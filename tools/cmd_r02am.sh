set -o pipefail
O=gpurun_out/r02am
mkdir -p $O
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base DEPTH=3 DEPTH=5 DEPTH=6 SIFT_KP_WGS=384 2>&1 | tee $O/ab1.txt || exit 1
