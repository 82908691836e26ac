set -o pipefail
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_KP_WGS=768 SIFT_KP_WGS=1024 SIFT_KP_WGS=384 SIFT_DESC_MODE=0 2>&1 | tee $O/ab1.txt || exit 1
timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 6 --steps 400 --depth 3 base 2>&1 | tee $O/ab_d3.txt || exit 1
timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 6 --steps 400 --depth 5 base 2>&1 | tee $O/ab_d5.txt || exit 1
