set -o pipefail
O=gpurun_out/r02ao
mkdir -p $O
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_BATCH_PX_LOG2=20 SIFT_BATCH_PX_LOG2=22 SIFT_BATCH_PX_LOG2=16 2>&1 | grep -v amdgpu.ids | tee $O/ab1.txt || exit 1
