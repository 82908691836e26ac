set -o pipefail
O=gpurun_out/r02ap
mkdir -p $O
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base SIFT_BATCH_PX_LOG2=20 SIFT_BATCH_PX_LOG2=22 SIFT_BATCH_PX_LOG2=24 2>&1 | grep -v amdgpu.ids | tee $O/ab1.txt || exit 1
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 100 --batch 8 --depth 2 base SIFT_BATCH_PX_LOG2=22 SIFT_BATCH_PX_LOG2=24 2>&1 | grep -v amdgpu.ids | tee $O/ab8.txt || exit 1
