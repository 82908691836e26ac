set -o pipefail
O=gpurun_out/r02as
mkdir -p $O
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 100 --batch 8 --depth 2 base SIFT_BATCH_PX_LOG2=18 SIFT_BATCH_PX_LOG2=20 2>&1 | grep -v amdgpu.ids | tee $O/ab8.txt || exit 1
