set -o pipefail
O=gpurun_out/r02an
mkdir -p $O
for rep in 1 2; do
for q in 4 8; do
  echo "== GPU_MAX_HW_QUEUES=$q" | tee -a $O/ab.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u tools/ab_interleaved.py --rounds 4 --steps 400 base SIFT_JOB_STREAMS=2 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
done
done
