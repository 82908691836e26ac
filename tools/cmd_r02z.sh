set -o pipefail
O=gpurun_out/r02z
mkdir -p $O
: > $O/q.txt
for rep in 1 2; do
for cfg in "4 4" "8 4" "8 6" "8 8" "16 8" "4 3"; do
  set -- $cfg
  r=$(GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python -u tools/ab_interleaved.py --rounds 2 --steps 800 --depth $2 base 2>/dev/null | grep base) || exit 1
  echo "queues $1 depth $2: $r" | tee -a $O/q.txt
done
done
