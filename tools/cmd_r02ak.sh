set -o pipefail
O=gpurun_out/r02ak
mkdir -p $O
timeout -k 10 500 python -u tools/ab_interleaved.py --rounds 8 --steps 400 base PROFILE=1 2>&1 | tee $O/ab1.txt || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 1500 --no-cpu-baseline --no-extra --no-matcher --no-alone 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('events', d['ms_per_step'])" || exit 1
  timeout -k 10 200 python bench.py --steps 1500 --no-cpu-baseline --no-extra --no-matcher --no-events 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('noevents', d['ms_per_step'])" || exit 1
done 2>&1 | tee $O/bench_pairs.txt
