set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02p
mkdir -p $O
SWEEP="base SIFT_DESC_MODE=1 SIFT_DESC_MODE=2" REPS=2 SWEEP_OUT=r02p/sw.txt tools/sweep.sh | grep mean || exit 1
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2; do
  SIFT_SERIAL=1 SIFT_DESC_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/m$m -o run -- python3 $R/bench.py --sync --steps 200 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/m$m.json 2> $O/m$m.err || { tail -5 $O/m$m.err; exit 1; }
  echo "mode $m"; find $O/m$m -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-5 | head -12
done
