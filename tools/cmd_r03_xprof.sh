# host profile (cProfile) of the bench loop with and without the RCCL exchange
set -o pipefail
O=gpurun_out/r03_xprof2; mkdir -p $O
for m in ex plain; do
  a=""; [ $m = ex ] && a=--exchange
  timeout -k 10 300 python3 -m cProfile -o $O/$m.prof bench.py $a --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/$m.json 2> $O/$m.err || { tail -20 $O/$m.err; exit 1; }
  python3 -c "
import pstats; p=pstats.Stats('$O/$m.prof'); p.sort_stats('tottime').print_stats(30)" > $O/$m.txt
done
echo DONE
