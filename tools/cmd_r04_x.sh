#!/bin/bash
# exchange path at world size 1: plain vs --exchange, new gather vs previous
# library, 400-step runs alternating; plus the GPU tests of the exchange
set -o pipefail
O=gpurun_out/r04_aa
mkdir -p $O
P=sift-project_amd/alt/prev/libsift_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in base prev; do
    envs=""; [ $v = prev ] && envs="SIFT_HIP_LIB=$P"
    for x in plain exch; do
      fl=""; [ $x = exch ] && fl="--exchange"
      env $envs timeout -k 10 200 python3 bench.py --steps 400 --warmup 20 $fl --no-extra --no-big \
          --no-cpu-baseline --no-matcher --no-alone > $O/${v}_${x}_$r.json 2> $O/${v}_${x}_$r.err \
          || { tail -20 $O/${v}_${x}_$r.err; exit 1; }
    done
  done
done
python3 - $O <<'PY'
import json, sys, statistics
o = sys.argv[1]
for v in ("base", "prev"):
    p = [json.load(open(f"{o}/{v}_plain_{r}.json"))["ms_per_step"] for r in (1, 2, 3)]
    e = [json.load(open(f"{o}/{v}_exch_{r}.json"))["ms_per_step"] for r in (1, 2, 3)]
    print(v, "plain", [round(x, 4) for x in p], "exchange", [round(x, 4) for x in e],
          "ratio", round(statistics.median(e) / statistics.median(p), 4))
PY
