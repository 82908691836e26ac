set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --extra-seconds 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"])
for k in ("alone", "alone_batch8"):
    a = d["roofline"][k]
    print(k, a["achieved"], a["frac"], a["us_per_image"], [(r["octave"], round(r["us_per_launch"], 1)) for r in a["per_octave"]])
    e = d["extrema_roofline"][k]; print("  extrema", e["achieved"], e["frac"], e["us_per_image"])
print("batch8", d["batch8"]["ms_per_image"], "api", d["api"]["value"], "latency", d["latency"]["ms_per_image"])
PY
