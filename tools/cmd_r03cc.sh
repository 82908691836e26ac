# round 3: stream policies 0 / 2 / 3 (four high-priority job streams) with the timed region's job timeline
O=gpurun_out/r03cc; mkdir -p $O
for i in 1 2 3; do for pol in 0 3 2; do
SIFT_STREAM_POLICY=$pol timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-alone --no-desc-f64 --no-extra --step-log > $O/p${pol}_$i.json 2> $O/p${pol}_$i.err || exit 1
python3 - $O/p${pol}_$i <<'PY'
import json, re, sys
b = sys.argv[1]
d = json.load(open(b + ".json"))
ev = {}
for line in open(b + ".err"):
    m = re.match(r"\s+(\w+)\s+job\s+(\d+)\s+([\d.]+)", line)
    if m: ev[(m.group(1), int(m.group(2)))] = float(m.group(3))
waits = [round(ev[("done", k)] - ev[("fetch", k)], 2) for k in range(20) if ("done", k) in ev]
print(b.split("/")[-1], round(d["ms_per_step"], 4), "fetch waits", waits)
PY
done; done
