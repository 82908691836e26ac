# round 3: the timed region's job timeline (submit / fetch / done) for the driver's bench shape
O=gpurun_out/r03bb; mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-alone --no-desc-f64 --no-extra --step-log > $O/b$i.json 2> $O/b$i.err || exit 1
grep -A80 "step log" $O/b$i.err | head -70; python3 -c "import json; print(json.load(open('$O/b$i.json'))['ms_per_step'])"
done
