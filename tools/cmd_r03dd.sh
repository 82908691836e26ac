# round 3: per-slot launch graphs: GPU tests, then the driver's bench command with graphs on / off and the timeline
bash tools/gpu_session.sh r03dd test || exit 1
O=gpurun_out/r03dd
for i in 1 2; do for g in 1 0; do
SIFT_GRAPHS=$g timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-alone --no-desc-f64 --step-log > $O/g${g}_$i.json 2> $O/g${g}_$i.err || exit 1
python3 -c "import json; d=json.load(open('$O/g${g}_$i.json')); h=d['host_busy']; print('graphs $g run $i', round(d['ms_per_step'],4), 'hostbusy', round(h['ms_per_step'],4), round(h['host_busy_ms'],4), json.dumps({k: round(v,4) for k,v in h['library_phases_ms'].items()}), 'lat', round(d['latency']['ms_per_image'],4), 'b8', round(d['batch8']['ms_per_image'],4), 'api', round(d['api']['ms_per_image'],4))"
grep "submit job" $O/g${g}_$i.err | head -8 | tr '\n' ' '; echo
done; done
