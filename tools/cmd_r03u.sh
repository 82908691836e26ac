# round 3: driver bench command under stream policy 0 / 1, twice each, alternating
O=gpurun_out/r03u; mkdir -p $O
for i in 1 2; do for pol in 0 2; do
  SIFT_STREAM_POLICY=$pol timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-alone --no-desc-f64 > $O/b_${pol}_$i.json 2> $O/b_${pol}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_${pol}_$i.json')); print('policy $pol run $i', round(d['ms_per_step'],4), 'host_busy leg', round(d['host_busy']['ms_per_step'],4), round(d['host_busy']['host_busy_ms'],4), 'lat', round(d['latency']['ms_per_image'],4), 'b8', round(d['batch8']['ms_per_image'],4))"
done; done
