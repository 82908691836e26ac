# latency (synchronous detects) A/B of the keypoint grid for jobs alone; separate processes
set -o pipefail
O=gpurun_out/r03_lat; mkdir -p $O
for r in 1 2 3; do for v in base SIFT_KP_WGS_ALONE=384 SIFT_KP_WGS_ALONE=512 SIFT_KP_WGS_ALONE=1024,SIFT_KP_WGS_MAX=1024; do
  envs=""; [ $v != base ] && envs=$(echo $v | tr ',' ' ')
  env $envs timeout -k 10 120 python3 bench.py --sync --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/lat_${v}_$r.json 2> $O/lat_${v}_$r.err || { tail -5 $O/lat_${v}_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/lat_${v}_$r.json'));print('$v', round(d['ms_per_step'],4))"
done; done
