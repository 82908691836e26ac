# round 3: tiny octaves on one wavefront in the LDS kernel: tests, per-octave alone times, bench A/B
bash tools/gpu_session.sh r03hh test || exit 1
O=gpurun_out/r03hh
for v in base small0; do
  if [ $v = base ]; then unset SIFT_HIP_LIB; else export SIFT_HIP_LIB=$(pwd)/sift-project_amd/alt/$v/libsift_hip.so; fi
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-desc-f64 > $O/$v.json 2> $O/$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/$v.json')); a=d['roofline']['alone']; print('$v', round(d['ms_per_step'],4), 'lat', round(d['latency']['ms_per_image'],4), 'alone us/img', round(a['us_per_image'],1), [(p['octave'], round(p['us_per_launch'],1)) for p in a['per_octave']])"
done
unset SIFT_HIP_LIB
bash tools/bench_ab.sh r03hh/ab 6 base SIFT_HIP_LIB=$(pwd)/sift-project_amd/alt/small0/libsift_hip.so
