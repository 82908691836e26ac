#!/bin/bash
# the driver's bench command on the current tree
set -o pipefail
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
    || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print({k: d[k] for k in ('value','ms_per_step','dtype')})
r=d['roofline']; print('roof', r['achieved'], r['frac'], r['traffic'], 'alone', r.get('alone',{}).get('frac'), r.get('alone',{}).get('us_per_image'), 'fp64', r['fp64'])
print('kp alone', d.get('keypoint_kernels_alone'))
for c in ('config3','config5'):
    x=d.get(c); print(c, x and {k:x[k] for k in ('value','ms_per_image','keypoints_per_image','speedup_vs_reference_cpu')}, x and x['roofline']['frac'], x and x['roofline']['alone']['frac'], x and x['roofline']['fp64'])
print('cpu', d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline_reference'))
print('lat', d.get('latency'), 'batch8', d.get('batch8',{}).get('ms_per_image'))
"
