#!/bin/bash
# round 6: bench.py's config 3 / 5 legs vs tools/big_profile.py, current library vs the round's first commit (alt/prefix)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_bigleg
mkdir -p $O
P=$R/sift-project_amd/alt/prefix/libsift_hip.so
for r in 1 2; do
  for v in base prefix; do
    lib=""; [ $v != base ] && lib=$P
    SIFT_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-alone --no-cpu-baseline --no-matcher > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('bench $v $r', round(d['ms_per_step'],4), [(c, round(d[c]['ms_per_image'],3), round(d[c]['host_phases_ms']['wait_device'],2)) for c in ('config3','config5')])"
  done
done
for v in base prefix; do
  lib=""; [ $v != base ] && lib=$P
  SIFT_HIP_LIB=$lib timeout -k 10 200 python3 tools/big_profile.py config3 --images 16 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); print('big_profile config3 $v', round(d['ms_per_image'],3))"
done
