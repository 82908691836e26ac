#!/bin/bash
# Kernel traces of bench variants in one GPU call:
#   tools/gpu_prof.sh <tag> "<bench args 1>" "<bench args 2>" ...
set -o pipefail
R=$(pwd)
T=$1; shift
mkdir -p $R/gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
i=0
for A in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/$T/p$i -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-matcher $A > $R/gpurun_out/$T/p$i.json 2> $R/gpurun_out/$T/p$i.err || { tail -5 $R/gpurun_out/$T/p$i.err; exit 1; }
  echo "p$i: $A"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['roofline']['avg_launch_us'])" $R/gpurun_out/$T/p$i.json
done
echo DONE
