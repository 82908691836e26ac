#!/bin/bash
# round 6: descriptor histogram layouts (alone + PMC), GPU suite on the default build, big configs with / without the DMA pair walk
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s3
mkdir -p $O
A=$R/sift-project_amd/alt
V="base bs9 rm2 rm2p rm1 p1s0"
args=""; for v in $V; do [ $v = base ] && args="$args base" || args="$args SIFT_HIP_LIB=$A/$v/libsift_hip.so"; done
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 $args base 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in $V; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex k_descriptor --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/sq.txt
  python3 $R/tools/sq_summary.py $O/pmc_$v/run_counter_collection.csv >> $O/sq.txt
  rm -rf $O/pmc_$v
done
cat $O/sq.txt
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for v in base nodma; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-extra > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print('$v', json.dumps(d['summary']))"
done
