#!/bin/bash
# round 6: the fused initial blur (one-channel input, x2) on the pair walk — parity, alone, A/B, config 5
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_pairup
mkdir -p $O
A=$R/sift-project_amd/alt
L() { echo SIFT_HIP_LIB=$A/$1/libsift_hip.so; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base $(L strip) base $(L strip) 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 3 base $(L strip) 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base strip; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib SIFT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser_$v -o run -- python3 $R/bench.py --sync --steps 50 --warmup 5 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-big > $O/ser_$v.json 2> $O/ser_$v.err || { tail -5 $O/ser_$v.err; exit 1; }
  python3 $R/tools/prof_summary.py $O/ser_$v/run_kernel_trace.csv > $O/summary_serial_$v.txt
  rm -rf $O/ser_$v
  head -12 $O/summary_serial_$v.txt
done
cd $R
bash tools/bench_ab.sh r06_pairup/ab 3 base $(L strip) 2>&1 | tee $O/ab.txt
