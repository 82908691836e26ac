#!/bin/bash
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_swz
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base swz0 swz1 swz3; do
  lib=""; [ $v != base ] && lib=$R/sift-project_amd/alt/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex k_descriptor --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python3 $R/tools/sq_summary.py $O/pmc_$v/run_counter_collection.csv | tee -a $O/sq.txt
done
cd $R
timeout -k 10 300 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=$R/sift-project_amd/alt/swz0/libsift_hip.so SIFT_HIP_LIB=$R/sift-project_amd/alt/swz1/libsift_hip.so SIFT_HIP_LIB=$R/sift-project_amd/alt/swz3/libsift_hip.so base 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "descriptor or big" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
