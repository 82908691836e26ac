#!/bin/bash
# round 6: LDS-DMA pair walk and descriptor lane permutation (lab + alone + PMC + parity)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s1
mkdir -p $O
A=$R/sift-project_amd/alt
for nb in 2 4 8; do
  LAB_NB=$nb timeout -k 10 120 tools/blur_lab pdma:2:32 3840 2160 2 4 5 6 8 10 > $O/lab_1080_nb$nb.txt 2>&1 || { cat $O/lab_1080_nb$nb.txt; exit 1; }
  cat $O/lab_1080_nb$nb.txt
done
for nb in 4 8; do
  LAB_NB=$nb timeout -k 10 120 tools/blur_lab pdma:2:32 8192 8192 1 5 7 10 14 > $O/lab_8k_nb$nb.txt 2>&1 || { cat $O/lab_8k_nb$nb.txt; exit 1; }
  cat $O/lab_8k_nb$nb.txt
done
timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=$A/dma4/libsift_hip.so SIFT_HIP_LIB=$A/dma8/libsift_hip.so SIFT_HIP_LIB=$A/p1s0/libsift_hip.so SIFT_HIP_LIB=$A/p1s1/libsift_hip.so SIFT_HIP_LIB=$A/p1s2/libsift_hip.so base SIFT_HIP_LIB=$A/dma4/libsift_hip.so SIFT_HIP_LIB=$A/p1s0/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base p1s0 p1s1 p1s2; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex k_descriptor --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/sq.txt
  python3 $R/tools/sq_summary.py $O/pmc_$v/run_counter_collection.csv >> $O/sq.txt
  rm -rf $O/pmc_$v
done
cat $O/sq.txt
cd $R
SIFT_HIP_LIB=$A/dma4/libsift_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_dma4.log 2>&1; tail -3 $O/pytest_dma4.log
SIFT_HIP_LIB=$A/p1s0/libsift_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "descriptor or big or golden" > $O/pytest_p1s0.log 2>&1; tail -3 $O/pytest_p1s0.log
