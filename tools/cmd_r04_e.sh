#!/bin/bash
set -o pipefail
O=gpurun_out/r04_e
mkdir -p $O
A=sift-project_amd/alt
timeout -k 10 120 tools/math64_check 4194304 > $O/math64.txt 2>&1 || { cat $O/math64.txt; exit 1; }
cat $O/math64.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/kernel_alone.py --n 40 base SIFT_HIP_LIB=$A/ori0/libsift_hip.so \
    SIFT_HIP_LIB=$A/ahead1/libsift_hip.so SIFT_HIP_LIB=$A/ahead3/libsift_hip.so SIFT_HIP_LIB=$A/oriahead2/libsift_hip.so \
    > $O/alone.txt 2>&1 || { tail -20 $O/alone.txt; exit 1; }
grep -v amdgpu.ids $O/alone.txt
timeout -k 10 700 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base \
    SIFT_HIP_LIB=$A/ori0/libsift_hip.so SIFT_HIP_LIB=$A/ahead1/libsift_hip.so \
    SIFT_HIP_LIB=$A/ahead3/libsift_hip.so SIFT_HIP_LIB=$A/oriahead2/libsift_hip.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
for i in 1 2; do
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher \
    --no-alone --no-extra --no-big --step-log > $O/steplog$i.json 2> $O/steplog$i.err || { tail -20 $O/steplog$i.err; exit 1; }
done
grep -A70 "step log" $O/steplog2.err | head -75
python3 -c "
import json
for i in (1,2):
    d=json.load(open('$O/steplog%d.json'%i)); print(d['value'], d['ms_per_step'])"
