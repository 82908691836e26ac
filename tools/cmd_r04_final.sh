#!/bin/bash
# round-4 deliverables, one GPU call: PMC traffic passes first (the bench
# reports roofline.traffic only when profiles/traffic.json matches the
# kernel sources), then the GPU suite, the driver's bench, rocprof
# (pipelined + serial kernel-alone) and the synchronous-latency timeline
set -o pipefail
N=${1:-r04_final}
shift
bash tools/pmc_session.sh ${N}_pmc || exit 1
python3 tools/pmc_traffic.py gpurun_out/${N}_pmc gpurun_out/${N}_pmc/traffic.json || exit 1
cp gpurun_out/${N}_pmc/traffic.json profiles/traffic.json
bash tools/gpu_session.sh $N ${@:-test bench prof timeline} || exit 1

# A/B of the tree against the previous build (kernels alone + latency)
if [ -f sift-project_amd/alt/prev/libsift_hip.so ]; then
  timeout -k 10 300 python3 tools/kernel_alone.py --n 60 base SIFT_HIP_LIB=sift-project_amd/alt/prev/libsift_hip.so \
      > gpurun_out/$N/kernel_alone_vs_prev.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$N/kernel_alone_vs_prev.txt
fi
echo FINAL_DONE
