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
echo FINAL_DONE
