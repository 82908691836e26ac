#!/bin/bash
# round-4 deliverables: GPU suite, the driver's bench, rocprof (pipelined +
# serial kernel-alone), PMC traffic passes
set -o pipefail
N=${1:-r04_final}
shift
bash tools/gpu_session.sh $N ${@:-test bench prof} || exit 1
bash tools/pmc_session.sh ${N}_pmc || exit 1
echo FINAL_DONE
