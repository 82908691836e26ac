#!/bin/bash
# round 6 final call on the final tree: kernels alone + latency, smoke, the driver's bench command,
# the GPU suite, serial / pipelined rocprof summaries, latency trace, configs 3 / 5 traces
set -o pipefail
R=$(pwd)
O=gpurun_out/r06_final
mkdir -p $O
timeout -k 10 400 python3 tools/kernel_alone.py --n 150 base 2>&1 | grep -v amdgpu.ids | tee $O/kalone.txt || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_session.sh r06_final bench test prof timeline big || exit 1
