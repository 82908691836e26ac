#!/bin/bash
# round 6: stream priorities of the pool's pair streams (pipelined jobs take them first): hi/hi/lo/lo (base), all high, all low
set -o pipefail
python3 -c "import ctypes; l=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); print('prio range', l.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), a.value, b.value)"
bash tools/bench_ab.sh r06_prio/ab 4 base SIFT_STREAM_PRIO=hh SIFT_STREAM_PRIO=ll 2>&1 | tee gpurun_out/r06_prio_ab.txt
