#!/bin/bash
# round 6: which pool streams pipelined jobs take (SIFT_PIPE_BASE 0: hi/hi/lo/lo priority first; 4: normal priority; 2: lo/lo/normal/normal)
set -o pipefail
bash tools/bench_ab.sh r06_pipe/ab 4 base SIFT_PIPE_BASE=4 SIFT_PIPE_BASE=2 2>&1 | tee gpurun_out/r06_pipe_ab.txt
