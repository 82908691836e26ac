#!/bin/bash
set -o pipefail
bash tools/bench_ab.sh r04_j/ab20 4 base SIFT_JOB_DEPTH=5 SIFT_JOB_DEPTH=6 SIFT_JOB_DEPTH=3 || exit 1
