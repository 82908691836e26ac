#!/bin/bash
# Blur-kernel lab on the GPU box (tools/blur_lab, built on the CPU side):
#   tools/lab_session.sh <name> "<env> <args>" ...
# each argument: environment assignments for the walk kernel's launcher
# followed by blur_lab's arguments (W H dec_at R...), e.g.
#   "LAB_BIN=blur_lab_np strip:2:32 3840 2160 2 4 5 6 8 10"
# (LAB_BIN: another build of blur_lab, e.g. with other k_blur macros)
# Every run has its own time limit; the session stops at the first failure.
set -o pipefail
N=${1:?name}
shift
O=gpurun_out/$N
mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i + 1))
  echo "== $spec" | tee -a $O/lab.txt
  # split the env assignments from the program arguments
  envs=(); args=()
  for w in $spec; do
    if [[ $w == *=* ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  bin=blur_lab
  for e in "${envs[@]}"; do [[ $e == LAB_BIN=* ]] && bin=${e#LAB_BIN=}; done
  env "${envs[@]}" timeout -k 10 120 tools/$bin "${args[@]}" >> $O/lab.txt 2>&1 \
      || { tail -20 $O/lab.txt; exit 1; }
done
cat $O/lab.txt
echo LAB_DONE
