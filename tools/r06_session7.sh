#!/bin/bash
# round 6: flow_lab — k_octaves_flow against per-level launches (exactness, counters, time)
set -o pipefail
O=gpurun_out/r06_s7
mkdir -p $O
for a in "1280 720 1 1 1 1" "1280 720 1 1 1 128" "1280 720 1 4 1 1" "1280 720 1 4 1 7" "1280 720 1 4 1 128" "3840 2160 3 5 1 128" "3840 2160 2 5 1 128" "3840 2160 3 5 8 128"; do
  echo "== $a" >> $O/lab.txt
  timeout -k 10 60 tools/flow_lab $a 20 >> $O/lab.txt 2>&1 || { echo "FAILED rc=$?" >> $O/lab.txt; cat $O/lab.txt; exit 1; }
done
cat $O/lab.txt
