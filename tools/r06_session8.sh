#!/bin/bash
set -o pipefail
O=gpurun_out/r06_s8
mkdir -p $O
for b in flow_lab_dbg flow_lab_dbg_inl flow_lab_dbg_nopad; do
  echo "== $b" >> $O/dbg.txt
  timeout -k 5 15 tools/$b 128 64 1 1 1 1 1 >> $O/dbg.txt 2>&1; echo "rc=$?" >> $O/dbg.txt
done
cat $O/dbg.txt | head -100
