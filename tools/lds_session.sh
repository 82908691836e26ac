#!/bin/bash
# k_octaves_lds lab on the GPU box: tools/lds_session.sh <name> <binary>...
# (builds of tools/lds_lab.hip with other k_octaves_lds macros), each on the
# 1080p small octaves (6-10, 5-10) and the 8K ones (8-10)
set -o pipefail
N=${1:?name}
shift
O=gpurun_out/$N
mkdir -p $O
for bin in "$@"; do
  for a in "3840 2160 6 10" "3840 2160 5 10" "15360 8640 8 10"; do
    echo "== $bin $a" >> $O/lds.txt
    timeout -k 10 60 tools/$bin $a >> $O/lds.txt 2>&1 || { tail -20 $O/lds.txt; exit 1; }
  done
done
grep -A0 "==\|per launch" $O/lds.txt
echo LDS_DONE
