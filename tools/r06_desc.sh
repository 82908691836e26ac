#!/bin/bash
# round 6: descriptor bin stride 9 vs 8 — SQ counters (1080p) and kernels alone at 8K (config 5)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_desc
mkdir -p $O
A=$R/sift-project_amd/alt
timeout -k 10 400 python3 tools/kernel_alone.py --big config5 --n 4 base SIFT_HIP_LIB=$A/bs8/libsift_hip.so base SIFT_HIP_LIB=$A/bs8/libsift_hip.so 2>&1 | grep -v amdgpu.ids | tee $O/alone_c5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $O/probe -o run -- $R/tools/lds_atomic_probe > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
python3 - $O/probe/run_counter_collection.csv <<'PY' | tee $O/probe.txt
import csv, collections, sys, re
t = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("(anonymous namespace)::", "")
    m = re.search(r"k_atomic<(\d)>", r["Kernel_Name"]); k = f"atomic<{m.group(1)}>" if m else k
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(t.items()):
    i = v["SQ_INSTS_LDS"]
    print(f"{k:16s} insts {i:10.4g}  active/inst {v['SQ_ACTIVE_INST_LDS']/i:6.2f}  conflict/inst {v['SQ_LDS_BANK_CONFLICT']/i:6.2f}  waitLDS/wave-cycles {v['SQ_WAIT_INST_LDS']/v['SQ_WAVE_CYCLES']:.3f}")
PY
rm -rf $O/probe
for v in base bs8; do
  lib=""; [ $v != base ] && lib=$A/$v/libsift_hip.so
  SIFT_HIP_LIB=$lib SIFT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex k_descriptor --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --sync --no-extra --no-cpu-baseline --no-matcher --no-events --no-alone --no-big > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  echo "== $v" >> $O/sq.txt
  python3 $R/tools/sq_summary.py $O/pmc_$v/run_counter_collection.csv >> $O/sq.txt
  rm -rf $O/pmc_$v
done
cat $O/sq.txt
