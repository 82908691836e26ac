#!/bin/bash
# round 6: LDS-DMA pair walk on big planes (lab) + what SQ_LDS_BANK_CONFLICT counts for ds_add_f64
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06_s2
mkdir -p $O
run() { echo "== $*" >> $O/lab.txt; env "$@" >> $O/lab.txt 2>&1 || { tail -20 $O/lab.txt; exit 1; }; }
run LAB_NB=4 timeout -k 10 120 tools/blur_lab pdma:2:32 3840 2160 2 4 5 6 8 10
for nb in 2 4 8; do run LAB_NB=$nb timeout -k 10 200 tools/blur_lab pdma:2:32 15360 8640 2 4 5 6 8 10; done
for nb in 2 4 8; do run LAB_NB=$nb timeout -k 10 120 tools/blur_lab pdma:2:32 8192 8192 1 5 7 10; done
for nb in 4; do run LAB_NB=$nb timeout -k 10 120 tools/blur_lab pdma:2:32 4096 4096 1 5 7 10; done
cat $O/lab.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $O/probe -o run -- $R/tools/lds_atomic_probe > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
python3 - $O/probe/run_counter_collection.csv <<'PY'
import csv, collections, sys, re
t = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("(anonymous namespace)::", "")
    m = re.search(r"k_atomic<(\d)>", r["Kernel_Name"]); k = f"atomic<{m.group(1)}>" if m else k
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(t.items()):
    i = v["SQ_INSTS_LDS"]
    print(f"{k:16s} insts {i:10.4g}  active/inst {v['SQ_ACTIVE_INST_LDS']/i:6.2f}  conflict/inst {v['SQ_LDS_BANK_CONFLICT']/i:6.2f}  waitLDS/wave-cycles {v['SQ_WAIT_INST_LDS']/v['SQ_WAVE_CYCLES']:.3f}")
PY
rm -rf $O/probe
