#!/bin/bash
# round 6 final: PMC passes in a call of their own (traffic: FETCH/WRITE_SIZE; SQ counters of every kernel alone)
set -o pipefail
R=$(pwd)
bash tools/pmc_session.sh r06_final_pmc2 || exit 1
bash tools/pmc_kp.sh r06_final_pmc2 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r06_final_pmc2 gpurun_out/r06_final_pmc2/traffic.json || exit 1
python3 tools/sq_summary.py gpurun_out/r06_final_pmc2/pass1/run_counter_collection.csv gpurun_out/r06_final_pmc2/pass2/run_counter_collection.csv > gpurun_out/r06_final_pmc2/sq_summary.txt || exit 1
cat gpurun_out/r06_final_pmc2/sq_summary.txt
rm -rf gpurun_out/r06_final_pmc2/bench_* gpurun_out/r06_final_pmc2/pass1 gpurun_out/r06_final_pmc2/pass2
