# round 3 final: GPU tests, PMC traffic of the final kernels, the driver's exact bench command,
# rocprof kernel-trace summaries (pipelined and serialised), SQ counters of the keypoint/pyramid kernels
N=${1:-r03_final}
O=gpurun_out/$N
mkdir -p $O
bash tools/gpu_session.sh $N test || exit 1
bash tools/pmc_session.sh $N/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc profiles/traffic.json > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
cp profiles/traffic.json $O/traffic.json
rm -rf $O/pmc/bench_* $O/pmc/calib_*
bash tools/gpu_session.sh $N bench prof || exit 1
bash tools/pmc_kp.sh $N/sq > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq/pass1/*counter_collection.csv $O/sq/pass2/*counter_collection.csv > $O/sq_summary.txt
rm -rf $O/sq
