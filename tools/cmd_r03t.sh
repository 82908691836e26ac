# round 3 checkpoint: GPU tests, PMC traffic of the current kernels, the driver's bench command, rocprof summaries
N=r03t
O=gpurun_out/$N
bash tools/gpu_session.sh $N test || exit 1
bash tools/pmc_session.sh $N/pmc > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc profiles/traffic.json > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
cp profiles/traffic.json $O/traffic.json
rm -rf $O/pmc/bench_* $O/pmc/calib_*/*.csv.gz
bash tools/gpu_session.sh $N bench prof
