# round 3 lab: where the descriptor's LDS bank-conflict cycles come from (no histogram atomics / one replica per LDS lane group)
L=$(pwd)/sift-project_amd/alt
for v in nohist rephi; do
  export SIFT_HIP_LIB=$L/$v/libsift_hip.so
  bash tools/pmc_kp.sh r03w/$v > gpurun_out/r03w_$v.log 2>&1 || { tail -5 gpurun_out/r03w_$v.log; exit 1; }
  python3 tools/sq_summary.py gpurun_out/r03w/$v/pass1/*counter_collection.csv gpurun_out/r03w/$v/pass2/*counter_collection.csv > gpurun_out/r03w/${v}_summary.txt
  rm -rf gpurun_out/r03w/$v/pass*/*.csv.gz
done
unset SIFT_HIP_LIB
bash tools/bench_ab.sh r03w/ab 6 base SIFT_HIP_LIB=$L/extnt/libsift_hip.so SIFT_LDS_PX=2100
