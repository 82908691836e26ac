# round 3: descriptor locate (binary search vs scalar walk), 16 interleaved replicas: tests, counters, bench A/B
L=$(pwd)/sift-project_amd/alt
bash tools/gpu_session.sh r03y test || exit 1
bash tools/pmc_kp.sh r03y/base > gpurun_out/r03y_base.log 2>&1 || { tail -5 gpurun_out/r03y_base.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r03y/base/pass1/*counter_collection.csv gpurun_out/r03y/base/pass2/*counter_collection.csv > gpurun_out/r03y/base_summary.txt
rm -rf gpurun_out/r03y/base/pass*/*.csv.gz
bash tools/bench_ab.sh r03y/ab 6 base SIFT_HIP_LIB=$L/walk/libsift_hip.so
