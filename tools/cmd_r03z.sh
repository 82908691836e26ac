# round 3: replica-interleaved orientation + descriptor histograms, binary-search locate vs the committed kernels
L=$(pwd)/sift-project_amd/alt
bash tools/gpu_session.sh r03z test || exit 1
bash tools/pmc_kp.sh r03z/base > gpurun_out/r03z_base.log 2>&1 || { tail -5 gpurun_out/r03z_base.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r03z/base/pass1/*counter_collection.csv gpurun_out/r03z/base/pass2/*counter_collection.csv > gpurun_out/r03z/base_summary.txt
rm -rf gpurun_out/r03z/base/pass*/*.csv.gz
bash tools/bench_ab.sh r03z/ab 8 base SIFT_HIP_LIB=$L/head/libsift_hip.so
