# round 3: the driver's bench command, variants in separate processes: descriptor replicas, wave priority, keypoint grids, kernel flavours
L=sift-project_amd/alt
bash tools/bench_ab.sh r03v 6 base SIFT_HIP_LIB=$L/reps16/libsift_hip.so SIFT_HIP_LIB=$L/prio0/libsift_hip.so SIFT_KP_WGS=512,SIFT_DESC_WGS=512 SIFT_ORI_MODE=0 SIFT_DESC_MODE=3 || exit 1
export SIFT_HIP_LIB=$(pwd)/$L/reps16/libsift_hip.so
bash tools/pmc_kp.sh r03v/sq16 > gpurun_out/r03v/sq16.log 2>&1 || { tail -5 gpurun_out/r03v/sq16.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r03v/sq16/pass1/*counter_collection.csv gpurun_out/r03v/sq16/pass2/*counter_collection.csv > gpurun_out/r03v/sq16_summary.txt && grep -E "kernel|descriptor" gpurun_out/r03v/sq16_summary.txt | cut -c1-200
rm -rf gpurun_out/r03v/sq16/pass*/*.csv.gz
