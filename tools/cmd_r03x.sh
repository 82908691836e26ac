# round 3: replica-interleaved descriptor histograms (8 default, 16, 4): GPU tests, LDS counters, the driver's bench command
L=$(pwd)/sift-project_amd/alt
bash tools/gpu_session.sh r03x test || exit 1
for v in base rep16; do
  if [ $v = base ]; then unset SIFT_HIP_LIB; else export SIFT_HIP_LIB=$L/$v/libsift_hip.so; fi
  bash tools/pmc_kp.sh r03x/$v > gpurun_out/r03x_$v.log 2>&1 || { tail -5 gpurun_out/r03x_$v.log; exit 1; }
  python3 tools/sq_summary.py gpurun_out/r03x/$v/pass1/*counter_collection.csv gpurun_out/r03x/$v/pass2/*counter_collection.csv > gpurun_out/r03x/${v}_summary.txt
  rm -rf gpurun_out/r03x/$v/pass*/*.csv.gz
done
unset SIFT_HIP_LIB
bash tools/bench_ab.sh r03x/ab 6 base SIFT_HIP_LIB=$L/rep16/libsift_hip.so SIFT_HIP_LIB=$L/rep4/libsift_hip.so SIFT_HIP_LIB=$L/r02/libsift_hip.so
