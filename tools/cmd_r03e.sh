export AB_ARGS="--rounds 6 --steps 300 base SIFT_HIP_LIB=sift-project_amd/alt/reps8/libsift_hip.so SIFT_HIP_LIB=sift-project_amd/alt/epf3/libsift_hip.so SIFT_HIP_LIB=sift-project_amd/alt/old/libsift_hip.so"
export AB2_ARGS="--rounds 4 --steps 100 SIFT_SERIAL=1,DEPTH=1 SIFT_SERIAL=1,DEPTH=1,SIFT_HIP_LIB=sift-project_amd/alt/reps8/libsift_hip.so SIFT_SERIAL=1,DEPTH=1,SIFT_HIP_LIB=sift-project_amd/alt/epf3/libsift_hip.so"
O=gpurun_out/r03e
bash tools/gpu_session.sh r03e test ab ab2 bench || exit 1
bash tools/pmc_kp.sh r03e/sq > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $(ls $O/sq/pass1/*counter_collection.csv $O/sq/pass2/*counter_collection.csv) > $O/sq_summary.txt && cat $O/sq_summary.txt
