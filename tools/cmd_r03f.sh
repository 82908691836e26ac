# round 3: wavefront-per-record descriptor (mode 1) vs the 256-thread f32 variant (mode 3)
export AB_ARGS="--rounds 6 --steps 300 base SIFT_DESC_MODE=3 SIFT_HIP_LIB=sift-project_amd/alt/reps8/libsift_hip.so SIFT_HIP_LIB=sift-project_amd/alt/occ6/libsift_hip.so"
export AB2_ARGS="--rounds 4 --steps 100 SIFT_SERIAL=1,DEPTH=1 SIFT_SERIAL=1,DEPTH=1,SIFT_DESC_MODE=3"
O=gpurun_out/r03f
bash tools/gpu_session.sh r03f test ab ab2 prof || exit 1
bash tools/pmc_kp.sh r03f/sq > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq/pass1/*counter_collection.csv $O/sq/pass2/*counter_collection.csv > $O/sq_summary.txt && cut -c1-200 $O/sq_summary.txt
