# round 3: pyramid wave priority variants; 20-step pipelined runs (the driver's bench shape) and steady state
L=sift-project_amd/alt
V="base SIFT_HIP_LIB=$L/prio_pyr/libsift_hip.so SIFT_HIP_LIB=$L/prio_lds/libsift_hip.so SIFT_HIP_LIB=$L/prio_tl/libsift_hip.so SIFT_HIP_LIB=$L/prio_all1/libsift_hip.so"
export AB_ARGS="--rounds 40 --steps 20 $V"
export AB2_ARGS="--rounds 6 --steps 300 $V"
export AB3_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 $V"
bash tools/gpu_session.sh r03o ab ab2 ab3
