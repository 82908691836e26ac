# round 3: pyramid wave priority (s_setprio), LDS-octave start, small-octave kernel flavour
L=sift-project_amd/alt
export AB_ARGS="--rounds 6 --steps 300 base SIFT_HIP_LIB=$L/prio_lds/libsift_hip.so SIFT_HIP_LIB=$L/prio_pyr/libsift_hip.so SIFT_LDS_PX=2100 SIFT_KP_SMALL_PX=1048576"
export AB2_ARGS="--rounds 6 --steps 150 DEPTH=1 DEPTH=1,SIFT_HIP_LIB=$L/prio_lds/libsift_hip.so DEPTH=1,SIFT_HIP_LIB=$L/prio_pyr/libsift_hip.so DEPTH=1,SIFT_LDS_PX=2100 DEPTH=1,SIFT_KP_SMALL_PX=1048576"
bash tools/gpu_session.sh r03n test ab ab2
