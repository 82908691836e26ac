# round 3: keypoint kernel flavour per batch size, alone-job grids, LDS-octave start; latency timeline
export AB_ARGS="--rounds 6 --steps 300 base SIFT_KP_SMALL_PX=0 SIFT_KP_SMALL_PX=4194304 SIFT_LDS_PX=2100 SIFT_HIP_LIB=sift-project_amd/alt/ext0/libsift_hip.so"
export AB2_ARGS="--rounds 6 --steps 150 DEPTH=1 DEPTH=1,SIFT_KP_SMALL_PX=0 DEPTH=1,SIFT_KP_WGS_ALONE=512 DEPTH=1,SIFT_KP_WGS_ALONE=2048 DEPTH=1,SIFT_LDS_PX=2100 DEPTH=1,SIFT_KP_SMALL_PX=4194304"
bash tools/gpu_session.sh r03m test ab ab2 bench || exit 1
TL_OUT=r03m/tl bash tools/cmd_r03l.sh
