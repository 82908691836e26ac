# round 3: orientation window staged in LDS vs gathers
L=sift-project_amd/alt
V="base SIFT_HIP_LIB=$L/nowin/libsift_hip.so SIFT_KP_WGS=128 SIFT_KP_WGS=256"
export AB_ARGS="--rounds 30 --steps 20 $V"
export AB2_ARGS="--rounds 6 --steps 300 $V"
export AB3_ARGS="--rounds 6 --steps 150 DEPTH=1 DEPTH=1,SIFT_HIP_LIB=$L/nowin/libsift_hip.so"
bash tools/gpu_session.sh r03p test ab ab2 ab3
