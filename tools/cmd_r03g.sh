# round 3: descriptor workgroups / prefetch depth, round-2 library vs now (single-image and 8-image jobs)
export AB_ARGS="--rounds 6 --steps 300 base SIFT_DESC_WGS=1024 SIFT_DESC_WGS=1536 SIFT_HIP_LIB=sift-project_amd/alt/ahead2/libsift_hip.so SIFT_HIP_LIB=sift-project_amd/alt/r02/libsift_hip.so"
export AB3_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 base SIFT_HIP_LIB=sift-project_amd/alt/r02/libsift_hip.so"
bash tools/gpu_session.sh r03g test ab ab3 bench
