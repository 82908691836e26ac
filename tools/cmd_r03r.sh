# round 3: workgroup-per-keypoint flavour for octaves >= 1 (SIFT_KP_SMALL_PX=4194304) and its grid
V="base SIFT_KP_SMALL_PX=4194304 SIFT_KP_SMALL_PX=4194304,SIFT_KP_WGS_SMALL=256 SIFT_KP_SMALL_PX=4194304,SIFT_KP_WGS_SMALL=1024"
export AB_ARGS="--rounds 40 --steps 20 $V"
export AB2_ARGS="--rounds 6 --steps 300 $V"
export AB3_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 $V"
bash tools/gpu_session.sh r03r ab ab2 ab3 || exit 1
export AB_ARGS="--rounds 6 --steps 150 DEPTH=1 DEPTH=1,SIFT_KP_SMALL_PX=4194304 DEPTH=1,SIFT_KP_SMALL_PX=4194304,SIFT_KP_WGS_SMALL=256 DEPTH=1,SIFT_KP_SMALL_PX=4194304,SIFT_KP_WGS_SMALL=1024"
bash tools/gpu_session.sh r03r/lat ab
