# round 3: per-image keypoint workgroups (cap 1024) for 8-image and single-image jobs
export AB_ARGS="--rounds 6 --steps 300 base SIFT_KP_WGS=160,SIFT_DESC_WGS=160 SIFT_KP_WGS=224,SIFT_DESC_WGS=224 SIFT_KP_WGS=160,SIFT_DESC_WGS=224 SIFT_ORI_MODE=0"
export AB2_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 base SIFT_KP_WGS=64,SIFT_DESC_WGS=64 SIFT_KP_WGS=96,SIFT_DESC_WGS=96 SIFT_KP_WGS=192,SIFT_DESC_WGS=192,SIFT_KP_WGS_MAX=1536"
bash tools/gpu_session.sh r03k test ab ab2 bench
