# round 3: wavefront-per-keypoint orientation vs the workgroup variant; keypoint workgroup counts
export AB_ARGS="--rounds 6 --steps 300 base SIFT_ORI_MODE=0 SIFT_KP_WGS=256 SIFT_KP_WGS=1024 SIFT_DESC_WGS=128 SIFT_DESC_WGS=192 SIFT_DESC_WGS=256 SIFT_DESC_WGS=256,SIFT_KP_WGS=256"
export AB2_ARGS="--rounds 4 --steps 100 SIFT_SERIAL=1,DEPTH=1 SIFT_SERIAL=1,DEPTH=1,SIFT_ORI_MODE=0"
bash tools/gpu_session.sh r03i test ab ab2
