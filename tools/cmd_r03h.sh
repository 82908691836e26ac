# round 3: marginal pipelined cost per kernel family (SIFT_LAB_DOUBLE), fewer keypoint workgroups
export AB_ARGS="--rounds 6 --steps 300 base SIFT_LAB_DOUBLE=1 SIFT_LAB_DOUBLE=2 SIFT_LAB_DOUBLE=4 SIFT_LAB_DOUBLE=8 SIFT_LAB_DOUBLE=16 SIFT_DESC_WGS=256 SIFT_DESC_WGS=384 SIFT_KP_WGS=256"
bash tools/gpu_session.sh r03h ab
