# round 3: stream policy (one normal-priority stream per pipelined job, burst hint)
V="base SIFT_STREAM_POLICY=1"
export AB_ARGS="--rounds 40 --steps 20 $V"
export AB2_ARGS="--rounds 6 --steps 300 $V"
export AB3_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 $V"
bash tools/gpu_session.sh r03s ab ab2 ab3 || exit 1
export AB_ARGS="--rounds 6 --steps 150 DEPTH=1 DEPTH=1,SIFT_STREAM_POLICY=1"
bash tools/gpu_session.sh r03s/lat ab || exit 1
O=gpurun_out/r03s/hq8; mkdir -p $O
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 40 --steps 20 $V > $O/ab20.txt 2>&1 && grep -v amdgpu.ids $O/ab20.txt
