# round 3: keypoint workgroup counts (orientation KP_WGS x descriptor DESC_WGS)
export AB_ARGS="--rounds 6 --steps 300 SIFT_KP_WGS=256,SIFT_DESC_WGS=256 SIFT_KP_WGS=128,SIFT_DESC_WGS=128 SIFT_KP_WGS=192,SIFT_DESC_WGS=192 SIFT_KP_WGS=128,SIFT_DESC_WGS=256 SIFT_KP_WGS=256,SIFT_DESC_WGS=128 SIFT_ORI_MODE=0,SIFT_KP_WGS=256,SIFT_DESC_WGS=256 SIFT_ORI_MODE=0,SIFT_KP_WGS=384,SIFT_DESC_WGS=256"
export AB2_ARGS="--rounds 4 --steps 30 --batch 8 --depth 2 base SIFT_KP_WGS=256,SIFT_DESC_WGS=256 SIFT_KP_WGS=128,SIFT_DESC_WGS=128"
bash tools/gpu_session.sh r03j ab ab2
O=gpurun_out/r03j
for v in "512 512" "256 256" "128 128"; do set -- $v
  SIFT_KP_WGS=$1 SIFT_DESC_WGS=$2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-alone --no-desc-f64 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_$1_$2.json')); print('$1 $2', d['ms_per_step'], d['latency']['ms_per_image'], d['batch8']['ms_per_image'], d['api']['ms_per_image'])"
done
