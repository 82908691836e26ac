SWEEP="base SIFT_SHARED_STREAMS=1,SIFT_TILE_PX_LOG2=-1 SIFT_TILE_PX_LOG2=19" REPS=2 SWEEP_OUT=sw_sync.txt BENCH_ARGS="--steps 500 --warmup 10 --sync" tools/sweep.sh | grep mean
SWEEP="base SIFT_SHARED_STREAMS=1 SIFT_SHARED_STREAMS=1,SIFT_TILE_PX_LOG2=-1" REPS=2 SWEEP_OUT=sw_b8.txt BENCH_ARGS="--steps 100 --warmup 5 --batch 8" tools/sweep.sh | grep mean
