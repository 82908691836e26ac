export AB_ARGS="--rounds 6 --steps 200 base SIFT_HIP_LIB=sift-project_amd/alt/old/libsift_hip.so SIFT_HIP_LIB=sift-project_amd/alt/pf2/libsift_hip.so"
export AB2_ARGS="--rounds 4 --steps 100 SIFT_SERIAL=1,DEPTH=1 SIFT_SERIAL=1,DEPTH=1,SIFT_HIP_LIB=sift-project_amd/alt/old/libsift_hip.so SIFT_SERIAL=1,DEPTH=1,SIFT_HIP_LIB=sift-project_amd/alt/pf2/libsift_hip.so"
O=gpurun_out/r03d
bash tools/gpu_session.sh r03d test ab ab2 || exit 1
timeout -k 10 300 python3 bench.py --exchange --steps 1000 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/bench_exchange.json 2> $O/bench_exchange.err || { tail -20 $O/bench_exchange.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/bench_noexchange.json 2> $O/bench_noexchange.err || exit 1
python3 -c "import json; a=json.load(open('$O/bench_exchange.json')); b=json.load(open('$O/bench_noexchange.json')); print('exchange', a['value'], a.get('exchange_check'), 'noexchange', b['value'])"
bash tools/gpu_session.sh r03d bench prof
