# world-size-1 RCCL exchange path against the plain pipelined path (the driver's N>1 runs use it)
O=gpurun_out/r03_exchange; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q -k "exchange or fetch_device" --timeout 120 --timeout-method thread 2>&1 | tail -2
for i in 1 2 3 4; do
timeout -k 10 300 python3 bench.py --exchange --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/ex_$i.json 2> $O/ex_$i.err || { tail -20 $O/ex_$i.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-matcher --no-alone --no-desc-f64 > $O/plain_$i.json 2> $O/plain_$i.err || exit 1
python3 -c "
import json
a=json.load(open('$O/ex_$i.json')); b=json.load(open('$O/plain_$i.json'))
print('exchange', round(a['ms_per_step'],4), 'plain', round(b['ms_per_step'],4), 'ratio', round(a['ms_per_step']/b['ms_per_step'],3), a['exchange_check']['records_match_peer_redetect'], a['exchange_check']['slot_checksum_mismatches'], a['exchange_check']['slots_checksummed'])"
done
