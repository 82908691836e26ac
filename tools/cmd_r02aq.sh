set -o pipefail
O=gpurun_out/r02aq
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 python -u bench.py --exchange --steps 800 --no-cpu-baseline --no-extra --no-matcher --no-alone > $O/bench_exchange.json 2> $O/bench_exchange.err || { tail -20 $O/bench_exchange.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_exchange.json')); print(d['value'], d['ms_per_step'], d.get('exchange_check'))"
