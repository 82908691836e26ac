set -o pipefail
O=gpurun_out/r02al
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-seconds 1 > $O/bench$i.json 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench$i.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['launches'], r['avg_launch_us'], r['sampled_jobs'], r['alone']['frac'], r['alone_batch8']['frac'])"
done
