# round 3: where the small-octave tail goes: kernel-alone per-octave pyramid times vs the first LDS-resident octave
O=gpurun_out/r03ff; mkdir -p $O
for px in 9088 2100 600 150; do
SIFT_LDS_PX=$px timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher --no-desc-f64 --no-extra > $O/lds$px.json 2> $O/lds$px.err || exit 1
python3 -c "import json; d=json.load(open('$O/lds$px.json')); a=d['roofline']['alone']; print('LDS_PX $px', round(d['ms_per_step'],4), 'alone us/img', round(a['us_per_image'],1), [(p['octave'], round(p['us_per_launch'],1)) for p in a['per_octave']])"
done
