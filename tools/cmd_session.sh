mkdir -p gpurun_out/r05_x && timeout -k 10 400 python3 tools/kernel_alone.py --n 100 base SIFT_HIP_LIB=sift-project_amd/alt/rep16/libsift_hip.so > gpurun_out/r05_x/alone.txt 2>&1 && grep -v amdgpu gpurun_out/r05_x/alone.txt && timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-extra --no-alone --no-cpu-baseline --no-matcher > gpurun_out/r05_x/big_base.json 2> gpurun_out/r05_x/big_base.err && SIFT_HIP_LIB=sift-project_amd/alt/rep16/libsift_hip.so timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-extra --no-alone --no-cpu-baseline --no-matcher > gpurun_out/r05_x/big_rep16.json 2> gpurun_out/r05_x/big_rep16.err && python3 -c "
import json
for f in ('base','rep16'):
    d=json.load(open('gpurun_out/r05_x/big_%s.json'%f)); print(f, d['ms_per_step'], [(c, round(d[c]['ms_per_image'],3), {k:round(v['us_per_image'],1) for k,v in d[c]['keypoint_kernels_alone'].items()}) for c in ('config3','config5')])
"
