# round 3: jobs in flight x hardware queues, 20-step runs (driver shape) and steady state
V="DEPTH=4 DEPTH=3 DEPTH=5 DEPTH=6 DEPTH=8"
O=gpurun_out/r03q; mkdir -p $O
for hq in 4 8; do
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 30 --steps 20 $V > $O/ab20_hq$hq.txt 2>&1 || { tail $O/ab20_hq$hq.txt; exit 1; }
  grep -v amdgpu.ids $O/ab20_hq$hq.txt
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 5 --steps 300 $V > $O/ab300_hq$hq.txt 2>&1 || { tail $O/ab300_hq$hq.txt; exit 1; }
  grep -v amdgpu.ids $O/ab300_hq$hq.txt
done
