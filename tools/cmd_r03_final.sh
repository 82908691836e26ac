# round 3 final: GPU tests, the driver's exact bench command, rocprof kernel-trace summaries (pipelined and serialised)
N=${1:-r03_final}
bash tools/gpu_session.sh $N test bench prof
