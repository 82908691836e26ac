mkdir -p gpurun_out/r05_lds8 && \
timeout -k 10 120 tools/lds_lab 3840 2160 6 10 > gpurun_out/r05_lds8/lds_1080p.txt 2>&1 && \
timeout -k 10 120 tools/lds_lab 15360 8640 8 10 > gpurun_out/r05_lds8/lds_8k.txt 2>&1 && \
timeout -k 10 120 tools/lds_lab 3840 2160 5 10 > gpurun_out/r05_lds8/lds_1080p_o5.txt 2>&1 && \
grep -A7 "per launch" gpurun_out/r05_lds8/*.txt && \
bash tools/gpu_session.sh r05_k test
