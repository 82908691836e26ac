bash tools/gpu_session.sh r05_check test bench
