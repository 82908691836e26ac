bash tools/gpu_session.sh r05_l test bench timeline
