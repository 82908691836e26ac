bash tools/gpu_session.sh r05_final3 big
