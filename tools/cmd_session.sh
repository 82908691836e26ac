bash tools/gpu_session.sh r05_final6 bench prof big
