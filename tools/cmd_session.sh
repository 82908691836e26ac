bash tools/gpu_session.sh r05_o test bench timeline && bash tools/bench_ab.sh r05_o/ab 3 base SIFT_HIP_LIB=sift-project_amd/alt/strip/libsift_hip.so
