# round 3: histogram replica layouts (descriptor 4/8/16, orientation 4/8/16) and locate form, driver's bench command
L=$(pwd)/sift-project_amd/alt
bash tools/bench_ab.sh r03aa 8 SIFT_HIP_LIB=$L/head/libsift_hip.so SIFT_HIP_LIB=$L/b/libsift_hip.so SIFT_HIP_LIB=$L/c/libsift_hip.so SIFT_HIP_LIB=$L/d/libsift_hip.so SIFT_HIP_LIB=$L/e/libsift_hip.so base
