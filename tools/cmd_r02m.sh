set -o pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 600 python -u -m pytest tests/test_stitch.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02m/t.log 2>&1 || { tail -40 gpurun_out/r02m/t.log; exit 1; }
tail -8 gpurun_out/r02m/t.log
timeout -k 10 120 python sift-project_amd/sift_stitch.py tests/golden/stitch --out gpurun_out/r02m/pano.png || exit 1
