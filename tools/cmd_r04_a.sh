set -o pipefail
mkdir -p gpurun_out/r04_a
timeout -k 10 120 tools/math64_check 4194304 > gpurun_out/r04_a/math64.txt 2>&1 && cat gpurun_out/r04_a/math64.txt && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "descriptor or math64 or reference_golden or deterministic or batch or async_fetch" > gpurun_out/r04_a/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r04_a/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 6 --steps 200 base SIFT_DESC_MODE=1 SIFT_DESC_MODE=2 > gpurun_out/r04_a/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04_a/ab.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_interleaved.py --rounds 4 --steps 100 --depth 1 base SIFT_DESC_MODE=1 > gpurun_out/r04_a/ab_sync.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04_a/ab_sync.txt; exit $rc
