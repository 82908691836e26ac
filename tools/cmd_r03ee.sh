# round 3: graph segments: the graph tests first, then the whole GPU suite and the bench with graphs on / off
SIFT_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q -k "u8_and_device or graph_replay" --timeout 120 --timeout-method thread > gpurun_out/r03ee_graph.log 2>&1
grep -i "sift_hip:\|passed\|failed" gpurun_out/r03ee_graph.log | head; grep -q "2 passed" gpurun_out/r03ee_graph.log || exit 1
bash tools/cmd_r03dd.sh
