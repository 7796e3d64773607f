#!/bin/bash
# round 6: windowed node-block build: its tests, then traces with side stream on / off
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r08d; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_blocks.py tests/test_gpu_edge_lds.py tests/test_gpu_capture.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_lib_trace.sh r08d_s1 "" gat-pytorch_amd/gatx/libgatx.so || exit 1
bash tools/gpu_lib_trace.sh r08d_s0 "--tune side_stream=0" gat-pytorch_amd/gatx/libgatx.so || exit 1
bash tools/gpu_ab.sh r08d_ab 3 "" "-" "--tune side_stream=0"
