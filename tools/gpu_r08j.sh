#!/bin/bash
# round 6: head-mean LDS pass: its tests, then traces and an interleaved A/B against the L2 gather
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r08j; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_args_trace.sh r08j_tr "" "-" "--tune edge_lds_mean=0" || exit 1
bash tools/gpu_ab.sh r08j_ab 3 "" "-" "--tune edge_lds_mean=0"
