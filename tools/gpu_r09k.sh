#!/bin/bash
# round 6 candidate (shared pass 2 rows in flight, max pass 2 edges per round, records reuse the
# first sweep's exps): tests, then windowed traces against the previous build
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09k; mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py tests/test_gpu_layer.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_lib_trace.sh r09k_tr "" tools/ab/libgatx_base.so tools/ab/libgatx_cand.so tools/ab/libgatx_base.so tools/ab/libgatx_cand.so
