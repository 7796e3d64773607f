#!/bin/bash
# round 6: head-mean LDS walk on 16 waves (3 set accumulators) instead of 12 (4): its tests, then
# an interleaved library A/B against the previous build and a trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09g; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py tests/test_gpu_capture.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_lib_ab.sh r09g_ab 3 "" tools/ab/libgatx_mean16.so tools/ab/libgatx_base.so || exit 1
bash tools/gpu_lib_trace.sh r09g_tr "" tools/ab/libgatx_mean16.so
