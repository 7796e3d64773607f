#!/bin/bash
# round 6: deferred epilogue of the concat LDS walk: its tests, a trace and an interleaved A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09c; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py tests/test_gpu_capture.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_args_trace.sh r09c_tr "" "-" "--tune lds_defer=0" || exit 1
bash tools/gpu_ab.sh r09c_ab 3 "" "-" "--tune lds_defer=0"
