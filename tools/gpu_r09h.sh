#!/bin/bash
# round 6: records pass with nontemporal alpha stores: tests, then an interleaved library A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09h; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_lib_ab.sh r09h_ab 3 "" tools/ab/libgatx_ntalpha.so tools/ab/libgatx_base.so
