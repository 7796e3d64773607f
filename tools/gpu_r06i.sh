#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06i; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_graph_blocks.py tests/test_gpu_capture.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06i_ab 2 "" "-" "--tune edge_lds=1" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_lds" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --tune edge_lds=1 > "$OUT/prof_lds.log" 2>&1 || exit 1
python3 "$R/tools/trace_window.py" "$OUT/prof_lds" | head -40
