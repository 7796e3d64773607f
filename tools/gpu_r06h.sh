#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06h; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_graph_blocks.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -15 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06h_ab 2 "" "-" "--tune edge_lds=1" && bash tools/gpu_lab.sh r06h_lab
