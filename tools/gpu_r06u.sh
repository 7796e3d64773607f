#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06u; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_capture.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06u_ab 3 "" "-" "--tune side_stream=0" || exit 1
bash tools/gpu_ab.sh r06u_abt 2 "--mode train" "-" "--tune side_stream=0" || exit 1
