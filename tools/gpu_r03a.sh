#!/bin/bash
# Round-3 check: the full GPU suite, then the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03a}; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu > $OUT/gpu_tests.log 2>&1; rc=$?; tail -5 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; head -c 1500 $OUT/bench.json; exit $rc
