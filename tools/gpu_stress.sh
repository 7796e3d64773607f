#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/stress; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u tools/stress_capture.py 600 > $OUT/stress.log 2>&1; rc=$?; tail -6 $OUT/stress.log; exit $rc
