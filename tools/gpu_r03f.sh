#!/bin/bash
# Round-3 iteration: full GPU suite, PATTERN G=8 train breakdown, PPI train step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03f}; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
TESTS="" BENCH_ARGS="--workload pattern --graphs 8 --mode train" bash tools/gpu_iter.sh ${1:-r03f}_pat > /dev/null 2>&1 || exit 1
head -3 gpurun_out/${1:-r03f}_pat/breakdown.txt; python -c "import json;print(json.load(open('gpurun_out/${1:-r03f}_pat/bench.json'))['ms_per_step'])"
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > $OUT/train.json 2> $OUT/train.err; python -c "import json;print('ppi train', json.load(open('$OUT/train.json'))['ms_per_step'])"
