#!/bin/bash
# Round-3 iteration: full GPU suite, PPI forward breakdown, PATTERN G=8 train breakdown, PPI
# train step.   bash tools/gpu_r03f.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03f}
OUT=$R/gpurun_out/$T; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
TESTS="" bash tools/gpu_iter.sh ${T}_fwd > /dev/null 2>&1 || exit 1
head -1 gpurun_out/${T}_fwd/breakdown.txt; python -c "import json;print('ppi fwd', json.load(open('gpurun_out/${T}_fwd/bench.json'))['ms_per_step'])"
TESTS="" BENCH_ARGS="--workload pattern --graphs 8 --mode train" bash tools/gpu_iter.sh ${T}_pat > /dev/null 2>&1 || exit 1
head -1 gpurun_out/${T}_pat/breakdown.txt; python -c "import json;print('pattern train', json.load(open('gpurun_out/${T}_pat/bench.json'))['ms_per_step'])"
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > $OUT/train.json 2> $OUT/train.err; python -c "import json;print('ppi train', json.load(open('$OUT/train.json'))['ms_per_step'])"
