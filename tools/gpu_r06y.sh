#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06y; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "--workload pattern --graphs 8 --mode train" "--graphs 2 --mode train" "" "--mode train"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > $OUT/b.json 2> $OUT/b.err || exit 1
  python -c "import json; d=json.load(open('$OUT/b.json')); print('$a', d['ms_per_step'])"
done
