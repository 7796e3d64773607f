#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06m; mkdir -p $OUT; cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --tune edge_lds=1 --verify > $OUT/b1.json 2> $OUT/b1.err; rc=$?; tail -2 $OUT/b1.err; [ $rc -ne 0 ] && exit $rc
python -c "import json;d=json.load(open('$OUT/b1.json'));print(d['ms_per_step'])"
