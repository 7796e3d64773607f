#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06q; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -15 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 1
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > $OUT/bt.json 2> $OUT/bt.err || exit 1
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline --tune edge_lds=0 > $OUT/bt0.json 2> $OUT/bt0.err || exit 1
python - $OUT <<'PY'
import json, sys
for f in ("b", "bt", "bt0"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["ms_per_step"], d.get("ms_per_step_alpha_deferred"))
PY
