#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06p; mkdir -p $OUT; cd $R
for a in mark zeros; do
  timeout -k 10 150 python -u tools/check_lds_replay.py $a > $OUT/$a.log 2>&1 || { tail -5 $OUT/$a.log; exit 1; }
  grep -E "replay [3-7]:|vs gather" $OUT/$a.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_blocks.py tests/test_gpu_edge_lds.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --tune edge_lds=1 > $OUT/b1.json 2> $OUT/b1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b0.json 2> $OUT/b0.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --tune edge_lds=1 > $OUT/b2.json 2> $OUT/b2.err || exit 1
python - $OUT <<'PY'
import json, sys
for f in ("b1", "b0", "b2"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, d["ms_per_step"], d.get("ms_per_step_alpha_deferred"), {k: round(v["avg_ms"] * 1e3, 1) for k, v in d["kernels"].items() if "edge" in k})
PY
