#!/bin/bash
# LDS-staged radix scatter (default) vs the direct scatter (GATX_RADIX_LDS=0): graph-build parity
# tests, then PPI and RMAT benches for both (graph-build share of the step).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/radix_ab; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider -k "graph or golden or hub or csr or build or sort or rmat or pattern" --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -n 1 "$OUT/tests.log"
for rep in 1 2; do
  for v in 1 0; do
    GATX_RADIX_LDS=$v timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline > "$OUT/p$v.json" 2> "$OUT/p$v.err" || exit 1
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print('ppi lds=' + sys.argv[2], d['ms_per_step'])" "$OUT/p$v.json" $v
  done
done
for v in 1 0; do
  GATX_RADIX_LDS=$v timeout -k 10 300 python "$R/bench.py" --workload rmat --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/r$v.json" 2> "$OUT/r$v.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('rmat lds=' + sys.argv[2], d['ms_per_step'])" "$OUT/r$v.json" $v
done
