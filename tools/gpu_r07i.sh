#!/bin/bash
# absmax_rows_cols geometry change: its tests, the gradient parity at the headline batch, train bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r07i; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_headline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > $OUT/bt_$r.json 2> $OUT/bt_$r.err || exit 1
python -c "import json; d=json.load(open('$OUT/bt_$r.json')); k=d['kernels']; print(d['ms_per_step'], {n: round(k[n]['avg_ms'],4) for n in ('bwd_gaug_stats','bwd_gemm_gw','bwd_gemm_gx') if n in k})"
done
