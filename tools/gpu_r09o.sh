#!/bin/bash
# round 6: the backward source pass on the LDS walk (edge_lds_bwd): tests, then windowed train
# traces and an interleaved train A/B against the gather source pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09o; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_args_trace.sh r09o_tr "--mode train" "-" "--tune edge_lds_bwd=0" || exit 1
grep -hE "edge_bwd_src|edge_records_src|edge_lds_kernel|steps in" "$OUT/../r09o_tr/breakdown_v1.txt" "$OUT/../r09o_tr/breakdown_v2.txt"
for r in 1 2; do
  for v in "-" "--tune edge_lds_bwd=0"; do
    [ "$v" = "-" ] && vv="" || vv="$v"
    timeout -k 10 300 python bench.py --mode train --no-cpu-baseline $vv > "$OUT/ab_${r}_${#vv}.json" 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/ab_${r}_${#vv}.json'));print('$v', d['ms_per_step'])"
  done
done
