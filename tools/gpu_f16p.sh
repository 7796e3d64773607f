#!/bin/bash
# f16p session: the new GEMM tests first, then the full GPU test suite, the A/B of the PPI forward
# and the two bench lines. Each step time-limited; the first failure ends the script.
#   bash tools/gpu_f16p.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
step new_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16p or wgrad or absmax" > "$OUT/new_tests.log" 2>&1
tail -8 "$OUT/new_tests.log"
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -3 "$OUT/gpu_tests.log"
step ab timeout -k 10 300 python tools/ab_f16p.py > "$OUT/ab.txt" 2>&1
cat "$OUT/ab.txt"
step bench timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench_train timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
python -c "import json
for f in ('bench','bench_train'):
    d=json.load(open('$OUT/'+f+'.json')); print(f, d['ms_per_step'], d['value'], d.get('ms_per_step_alpha_eager'), d.get('gemm_f16x3_fallback_tiles_per_step'), d['roofline']['kernel'], d['roofline']['frac'], d.get('roofline_time_frac'))
    print({k: round(v['total_ms_per_step'], 4) for k, v in d['kernels'].items()})"
echo "all done"
