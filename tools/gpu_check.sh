#!/bin/bash
# Parity + bench check: full GPU tests, then the default bench, PATTERN train, PPI train and RMAT.
#   bash tools/gpu_check.sh TAG [pytest -k expr]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
K=${2:-}
step tests timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -x -q ${K:+-k "$K"} -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], 'rtf', d.get('roofline_time_frac'), 'uniq', d.get('unique_GBps'), 'roof', (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))" "$1"; }
step bench timeout -k 10 300 python "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"; summ "$OUT/bench.json"
step pat_train timeout -k 10 200 python "$R/bench.py" --workload pattern --graphs 8 --mode train --no-cpu-baseline > "$OUT/pat_train.json" 2> "$OUT/pat_train.err"; summ "$OUT/pat_train.json"
step ppi_train timeout -k 10 200 python "$R/bench.py" --mode train --no-cpu-baseline > "$OUT/ppi_train.json" 2> "$OUT/ppi_train.err"; summ "$OUT/ppi_train.json"
step rmat timeout -k 10 400 python "$R/bench.py" --workload rmat --steps 5 --warmup 2 > "$OUT/rmat.json" 2> "$OUT/rmat.err"; summ "$OUT/rmat.json"
echo "all done"
