#!/bin/bash
# Full GPU test suite + the four bench lines (fwd, train, RMAT, PATTERN train), no profiler.
# Every GPU step has its own time limit; the first failure ends the script.
#   bash tools/gpu_quick.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
step bench timeout -k 10 300 python bench.py --no-cpu-baseline --no-train-leg > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench_train timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
step bench_rmat timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_rmat.json" 2> "$OUT/bench_rmat.err"
step bench_pattern timeout -k 10 300 python bench.py --workload pattern --graphs 8 --mode train --no-cpu-baseline > "$OUT/bench_pattern_train.json" 2> "$OUT/bench_pattern_train.err"
for f in bench bench_train bench_rmat bench_pattern_train; do
  python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['ms_per_step'], d['value'])"
done
