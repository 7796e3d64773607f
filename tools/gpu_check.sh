#!/bin/bash
# GPU tests (full -m gpu suite or the given test files), one default bench line and a windowed
# kernel trace of the forward.   bash tools/gpu_check.sh TAG [TEST FILES...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$R"
TESTS=${*:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('fwd', d['ms_per_step'], 'train', d.get('train_ms_per_step'), 'replay', d.get('replay_verified'))"
bash tools/gpu_args_trace.sh "$TAG/tr" "" "-" || exit 1
head -24 "$OUT/tr/breakdown_v1.txt"
