#!/bin/bash
# One iteration on the box: selected GPU tests (TESTS, default the layer / hub / golden files),
# the default bench line, and a kernel trace of the forward bench (per-step breakdown with
# tools/trace_window.py). Every GPU step has its own time limit; the first failure ends it.
#   TESTS="tests/test_gpu_hubs.py" BENCH_ARGS="" bash tools/gpu_iter.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
T=${TESTS-tests/test_gpu_layer.py tests/test_gpu_hubs.py}
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider $T -m gpu > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms_per_step',d['ms_per_step'],'value',d['value'])"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $BENCH_ARGS > "$OUT/prof.log" 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 "$R/tools/trace_window.py" "$OUT/prof" "$OUT/breakdown.txt" | head -30
