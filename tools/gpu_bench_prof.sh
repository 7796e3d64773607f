#!/bin/bash
# One GPU session on the box: bench.py (with its CPU baseline), then a rocprofv3 kernel-trace
# --stats run of a short bench. Each GPU step runs under its own time limit; any non-zero exit
# ends the script (no further GPU work after a failure).
#   bash tools/gpu_bench_prof.sh TAG [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
shift
timeout -k 10 500 python "$R/bench.py" "$@" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?
echo "bench rc=$rc"
tail -c 4000 "$OUT/bench_$TAG.json"
[ $rc -ne 0 ] && { tail -20 "$OUT/bench_$TAG.err"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$OUT/prof_$TAG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT/prof_$TAG" -name "*stats*"
exit $rc
