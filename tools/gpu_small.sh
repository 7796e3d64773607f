#!/bin/bash
# Small-batch launch overhead: step time vs summed kernel time (rocprofv3 kernel trace) for the
# launch-bound workloads, with the bench's default launch mode (hipGraph replay where it applies).
#   bash tools/gpu_small.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
cd /tmp && export TMPDIR=/tmp
for cfg in "pat8_fwd --workload pattern --graphs 8" "pat8_train --workload pattern --graphs 8 --mode train" "ppi2_fwd --graphs 2" "ppi2_train --graphs 2 --mode train"; do
  set -- $cfg
  n=$1; shift
  step "$n" timeout -k 10 200 python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err"
  step "prof_$n" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline "$@" > "$OUT/prof_$n.log" 2>&1
done
echo "all done"
