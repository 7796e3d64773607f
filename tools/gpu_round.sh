#!/bin/bash
# One GPU session that refreshes everything the round reports: GPU parity tests, the default
# bench (with CPU baseline), the train / RMAT / PATTERN benches, rocprofv3 kernel traces of the
# forward / train / RMAT / PATTERN-train benches and the windowed PMC passes for the forward and
# RMAT. Every GPU step has its own time limit; the first failure ends the script.
#   bash tools/gpu_round.sh TAG [PART]   (then: bash tools/snapshot_round.sh TAG)
# PART: all (default) | bench (tests, benches, traces) | pmc (the counter passes): a whole refresh
# can outlast one gpurun call's time limit, so it can run as two calls into the same TAG.
R=${GRAFT_REPO_ROOT:-$(pwd)}
PART=${2:-all}
OUT=$R/gpurun_out/$1
mkdir -p "$OUT"
exec 3>&1   # progress lines go to the call's stdout, never into a step's redirected output
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "$PART" != pmc ]; then
step tests timeout -k 10 900 python -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  --junitxml="$OUT/gpu_tests.xml" > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
step bench timeout -k 10 300 python "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench_train timeout -k 10 300 python "$R/bench.py" --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
step bench_rmat timeout -k 10 400 python "$R/bench.py" --workload rmat --steps 5 --warmup 2 > "$OUT/bench_rmat.json" 2> "$OUT/bench_rmat.err"
step bench_ppi2 timeout -k 10 300 python "$R/bench.py" --graphs 2 --mode train --no-cpu-baseline > "$OUT/bench_ppi2_train.json" 2> "$OUT/bench_ppi2_train.err"
step bench_pattern timeout -k 10 300 python "$R/bench.py" --workload pattern --graphs 8 --mode train --no-cpu-baseline > "$OUT/bench_pattern_train.json" 2> "$OUT/bench_pattern_train.err"
cd /tmp && export TMPDIR=/tmp
step prof_fwd timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fwd" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-leg > "$OUT/prof_fwd.log" 2>&1
step prof_train timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.log" 2>&1
step prof_rmat timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat" -o run --output-format csv -- python3 "$R/bench.py" --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_rmat.log" 2>&1
step prof_pattern timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pattern" -o run --output-format csv -- python3 "$R/bench.py" --workload pattern --graphs 8 --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_pattern.log" 2>&1
fi
[ "$PART" = bench ] && { echo "bench part done"; exit 0; }
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  step pmc$i timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmc_p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-train-leg > "$OUT/pmc_p$i.log" 2>&1
done
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  step pmct$i timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmct_p$i" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmct_p$i.log" 2>&1
done
step pmc_rmat bash "$R/tools/gpu_pmc_rmat.sh" "$1"
echo "all done"
