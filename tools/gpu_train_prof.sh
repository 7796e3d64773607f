#!/bin/bash
# GPU parity tests, the forward and train bench lines, the rocprofv3 kernel trace of the train
# step and its windowed PMC passes (FETCH / WRITE / L2 / clock), one per counter group.
#   bash tools/gpu_train_prof.sh TAG      (then: python tools/pmc_summary.py gpurun_out/TAG/pmct ...)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log"
fi
step bench timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench_train timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
cd /tmp && export TMPDIR=/tmp
step prof_fwd timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fwd" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_fwd.log" 2>&1
step prof_train timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  step pmct$i timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmct_p$i" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmct_p$i.log" 2>&1
done
echo "all done"
