#!/bin/bash
# Round-5 working session: GPU suite (optional), the forward / train bench lines, and the
# forward + train kernel traces cut to the timed steps. Every GPU step has its own time limit;
# the first failure ends the script.
#   bash tools/gpu_r06.sh TAG        (TESTS=0: skip the suite; TRAIN=0: skip the train legs)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "${TESTS:-1}" = 1 ]; then
  step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log" >&3
fi
step bench timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
if [ "${TRAIN:-1}" = 1 ]; then
  step bench_train timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
fi
cd /tmp && export TMPDIR=/tmp
step prof_fwd timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fwd" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_fwd.log" 2>&1
if [ "${TRAIN:-1}" = 1 ]; then
  step prof_train timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.log" 2>&1
fi
cd "$R"
python - "$OUT" >&3 <<'PY'
import json, sys, os
o = sys.argv[1]
for f in ("bench", "bench_train"):
    if not os.path.exists(f"{o}/{f}.json"):
        continue
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["ms_per_step"], d.get("ms_per_step_alpha_deferred"), d["roofline"]["kernel"],
          d["roofline"]["frac"], d.get("roofline_time_frac"))
    print("  ", {k: round(v["total_ms_per_step"], 4) for k, v in d.get("kernels", {}).items()})
PY
echo "all done" >&3
