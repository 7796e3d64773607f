#!/bin/bash
# Working session: full GPU suite, the forward / train / PATTERN-train bench lines, the train
# step's kernel trace, and the train bench with the f16p / f16rc kernels off (A/B).
#   bash tools/gpu_session.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log" >&3
fi
step bench timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench_train timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
step bench_train_nof16p env GATX_F16P=0 timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train_nof16p.json" 2> "$OUT/bench_train_nof16p.err"
if [ "${PPAB:-0}" = 1 ]; then
  step bench_nopp env GATX_F16P_PP=0 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_nopp.json" 2> "$OUT/bench_nopp.err"
  step bench_train_nopp env GATX_F16P_PP=0 timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > "$OUT/bench_train_nopp.json" 2> "$OUT/bench_train_nopp.err"
fi
step bench_pattern timeout -k 10 300 python bench.py --workload pattern --graphs 8 --mode train --no-cpu-baseline > "$OUT/bench_pattern_train.json" 2> "$OUT/bench_pattern_train.err"
cd /tmp && export TMPDIR=/tmp
step prof_train timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.log" 2>&1
step prof_pattern timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pattern" -o run --output-format csv -- python3 "$R/bench.py" --workload pattern --graphs 8 --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_pattern.log" 2>&1
cd "$R"
if [ "${LAB:-1}" = 1 ]; then
  step lab timeout -k 10 300 python tools/gemm_lab/run_lab.py > "$OUT/lab.txt" 2>&1
  cat "$OUT/lab.txt" >&3
fi
python - "$OUT" >&3 <<'PY'
import json, sys
o = sys.argv[1]
import os
for f in ("bench", "bench_train", "bench_train_nof16p", "bench_bk32", "bench_train_bk32",
          "bench_nopp", "bench_train_nopp", "bench_pattern_train"):
    if not os.path.exists(f"{o}/{f}.json"):
        continue
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d.get("roofline_time_frac"))
    print("  ", {k: round(v["total_ms_per_step"], 4) for k, v in d.get("kernels", {}).items()})
PY
echo "all done" >&3
