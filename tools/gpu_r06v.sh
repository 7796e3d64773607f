#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06v; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06v_ab 2 "" "-" "--tune edge_lds=0" || exit 1
cd /tmp && export TMPDIR=/tmp
for sd in 1 0; do
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_t$sd" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline --tune side_stream=$sd > "$OUT/prof_t$sd.log" 2>&1 || exit 1
python3 - "$OUT/prof_t$sd" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "region_mark" in r["Kernel_Name"]]
win = rows[marks[0] + 1: marks[1]]
t0, t1 = int(win[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in win)
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
qs = {}
for r in win: qs[r["Queue_Id"]] = qs.get(r["Queue_Id"], 0) + 1
print(sys.argv[1][-8:], "window us", (t1 - t0) / 1e3, "kernel-sum us", busy / 1e3, "launches", len(win), "queues", qs)
PY
done
