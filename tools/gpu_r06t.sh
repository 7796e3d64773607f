#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06t; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_graph_blocks.py tests/test_gpu_capture.py tests/test_gpu_headline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06t_ab 3 "" "-" "--tune edge_lds=0" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "region_mark" in r["Kernel_Name"]]
win = rows[marks[0] + 1: marks[1]]
t0 = int(win[0]["Start_Timestamp"])
for r in win[:60]:
    print(f'{r["Kernel_Name"][:38]:38s} q{r["Queue_Id"]} {(int(r["Start_Timestamp"]) - t0) / 1e3:9.2f} {(int(r["End_Timestamp"]) - t0) / 1e3:9.2f}')
PY
