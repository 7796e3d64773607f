#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06n; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --tune edge_lds=1 > "$OUT/prof.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
for r in rows:
    n = r["Kernel_Name"]
    if "edge_lds" in n or "region_mark" in n:
        print(r["Dispatch_Id"], n[:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY
grep -o '"ms_per_step": [0-9.]*' "$OUT/prof.log"
