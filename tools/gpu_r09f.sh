#!/bin/bash
# round 6 evidence on the current library: forward PMC passes (the head-mean LDS pass's traffic)
# and the train-step kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09f; mkdir -p "$OUT"
bash "$R/tools/gpu_pmc.sh" r09f pmc --steps 3 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train" -o run --output-format csv -- python3 "$R/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_train.log" 2>&1 || exit 1
python3 "$R/tools/trace_window.py" "$OUT/prof_train" "$OUT/train_breakdown.txt" | head -40
