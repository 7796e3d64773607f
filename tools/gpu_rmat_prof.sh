#!/bin/bash
# Kernel-trace breakdown of the full-size RMAT fwd+bwd step, backward hub splitting on and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for h in 1 0; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_h$h" -o run --output-format csv -- python3 "$R/bench.py" --tune bwd_hubs=$h --workload rmat --mode train --steps 2 --warmup 2 --no-cpu-baseline > "$OUT/prof_h$h.log" 2>&1 || exit 1
  python3 "$R/tools/trace_window.py" "$OUT/prof_h$h" "$OUT/breakdown_h$h.txt" | head -16
done
