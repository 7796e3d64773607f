#!/bin/bash
# Kernel traces of bench.py argument variants (e.g. --tune switches), windowed to the timed steps
# (tools/trace_window.py).   bash tools/gpu_args_trace.sh TAG "COMMON ARGS" "VARIANT A" "VARIANT B" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"; shift
COMMON=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  [ "$v" = "-" ] && v=""
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_v$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-leg $COMMON $v > "$OUT/prof_v$i.log" 2>&1 || { echo "variant $i failed rc=$?"; tail -5 "$OUT/prof_v$i.log"; exit 1; }
  echo "== $v"
  python3 "$R/tools/trace_window.py" "$OUT/prof_v$i" "$OUT/breakdown_v$i.txt" | head -3
done
