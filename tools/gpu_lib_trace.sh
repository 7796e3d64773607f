#!/bin/bash
# Kernel traces of one bench.py command against each library build (GATX_LIB), windowed to the
# timed steps (tools/trace_window.py): per-kernel time per step, variant by variant.
#   bash tools/gpu_lib_trace.sh TAG "BENCH ARGS" LIB_A LIB_B ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"; shift
COMMON=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  GATX_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_v$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-leg $COMMON > "$OUT/prof_v$i.log" 2>&1 || { echo "variant $i failed rc=$?"; tail -5 "$OUT/prof_v$i.log"; exit 1; }
  echo "== $lib"
  python3 "$R/tools/trace_window.py" "$OUT/prof_v$i" "$OUT/breakdown_v$i.txt" | head -24
done
