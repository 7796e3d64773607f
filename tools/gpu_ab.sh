#!/bin/bash
# Interleaved A/B of bench.py argument variants on one box (e.g. --tune switches).
#   bash tools/gpu_ab.sh TAG ROUNDS "COMMON ARGS" "VARIANT A ARGS" "VARIANT B ARGS" ...   ("-" = none)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"; shift
ROUNDS=$1; shift
COMMON=$1; shift
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    [ "$v" = "-" ] && v=""
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-train-leg $COMMON $v > "$OUT/v${i}_r${r}.json" 2> "$OUT/v${i}_r${r}.err" || { echo "variant $i round $r failed rc=$?"; tail -5 "$OUT/v${i}_r${r}.err"; exit 1; }
    python - "$OUT/v${i}_r${r}.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {a: round(b["total_ms_per_step"], 4) for a, b in d.get("kernels", {}).items()}
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} {k}")
PY
  done
done
