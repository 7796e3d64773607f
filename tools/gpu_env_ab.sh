#!/bin/bash
# Interleaved A/B of environment switches on the forward bench: for each round, one kernel trace
# per variant (rocprofv3 --kernel-trace, 5 timed steps) and its per-step breakdown filtered by
# KFILTER. Variants are "NAME=VALUE" strings ("-" = no switch).
#   KFILTER=smallk ROUNDS=2 bash tools/gpu_env_ab.sh TAG "-" "GATX_SMALLK_CB=4"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    d="$OUT/r${round}_v$i"
    if [ "$v" = "-" ]; then
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $BENCH_ARGS > "$d.log" 2>&1
    else
      timeout -k 10 300 env "$v" rocprofv3 --kernel-trace -d "$d" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 $BENCH_ARGS > "$d.log" 2>&1
    fi
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$d.log"; exit $rc; }
    python3 "$R/tools/trace_window.py" "$d" "$d.txt" > /dev/null
    echo "== round $round variant $i ($v): $(head -1 "$d.txt")"
    grep -E "${KFILTER:-.}" "$d.txt" | head -${KLINES:-6}
  done
done
