#!/bin/bash
# In-situ A/B of the projection GEMM's epilogue options on the PPI forward: kernel traces of the
# bench forward with the node scores fused into the GEMM (default) and computed by the separate
# score pass (GATX_FUSED_SCORES=0).   bash tools/gpu_gemm_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
cd /tmp && export TMPDIR=/tmp
step fused timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/fused" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/fused.log" 2>&1
step unfused env GATX_FUSED_SCORES=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/unfused" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/unfused.log" 2>&1
cd "$R"
for v in fused unfused; do echo "-- $v" >&3; python tools/trace_window.py "$OUT/$v" 2>&1 | head -12 >&3; done
