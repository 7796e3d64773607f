#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06r; mkdir -p $OUT; cd $R
bash tools/gpu_ab.sh r06r_ab 3 "" "-" "--tune edge_lds=0" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
python3 "$R/tools/trace_window.py" "$OUT/prof" > $OUT/window.txt && head -30 $OUT/window.txt
