#!/bin/bash
# GEMM lab, library kernel against the lab's ping-pong references only (tuning only), then the
# PPI forward bench.   bash tools/gemm_lab/lab_lib.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
LAB_ONLY="lib f16p,v6,v7" timeout -k 10 300 python -u tools/gemm_lab/run_lab.py > "$OUT/lab.txt" 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/fwd_a.json" 2> "$OUT/fwd_a.err" &&
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/fwd_b.json" 2> "$OUT/fwd_b.err" &&
python -c "
import json
for f in ('fwd_a', 'fwd_b'):
    d = json.load(open('$OUT/' + f + '.json'))
    print(f, d['ms_per_step'], d['kernels']['gemm'])
"
