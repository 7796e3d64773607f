#!/bin/bash
# Interleaved A/B of env settings on the PPI forward bench: per run, the step time and the
# projection GEMM's mean launch time from the bench line.
#   ENVS="A=1;A=2" bash tools/gpu_env_ab2.sh TAG [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
n=${2:-2}
IFS=';' read -ra LIST <<< "$ENVS"
for i in $(seq 1 $n); do
  for e in "${LIST[@]}"; do
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > "$OUT/ab.json" 2> "$OUT/ab.err" || exit $?
    python -c "
import json;d=json.load(open('$OUT/ab.json'));r=d['roofline'];o=d.get('roofline_other') or {}
g=r if r.get('unit')=='TFLOP/s' else o
print('$e', d['ms_per_step'], 'gemm_ms', round(g.get('avg_launch_ms',0),4))"
  done
done
