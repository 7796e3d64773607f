#!/bin/bash
# Head-group sweep for the head-mean edge pass (PPI L2): GATX_MEAN_HEADS = 1, 2, 3, 6 in the
# forward bench; per-kernel times from the bench's HIP events.   bash tools/gpu_sweep_mean.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
for hm in 6 3 2 1; do
  step "mean_heads=$hm" env GATX_MEAN_HEADS=$hm timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline > "$OUT/mean$hm.json" 2> "$OUT/mean$hm.err"
  python - "$OUT/mean$hm.json" <<'PY' >&3
import json,sys
d=json.load(open(sys.argv[1]))
print(d['ms_per_step'], {k: round(v['total_ms_per_step'],4) for k,v in d['kernels'].items() if k in ('edge_forward','attention_alpha')})
PY
done
echo done
