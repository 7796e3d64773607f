#!/bin/bash
# PlanetoidGAT steps (Cora / Citeseer / Pubmed), train + fwd, one line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['ms_per_step'], round(d['value']/1e6,1), 'M', d['config'].get('launch'), (d.get('cpu_baseline') or {}).get('value'))" "$1" >&3; }
for w in cora citeseer pubmed; do
  for m in train fwd; do
    step "$w/$m" timeout -k 10 200 python "$R/bench.py" --workload $w --mode $m > "$OUT/${w}_$m.json" 2> "$OUT/${w}_$m.err"
    summ "$OUT/${w}_$m.json"
  done
done
echo "all done"
