#!/bin/bash
# hipGraph vs eager on the small, launch-bound workloads (+ the headline), one line each.
#   bash tools/gpu_graphs.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['ms_per_step'], round(d['value']/1e6,1), 'M', d['config'].get('launch'))" "$1" >&3; }
for cfg in "pat8_fwd --workload pattern --graphs 8" "pat8_train --workload pattern --graphs 8 --mode train" "pat32_train --workload pattern --graphs 32 --mode train" "ppi2_fwd --graphs 2" "ppi20_fwd"; do
  set -- $cfg; n=$1; shift
  for g in off on; do
    step "$n/$g" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --hipgraph $g "$@" > "$OUT/${n}_$g.json" 2> "$OUT/${n}_$g.err"
    summ "$OUT/${n}_$g.json"
  done
done
echo "all done"
