#!/bin/bash
# The INTEGRATION.md drop-in (the reference's GATModel.forward around gatx GATLayers, bench.py
# --wiring reference) timed beside gatx's fused wiring: PPI G=20 fwd / train, PATTERN G=8
# fwd / train.   bash tools/gpu_wiring.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['ms_per_step'], round(d['value']/1e9,4), 'G')" "$1" >&3; }
for w in gatx reference; do
  for cfg in "ppi_fwd --workload ppi" "ppi_train --workload ppi --mode train" "pat8_fwd --workload pattern --graphs 8" "pat8_train --workload pattern --graphs 8 --mode train"; do
    set -- $cfg
    n=$1; shift
    step "$w/$n" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --wiring $w "$@" > "$OUT/${n}_$w.json" 2> "$OUT/${n}_$w.err"
    summ "$OUT/${n}_$w.json"
  done
done
echo "all done"
