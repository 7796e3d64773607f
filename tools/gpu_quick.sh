#!/bin/bash
# Quick GPU iteration: selected GPU tests, optional lab tools, fwd (and train) bench kernel
# breakdown.   bash tools/gpu_quick.sh "<pytest -k expr>" "<tool.py ...>;<tool2.py ...>" [train]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/quick; mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ -n "$1" ]; then
  step tests timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -q -k "$1" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  tail -2 "$OUT/tests.log"
fi
IFS=';' read -ra TOOLS <<< "$2"
for t in "${TOOLS[@]}"; do
  [ -z "$t" ] && continue
  step "tool $t" timeout -k 10 300 python $R/tools/$t > "$OUT/tool.log" 2>&1
  grep -v amdgpu.ids "$OUT/tool.log"
done
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],{k:round(v['total_ms_per_step'],3) for k,v in d['kernels'].items()})" "$1"; }
step bench timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline > "$OUT/b.json" 2> "$OUT/b.err"
summ "$OUT/b.json"
if [ "$3" = "train" ]; then
  step train timeout -k 10 200 python "$R/bench.py" --mode train --no-cpu-baseline > "$OUT/t.json" 2> "$OUT/t.err"
  summ "$OUT/t.json"
fi
