#!/bin/bash
# Small-batch host-overhead probe: PATTERN (G=8, 32) and PPI G=2 benches, fwd and train, plus a
# rocprofv3 kernel-trace of each so step time can be compared with summed kernel time.
#   bash tools/gpu_small.sh TAG [extra bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p "$OUT"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
run() {   # name, bench args
  local n=$1; shift
  step "$n" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['ms_per_step'], d['value'])" "$OUT/$n.json" "$n" >&3
}
run pat8_fwd --workload pattern --graphs 8 "$@"
run pat8_train --workload pattern --graphs 8 --mode train "$@"
run pat32_train --workload pattern --graphs 32 --mode train "$@"
run ppi2_fwd --graphs 2 "$@"
run ppi2_train --graphs 2 --mode train "$@"
cd /tmp && export TMPDIR=/tmp
for cfg in "pat8_fwd --workload pattern --graphs 8" "pat8_train --workload pattern --graphs 8 --mode train" "ppi2_fwd --graphs 2" "ppi2_train --graphs 2 --mode train"; do
  set -- $cfg
  n=$1; shift
  step "prof_$n" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline "$@" > "$OUT/prof_$n.log" 2>&1
done
echo "all done"
