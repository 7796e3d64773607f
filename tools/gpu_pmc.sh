#!/bin/bash
# HBM / L2 counters per kernel over bench.py's timed steps, one rocprofv3 --pmc pass per counter
# group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; counters only with
# --kernel-trace). tools/pmc_summary.py then keeps the dispatches between bench.py's region marks.
#   bash tools/gpu_pmc.sh TAG NAME [bench args...]   -> gpurun_out/TAG/NAME_p1..p4
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}; NAME=${2:-pmc}
shift 2
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/${NAME}_p$i" -o run \
    --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-train-leg "$@" \
    > "$OUT/${NAME}_p$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
