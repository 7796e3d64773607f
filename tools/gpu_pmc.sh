#!/bin/bash
# HBM / L2 counters per kernel for a short bench run, one rocprofv3 --pmc pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Counters only with --kernel-trace.
#   bash tools/gpu_pmc.sh TAG [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-pmc}
shift
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/${TAG}_p$i" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" \
    > "$OUT/${TAG}_p$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
