#!/bin/bash
# One rocprofv3 pass of SQ stall counters over the forward bench's timed steps:
#   bash tools/gpu_pmc_sq.sh TAG [bench args...]  -> gpurun_out/TAG/sq_p1
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$OUT/sq_p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-train-leg --steps 3 --warmup 1 "$@" > "$OUT/sq_p1.log" 2>&1
rc=$?; echo "sq pass rc=$rc"; exit $rc
