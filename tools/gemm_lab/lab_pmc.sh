#!/bin/bash
# SQ counters of the GEMM lab's library kernel vs the lab's v6 (tuning only), two passes.
#   bash tools/gemm_lab/lab_pmc.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export LAB_SHAPES=waves LAB_ONLY="lib f16p,v6 ping"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$OUT/p1" -o run --output-format csv -- python3 "$R/tools/gemm_lab/run_lab.py" > "$OUT/p1.log" 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES --kernel-trace -d "$OUT/p2" -o run --output-format csv -- python3 "$R/tools/gemm_lab/run_lab.py" > "$OUT/p2.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
