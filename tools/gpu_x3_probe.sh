#!/bin/bash
# Where the x3 GEMM's time goes on the PPI L1 projection shape (44900 x 1024 x 1024): the kernel
# as built and its tuning probes (GATX_X3_DBG=1..4, wrong results), then PMC passes on the
# shipped kernel.   bash tools/gpu_x3_probe.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
SHAPE="44900 1024 1024"
for d in ${DBGS:-0 1 2 3 4}; do
  step "dbg$d" env GATX_X3_DBG=$d timeout -k 10 60 python "$R/tools/gemm_one.py" 1 nt $SHAPE 20 > "$O/dbg$d.txt" 2>&1
  cat "$O/dbg$d.txt" >&3
done
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  step "pmc$i" timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$O/p$i" -o run --output-format csv -- python3 "$R/tools/gemm_one.py" 1 nt $SHAPE 5 > "$O/p$i.log" 2>&1
done
echo done
