#!/bin/bash
# gemm_out (PPI layer 0 output projection, small-K path) under rocprofv3: kernel stats + PMC.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/skpmc; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks -o run --output-format csv -- python3 $R/tools/gemm_out_lab.py > $O/ks.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/tools/gemm_out_lab.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
