#!/bin/bash
# A/B of x3 GEMM main-loop variants (GATX_X3_DBG values in $VARIANTS, 0 = as shipped) on the PPI
# projection / g_x shapes, interleaved so all variants see the same clocks; the first round also
# checks each variant's result against fp64.   VARIANTS="0 10 11" bash tools/gpu_x3_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
run() { timeout -k 10 60 env GATX_X3_DBG=$1 python "$R/tools/gemm_one.py" 1 $2 $3 $4 $5 30 >> "$O/ab.txt" 2>&1 || exit $?; }
for rep in 1 2 3; do
  for shp in "nt 44900 1024 50" "nt 44900 1024 1024" "nt 44900 847 1024" "nt 8192 4096 4096"; do
    for v in ${VARIANTS:-0}; do
      echo "dbg=$v $shp" >> "$O/ab.txt"
      if [ $rep = 1 ]; then GEMM_CHECK=1 run $v $shp; else run $v $shp; fi
    done
  done
done
grep -v amdgpu.ids "$O/ab.txt"
