#!/bin/bash
# PMC passes (HBM bytes, L2 hits, clock) over the RMAT bench: bash tools/gpu_pmc_rmat.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  echo "== rmat pmc$i"
  timeout -k 10 400 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/pmcr_p$i" -o run --output-format csv -- python3 "$R/bench.py" --workload rmat --steps 1 --warmup 2 --no-cpu-baseline > "$OUT/pmcr_p$i.log" 2>&1 || exit 1
done
echo done
