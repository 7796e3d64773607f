#!/bin/bash
# RMAT edge pass vs hub piece size: HUBS="2048 4096 16384" bash tools/gpu_rmat_sweep.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
for t in ${HUBS:-2048 4096 8192 16384}; do
  GATX_HUB_EDGES=$t timeout -k 10 400 python "$R/bench.py" --workload rmat --steps 5 --warmup 2 --no-cpu-baseline > "$O/rmat_$t.json" 2> "$O/rmat_$t.err" || exit 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('T', sys.argv[2], d['ms_per_step'], round(d['kernels']['edge_forward']['avg_ms'],2))" "$O/rmat_$t.json" $t
done
