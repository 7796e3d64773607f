#!/bin/bash
# RMAT bench with and without hub splitting, then the whole GPU suite.  bash tools/gpu_rmat_hubs.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
step rmat_hub timeout -k 10 400 python "$R/bench.py" --workload rmat --steps 5 --warmup 2 --no-cpu-baseline > "$O/rmat_hub.json" 2> "$O/rmat_hub.err"
step rmat_nohub env GATX_HUB_EDGES=0 timeout -k 10 400 python "$R/bench.py" --workload rmat --steps 5 --warmup 2 --no-cpu-baseline > "$O/rmat_nohub.json" 2> "$O/rmat_nohub.err"
for f in rmat_hub rmat_nohub; do python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['kernels']['edge_forward'])" "$O/$f.json" >&3; done
echo done
