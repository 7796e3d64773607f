#!/bin/bash
# bench.py's multi-rank path on one GPU (2 ranks, gloo, both on cuda:0): fwd + train for PPI and
# PATTERN.   bash tools/gpu_multirank.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
export GATX_BENCH_BACKEND=gloo GATX_BENCH_ONE_DEVICE=1
i=0
for args in "--workload ppi" "--workload ppi --mode train" "--workload pattern --graphs 8" "--workload pattern --graphs 8 --mode train"; do
  i=$((i+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500+i)) "$R/bench.py" --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline $args > "$O/mr$i.json" 2> "$O/mr$i.err" || { echo "run $i failed"; tail -20 "$O/mr$i.err"; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['n_gpus'], d['ms_per_step'], round(d['value']/1e9,3), d['config']['parallelism'], d['scaling'])" "$O/mr$i.json" "$args"
done
