#!/bin/bash
# Scaled-RMAT hub-split backward test, then the full-size RMAT fwd+bwd step with the backward's
# hub splitting on and off (--tune bwd_hubs=0|1).   bash tools/gpu_rmat_train.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_hubs.py -m gpu -k rmat > "$OUT/rmat_hub_test.log" 2>&1
rc=$?; tail -3 "$OUT/rmat_hub_test.log"; [ $rc -ne 0 ] && exit $rc
for h in 1 0; do
  timeout -k 10 400 python bench.py --tune bwd_hubs=$h --workload rmat --mode train --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/rmat_train_h$h.json" 2> "$OUT/rmat_train_h$h.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/rmat_train_h$h.json'));print('bwd hubs', $h, d['ms_per_step'])"
done
