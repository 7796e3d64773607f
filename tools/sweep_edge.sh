#!/bin/bash
# In-situ sweep of the edge-pass work-item shape inside the full PPI forward bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for cfg in "1 2048" "2 2048" "2 4096" "1 4096" "4 2048"; do
  set -- $cfg
  GATX_HEADS_PER_ITEM=$1 GATX_EDGE_CHUNK=$2 timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$R/gpurun_out/sw.json'));k=d['kernels'];print('hs=$1 chunk=$2', d['ms_per_step'], round(k['edge_forward']['total_ms_per_step'],3), round(k['gemm']['total_ms_per_step'],3))"
done
