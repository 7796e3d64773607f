#!/bin/bash
# The edge-pass lab (tools/edge_lab) on one box.   bash tools/gpu_lab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R/tools/edge_lab" && timeout -k 10 150 ./edge_lab > "$OUT/edge_lab.txt" 2>&1; rc=$?; cat "$OUT/edge_lab.txt"; exit $rc
