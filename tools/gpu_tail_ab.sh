#!/bin/bash
# In-situ A/B of the GEMM tail split on the PPI forward / train benches (tuning only).
#   bash tools/gpu_tail_ab.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd "$R"
exec 3>&1
step() { echo "== $1" >&3; shift; "$@"; rc=$?; echo "rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
for ts in auto 1 2 4; do
  if [ $ts = auto ]; then e=""; else e="GATX_TAIL_SPLIT=$ts"; fi
  step fwd_$ts env $e timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/fwd_$ts.json" 2> "$OUT/fwd_$ts.err"
done
for ts in auto 1 2 4; do
  python -c "import json;d=json.load(open('$OUT/fwd_$ts.json'));print('$ts', d['ms_per_step'], d['kernels']['gemm'])" >&3
done
