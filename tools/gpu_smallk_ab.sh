#!/bin/bash
# A/B of the small-K output projection's column slice (GATX_SMALLK_NM=128: two 48-KB workgroups
# per CU, vs 256: one 96-KB workgroup): parity tests under the variant, then interleaved PPI
# forward benches (per-kernel ms/step of the first layer's output projection, "gemm_out").
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/smallk_ab; mkdir -p "$OUT"
GATX_SMALLK_NM=128 timeout -k 10 600 python -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider -k "ppi or reassoc or smallk or skip or pattern" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -n 1 "$OUT/tests.log"
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernels'];print(sys.argv[2], d['ms_per_step'], round(k['gemm_out']['total_ms_per_step'],4))" "$1" "$2"; }
for rep in 1 2 3; do
  for nm in 256 128; do
    GATX_SMALLK_NM=$nm timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline > "$OUT/b$nm.json" 2> "$OUT/b$nm.err" || exit 1
    summ "$OUT/b$nm.json" "nm=$nm"
  done
done
