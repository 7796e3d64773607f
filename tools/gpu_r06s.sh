#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06s; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_lds.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r06s_ab 2 "" "-" "--tune edge_lds=0" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU -d "$OUT/p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/p1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/p2" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/p2.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for p in ("p1", "p2"):
    f = glob.glob(f"{o}/{p}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        if "edge_lds" in k or "edge_forward_kernel" in k:
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        print(p, k, {a: round(b) for a, b in d.items()})
PY
