#!/bin/bash
# SQ counters of the edge-pass lab's gather and LDS kernels (one pass per counter group).
#   bash tools/gpu_lab_pmc.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/$1; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
L=$R/tools/edge_lab/edge_lab
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU -d "$OUT/p1" -o run --output-format csv -- "$L" q > "$OUT/p1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/p2" -o run --output-format csv -- "$L" q > "$OUT/p2.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for p in ("p1", "p2"):
    f = glob.glob(f"{o}/{p}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(p, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        print(p, k, {a: round(b) for a, b in d.items()})
PY
