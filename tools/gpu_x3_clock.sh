#!/bin/bash
# Effective clock and MFMA-busy per x3 GEMM variant (GATX_X3_DBG=...), PPI L1 projection shape.
#   DBGS="0 5 6" bash tools/gpu_x3_clock.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 5}; do
  echo "== dbg$d"
  GATX_X3_DBG=$d timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d "$O/c$d" -o run --output-format csv -- python3 "$R/tools/gemm_one.py" 1 nt 44900 1024 1024 20 > "$O/c$d.log" 2>&1 || exit 1
  python3 - "$O/c$d" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list); dur = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_x3" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
d = sum(dur.values()) / len(dur)
m = {k: sum(v) / len(v) for k, v in acc.items()}
print(f"dur {d:.1f} us  clk {m['GRBM_GUI_ACTIVE']/8/(d*1e-6)/1e9:.2f} GHz  mfma_busy/cu-cycle "
      f"{m['SQ_VALU_MFMA_BUSY_CYCLES']/(m['GRBM_GUI_ACTIVE']/8*256*4):.3f}  valu/mfma {m['SQ_INSTS_VALU']/m['SQ_INSTS_MFMA']:.2f}"
      f"  lds/mfma {m['SQ_INSTS_LDS']/m['SQ_INSTS_MFMA']:.2f}")
PY
done
