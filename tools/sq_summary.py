"""Per-kernel SQ stall shares from tools/gpu_pmc_sq.sh (windowed like tools/pmc_summary.py):
wait (s_waitcnt / barrier) / issue-stall / active instruction cycles as fractions of wave cycles,
and MFMA-busy over busy cycles.   python tools/sq_summary.py gpurun_out/TAG/sq"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import glob  # noqa: E402

from pmc_summary import read_pass, summarize  # noqa: E402

files = sorted(glob.glob(os.path.join(sys.argv[1] + "_p*", "**", "*counter_collection.csv"),
                         recursive=True))
rows = read_pass(files[0])
from collections import defaultdict  # noqa: E402
from pmc_summary import window, short  # noqa: E402
steps, win = window(rows)
acc = defaultdict(lambda: defaultdict(float))
for r in win:
    acc[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':60s} {'wait':>6s} {'issue':>6s} {'active':>6s} {'mfma/busy':>9s}")
for n, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    bc = c.get("SQ_BUSY_CYCLES", 0) or 1
    print(f"{n:60s} {c['SQ_WAIT_ANY'] / wc:6.2f} {c['SQ_WAIT_INST_ANY'] / wc:6.2f} "
          f"{c['SQ_ACTIVE_INST_ANY'] / wc:6.2f} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / bc:9.2f}")
