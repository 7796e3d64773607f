"""Per-step kernel breakdown of a bench.py run under `rocprofv3 --kernel-trace`: the dispatches
between bench.py's two region marks (tools/pmc_summary.py), grouped by kernel: launches per step,
mean duration, time per step; plus the launch count and summed kernel time per step.
    python tools/trace_window.py gpurun_out/TAG/prof_fwd [out.txt]"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import MARK, short  # noqa: E402


def breakdown(rows):
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if MARK in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"{len(marks)} region marks in the trace (need 2)")
    m0, m1 = marks[0], marks[1]
    steps = int(rows[m0]["Grid_Size_X"]) // 64 if "Grid_Size_X" in rows[m0] else \
        int(rows[m0]["Grid_Size"]) // 64
    acc = {}
    for r in rows[m0 + 1:m1]:
        n = short(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c, t = acc.get(n, (0, 0.0))
        acc[n] = (c + 1, t + d)
    return steps, acc


def main(argv):
    f = glob.glob(os.path.join(argv[1], "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel_trace.csv under {argv[1]}")
    steps, acc = breakdown(list(csv.DictReader(open(f[0]))))
    launches = sum(c for c, _ in acc.values()) / steps
    total = sum(t for _, t in acc.values()) / steps
    out = [f"steps in window: {steps}; launches per step {launches:.1f}; "
           f"summed kernel time per step {total:.1f} us",
           f"{'kernel':60s} {'per_step':>8s} {'avg_us':>8s} {'us/step':>8s}"]
    for n, (c, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        out.append(f"{n:60s} {c / steps:8.2f} {t / c:8.1f} {t / steps:8.1f}")
    text = "\n".join(out)
    print(text)
    if len(argv) > 2:
        open(argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main(sys.argv)
