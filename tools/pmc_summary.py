"""Summarise rocprofv3 --pmc passes over a bench.py run into per-STEP counter figures.

bench.py brackets its timed region with two gatx_region_mark_kernel dispatches (the first one's
grid is `steps` workgroups of 64 lanes). Every pass directory is cut to the dispatches strictly
between its first two marks, so one-off setup kernels (input generators, weight assembly, the
hipGraph capture warm-ups, the post-timing graph rebuild) never count, and the step count comes
from the trace itself, not from a constant. Per kernel: launches per step, mean counter values per
dispatch and mean duration. FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half
the bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md §HBM), so read bytes =
2 x FETCH_SIZE x 1024.

    python tools/pmc_summary.py gpurun_out/TAG/pmc [profiles/pmc_latest.json] [> summary.txt]
(reads every gpurun_out/TAG/pmc_p*/ directory)"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

MARK = "gatx_region_mark_kernel"


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("gatx::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)\(", n)
    return (m.group(1) if m else n)[:60]


def window(rows):
    """rows: dicts with Dispatch_Id, Kernel_Name, Grid_Size (+ counters). Returns (steps, rows of
    the dispatches strictly between the first two region marks)."""
    marks = sorted({int(r["Dispatch_Id"]): r for r in rows if MARK in r["Kernel_Name"]}.items())
    if len(marks) < 2:
        raise ValueError(f"pmc: {len(marks)} region marks in the trace (need 2: run bench.py)")
    (d0, m0), (d1, _) = marks[0], marks[1]
    steps = int(m0["Grid_Size"]) // 64
    if steps <= 0:
        raise ValueError("pmc: region mark without a step count")
    return steps, [r for r in rows if d0 < int(r["Dispatch_Id"]) < d1]


def summarize(passes, source: str = "") -> dict:
    """passes: one list of counter-collection rows per rocprofv3 pass (same program, same
    arguments). Every pass must see the same step count and the same launches per kernel."""
    acc = defaultdict(lambda: defaultdict(list))
    launches = {}
    steps_seen = set()
    for rows in passes:
        steps, win = window(rows)
        steps_seen.add(steps)
        per_kernel = defaultdict(set)
        for r in win:
            name = short(r["Kernel_Name"])
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Dispatch_Id"] not in per_kernel[name]:
                per_kernel[name].add(r["Dispatch_Id"])
                acc[name]["_dur_us"].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for name, ids in per_kernel.items():
            prev = launches.setdefault(name, len(ids))
            if prev != len(ids):
                raise ValueError(f"pmc: {name} launched {prev} vs {len(ids)} times across passes")
    if len(steps_seen) != 1:
        raise ValueError(f"pmc: passes disagree on the step count {sorted(steps_seen)}")
    steps = steps_seen.pop()
    out = {"source": source, "steps": steps,
           "window": "dispatches between bench.py's two gatx_region_mark_kernel marks",
           "kernels": {}}
    for n, cs in acc.items():
        d = {k: sum(v) / len(v) for k, v in cs.items()}
        hit, miss = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
        dur = d.get("_dur_us", 0.0)
        out["kernels"][n] = {
            "launches": launches[n],
            "launches_per_step": launches[n] / steps,
            "dur_us": dur,
            "hbm_read_bytes": 2 * d.get("FETCH_SIZE", 0.0) * 1024,
            "hbm_write_bytes": d.get("WRITE_SIZE", 0.0) * 1024,
            "l2_hit": hit / (hit + miss) if hit + miss else None,
            "clk_GHz": (d["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-6) / 1e9
                        if dur and "GRBM_GUI_ACTIVE" in d else None),
        }
    return out


def step_bytes(pm: dict) -> float:
    """Fabric bytes (read x2-corrected + write) per step: every dispatch in the window counts."""
    return sum((v["hbm_read_bytes"] + v["hbm_write_bytes"]) * v["launches"]
               for v in pm["kernels"].values()) / pm["steps"]


def prefix_bytes_per_step(pm: dict, prefix: str) -> float:
    """Fabric bytes per step of the kernels whose short name starts with `prefix`."""
    return sum((v["hbm_read_bytes"] + v["hbm_write_bytes"]) * v["launches"]
               for k, v in pm["kernels"].items() if k.startswith(prefix)) / pm["steps"]


def read_pass(path: str):
    return list(csv.DictReader(open(path)))


def main(argv):
    base = argv[1]
    files = sorted(glob.glob(os.path.join(base + "_p*", "**", "*counter_collection.csv"),
                             recursive=True))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {base}_p*")
    label = os.environ.get("PMC_SOURCE", "bench.py --steps 3 --warmup 1")
    tag = os.path.basename(os.path.dirname(base.rstrip("/")))
    pm = summarize([read_pass(f) for f in files], f"rocprofv3 --pmc, {label}: {tag}")
    if len(argv) > 2:
        json.dump(pm, open(argv[2], "w"), indent=1)
    print(f"steps in window: {pm['steps']}; fabric bytes per step {step_bytes(pm) / 1e6:.1f} MB")
    print(f"{'kernel':60s} {'per_step':>8s} {'dur_us':>8s} {'FETCHx2_MB':>10s} {'WRITE_MB':>9s} "
          f"{'GB/s':>7s} {'L2hit':>6s} {'clk_GHz':>7s}")
    rows = sorted(pm["kernels"].items(), key=lambda kv: -kv[1]["dur_us"] * kv[1]["launches"])
    for name, v in rows[:28]:
        dur = v["dur_us"]
        by = v["hbm_read_bytes"] + v["hbm_write_bytes"]
        gbs = by / (dur * 1e-6) / 1e9 if dur else 0.0
        hit = v["l2_hit"] if v["l2_hit"] is not None else float("nan")
        clk = v["clk_GHz"] if v["clk_GHz"] is not None else float("nan")
        print(f"{name:60s} {v['launches_per_step']:8.2f} {dur:8.1f} "
              f"{v['hbm_read_bytes'] / 1e6:10.1f} {v['hbm_write_bytes'] / 1e6:9.1f} {gbs:7.0f} "
              f"{hit:6.3f} {clk:7.2f}")


if __name__ == "__main__":
    main(sys.argv)
