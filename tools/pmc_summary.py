"""Summarise rocprofv3 --pmc CSVs (tools/gpu_pmc.sh): per kernel, mean counter value per
dispatch and mean duration. FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports
half the bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md §HBM), so HBM read
bytes = 2 x FETCH_SIZE x 1024 for such kernels.
    python tools/pmc_summary.py gpurun_out/pmc1 [profiles/pmc_latest.json] [> summary.txt]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("gatx::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)\(", n)
    return (m.group(1) if m else n)[:60]


base = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(base + "_p*", "**", "*counter_collection.csv"),
                          recursive=True)):
    seen = set()
    for r in csv.DictReader(open(f)):
        name = short(r["Kernel_Name"])
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (r["Dispatch_Id"],)
        if key not in seen:
            seen.add(key)
            acc[name]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
import json
label = os.environ.get("PMC_SOURCE", "bench.py --steps 3 --warmup 1")
out_json = {"source": "rocprofv3 --pmc, " + label + ": " + os.path.basename(base.rstrip("/").rsplit("/pmc", 1)[0]),
            "steps": int(os.environ.get("PMC_STEPS", "4")), "kernels": {}}
for n, cs in acc.items():
    d = {k: sum(v) / len(v) for k, v in cs.items()}
    out_json["kernels"][n] = {
        "launches": len(cs["_dur_us"]) // max(1, len([d for d in glob.glob(base + "_p*")
                                                       if os.path.isdir(d)])),
        "dur_us": d.get("_dur_us", 0.0),
        # gfx950: FETCH_SIZE counts half the bytes of 16-B/lane coalesced reads -> x2
        "hbm_read_bytes": 2 * d.get("FETCH_SIZE", 0.0) * 1024,
        "hbm_write_bytes": d.get("WRITE_SIZE", 0.0) * 1024,
        "l2_hit": (d.get("TCC_HIT_sum", 0) / (d.get("TCC_HIT_sum", 0) + d.get("TCC_MISS_sum", 0))
                   if d.get("TCC_HIT_sum", 0) + d.get("TCC_MISS_sum", 0) else None)}
if len(sys.argv) > 2:
    json.dump(out_json, open(sys.argv[2], "w"), indent=1)
rows = sorted(((n, {k: sum(v) / len(v) for k, v in cs.items()}) for n, cs in acc.items()),
              key=lambda x: -x[1].get("_dur_us", 0) * len(acc[x[0]]["_dur_us"]))
print(f"{'kernel':60s} {'dur_us':>8s} {'FETCHx2_MB':>10s} {'WRITE_MB':>9s} {'HBM_GB/s':>9s} "
      f"{'L2hit':>6s} {'clk_GHz':>7s}")
for name, d in rows[:24]:
    fs, ws, dur = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0), d.get("_dur_us", 0.0)
    hit, miss = d.get("TCC_HIT_sum", 0), d.get("TCC_MISS_sum", 0)
    hr = hit / (hit + miss) if hit + miss else float("nan")
    hbm = (2 * fs + ws) * 1024 / (dur * 1e-6) / 1e9 if dur else 0.0
    clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (dur * 1e-6) / 1e9 if dur else 0.0
    print(f"{name:60s} {dur:8.1f} {2 * fs / 1024:10.1f} {ws / 1024:9.1f} {hbm:9.0f} {hr:6.3f} "
          f"{clk:7.2f}")
