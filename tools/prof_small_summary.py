"""Step time (bench JSON) vs summed kernel time per step (rocprofv3 kernel stats) for the
small-batch runs of tools/gpu_small.sh. The profiled run executes warmup + steps timed steps plus
the CapturedStep warm-up (2) and the eager instrumented tail; kernels per step are counted over
all executed steps.   python tools/prof_small_summary.py gpurun_out/TAG [out.md]"""
import csv
import json
import os
import sys

base = sys.argv[1]
lines = ["| workload | launch | step ms | kernel ms/step | ratio | launches/step |",
         "|---|---|---|---|---|---|"]
for n in ["pat8_fwd", "pat8_train", "ppi2_fwd", "ppi2_train"]:
    jf = os.path.join(base, f"{n}.json")
    sf = os.path.join(base, f"prof_{n}", "run_kernel_stats.csv")
    if not (os.path.exists(jf) and os.path.exists(sf)):
        continue
    d = json.load(open(jf))
    rows = list(csv.DictReader(open(sf)))
    graph = "hipGraph" in d["config"].get("launch", "")
    steps = d["steps"] + d["warmup"] + (2 if graph else 0)
    # one-off setup kernels (data generation, weight init) launch once: drop them
    per = [r for r in rows if int(r["Calls"]) >= steps]
    tot = sum(float(r["TotalDurationNs"]) for r in per) / steps / 1e6
    calls = sum(int(r["Calls"]) for r in per) / steps
    lines.append(f"| {n} | {'hipGraph' if graph else 'eager'} | {d['ms_per_step']:.4f} | "
                 f"{tot:.4f} | {d['ms_per_step'] / tot:.2f} | {calls:.0f} |")
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
