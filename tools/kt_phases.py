"""Split a bench.py kernel trace into its phases by dispatch order and summarise one kernel per phase.

bench.py --no-extra (N = 1) launches the dominant kernel in this order:
  warmup + steps calls of the metric's step, where the kernel stores (score, end) straight into pinned
  host memory (PCIe-bound); then 3 + max(steps, 20) kernel-only launches on device outputs (HIP events;
  roofline.kernel_ms); then 5 more step calls (step_breakdown).  "step" below joins both step runs.
usage: python tools/kt_phases.py <kernel_trace.csv> <kernel-substring> <warmup> <steps> [out.json]
"""
import csv
import json
import sys

path, name, warmup, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
n_step = warmup + steps
n_ko = 3 + max(steps, 20)
out = {"kernel": name, "dispatches": len(dur), "expected": n_step + n_ko + 5}
for label, idx in (("step", list(range(n_step)) + list(range(n_step + n_ko, len(dur)))),
                   ("kernel_only", list(range(n_step, n_step + n_ko)))):
    x = [dur[i] for i in idx if i < len(dur)]
    if x:
        s = sorted(x)
        out[label] = {"dispatches": len(x), "mean_us": sum(x) / len(x), "median_us": s[len(s) // 2],
                      "min_us": s[0], "max_us": s[-1]}
print(json.dumps(out, indent=1))
if len(sys.argv) > 5:
    json.dump(out, open(sys.argv[5], "w"), indent=1)
