"""HBM traffic per dispatch of one kernel from separate FETCH_SIZE and WRITE_SIZE rocprofv3 passes over the
same bench.py command, split into the phases of tools/kt_phases.py (dispatch order).

HBM bytes = 2 * FETCH_SIZE * 1 KiB + WRITE_SIZE * 1 KiB: on gfx950 FETCH_SIZE reports half the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM / rocprofv3 section); both are L2 fabric-side request counts, so
Infinity Cache hits are included.  In the step phase WRITE_SIZE also counts the kernel's stores to host memory.
usage: python tools/pmc_phases.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel> <warmup>
       <steps> <workload> <algorithmic bytes per launch> [out.json]
"""
import csv
import json
import sys


def per_dispatch(path, name, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
            k = int(r["Dispatch_Id"])
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


fetch = per_dispatch(sys.argv[1], sys.argv[3], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], sys.argv[3], "WRITE_SIZE")
warmup, steps, workload, algo = int(sys.argv[4]), int(sys.argv[5]), sys.argv[6], int(sys.argv[7])
n_step, n_ko = warmup + steps, 3 + max(steps, 20)
phases = {"step": list(range(n_step)) + list(range(n_step + n_ko, len(fetch))),
          "kernel_only": list(range(n_step, n_step + n_ko))}
out = {"workload": workload, "kernel": sys.argv[3], "dispatches": [len(fetch), len(write)],
       "algorithmic_bytes_per_launch": algo,
       "formula": "hbm bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)"}
for label, idx in phases.items():
    idx = [i for i in idx if i < min(len(fetch), len(write))]
    if not idx:
        continue
    f = sum(fetch[i] for i in idx) / len(idx) * 1024 * 2
    w = sum(write[i] for i in idx) / len(idx) * 1024
    out[label] = {"dispatches": len(idx), "fetch_bytes": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
                  "traffic_over_algorithmic": (f + w) / algo}
out["hbm_bytes_per_launch"] = out["kernel_only"]["hbm_bytes_per_launch"]  # bench.py load_traffic (roofline)
print(json.dumps(out, indent=1))
if len(sys.argv) > 8:
    json.dump(out, open(sys.argv[8], "w"), indent=1)
