"""Turn a tools/gpu_profile.sh run into committed artefacts under profiles/.

    python tools/make_profile_summary.py gpurun_out/<tag> <round> <config> [kernel] [valu-pmc-dir]

Writes profiles/<round>_<config>_kernel_stats.csv (rocprofv3 --stats), and
profiles/<round>_<config>_pmc.json with the dominant kernel's per-launch HBM
traffic from the separate FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md's HBM section prescribes for gfx950 (FETCH_SIZE reads half of
a wide read stream: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024; FETCH_SIZE and
WRITE_SIZE are in KiB).  The correction is calibrated for 16-B/lane streaming
loads; this kernel's gathers are uncalibrated, so the raw counters are kept too.
"""
import csv
import glob
import json
import os
import shutil
import sys


def mean_counter(path, kernel, name):
    vals = []
    for f in glob.glob(os.path.join(path, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    run, rnd, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "uniform_kernel"
    valu_dir = sys.argv[5] if len(sys.argv) > 5 else None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pdir = os.path.join(root, "profiles")
    os.makedirs(pdir, exist_ok=True)
    shutil.copy(os.path.join(run, "kt", "kt_kernel_stats.csv"), os.path.join(pdir, f"{rnd}_{cfg}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(run, "kt", "kt_kernel_stats.csv")))}
    fetch, nf = mean_counter(os.path.join(run, "fetch"), kernel, "FETCH_SIZE")
    write, nw = mean_counter(os.path.join(run, "write"), kernel, "WRITE_SIZE")
    bench = json.loads(open(os.path.join(run, "bench.json")).read().strip().splitlines()[-1])
    out = {
        "workload": cfg,
        "kernel": kernel,
        "rocprof_avg_duration_ns": float(stats[kernel]["AverageNs"]) if kernel in stats else None,
        "rocprof_calls": int(stats[kernel]["Calls"]) if kernel in stats else None,
        "bench_kernel_ms": bench["roofline"]["kernel_ms"],
        "FETCH_SIZE_KiB_per_launch": fetch,
        "WRITE_SIZE_KiB_per_launch": write,
        "pmc_dispatches": [nf, nw],
        "hbm_bytes_per_launch": int((2 * fetch + write) * 1024) if fetch is not None and write is not None else None,
        "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM, gfx950); "
                      "uncalibrated for gather loads",
    }
    if valu_dir:
        # SQ counters from tools/gpu_pmc.sh passes (p1, p2, ...): VALU / SALU / LDS / VMEM instructions per launch
        for name in ("SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_INSTS_SALU",
                     "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            vals = []
            for d in sorted(glob.glob(os.path.join(valu_dir, "p*"))):
                v, n = mean_counter(d, kernel, name)
                if v is not None:
                    vals.append(v)
            out[name + "_per_launch"] = vals[0] if vals else None
    json.dump(out, open(os.path.join(pdir, f"{rnd}_{cfg}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
