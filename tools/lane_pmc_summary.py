"""Summarise tools/gpu_profiles_lane.sh PMC passes for one gapped kernel into profiles/<round>_<name>_pmc.json.

    python tools/lane_pmc_summary.py gpurun_out/<tag> <round> <name> <kernel> <profile-name>

Per launch: rocprof duration, SQ instruction counts, the VALU issue rate against the
measured per-SIMD issue model (profiles/r01_valu_rates.txt), and HBM bytes from the
separate FETCH_SIZE / WRITE_SIZE passes corrected as MI355X_MICROARCH.md prescribes for
gfx950 ((2 * FETCH_SIZE + WRITE_SIZE) KiB).
"""
import csv
import glob
import json
import os
import sys


def counters(d, kernel):
    out = {}
    for f in glob.glob(os.path.join(d, "p*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def trace(d, kernel):
    durs, meta = [], {}
    for f in glob.glob(os.path.join(d, "p1", "*_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                meta = {k: r[k] for k in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size",
                                          "Workgroup_Size_X", "Grid_Size_X") if k in r}
    return (sum(durs) / len(durs) if durs else None), meta


def main():
    run, rnd, name, kernel, pname = sys.argv[1:6]
    d = os.path.join(run, f"pmc_{name}")
    c = counters(d, kernel)
    dur, meta = trace(d, kernel)
    bench = json.loads(open(os.path.join(run, f"bench_{name}.json")).read().strip().splitlines()[-1])
    clock_hz = c["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9) if dur and c.get("GRBM_GUI_ACTIVE") else None
    issue_cycles = 3.66  # measured mix model (profiles/r01_valu_rates.txt); 1024 SIMDs
    out = {
        "workload": bench["config"]["workload"], "kernel": kernel, "scoring": bench["config"]["scoring"],
        "pairs": bench["config"]["pairs_per_gpu"], "rocprof_pmc_pass_avg_duration_ns": dur, "dispatch": meta,
        "SQ_INSTS_VALU_per_launch": c.get("SQ_INSTS_VALU"), "SQ_INSTS_SALU_per_launch": c.get("SQ_INSTS_SALU"),
        "SQ_INSTS_VMEM_RD_per_launch": c.get("SQ_INSTS_VMEM_RD"), "SQ_INSTS_VMEM_WR_per_launch": c.get("SQ_INSTS_VMEM_WR"),
        "SQ_WAVES_per_launch": c.get("SQ_WAVES"), "SQ_BUSY_CYCLES_per_launch": c.get("SQ_BUSY_CYCLES"),
        "shader_clock_hz_from_GRBM_GUI_ACTIVE": clock_hz,
        "valu_issue_cycles_per_instruction_per_simd":
            (dur * 1e-9 * clock_hz * 1024 / c["SQ_INSTS_VALU"]) if clock_hz and c.get("SQ_INSTS_VALU") else None,
        "valu_issue_frac_vs_mix_model": (c["SQ_INSTS_VALU"] * issue_cycles / (1024 * clock_hz * dur * 1e-9))
            if clock_hz and c.get("SQ_INSTS_VALU") else None,
        "FETCH_SIZE_KiB_per_launch": c.get("FETCH_SIZE"), "WRITE_SIZE_KiB_per_launch": c.get("WRITE_SIZE"),
        "hbm_bytes_per_launch": int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            if c.get("FETCH_SIZE") is not None and c.get("WRITE_SIZE") is not None else None,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM, gfx950)",
        "bench_kernel_ms_incl_seed": bench["roofline"]["kernel_ms"],
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", f"{rnd}_{pname}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
