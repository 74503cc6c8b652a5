"""Summarise tools/gpu_r05_cfg5_pmc.sh into profiles/<round>_cfg5_pmc.json (BASELINE configs[4], the kernel of every
point of the cfg5 band sweep; <round> from CFG5_PMC_ROUND, default r06).

    python tools/cfg5_pmc_summary.py gpurun_out/r06cfg5a [gpurun_out/<later run> ...]   (a later run's bands win)

Per kernel (averaged per launch, each counter from its own pass):
  waves_per_simd = 4 * SQ_WAVE_CYCLES / (duration * shader clock * 1024 SIMDs)  (SQ_WAVE_CYCLES counts quad-cycles);
  valu_isa_frac = 4 * SQ_INSTS_VALU / (duration * shader clock * 1024 SIMDs): the VALU pipe's issue share, one wave64
      VALU instruction per 4 cycles per SIMD (the 32-bit rate);
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over all LDS-array cycles,
      MI355X_MICROARCH.md LDS section);
  shader clock = GRBM_GUI_ACTIVE / 8 XCDs / duration of the same dispatch;
  hbm_fetch_bytes = 2 * FETCH_SIZE KiB (the gfx950 halving, MI355X_MICROARCH.md HBM section).
bench.py reads the per-band fields back into every cfg5_band_sweep point (``pmc``).
"""
import csv
import glob
import json
import os
import sys

SIMDS = 1024


def short(name):
    return name.split("(")[0].replace("void ", "").replace("ovl::", "").strip()


def passes(d):
    """kernel -> counter -> [per-dispatch value]; kernel -> counter -> [dispatch duration ns]."""
    vals, durs = {}, {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per, dur = {}, {}
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            key = (k, r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for key, v in per.items():
            k, c, _ = key
            vals.setdefault(k, {}).setdefault(c, []).append(v)
            durs.setdefault(k, {}).setdefault(c, []).append(dur[key])
    return vals, durs


def mean(x):
    return sum(x) / len(x) if x else None


def kernel_entry(cs, ds):
    m = {c: mean(v) for c, v in cs.items()}
    dm = {c: mean(v) for c, v in ds.items()}
    e = {"counters_per_launch": m, "launches_profiled": max(len(v) for v in cs.values())}

    # GRBM_GUI_ACTIVE (summed over the 8 XCDs) rides in passes 1 and 2; its dispatches' mean duration goes with it
    clk = m["GRBM_GUI_ACTIVE"] / 8 / (dm["GRBM_GUI_ACTIVE"] * 1e-9) if "GRBM_GUI_ACTIVE" in m else None
    if clk:
        e["shader_clock_hz"] = clk
    if clk and "SQ_WAVE_CYCLES" in m:
        e["waves_per_simd"] = 4 * m["SQ_WAVE_CYCLES"] / (dm["SQ_WAVE_CYCLES"] * 1e-9 * clk * SIMDS)
        wc = m["SQ_WAVE_CYCLES"]
        e["wave_cycles_breakdown"] = {"parked_s_waitcnt_frac": m.get("SQ_WAIT_ANY", 0) / wc,
                                      "issue_stalled_frac": m.get("SQ_WAIT_INST_ANY", 0) / wc,
                                      "lds_issue_stalled_frac": m.get("SQ_WAIT_INST_LDS", 0) / wc,
                                      "issuing_frac": m.get("SQ_ACTIVE_INST_ANY", 0) / wc}
    if clk and "SQ_INSTS_VALU" in m:
        e["valu_isa_frac"] = 4 * m["SQ_INSTS_VALU"] / (dm["SQ_INSTS_VALU"] * 1e-9 * clk * SIMDS)
        e["valu_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        e["lds_insts_per_wave"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"]
        tot = m["SQ_INSTS_VALU"] + m.get("SQ_INSTS_SALU", 0) + m.get("SQ_INSTS_LDS", 0)
        e["valu_share_of_valu_salu_lds_insts"] = m["SQ_INSTS_VALU"] / tot
    if m.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
    if "FETCH_SIZE" in m:
        e["hbm_fetch_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024
    e["pmc_pass_duration_ns"] = mean([mean(v) for v in ds.values()])
    return e


def main():
    runs = sys.argv[1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {"workload": "cfg5 (BASELINE configs[4]) band sweep at indel -2, the bench's points (-1 = full DP)",
           "command": "bash tools/gpu_r05_cfg5_pmc.sh <tag> (BANDS=...); python tools/cfg5_pmc_summary.py " + " ".join(runs),
           "definitions": __doc__.strip().split("\n\n")[2], "bands": {}}
    dirs = {}
    for run in runs:
        dirs.update({int(os.path.basename(d)[1:]): d for d in glob.glob(os.path.join(run, "b*"))})
    for b in sorted(dirs, key=lambda x: (x < 0, x)):  # (widths ascending, then the full DP)
        d, band = dirs[b], str(b)
        vals, durs = passes(d)
        want = "dp_lane" if band == "-1" else "band_lane"
        ks = {k: kernel_entry(vals[k], durs[k]) for k in vals if want in k}
        stats = glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True)
        trace = {}
        if stats:
            for r in csv.DictReader(open(stats[0])):
                if want in r["Name"]:
                    trace[short(r["Name"])] = {"calls": int(r["Calls"]), "average_ns": float(r["AverageNs"])}
        for k in ks:
            if k in trace:
                ks[k]["kernel_trace"] = trace[k]
        line = next((json.loads(x) for x in open(os.path.join(d, "kt.log")) if x.startswith('{"metric"')), None)
        pt = None
        if line and line.get("band_sweep"):
            pt = line["band_sweep"]["points"][0]
        out["bands"][band] = {"kernels": ks, "bench_point_same_run": pt, "run": os.path.basename(os.path.dirname(d))}
    path = os.path.join(root, "profiles", os.environ.get("CFG5_PMC_ROUND", "r06") + "_cfg5_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1)[:6000])


if __name__ == "__main__":
    main()
