"""Summarise tools/gpu_profile.sh into profiles/<round>_<config>_{kernel_stats.csv,pmc.json} (a shard run,
SHARD=r/N: workload "<config>/shard<r>of<N>", files <round>_<config>_shard<r>of<N>_*).

One entry per uniform_kernel instantiation (their names differ by the result sink: <W, 0, false, 2> packed chunks
and <W, 0, false, 1> the direct chunk inside the step, <W, 0, false, 0> the HBM-output launch of
kernel_only_roofline), averaged per launch of that kernel:
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1 KiB (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md; the in-step
kernels' result stores go to host memory through the fabric, which TCC's WRITE_SIZE also counts);
mean resident wavefronts per SIMD = 4 * SQ_WAVE_CYCLES / (duration * shader clock * 1024 SIMDs); the wave-cycle
breakdown: SQ_WAIT_ANY (parked on s_waitcnt: loads, and the stores to host memory of the in-step kernels),
SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY (issuing), each a fraction of SQ_WAVE_CYCLES.
``headline_kernel`` is the bench line's roofline.kernel (the in-step kernel scoring most of the pairs).

    python tools/profile_summary.py gpurun_out/r04prof r04 target [shard_tag]
"""
import csv
import glob
import json
import os
import shutil
import sys

SIMDS = 1024
LDS_PER_CU = 160 * 1024


def rows(path):
    return list(csv.DictReader(open(path)))


def short(name):
    return name.split("(")[0].replace("void ", "").replace("ovl::", "").strip()


def main():
    run, rnd, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    shard = sys.argv[4] if len(sys.argv) > 4 else None  # e.g. shard0of8
    workload = f"{cfg}/{shard}" if shard else cfg
    stem = f"{rnd}_{cfg}_{shard}" if shard else f"{rnd}_{cfg}"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = glob.glob(os.path.join(run, "kt", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(root, "profiles", f"{stem}_kernel_stats.csv"))
    st = {short(r["Name"]): r for r in rows(stats)}
    bench = next(json.loads(line) for line in open(os.path.join(run, "kt.log"))
                 if line.startswith('{"metric"') or line.startswith('{"shard"'))
    # per kernel: counter -> per-dispatch values; durations of the SQ_WAVE_CYCLES and GRBM passes; LDS size
    ctr, durs, gdurs, lds = {}, {}, {}, {}
    for f in sorted(glob.glob(os.path.join(run, "p*", "*_counter_collection.csv"))):
        per = {}
        for r in rows(f):
            if "uniform_kernel" not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            key = (k, r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if r["Counter_Name"] == "SQ_WAVE_CYCLES":
                durs.setdefault(k, []).append(dur)
                lds[k] = int(r.get("LDS_Block_Size") or r.get("Lds_Size") or 0)
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                gdurs.setdefault(k, []).append(dur)
        for (k, c, _), v in per.items():
            ctr.setdefault(k, {}).setdefault(c, []).append(v)
    kernels = {}
    for k, cs in ctr.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"launches_profiled": len(cs.get("FETCH_SIZE", [])), "formula": "hbm bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024"}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            e.update(FETCH_SIZE_kib=m["FETCH_SIZE"], WRITE_SIZE_kib=m["WRITE_SIZE"],
                     hbm_bytes_per_launch=(2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024)
        if "SQ_INSTS_VALU" in m:
            e.update(SQ_INSTS_VALU_per_launch=m["SQ_INSTS_VALU"], SQ_INSTS_SALU_per_launch=m["SQ_INSTS_SALU"],
                     SQ_WAVES_per_launch=m["SQ_WAVES"], VALU_per_wave=m["SQ_INSTS_VALU"] / m["SQ_WAVES"])
        if k in gdurs and "GRBM_GUI_ACTIVE" in m:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs
            e["shader_clock_hz"] = m["GRBM_GUI_ACTIVE"] / 8 / (sum(gdurs[k]) / len(gdurs[k]) * 1e-9)
        if k in durs and "SQ_WAVE_CYCLES" in m and e.get("shader_clock_hz"):
            dur_ns = sum(durs[k]) / len(durs[k])
            waves = 4 * m["SQ_WAVE_CYCLES"] / (dur_ns * 1e-9 * e["shader_clock_hz"] * SIMDS)
            e["occupancy"] = {
                "kernel": k, "pmc_pass_duration_ns": dur_ns, "SQ_WAVE_CYCLES_per_launch": m["SQ_WAVE_CYCLES"],
                "SQ_BUSY_CYCLES_per_launch": m.get("SQ_BUSY_CYCLES"), "mean_resident_waves_per_simd": waves,
                "waves_per_simd_limit": 8, "achieved_occupancy_frac": waves / 8, "lds_bytes_per_block": lds.get(k),
                "lds_bytes_per_cu_at_limit": (lds.get(k) or 0) * 8,
                "lds_frac_of_160KiB_at_limit": (lds.get(k) or 0) * 8 / LDS_PER_CU,
                "SQ_INSTS_LDS_per_launch": m.get("SQ_INSTS_LDS"),
                "SQ_LDS_BANK_CONFLICT_per_launch": m.get("SQ_LDS_BANK_CONFLICT"),
                "SQ_LDS_IDX_ACTIVE_per_launch": m.get("SQ_LDS_IDX_ACTIVE"),
                "lds_bank_conflict_frac": (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"])
                if m.get("SQ_LDS_IDX_ACTIVE") else None}
            if m.get("SQ_LDS_IDX_ACTIVE") is not None:
                # LDS-array busy cycles per CU cycle of the launch (the LDS's own peak is one array access per
                # cycle per CU); LDS instructions per wave, and how much of the waves' time they held issue
                cu_cycles = dur_ns * 1e-9 * e["shader_clock_hz"] * (SIMDS // 4)
                e["occupancy"]["lds_array_busy_frac_of_cu_cycles"] = m["SQ_LDS_IDX_ACTIVE"] / cu_cycles
                if m.get("SQ_WAVES"):
                    e["occupancy"]["lds_insts_per_wave"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"]
                e["occupancy"]["SQ_ACTIVE_INST_LDS_per_launch"] = m.get("SQ_ACTIVE_INST_LDS")
                e["occupancy"]["SQ_WAIT_INST_LDS_per_launch"] = m.get("SQ_WAIT_INST_LDS")
            if "SQ_WAIT_ANY" in m:
                wc = m["SQ_WAVE_CYCLES"]
                e["occupancy"]["wave_cycles_breakdown"] = {
                    "waiting_on_memory_frac": m["SQ_WAIT_ANY"] / wc, "issue_stalled_frac": m["SQ_WAIT_INST_ANY"] / wc,
                    "issuing_frac": m["SQ_ACTIVE_INST_ANY"] / wc,
                    "what": "SQ_WAIT_ANY (parked on s_waitcnt) / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over "
                            "SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md PMC table)"}
        if k in st:
            e["kernel_trace"] = {"calls": int(st[k]["Calls"]), "average_ns": float(st[k]["AverageNs"])}
        kernels[k] = e
    in_step = {t["kernel"]: t for t in bench.get("in_step_kernels", [])}
    for k, t in in_step.items():
        if k in kernels:
            kernels[k]["bench_same_run"] = {"launch_ms": t["launch_ms"], "pairs_per_launch": t["pairs_per_launch"],
                                            "algorithmic_bytes_per_launch": t["algorithmic_bytes_per_launch"]}
            if "hbm_bytes_per_launch" in kernels[k]:
                kernels[k]["traffic_over_algorithmic"] = (kernels[k]["hbm_bytes_per_launch"] /
                                                          t["algorithmic_bytes_per_launch"])
    ko = bench.get("kernel_only_roofline") or {}
    if ko.get("kernel") in kernels:
        kernels[ko["kernel"]]["bench_same_run"] = {"launch_ms": ko["kernel_ms"],
                                                   "algorithmic_bytes_per_launch": ko["algorithmic_bytes_per_launch"]}
        if "hbm_bytes_per_launch" in kernels[ko["kernel"]]:
            kernels[ko["kernel"]]["traffic_over_algorithmic"] = (kernels[ko["kernel"]]["hbm_bytes_per_launch"] /
                                                                 ko["algorithmic_bytes_per_launch"])
    cmd = "bench.py --config %s --steps 20 --warmup 5 --no-cpu-baseline --no-extra" % cfg
    if shard:
        cmd += " --shard " + shard.replace("shard", "").replace("of", "/")
    out = {"workload": workload, "headline_kernel": bench["roofline"]["kernel"], "command": cmd,
           "bench_roofline_same_run": bench["roofline"], "kernels": kernels,
           "source": "tools/gpu_profile.sh, tools/profile_summary.py"}
    json.dump(out, open(os.path.join(root, "profiles", f"{stem}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1)[:4000])


if __name__ == "__main__":
    main()
