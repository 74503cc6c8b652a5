"""Summarise tools/gpu_r02_profile.sh into profiles/<round>_<config>_{kernel_stats.csv,pmc.json}.

The step launches uniform_kernel<W, 0, false, 3> (the progressive transport, reads <= 128 bases) or
uniform_kernel<W, 0, false, 2> (packed chunks into pinned staging slots) and uniform_kernel<W, 0, false, 1>
(the last chunk, int32 straight into the pinned arrays), and roofline.kernel_ms times uniform_kernel<W, 0, false, 0> (device outputs); their names differ, so the
rocprofv3 --stats rows are already one per phase.  PMC passes cover the kernel-only variant:
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1 KiB (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md);
mean resident wavefronts per SIMD = 4 * SQ_WAVE_CYCLES / (duration * shader clock * 1024 SIMDs).

    python tools/profile_summary_r02.py gpurun_out/r02prof r02 target
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


def main():
    run, rnd, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = glob.glob(os.path.join(run, "kt", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(root, "profiles", f"{rnd}_{cfg}_kernel_stats.csv"))
    st = {r["Name"]: r for r in rows(stats)}
    bench = next(json.loads(line) for line in open(os.path.join(run, "kt.log")) if line.startswith('{"metric"'))
    ctr, durs, gdurs, meta, name = {}, [], [], {}, None
    for f in sorted(glob.glob(os.path.join(run, "p*", "*_counter_collection.csv"))):
        per = {}
        for r in rows(f):
            if "uniform_kernel" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            key = (r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            if r["Counter_Name"] == "SQ_WAVE_CYCLES":
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                meta = r
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                gdurs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for (c, _), v in per.items():
            ctr.setdefault(c, []).append(v)
    m = {c: sum(v) / len(v) for c, v in ctr.items()}
    algo = bench["roofline"]["algorithmic_bytes_per_launch"]
    hbm = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    dur_ns = sum(durs) / len(durs)
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (tools/lane_pmc_summary.py); its pass ran the same launches
    clock = m["GRBM_GUI_ACTIVE"] / 8 / (sum(gdurs) / len(gdurs) * 1e-9)
    waves = 4 * m["SQ_WAVE_CYCLES"] / (dur_ns * 1e-9 * clock * SIMDS)
    lds_block = int(meta.get("LDS_Block_Size") or meta.get("Lds_Size") or 0)
    step_names = [k for k in st if "uniform_kernel" in k and k.split("(")[0].endswith((", 1>", ", 2>", ", 3>"))]
    ko_name = next((k for k in st if "uniform_kernel" in k and k.split("(")[0].endswith(", 0>")), None)
    out = {
        "workload": cfg, "kernel": name.split("(")[0] if name else None,
        "command": "bench.py --config %s --steps 20 --warmup 5 --no-cpu-baseline --no-extra" % cfg,
        "rocprof_stats": {
            # the step's chunks: sink 2 (packed into the staging slots) and sink 1 (int32 into the pinned arrays)
            "step_kernels": {k.split("(")[0]: {"calls": int(st[k]["Calls"]), "average_ns": float(st[k]["AverageNs"])}
                             for k in step_names},
            "kernel_only": ko_name.split("(")[0] if ko_name else None,
            "kernel_only_average_ns": float(st[ko_name]["AverageNs"]) if ko_name else None,
            "bench_roofline_kernel_ms_same_run": bench["roofline"]["kernel_ms"],
        },
        "algorithmic_bytes_per_launch": algo,
        "formula": "hbm bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
        "FETCH_SIZE_kib": m["FETCH_SIZE"], "WRITE_SIZE_kib": m["WRITE_SIZE"],
        "hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / algo,
        "SQ_INSTS_VALU_per_launch": m["SQ_INSTS_VALU"], "SQ_INSTS_SALU_per_launch": m["SQ_INSTS_SALU"],
        "SQ_WAVES_per_launch": m["SQ_WAVES"], "VALU_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
        "shader_clock_hz": clock,
        "occupancy": {
            "kernel": name.split("(")[0] if name else None, "pmc_pass_duration_ns": dur_ns,
            "SQ_WAVE_CYCLES_per_launch": m["SQ_WAVE_CYCLES"], "SQ_BUSY_CYCLES_per_launch": m["SQ_BUSY_CYCLES"],
            "mean_resident_waves_per_simd": waves, "waves_per_simd_limit": 8,
            "achieved_occupancy_frac": waves / 8, "lds_bytes_per_block": lds_block,
            "lds_bytes_per_cu_at_limit": lds_block * 8, "lds_frac_of_160KiB_at_limit": lds_block * 8 / LDS_PER_CU,
            "SQ_INSTS_LDS_per_launch": m.get("SQ_INSTS_LDS"),
            "SQ_LDS_BANK_CONFLICT_per_launch": m.get("SQ_LDS_BANK_CONFLICT"),
            "SQ_LDS_IDX_ACTIVE_per_launch": m.get("SQ_LDS_IDX_ACTIVE"),
            "lds_bank_conflict_frac": (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"])
            if m.get("SQ_LDS_IDX_ACTIVE") else None,
        },
        "source": "tools/gpu_r02_profile.sh, tools/profile_summary_r02.py",
    }
    json.dump(out, open(os.path.join(root, "profiles", f"{rnd}_{cfg}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
