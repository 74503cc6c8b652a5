"""Merge tools/gpu_occupancy.sh passes into profiles/<round>_<config>_pmc.json as an "occupancy" section.

    python tools/occupancy_summary.py gpurun_out/<tag> <round> [kernel]

Mean resident wavefronts per SIMD = 4 * SQ_WAVE_CYCLES (quad-cycles, MI355X_MICROARCH.md PMC units)
/ (kernel duration in shader cycles * 1024 SIMDs), against the kernel's own limit (waves per SIMD its
VGPRs / launch bounds allow) and the hardware's 8 (wavefront slots per SIMD at this register size).
LDS: bytes per block from the kernel trace, the LDS held per CU when every SIMD holds its limit of
wavefronts, and the LDS counters (instructions, bank-conflict cycles over LDS-active cycles).
"""
import csv
import glob
import json
import os
import sys

LDS_PER_CU = 160 * 1024
SIMDS = 1024


def main():
    run, rnd = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "uniform_kernel"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for cfg in ("cfg2", "target"):
        d = os.path.join(run, cfg)
        c, durs, meta = {}, [], {}
        for f in glob.glob(os.path.join(d, "p*", "*_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if kernel in r["Kernel_Name"]:
                    c.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "p1", "*_kernel_trace.csv")):
            for r in csv.DictReader(open(f)):
                if kernel in r["Kernel_Name"]:
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    meta = r
        c = {k: sum(v) / len(v) for k, v in c.items()}
        dur_ns = sum(durs) / len(durs)
        pj = os.path.join(root, "profiles", f"{rnd}_{cfg}_pmc.json")
        prof = json.load(open(pj))
        clock = prof.get("shader_clock_hz") or 2.35e9
        waves_per_simd = 4 * c["SQ_WAVE_CYCLES"] / (dur_ns * 1e-9 * clock * SIMDS)
        lds_block = int(meta["LDS_Block_Size"])
        wg_waves = int(meta["Workgroup_Size_X"]) // 64
        limit = 8  # uniform_kernel W <= 4, int32 keys: launch bounds for 8 waves/SIMD (UNI_OCC)
        blocks_per_cu = limit * 4 // wg_waves
        prof["occupancy"] = {
            "kernel": kernel, "pmc_pass_duration_ns": dur_ns, "shader_clock_hz_assumed": clock,
            "SQ_WAVE_CYCLES_per_launch": c["SQ_WAVE_CYCLES"], "SQ_WAVES_per_launch": c["SQ_WAVES"],
            "mean_resident_waves_per_simd": waves_per_simd, "waves_per_simd_limit": limit,
            "achieved_occupancy_frac": waves_per_simd / limit,
            "lds_bytes_per_block": lds_block, "lds_bytes_per_cu_at_limit": lds_block * blocks_per_cu,
            "lds_frac_of_160KiB_at_limit": lds_block * blocks_per_cu / LDS_PER_CU,
            "SQ_INSTS_LDS_per_launch": c.get("SQ_INSTS_LDS"),
            "SQ_LDS_BANK_CONFLICT_per_launch": c.get("SQ_LDS_BANK_CONFLICT"),
            "SQ_LDS_IDX_ACTIVE_per_launch": c.get("SQ_LDS_IDX_ACTIVE"),
            "lds_bank_conflict_frac": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"])
            if c.get("SQ_LDS_IDX_ACTIVE") else None,
            "source": f"tools/gpu_occupancy.sh ({os.path.basename(run)}), tools/occupancy_summary.py",
        }
        json.dump(prof, open(pj, "w"), indent=1)
        print(cfg, json.dumps(prof["occupancy"], indent=1))


if __name__ == "__main__":
    main()
