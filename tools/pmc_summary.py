"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch), with derived metrics."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(tagdir):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values per dispatch]
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(tagdir, "p*", "*_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        by_dispatch = defaultdict(dict)
        for r in rows:
            k = r["Kernel_Name"]
            by_dispatch[(k, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            by_dispatch[(k, r["Dispatch_Id"])]["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (k, _), ctrs in by_dispatch.items():
            for c, v in ctrs.items():
                if c == "_dur":
                    dur[k].append(v)
                else:
                    per[k][c].append(v)
    out = {}
    for k, ctrs in per.items():
        m = {c: sum(v) / len(v) for c, v in ctrs.items()}
        m["dispatches"] = max(len(v) for v in ctrs.values())
        out[k] = m
    return out


if __name__ == "__main__":
    res = load(sys.argv[1])
    for k, m in res.items():
        print(f"== {k}  ({m['dispatches']} dispatches)")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:.4g}")
        if "GRBM_GUI_ACTIVE" in m:
            pass
        if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
            print(f"   VALU insts per wave        {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:.1f}")
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            print(f"   VALU-active / wave-cycles  {m['SQ_ACTIVE_INST_VALU'] / m['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
            print(f"   wait-any / wave-cycles     {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
            print(f"   wait-inst / wave-cycles    {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
