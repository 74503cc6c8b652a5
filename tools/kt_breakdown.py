"""Per-config median kernel durations from a bench kernel trace (cfg2 x105, target x28, cfg3 x28 dispatches)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted(((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Start_Timestamp"]))
              for r in rows), key=lambda x: x[2])
names = sorted({n for n, _, _ in seq if "rocclr" not in n and "pack" not in n and "map_codes" not in n})
for name in names:
    ds = [d for n, d, t in seq if n == name]
    bounds = [(0, 105, "cfg2"), (105, 133, "target"), (133, 161, "cfg3")] if len(ds) == 161 else [(0, len(ds), "all")]
    for lo, hi, lab in bounds:
        x = sorted(ds[lo:hi])
        if x:
            print(f"{name:20s} {lab:7s} median {x[len(x)//2]/1000:8.2f} us  min {x[0]/1000:8.2f} us")
