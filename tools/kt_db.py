"""Kernel durations and inter-kernel gaps from a rocprofv3 results database (rocpd sqlite):
    python tools/kt_db.py <results.db> [last_n]"""
import collections
import sqlite3
import statistics
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    last_n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    g = collections.defaultdict(list)
    for n, s, e, gx in rows:
        g[(n.split("(")[0][:70], gx)].append((e - s) / 1000)
    print(f"{len(rows)} dispatches; median us per (kernel, grid_x):")
    for k, v in sorted(g.items(), key=lambda x: -len(x[1]))[:16]:
        print(f"  {len(v):6d} x {statistics.median(v):9.2f}  {k[0]}  grid {k[1]}")
    last = rows[-last_n:]
    print(f"last {last_n}: duration, gap to the previous end (us)")
    for i in range(1, len(last)):
        n, s, e, gx = last[i]
        print(f"  {n.split('(')[0][:50]:50s} grid {gx:8d} {(e - s) / 1000:8.2f}  gap {(s - last[i - 1][2]) / 1000:8.2f}")


if __name__ == "__main__":
    main()
