"""Print the kernel timeline of the last calls in a rocprofv3 --kernel-trace database (calls separated by
gaps of more than 1 ms): start / end / duration in microseconds relative to each call's first kernel.

    python tools/kernel_timeline.py DB [calls]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, stream_id from kernels order by start"))
    try:  # memory copies too, when traced (--memory-copy-trace)
        cols = [r[1] for r in c.execute("pragma table_info(memory_copies)")]
        if cols:
            nm = "name" if "name" in cols else cols[0]
            rows += [("copy " + str(r[0]) + " " + str(r[3]) + " B", r[1], r[2], -1)
                     for r in c.execute(f"select {nm}, start, end, size from memory_copies")]
            rows.sort(key=lambda r: r[1])
    except sqlite3.Error:
        pass
    groups, cur, end = [], [], None
    for r in rows:
        if end is not None and r[1] - end > 1_000_000:
            groups.append(cur)
            cur = []
        cur.append(r)
        end = r[2] if end is None else max(end, r[2])
    groups.append(cur)
    for g in groups[-last:]:
        t0 = g[0][1]
        print(f"--- {len(g)} kernels, {(max(r[2] for r in g) - t0) / 1e3:.1f} us")
        for name, s, e, st in g:
            print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} s{st} {name[:70]}")


if __name__ == "__main__":
    main()
