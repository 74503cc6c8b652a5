"""Per-wavefront timeline of one uniform-kernel launch (diagnostic; needs the `make trace` build).

    OVL_LIB_PATH=genome-assembly-using-overlap-graphs_amd/build/trace/libovl.so \
        python tools/trace_waves.py [config] [OVL_SPLIT]

Record per wavefront (s_memtime, shader clock): t0 start, t1 rows loaded, t2 side
pairs scored (latency mode), t3 sweep done, t4 tile stored (latency mode), plus
HW_ID / XCC_ID and the tile's side-pair count.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    import torch
    import bench
    from ovlgraph import _lib
    dev = torch.device("cuda", 0)
    w = bench.Workload(cfg, 0, dev)
    for _ in range(20):
        w.launch()
    torch.cuda.synchronize()
    lib = _lib.load()
    n = 65536 * 8
    buf = np.zeros(n, dtype=np.uint64)
    w.launch()
    torch.cuda.synchronize()
    rc = lib.ovl_debug_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    assert rc == 0, rc
    tr = buf.reshape(65536, 8).astype(np.int64)
    tr = tr[tr[:, 0] != 0]
    hw = tr[:, 5]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = tr[:, 6] & 0xF
    role = (tr[:, 6] >> 8) & 1
    side = tr[:, 7]
    # s_memtime bases differ per XCD: times relative to the XCD's first wave start
    rel = np.zeros((tr.shape[0], 5), np.int64)
    for x in np.unique(xcc):
        m = xcc == x
        rel[m] = np.where(tr[m, :5] != 0, tr[m, :5] - tr[m, 0].min(), -1)

    def pct(x):
        if x.size == 0:
            return "-"
        return "min %6d p50 %6d p90 %6d max %6d" % (x.min(), np.median(x), np.percentile(x, 90), x.max())

    print(f"{cfg}: {tr.shape[0]} wavefronts (s_memtime ticks, per-XCD origin); roles: {np.bincount(role)}")
    for rl in np.unique(role):
        m = role == rl
        r = rel[m]
        print(f"-- role {rl}: {m.sum()} waves")
        print("start          ", pct(r[:, 0]))
        print("rows loaded dt ", pct(r[:, 1] - r[:, 0]))
        if (r[:, 2] >= 0).any() and rl == 1:
            print("side dt        ", pct(r[:, 2] - r[:, 1]))
            print("end            ", pct(r[:, 2]))
            sd = side[m]
            for c in sorted(set(sd.tolist()))[:12]:
                mm = sd == c
                print(f"  side={c:2d}: n={mm.sum():5d} side dt p50 {np.median(r[mm, 2] - r[mm, 1]):8.0f}")
        if (r[:, 3] >= 0).any():
            ok = r[:, 3] >= 0
            print("sweep dt       ", pct(r[ok, 3] - r[ok, 1]))
            print("store dt       ", pct(r[ok, 4] - r[ok, 3]))
            print("end            ", pct(r[ok, 4]))
    key = (xcc * 8 + se) * 2 * 16 * 4 + sh * 64 + cu * 4 + simd
    for rl in np.unique(role):
        _, counts = np.unique(key[role == rl], return_counts=True)
        print(f"role {rl} waves per SIMD (histogram):", np.bincount(counts), "SIMDs used", len(counts))
    _, counts = np.unique(key, return_counts=True)
    print("all waves per SIMD (histogram):", np.bincount(counts))
    endc = np.maximum(rel[:, 4], rel[:, 2])
    print("kernel span per XCD (ticks):", [int(endc[xcc == x].max()) for x in np.unique(xcc)])
    for i in np.argsort(-endc)[:6]:
        print("  late wave role", role[i], "t", rel[i].tolist(), "nside", side[i], "SIMD shared by",
              (key == key[i]).sum(), "waves; roles there", np.bincount(role[key == key[i]], minlength=2).tolist())


if __name__ == "__main__":
    main()
