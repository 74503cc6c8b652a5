"""Host-pair-list calls (ovl_score_host, the target list in pinned and pageable host memory, results into
pinned arrays) under environment settings read at context creation: one engine per setting, interleaved
rounds of `reps` calls, medians per setting.

    HOST_LIST_AB="name=KNOB:value,KNOB:value;name=..." python tools/host_list_ab.py [config] [rounds] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    settings = [(nm, dict(kv.split(":") for kv in spec.split(",") if kv))
                for nm, spec in (x.split("=", 1) for x in os.environ["HOST_LIST_AB"].split(";"))]
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    engines = {}
    for name, env in settings:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        engines[name] = OverlapEngine(0)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        engines[name].set_reads(reads)
    a, b = engines[settings[0][0]].candidates(5)
    a, b = np.array(a), np.array(b)
    n = a.shape[0]
    pa, pb = pinned_empty(n), pinned_empty(n)
    pa[:], pb[:] = a, b
    out = (pinned_empty(n), pinned_empty(n))
    lists = {"pinned": (pa, pb), "pageable": (a, b)}
    times = {(s, l): [] for s, _ in settings for l in lists}
    ref = None
    for _ in range(rounds):
        for name, _ in settings:
            for lname, (x, y) in lists.items():
                eng = engines[name]
                for _ in range(3):
                    eng.score(x, y, out=out)
                t0 = time.perf_counter()
                for _ in range(reps):
                    eng.score(x, y, out=out)
                times[(name, lname)].append((time.perf_counter() - t0) / reps * 1e3)
                if ref is None:
                    ref = (out[0].copy(), out[1].copy())
                assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]), name
    res = {"config": cfg, "pairs": int(n), "rounds": rounds, "reps": reps}
    for (name, lname), v in times.items():
        res.setdefault(name, {})[lname] = {"median_ms": round(float(np.median(v)), 4),
                                           "min_ms": round(float(np.min(v)), 4)}
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
