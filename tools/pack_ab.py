"""Packed result transport A/B with the modes interleaved: one engine per setting (env knobs read at context
creation), the same output arrays (pinned from the pool, pageable; PACK_AB_KINDS=1 adds pinned coherent /
non-coherent), R rounds of `reps` steps per setting, medians per setting.  Resident
candidate list -> pinned (the bench's step) and pageable arrays.

    python tools/pack_ab.py [config] [rounds] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402

KNOBS = ("OVL_PACK", "OVL_PACK_DIRECT_PCT", "OVL_PACK_NT", "OVL_PIPE_CHUNK", "OVL_PACK_MIN")
SETTINGS = (("int32", {"OVL_PACK": "0"}),
            ("packed_adaptive", {}),
            ("packed_pct18", {"OVL_PACK_DIRECT_PCT": "18"}))
if os.environ.get("PACK_AB_SETTINGS"):  # name=KNOB:value,KNOB:value;name=...
    SETTINGS = tuple((nm, dict(kv.split(":") for kv in spec.split(",") if kv))
                     for nm, spec in (x.split("=", 1) for x in os.environ["PACK_AB_SETTINGS"].split(";")))


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import PinnedPool, pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    engines = {}
    settings = SETTINGS
    if os.environ.get("PACK_AB_MIN0"):  # small lists: packed settings below the default 1 M-pair threshold
        settings = tuple((nm, dict(env, **({} if env.get("OVL_PACK") == "0" else {"OVL_PACK_MIN": "0"})))
                         for nm, env in SETTINGS)
    for name, env in settings:
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = OverlapEngine(0)
        for k in KNOBS:
            os.environ.pop(k, None)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
        engines[name] = eng
    outs = {"pinned": (pinned_empty(n), pinned_empty(n))}
    if os.environ.get("PACK_AB_KINDS"):
        # pinned arrays of each host-memory kind (ovl_host_alloc reads OVL_HOST_COHERENT per allocation)
        for kind, v in (("pinned_coherent", "1"), ("pinned_noncoherent", "0")):
            os.environ["OVL_HOST_COHERENT"] = v
            pool = PinnedPool()
            outs[kind] = (pool.empty(n), pool.empty(n))
            os.environ.pop("OVL_HOST_COHERENT", None)
    outs["pageable"] = (np.empty(n, np.int32), np.empty(n, np.int32))
    times = {(s, o): [] for s, _ in settings for o in outs}
    shares = {}
    ref = None
    for _ in range(rounds):
        for name, _ in settings:
            eng = engines[name]
            for oname, out in outs.items():
                for _ in range(3):
                    eng.score_candidates(out=out)
                t0 = time.perf_counter()
                for _ in range(reps):
                    eng.score_candidates(out=out)
                times[(name, oname)].append((time.perf_counter() - t0) / reps * 1e3)
                if oname == "pinned":
                    shares[name] = eng.last_transfer()["packed_pairs"] / n
                if ref is None:
                    ref = (out[0].copy(), out[1].copy())
                assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]), (name, oname)
    res = {"config": cfg, "pairs": int(n), "rounds": rounds, "reps": reps}
    for (name, oname), v in times.items():
        res.setdefault(name, {})[oname] = {"median_ms": round(float(np.median(v)), 4),
                                           "min_ms": round(float(np.min(v)), 4),
                                           "max_ms": round(float(np.max(v)), 4)}
    for name, v in shares.items():
        res[name]["packed_share_pinned"] = round(v, 3)
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
