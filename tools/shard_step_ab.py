"""Per-rank step at N > 1: rank 0's shard of the target list (what one rank scores when the list is sharded over
N ranks; candidate_shards, sum n*m) scored alone into pinned arrays, under pipeline settings (env knobs read at
context creation), interleaved: R rounds x `reps` steps per (setting, N), medians.

    python tools/shard_step_ab.py [rounds] [reps]        SHARD_AB_SETTINGS="name=KNOB:v,KNOB:v;name=..."
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402

KNOBS = ("OVL_PACK", "OVL_PACK_DIRECT_PCT", "OVL_PIPE_CHUNK", "OVL_PACK_MIN", "OVL_RESIDENT")
SETTINGS = (("default", {}),)
if os.environ.get("SHARD_AB_SETTINGS"):
    SETTINGS = tuple((nm, dict(kv.split(":") for kv in spec.split(",") if kv))
                     for nm, spec in (x.split("=", 1) for x in os.environ["SHARD_AB_SETTINGS"].split(";")))
NS = [int(x) for x in os.environ.get("SHARD_AB_NS", "1,2,4,8").split(",")]


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    cfg = os.environ.get("SHARD_AB_CONFIG", "target")
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    # one engine per (setting, N): the adaptive direct share (pack_share) follows the call size it sees, as in a
    # rank that scores the same shard every step
    engines = {}
    for name, env in SETTINGS:
        for N in NS:
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            eng = OverlapEngine(0)
            for k in KNOBS:
                os.environ.pop(k, None)
            eng.set_reads(reads)
            n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
            engines[(name, N)] = eng
    first = engines[(SETTINGS[0][0], NS[0])]
    cuts = {N: first.candidate_shards(N) for N in NS}
    out = (pinned_empty(n), pinned_empty(n))
    ref = first.score_candidates()
    ref = (np.array(ref[0]), np.array(ref[1]))
    times = {(s, N): [] for s, _ in SETTINGS for N in NS}
    plan = {}
    for r in range(rounds):
        for name, _ in SETTINGS:
            for N in NS:
                eng = engines[(name, N)]
                lo, hi = cuts[N][0], cuts[N][1]
                o = (out[0][lo:hi], out[1][lo:hi])
                # (the pre-bound call a rank's ShardedStep makes every step: one foreign call)
                step = eng.range_scorer(lo, hi, o)
                for _ in range(60 if r == 0 else 3):
                    step()
                t0 = time.perf_counter()
                for _ in range(reps):
                    step()
                times[(name, N)].append((time.perf_counter() - t0) / reps * 1e3)
                assert np.array_equal(o[0], ref[0][lo:hi]) and np.array_equal(o[1], ref[1][lo:hi]), (name, N)
                eng.set_timing(True)
                eng.score_candidates_range(lo, hi, out=o)
                plan[(name, N)] = [(r_["sink"], r_["pairs"], round(r_["ms"], 4)) for r_ in eng.last_launches()]
                eng.set_timing(False)
    res = {"config": cfg, "pairs": int(n), "rounds": rounds, "reps": reps, "results": []}
    for (name, N), v in times.items():
        lo, hi = cuts[N][0], cuts[N][1]
        res["results"].append({"setting": name, "env": dict(SETTINGS)[name], "ranks": N, "shard_pairs": hi - lo,
                               "median_ms": round(float(np.median(v)), 4), "min_ms": round(float(np.min(v)), 4),
                               "max_ms": round(float(np.max(v)), 4),
                               "projected_pairs_per_s": n / (float(np.median(v)) * 1e-3),
                               "launches_sink_pairs_ms": plan[(name, N)]})
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
