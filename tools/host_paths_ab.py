"""Host-array entry points at one config (default: target): every combination of where the pair list
lives (device-enumerated / pinned host / pageable host) and where results go (pinned / pageable), in direct
mode (kernels read and store host memory through its mapping; OVL_PIPE_DIRECT=1, the default) with packed
results (the default) or int32 results (OVL_PACK=0) and a few chunk sizes, and copy-engine mode
(OVL_PIPE_DIRECT=0), with the host staging copies on 1 thread or the pool's default.

    python tools/host_paths_ab.py [config] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def run_setting(reads, k, env, reps):
    from ovlgraph import OverlapEngine
    from ovlgraph.hostmem import PinnedPool
    keep = {x: os.environ.get(x) for x in ("OVL_PIPE_DIRECT", "OVL_PACK", "OVL_PIPE_CHUNK", "OVL_PACK_MIN",
                                           "OVL_PACK_NT", "OVL_PACK_DIRECT_PCT")}
    os.environ.update(env)
    try:
        eng = OverlapEngine(0)
    finally:
        for x, v in keep.items():
            os.environ.pop(x, None)
            if v is not None:
                os.environ[x] = v
    pool = PinnedPool()
    eng.set_reads(reads)
    n = eng.enumerate_candidates(k)
    a, b = eng.candidates(k)
    a, b = np.array(a), np.array(b)
    pa, pb = pool.empty(n), pool.empty(n)
    pa[:], pb[:] = a, b
    outs = {"pinned": (pool.empty(n), pool.empty(n)), "pageable": (np.empty(n, np.int32), np.empty(n, np.int32))}
    ins = {"device_list": None, "pinned_list": (pa, pb), "pageable_list": (a, b)}
    res, ref = {}, None
    for iname, lst in ins.items():
        for oname, out in outs.items():
            def call():
                if lst is None:
                    eng.score_candidates(out=out)
                else:
                    eng.score(lst[0], lst[1], out=out)
            for _ in range(3):
                call()
            t0 = time.perf_counter()
            for _ in range(reps):
                call()
            dt = (time.perf_counter() - t0) / reps
            if ref is None:
                ref = (out[0].copy(), out[1].copy())
            same = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
            res[f"{iname}->{oname}"] = {"ms": round(dt * 1e3, 4), "pairs_per_s": n / dt, "same": same}
    eng.close()
    pool.trim()
    return res, ref


def main():
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    out = {"config": cfg, "host_threads_env": os.environ.get("OVL_HOST_THREADS")}
    refs = []
    modes = (("direct", {"OVL_PIPE_DIRECT": "1"}),
             ("direct_unpacked", {"OVL_PIPE_DIRECT": "1", "OVL_PACK": "0"}),
             ("packed_any_size", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_MIN": "0"}),
             ("packed_direct_0pct", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_DIRECT_PCT": "0"}),
             ("packed_direct_15pct", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_DIRECT_PCT": "15"}),
             ("packed_direct_35pct", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_DIRECT_PCT": "35"}),
             ("packed_direct_50pct", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_DIRECT_PCT": "50"}),
             ("packed_plain_stores", {"OVL_PIPE_DIRECT": "1", "OVL_PACK_NT": "0"}),
             ("packed_chunk512k", {"OVL_PIPE_DIRECT": "1", "OVL_PIPE_CHUNK": "524288"}),
             ("packed_chunk2m", {"OVL_PIPE_DIRECT": "1", "OVL_PIPE_CHUNK": "2097152"}),
             ("copy_engine", {"OVL_PIPE_DIRECT": "0"}))
    for name, env in modes:
        out[name], r = run_setting(reads, CONFIGS[cfg]["k"], env, reps)
        refs.append(r)
    out["modes_agree"] = all(bool(np.array_equal(refs[0][0], r[0]) and np.array_equal(refs[0][1], r[1])) for r in refs)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
