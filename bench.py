"""Benchmark: overlap-pairs/s of the GPU scoring step (BASELINE.json metric).

A step = one pass of the hot path (aligners.py:27-57 for every candidate pair
of overlapGraphs.py:43-53) over the candidate list of one synthetic read set,
with reads (bit-plane packed) and pairs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W --config cfg2]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

N > 1: one process per GPU; rank r scores its own seeded read set of the same
config (weak scaling: per-GPU work fixed, no data-path collective).  The time
is the max over ranks between barriers; value = pairs of all ranks / time.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))

METRIC = "overlap-pairs/sec (candidate read-pair alignments) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
WORKLOAD_DESC = {
    "cfg1": "PhiX N=500 l=100 p=0.0 k=5 (BASELINE configs[0])",
    "cfg2": "PhiX N=10000 l=100 p=0.01 k=5 (BASELINE configs[1], the 1xMI355X metric config)",
    "cfg3": "PhiX N=50000 l=150 p=0.02 k=5 (BASELINE configs[2])",
    "cfg4": "random 1 Mbp genome N=200000 l=100 p=0.01 k=5 (BASELINE configs[3])",
    "cfg5": "PhiX N=50000 l=250 p=0.05 k=5 (BASELINE configs[4], full band)",
    "target": "PhiX N=50000 l=100 p=0.01 k=5 (north_star target point)",
}


def algorithmic_bytes(lens: np.ndarray, a: np.ndarray, b: np.ndarray) -> int:
    """ceil(n/4) + ceil(m/4) 2-bit read bytes + 8 B indices + 8 B (score, end) per pair."""
    q = (lens + 3) // 4
    return int(q[a].sum() + q[b].sum() + 16 * a.shape[0])


def load_profile(workload: str):
    """The committed PMC summary (profiles/*pmc*.json, newest round first) for this workload, or {}."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return {}
    for name in sorted(os.listdir(pdir), reverse=True):
        if "pmc" in name and name.endswith(".json"):
            try:
                d = json.load(open(os.path.join(pdir, name)))
            except Exception:
                continue
            if d.get("workload") == workload:
                return d
    return {}


def load_traffic(workload: str):
    """HBM bytes per launch from the committed PMC summary for this workload."""
    d = load_profile(workload)
    return int(d["hbm_bytes_per_launch"]) if d.get("hbm_bytes_per_launch") else None


# VALU issue model (profiles/r01_valu_rates.txt, tools/valu_rates.hip): a wave64 integer VALU instruction
# occupies its SIMD ~2.6 (xor/or/and/add/sub/bitop3/lshr) or ~4.3 (bcnt/alignbit/mad24/max/min/cndmask...)
# shader cycles; the uniform sweep's loop mix (tools/isa_mix.py) averages 3.66.  Peak = every SIMD issuing.
VALU_CYCLES_PER_INST = 3.66
SIMD_COUNT = 1024
SHADER_CLOCK_HZ = 2.4e9


def valu_roofline(workload: str, kernel_ms: float):
    """Second bound next to HBM: VALU issue (the one this kernel is actually limited by)."""
    d = load_profile(workload)
    n = d.get("SQ_INSTS_VALU_per_launch")
    if not n or kernel_ms <= 0:
        return None
    achieved = n / (kernel_ms * 1e-3)  # wave64 VALU instructions per second
    peak = SIMD_COUNT * SHADER_CLOCK_HZ / VALU_CYCLES_PER_INST
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "wave64 VALU instructions/s",
            "frac": achieved / peak, "valu_instructions_per_launch": n,
            "model": f"{VALU_CYCLES_PER_INST} SIMD cycles per instruction (measured mix), {SIMD_COUNT} SIMDs "
                     f"x {SHADER_CLOCK_HZ / 1e9} GHz; instruction count from the committed PMC profile"}
    return None


def cpu_baseline(reads, a, b, budget_s: float = 10.0):
    """The oracle's C restatement of aligners.py:27-57 (full DP, per-pair tables) on host cores.

    The whole candidate list is scored repeatedly until ~budget_s of wall time
    (at least once); a strided sample is used instead when one pass would
    exceed the budget.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    threads = max(1, min(16, os.cpu_count() or 1))
    enc = oracle.encode(reads)
    cal = min(a.shape[0], 4000)
    t0 = time.perf_counter()
    oracle.batch_dp(reads, a[:cal], b[:cal], threads=threads, encoded=enc)
    per_pair = (time.perf_counter() - t0) / max(cal, 1)
    n_fit = int(budget_s / max(per_pair, 1e-9))
    if n_fit < a.shape[0]:
        idx = np.linspace(0, a.shape[0] - 1, max(n_fit, cal)).astype(np.int64)
        sa, sb = a[idx], b[idx]
        what = f"{idx.shape[0]} of {a.shape[0]} candidate pairs (evenly strided)"
    else:
        sa, sb = a, b
        what = f"all {a.shape[0]} candidate pairs"
    # whole passes until the budget is spent (at least one)
    reps = 0
    t0 = time.perf_counter()
    while True:
        oracle.batch_dp(reads, sa, sb, threads=threads, encoded=enc)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    what += f" x {reps} passes"
    return {"value": sa.shape[0] * reps / dt, "unit": "overlap-pairs/s", "cores": threads, "kind": "port",
            "sample": f"{what} through oracle/ovl_oracle.c oracle_batch_dp (full int32 DP + int8 traceback "
                      f"per pair, as aligners.py:27-57; OpenMP {threads} threads), {dt:.1f} s"}


class Workload:
    """One rank's read set + candidate list resident on its GPU."""

    def __init__(self, name: str, seed: int, dev, engine=None, indel: int = None, band: int = -1):
        import torch
        from ovlgraph import OverlapEngine
        from ovlgraph.candidates import dedup_reads, enumerate_candidates
        from ovlgraph.reads import CONFIGS, config_reads

        self.name = name
        self.cfg = CONFIGS[name]
        t0 = time.perf_counter()
        self.reads, _ = dedup_reads(config_reads(name, seed=seed))
        self.a, self.b = enumerate_candidates(self.reads, self.cfg["k"])
        self.t_enum = time.perf_counter() - t0
        self.eng = engine or OverlapEngine(dev.index)
        t0 = time.perf_counter()
        self.eng.set_reads(self.reads)
        self.t_pack = time.perf_counter() - t0
        from ovlgraph.engine import INDEL_DEFAULT
        self.indel = INDEL_DEFAULT if indel is None else indel
        self.band = band
        self.kernel = self.eng.plan(10, -1, self.indel, band)
        self.n_pairs = int(self.a.shape[0])
        self.da = torch.as_tensor(self.a, device=dev)
        self.db = torch.as_tensor(self.b, device=dev)
        self.ds = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        self.de = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        self.launch = self.eng.launcher(self.da, self.db, self.ds, self.de, 10, -1, self.indel, band)

    def rebind(self, indel: int, band: int) -> None:
        """Same resident reads and pairs, other scoring (band sweep)."""
        self.indel, self.band = indel, band
        self.kernel = self.eng.plan(10, -1, indel, band)
        self.launch = self.eng.launcher(self.da, self.db, self.ds, self.de, 10, -1, indel, band)

    def algo_bytes(self) -> int:
        lens = np.fromiter((len(r) for r in self.reads), dtype=np.int64, count=len(self.reads))
        return algorithmic_bytes(lens, self.a, self.b)


def timed_steps(w: Workload, steps: int, warmup: int, dev, world: int):
    """Warmup, then K steps between barriers; returns (wall seconds, HIP-event ms per launch)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        w.launch()
    torch.cuda.synchronize(dev)
    w.eng.check_device_errors()
    stream = torch.cuda.current_stream(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        w.launch()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()  # this rank's own end; the caller takes the max over ranks
    if world > 1:
        dist.barrier()
    return t1 - t0, ev0.elapsed_time(ev1) / max(steps, 1)


def host_buffer_timing(w: Workload, reps: int = 20):
    """The same pairs through ovl_score_host: pair list in host memory, (score, end) back in host
    memory, so PCIe copies are included (SURVEY.md §8d's ABI-call step).  Not the metric."""
    w.eng.score(w.a, w.b, 10, -1, w.indel, w.band)  # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        w.eng.score(w.a, w.b, 10, -1, w.indel, w.band)
    dt = (time.perf_counter() - t0) / reps
    return {"pairs": w.n_pairs, "ms_per_call": dt * 1e3, "pairs_per_s": w.n_pairs / dt,
            "what": "ovl_score_host: H2D of a_idx/b_idx, scoring, D2H of score/end (reads resident)"}


def candidate_timing(w: Workload, reps: int = 5):
    """Candidate enumeration (overlapGraphs.py:30-52) for this workload: the device path
    (ovl_candidates: keys, radix sort, lookup, scan, ordered emit; synchronous, list left
    in HBM) vs the host restatement (candidates.enumerate_candidates, numpy)."""
    from ovlgraph.candidates import enumerate_candidates
    k = w.cfg["k"]
    n = w.eng.enumerate_candidates(k)  # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        n = w.eng.enumerate_candidates(k)
    dev_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    a, _ = enumerate_candidates(w.reads, k)
    host_s = time.perf_counter() - t0
    return {"k": k, "pairs": int(n), "same_count_as_host": int(n) == int(a.shape[0]),
            "device_ms": dev_s * 1e3, "host_ms": host_s * 1e3,
            "device_pairs_per_s": n / dev_s if dev_s > 0 else None}


def end_to_end(w: Workload, seed: int = 0):
    """``construct_overlap_graph_nx_k`` for this workload, split into its stages (not the metric):
    dedup + device enumeration + scoring with results on the host, then the DiGraph via the
    direct builder and, for comparison, via networkx ``add_edges_from`` (the reference's way);
    then cycle removal on that graph and the whole ``assemble_contigs_using_overlap_graphs``."""
    from ovlgraph import overlapGraphs as og
    from ovlgraph.reads import config_reads
    raw = config_reads(w.name, seed=seed)
    t0 = time.perf_counter()
    edges = og.overlap_edges_k(raw, w.cfg["k"], engine=w.eng)
    t1 = time.perf_counter()
    G = edges.to_digraph()
    t2 = time.perf_counter()
    G2 = og.assemble_graph(edges.reads, edges.counts, edges.a, edges.b, edges.score, edges.end)
    t3 = time.perf_counter()
    n_e = G.number_of_edges()
    assert n_e == G2.number_of_edges()
    del G2
    # the rest of the reference pipeline (overlapGraphs.py:151-193): cycle removal (native replay of
    # overlapGraphs.py:106-130), topological order, contig walks
    t4 = time.perf_counter()
    og.remove_cycles_from_graph(G)
    t5 = time.perf_counter()
    n_dag = G.number_of_edges()
    del G
    import contextlib
    import io
    t6 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        contigs = og.assemble_contigs_using_overlap_graphs(raw, w.cfg["k"], engine=w.eng)
    t7 = time.perf_counter()
    return {"reads": len(raw), "pairs": len(edges), "edges": n_e,
            "dedup_enumerate_score_s": round(t1 - t0, 4), "digraph_direct_s": round(t2 - t1, 4),
            "digraph_networkx_s": round(t3 - t2, 4),
            "end_to_end_s": round(t2 - t0, 4),
            "remove_cycles_s": round(t5 - t4, 4), "edges_removed": n_e - n_dag,
            "assemble_contigs_s": round(t7 - t6, 4), "contigs": len(contigs)}


def local_alignment_timing(eng, reps: int = 5):
    """local_alignment (aligners.py:85-167, §8f rank 3) of a 4,000-base contig against the whole PhiX
    genome: GPU with and without the traceback walk, beside the oracle's C port on one core."""
    import random
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from ovlgraph.reads import read_genome_from_fasta
    genome = read_genome_from_fasta()
    rng = random.Random(11)
    st = rng.randint(0, len(genome) - 4000)
    contig = "".join(rng.choice("ACGT") if rng.random() < 0.02 else ch for ch in genome[st:st + 4000])
    eng.local_align(contig, genome)  # warm
    t0 = time.perf_counter()
    for _ in range(reps):
        res = eng.local_align(contig, genome)
    tb_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.local_align(contig, genome, traceback=False)
    sc_s = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    exp = oracle.local_alignment(contig, genome)
    cpu_s = time.perf_counter() - t0
    cells = len(contig) * len(genome)
    return {"query": len(contig), "reference": len(genome), "cells": cells, "score": res[0],
            "matches_oracle": res[0] == exp[3] and res[2] == exp[5],
            "gpu_ms_with_traceback": tb_s * 1e3, "gpu_ms_score_only": sc_s * 1e3,
            "gpu_cells_per_s_score_only": cells / sc_s, "cpu_port_ms_1core": cpu_s * 1e3}


def device_list_timing(eng, name: str, steps: int, dev):
    """A whole config scored from its device-enumerated candidate list (no host list): BASELINE
    configs[3] (cfg4, 38 M pairs) fits one GPU; the 8-GPU run shards the same list 8 ways."""
    import torch
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    t0 = time.perf_counter()
    reads, _ = dedup_reads(config_reads(name, seed=0))
    eng.set_reads(reads)
    n = eng.enumerate_candidates(CONFIGS[name]["k"])
    torch.cuda.synchronize(dev)
    t_setup = time.perf_counter() - t0
    pa, pb, n = eng.candidates_device()
    ds = torch.empty(n, dtype=torch.int32, device=dev)
    de = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    launch = lambda: eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(), stream=stream.cuda_stream)
    launch()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        launch()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    km = ev0.elapsed_time(ev1) / steps
    lens = np.fromiter((len(r) for r in reads), dtype=np.int64, count=len(reads))
    algo = int(n) * (2 * int((lens.max() + 3) // 4) + 16)  # uniform-length estimate of SURVEY §8d bytes
    return {"workload": WORKLOAD_DESC[name], "reads": len(reads), "pairs": int(n),
            "setup_s (simulate, upload, device enumeration)": round(t_setup, 3),
            "value": n * steps / el, "kernel_ms": km, "kernel_pairs_per_s": n / (km * 1e-3),
            "roofline_frac": algo / (km * 1e-3) / 1e9 / HBM_PEAK_GBS}


def sharded_gather_timing(eng, dev, world: int, backend: str, steps: int):
    """N > 1, every rank: ONE candidate list (the target point, seed 0, the same on every rank) scored
    pair-sharded with the RCCL all_gather of (score, end) that restores reference order
    (ovlgraph.sharded.ShardedStep) -- the multi-GPU drop-in, strong scaling.  Also
    checks the gathered result against this rank scoring the whole list alone."""
    import torch
    import torch.distributed as dist
    from ovlgraph.sharded import ShardedStep
    x = Workload("target", seed=0, dev=dev, engine=eng)
    st = ShardedStep(x.reads, x.a, x.b, engine=eng)
    for _ in range(3):
        st.step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        st.step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    sc, en = st.results()
    x.launch()
    torch.cuda.synchronize(dev)
    ok = bool(np.array_equal(sc, x.ds.cpu().numpy()) and np.array_equal(en, x.de.cpu().numpy()))
    red = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(red, op=dist.ReduceOp.MAX)
    el, bad = float(red[0]), float(red[1])
    return {"workload": WORKLOAD_DESC["target"], "pairs": x.n_pairs, "ranks": world, "scaling": "strong",
            "steps": steps, "ms_per_step": el / steps * 1e3, "pairs_per_s": x.n_pairs * steps / el,
            "gather_bytes_per_rank_per_step": st.gather_bytes(),
            "collective": "all_gather_into_tensor (RCCL over xGMI)" if backend == "nccl" else "all_gather (gloo, host)",
            "matches_single_gpu": bad == 0.0}


def band_sweep(w: Workload, bands, indel: int, steps: int, dev):
    """Config 5's band-width sweep: the same resident pairs at each band (-1 = full DP).

    band >= 0 is the build's seed-and-extend knob (ungapped seed j*, DP on
    |(i - j) - (n - j*)| <= band), not a reference mode; cells_per_pair counts
    the DP cells inside the band (full: n * m).
    """
    lens = np.fromiter((len(r) for r in w.reads), dtype=np.int64, count=len(w.reads))
    n, m = lens[w.a].astype(np.float64), lens[w.b].astype(np.float64)
    out = {"indel": indel, "match": 10, "mismatch": -1, "pairs": w.n_pairs, "points": []}
    for band in bands:
        w.rebind(indel, band)
        el, km = timed_steps(w, steps, 1, dev, 1)
        cells = float((n * m).mean()) if band < 0 else float(np.minimum(n * m, (2 * band + 1) * n).mean())
        out["points"].append({"band": band, "kernel": w.kernel, "ms_per_step": el / steps * 1e3,
                              "kernel_ms": km, "pairs_per_s": w.n_pairs * steps / el,
                              "cells_per_pair_upper": round(cells, 1),
                              "cells_per_s": w.n_pairs * cells / (km * 1e-3)})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg2", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra single-GPU configs")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (>= 10)")
    ap.add_argument("--indel", type=int, default=None, help="indel score (default: the reference's -2**31)")
    ap.add_argument("--band", type=int, default=-1, help="band half-width (-1 = full DP, the reference)")
    ap.add_argument("--band-sweep", default=None,
                    help="comma list of bands (-1 = full) timed on the same workload at --sweep-indel "
                         "(config 5's sweep: 8,16,32,64,-1); reported under band_sweep")
    ap.add_argument("--sweep-indel", type=int, default=-2)
    ap.add_argument("--sweep-steps", type=int, default=5)
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the sharded one-list RCCL-gather timing")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; ranks beyond the visible devices (flow rehearsal on a 1-GPU box) share them
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("OVL_BENCH_BACKEND", "nccl")  # nccl = RCCL on ROCm; gloo only for rehearsal
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    w = Workload(args.config, seed=rank, dev=dev, indel=args.indel, band=args.band)
    elapsed, kernel_ms = timed_steps(w, args.steps, args.warmup, dev, world)

    stats = torch.tensor([elapsed, kernel_ms, float(w.n_pairs)], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, kernel_ms = float(mx[0]), float(mx[1])
        total_pairs = int(tot[2])
    else:
        total_pairs = w.n_pairs

    gather = None
    if world > 1 and not args.no_gather:
        gather = sharded_gather_timing(w.eng, dev, world, backend, max(20, args.steps // 10))

    if rank == 0:
        algo = w.algo_bytes()
        achieved = algo / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
        line = {
            "metric": METRIC,
            "value": total_pairs * args.steps / elapsed,
            "unit": "overlap-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: {WORKLOAD_DESC[args.config]}",
                "reads_per_gpu": len(w.reads),
                "pairs_per_gpu": w.n_pairs,
                "read_length": w.cfg["l"],
                "parallelism": f"pair-sharded x{world} (one process per GPU, own seeded read set per rank)",
                "kernel": w.kernel,
                "scoring": {"match": 10, "mismatch": -1, "indel": w.indel, "band": w.band},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic(args.config),
                "kernel_ms": kernel_ms,
                "algorithmic_bytes_per_launch": algo,
            },
            "valu_roofline": valu_roofline(args.config, kernel_ms),
            "occupancy": load_profile(args.config).get("occupancy"),
            "host_setup_s": {"read_sim_and_enumeration": round(w.t_enum, 3), "upload_and_pack": round(w.t_pack, 4)},
        }
        if gather is not None:
            line["sharded_gather"] = gather
        if world == 1:
            line["candidates"] = candidate_timing(w)
            line["host_buffers"] = host_buffer_timing(w)
            if not args.no_extra:
                line["end_to_end"] = end_to_end(w)
                line["local_alignment"] = local_alignment_timing(w.eng)
        if world == 1 and args.band_sweep:
            line["band_sweep"] = band_sweep(w, [int(x) for x in args.band_sweep.split(",")], args.sweep_indel,
                                            args.sweep_steps, dev)
            w.rebind(w.indel if args.indel is None else args.indel, args.band)
        if world == 1 and not args.no_extra:
            extra = {}
            for name in ("target", "cfg3"):
                if name == args.config:
                    continue
                x = Workload(name, seed=0, dev=dev, engine=w.eng)
                el, km = timed_steps(x, max(20, args.steps // 4), 3, dev, 1)
                xa = x.algo_bytes()
                extra[name] = {"workload": WORKLOAD_DESC[name], "pairs": x.n_pairs,
                               "value": x.n_pairs * max(20, args.steps // 4) / el, "kernel_ms": km,
                               "kernel_pairs_per_s": x.n_pairs / (km * 1e-3),
                               "roofline_frac": xa / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel": x.kernel}
                del x
            line["extra_configs"] = extra
            if args.config != "cfg4":
                extra["cfg4"] = device_list_timing(w.eng, "cfg4", 10, dev)
            if args.config != "cfg5" and not args.band_sweep:
                # BASELINE configs[4]: the cfg5 band-width sweep at indel -2 (gaps can win), per-GPU kernels
                x = Workload("cfg5", seed=0, dev=dev, engine=w.eng)
                line["cfg5_band_sweep"] = band_sweep(x, [4, 8, 16, 32, 64, -1], args.sweep_indel, 3, dev)
                del x
            w.eng.set_reads(w.reads)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(w.reads, w.a, w.b, args.cpu_budget)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
