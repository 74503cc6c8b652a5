"""Benchmark: overlap-pairs/s of the scoring step (BASELINE.json metric).

A step is one scoring call over the candidate list of one synthetic read
set: the distinct reads and the reference-ordered candidate list (aligners.py:27-57 for
every pair of overlapGraphs.py:43-53) are resident in HBM when the timed region starts
(the list is enumerated on the device, ovl_candidates), and the step ends with every
pair's (score, end) in host memory: the ABI call ``ovl_score_candidates`` runs the
kernels, which store their results over the link into host memory packed (end and
mismatch count, 2 B per pair) and host threads expand them into the caller's pinned
int32 arrays: packed chunks expanded while the next chunk scores, and the last ~20 % of
the pairs stored as int32 straight into the arrays (OVL_PROGRESSIVE=1 selects the measured
alternative: one launch whose tiles publish packed lines as they finish).

    python bench.py [--gpus 1 --steps K --warmup W --config target]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

N = 1: the north_star target point (PhiX N=50k l=100 p=0.01 k=5, ~2.0 M pairs).
N > 1: one process per GPU, ONE shared list -- BASELINE configs[3] (cfg4: 1 Mbp genome,
N=200k reads, ~38 M pairs) -- sharded by sum n*m; every rank copies its (score, end)
slice into rank 0's shared pinned host buffer (ovlgraph.sharded.ShardedStep, dest="host"),
so the step ends with the whole reference-ordered result on rank 0's host: strong
scaling.  Time = max over ranks between barriers; value = pairs / time.  Rank 0 prints
one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))

METRIC = "overlap-pairs/sec (candidate read-pair alignments) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md)
PCIE_PEAK_GBS = 63.0    # PCIe Gen5 x16 host link, per direction (MI355X_MICROARCH.md "Host link")
WORKLOAD_DESC = {
    "cfg1": "PhiX N=500 l=100 p=0.0 k=5 (BASELINE configs[0])",
    "cfg2": "PhiX N=10000 l=100 p=0.01 k=5 (BASELINE configs[1])",
    "cfg3": "PhiX N=50000 l=150 p=0.02 k=5 (BASELINE configs[2])",
    "cfg4": "random 1 Mbp genome N=200000 l=100 p=0.01 k=5 (BASELINE configs[3], pair-sharded)",
    "cfg5": "PhiX N=50000 l=250 p=0.05 k=5 (BASELINE configs[4])",
    "target": "PhiX N=50000 l=100 p=0.01 k=5 (north_star target point: >=100x the CPU baseline at 1 GPU)",
}

# VALU issue model (profiles/r01_valu_rates.txt, tools/valu_rates.hip): a wave64 integer VALU instruction
# occupies its SIMD ~2.6 (xor/or/and/add/sub/bitop3/lshr) or ~4.3 (bcnt/alignbit/mad24/max/min/cndmask...)
# shader cycles; the uniform sweep's loop mix (tools/isa_mix.py) averages 3.66.  The ISA peak is 2 cycles
# per wave64 instruction on a SIMD-32 (MI355X_MICROARCH.md, "Wave scheduling").
VALU_CYCLES_PER_INST = 3.66
ISA_CYCLES_PER_INST = 2.0
SIMD_COUNT = 1024
SHADER_CLOCK_HZ = 2.4e9


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
                with open(os.path.join(pdir, name)) as fh:
                    d = json.load(fh)
            except Exception:
                continue
            if d.get("workload") == workload:
                return d
    return {}


def load_traffic(workload: str):
    """HBM bytes per launch from the committed PMC summary for this workload."""
    d = load_profile(workload)
    return int(d["hbm_bytes_per_launch"]) if d.get("hbm_bytes_per_launch") else None


def valu_roofline(workload: str, kernel_ms: float):
    """Second bound next to HBM: VALU issue (what the ungapped kernel is limited by), against both the
    measured-mix issue model and the ISA peak (2 cycles per wave64 instruction)."""
    d = load_profile(workload)
    n = d.get("SQ_INSTS_VALU_per_launch")
    if not n or kernel_ms <= 0:
        return None
    achieved = n / (kernel_ms * 1e-3)  # wave64 VALU instructions per second
    peak = SIMD_COUNT * SHADER_CLOCK_HZ / VALU_CYCLES_PER_INST
    isa_peak = SIMD_COUNT * SHADER_CLOCK_HZ / ISA_CYCLES_PER_INST
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "wave64 VALU instructions/s",
            "frac": achieved / peak, "isa_peak": isa_peak, "isa_frac": achieved / isa_peak,
            "valu_instructions_per_launch": n,
            "model": f"peak: {VALU_CYCLES_PER_INST} SIMD cycles per instruction (the kernel's measured mix); "
                     f"isa_peak: {ISA_CYCLES_PER_INST} cycles (wave64 on SIMD-32); {SIMD_COUNT} SIMDs x "
                     f"{SHADER_CLOCK_HZ / 1e9} GHz; instruction count from the committed PMC profile"}


def host_cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        nproc = None
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"model": model, "os_cpu_count": os.cpu_count(), "nproc": nproc, "affinity_cpus": affinity,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(reads, a, b, gpu_score, gpu_end, budget_s: float = 10.0):
    """The oracle's C restatement of aligners.py:27-57 (full int32 DP + int8 traceback table per pair,
    the reference's algorithm) on the GPU box's host cores, on an evenly strided sample of the same
    candidate list; plus a 1-core run and the optimised closed-form CPU path.  Each
    sample's results are compared with the GPU's (the same pairs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    info = host_cpu_info()
    # the box's CPU share for one GPU (OMP_NUM_THREADS, 16 there); the machine's count is reported beside it
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (info["affinity_cpus"] or os.cpu_count() or 1)
    enc = oracle.encode(reads)
    n = a.shape[0]

    def run(fn, t, secs):
        # size an evenly strided sample from a calibration pass, then whole passes over it until `secs`
        cal = min(n, max(1024, 256 * t))
        idx = np.linspace(0, n - 1, cal).astype(np.int64)
        t0 = time.perf_counter()
        fn(reads, a[idx], b[idx], threads=t, encoded=enc)
        per = (time.perf_counter() - t0) / cal
        m = int(min(n, max(cal, secs / max(per, 1e-12))))
        idx = np.linspace(0, n - 1, m).astype(np.int64)
        sa, sb = a[idx], b[idx]
        ok, passes = True, 0
        t0 = time.perf_counter()
        while True:
            sc, en = fn(reads, sa, sb, threads=t, encoded=enc)
            passes += 1
            if passes == 1:
                ok = bool(np.array_equal(sc, gpu_score[idx]) and np.array_equal(en, gpu_end[idx]))
            if time.perf_counter() - t0 >= secs:
                break
        dt = time.perf_counter() - t0
        return {"value": m * passes / dt, "pairs": m, "passes": passes, "seconds": round(dt, 2), "threads": t,
                "matches_gpu": ok}

    full = run(oracle.batch_dp, threads, budget_s)
    one = run(oracle.batch_dp, 1, budget_s / 2)
    cf = run(oracle.batch_closed_form, threads, 2.0)
    cf1 = run(oracle.batch_closed_form, 1, 2.0)
    return {"value": full["value"], "unit": "overlap-pairs/s", "cores": threads, "kind": "port",
            "sample": f"{full['pairs']} of {n} candidate pairs of the same list (evenly strided) x "
                      f"{full['passes']} passes, {full['seconds']} s, through oracle/ovl_oracle.c oracle_batch_dp: the full int32 DP + "
                      f"int8 traceback table per pair of aligners.py:27-57, OpenMP {threads} threads (the box's "
                      f"CPU share per GPU; cpu below lists the machine)",
            "matches_gpu": full["matches_gpu"],
            "one_core": one,
            "closed_form": dict(cf, what="oracle_batch_closed_form: the optimised CPU closed form (2-bit planes, "
                                         "64-base XOR/popcount per diagonal, OpenMP), exact when gaps cannot win"),
            "closed_form_one_core": cf1,
            "cpu": info}


class Workload:
    """One read set resident on the GPU with its device-enumerated candidate list."""

    def __init__(self, name: str, seed: int, dev, engine=None, indel: int = None, band: int = -1,
                 host_list: bool = True):
        import torch
        from ovlgraph import OverlapEngine
        from ovlgraph.candidates import dedup_reads
        from ovlgraph.engine import INDEL_DEFAULT
        from ovlgraph.reads import CONFIGS, config_reads

        self.name = name
        self.cfg = CONFIGS[name]
        self.dev = dev
        t0 = time.perf_counter()
        self.reads, _ = dedup_reads(config_reads(name, seed=seed))
        self.t_sim = time.perf_counter() - t0
        self.eng = engine or OverlapEngine(dev.index)
        t0 = time.perf_counter()
        self.eng.set_reads(self.reads)
        self.n_pairs = self.eng.enumerate_candidates(self.cfg["k"])
        torch.cuda.synchronize(dev)
        self.t_setup = time.perf_counter() - t0
        self.indel = INDEL_DEFAULT if indel is None else indel
        self.band = band
        self.kernel = self.eng.plan(10, -1, self.indel, band)
        self.a = self.b = None
        if host_list:
            self.a, self.b = self.eng.candidates(self.cfg["k"])
            self.a, self.b = np.array(self.a), np.array(self.b)
        self.pa, self.pb, _ = self.eng.candidates_device()
        self.ds = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        self.de = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        from ovlgraph.hostmem import pinned_empty
        self.out = (pinned_empty(self.n_pairs), pinned_empty(self.n_pairs))

    def lens(self) -> np.ndarray:
        return np.fromiter((len(r) for r in self.reads), dtype=np.int64, count=len(self.reads))

    def algo_bytes(self) -> int:
        if self.a is None:
            return int(self.n_pairs) * (2 * int((self.lens().max() + 3) // 4) + 16)
        return algorithmic_bytes(self.lens(), self.a, self.b)

    def step(self) -> None:
        """The metric's step: resident list -> kernels -> (score, end) in pinned host memory."""
        self.eng.score_candidates(10, -1, self.indel, self.band, out=self.out)

    def launch(self, stream) -> None:
        """Kernel only (device outputs), on `stream`: the dominant kernel's timing for the roofline."""
        self.eng.score_device(self.pa, self.pb, self.n_pairs, self.ds.data_ptr(), self.de.data_ptr(),
                              10, -1, self.indel, self.band, stream=stream.cuda_stream)

    def rebind(self, indel: int, band: int) -> None:
        self.indel, self.band = indel, band
        self.kernel = self.eng.plan(10, -1, indel, band)


def timed_steps(fn, steps: int, warmup: int, dev, world: int, group=None) -> float:
    """Warmup, then `steps` calls of fn between barriers + synchronize; this rank's seconds."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier(group=group)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier(group=group)
    return t1 - t0


def kernel_timing(w: Workload, steps: int, dev):
    """The dominant kernel alone over the whole list, HIP events on the stream it is launched on."""
    import torch
    stream = torch.cuda.current_stream(dev)
    for _ in range(3):
        w.launch(stream)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(steps):
        w.launch(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    w.eng.check_device_errors()
    return ev0.elapsed_time(ev1) / max(steps, 1)


def step_breakdown(w: Workload, ms_per_step: float, reps: int = 5):
    """Inside the step: summed kernel time (HIP events per chunk, ovl_set_timing) and the D2H rate."""
    w.eng.set_timing(True)
    k = []
    for _ in range(reps):
        w.step()
        k.append(w.eng.last_timing()["kernel_ms"])
    w.eng.set_timing(False)
    x = w.eng.last_transfer()
    d2h = x["link_bytes"]
    gbs = d2h / (ms_per_step * 1e-3) / 1e9
    return {"kernels_ms_in_step": float(np.median(k)), "d2h_bytes_per_step": d2h,
            "packed_pairs_per_step": x["packed_pairs"], "d2h_gbs_over_step": gbs,
            "pcie_roofline": {"bound": "pcie", "achieved": gbs, "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                              "frac": gbs / PCIE_PEAK_GBS,
                              "what": "result bytes over the link (ovl_last_transfer: 2 B per pair in packed "
                                      "chunks, expanded on the host; 8 B per pair stored straight into the "
                                      "pinned arrays) over the whole step time"}}


def host_paths(w: Workload, reps: int = 10):
    """The same pairs through the other host-array entry points (not the metric):
    ovl_score_host with the pair list in (pageable) host memory -- H2D of a/b + kernels + D2H, the
    PCIe-inclusive rate of the one-shot ABI -- and ovl_score_candidates into pageable numpy arrays."""
    res = {}
    out_pg = (np.empty(w.n_pairs, np.int32), np.empty(w.n_pairs, np.int32))
    cases = {
        "host_pair_list_pinned_out": lambda: w.eng.score(w.a, w.b, 10, -1, w.indel, w.band, out=w.out),
        "device_list_pageable_out": lambda: w.eng.score_candidates(10, -1, w.indel, w.band, out=out_pg),
    }
    for name, fn in cases.items():
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        res[name] = {"ms_per_call": dt * 1e3, "pairs_per_s": w.n_pairs / dt}
    ok = np.array_equal(out_pg[0], w.out[0]) and np.array_equal(out_pg[1], w.out[1])
    res["same_results"] = bool(ok)
    return res


def candidate_timing(w: Workload, reps: int = 5):
    """Candidate enumeration (overlapGraphs.py:30-52): the device path (ovl_candidates, list left in
    HBM) vs the host restatement (candidates.enumerate_candidates, numpy)."""
    from ovlgraph.candidates import enumerate_candidates
    k = w.cfg["k"]
    n = w.eng.enumerate_candidates(k)
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
    """``construct_overlap_graph_nx_k`` for this workload split into stages (not the metric): dedup +
    device enumeration + scoring with results on the host; the DiGraph (direct builder vs networkx
    ``add_edges_from``); then cycle removal (overlapGraphs.py:106-130) on that graph."""
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
    t4 = time.perf_counter()
    stages = {}
    og.remove_cycles_from_graph(G, timing=stages)
    t5 = time.perf_counter()
    return {"reads": len(raw), "pairs": len(edges), "edges": n_e,
            "dedup_enumerate_score_s": round(t1 - t0, 4), "digraph_direct_s": round(t2 - t1, 4),
            "digraph_networkx_s": round(t3 - t2, 4), "end_to_end_s": round(t2 - t0, 4),
            "remove_cycles_s": round(t5 - t4, 4), "edges_removed": n_e - G.number_of_edges(),
            "remove_cycles_stages_s": {k: round(stages[k], 4) for k in ("csr", "replay", "remove")}}


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


def config_line(w: Workload, steps: int, dev):
    """One config's step (results to pinned host) and kernel-only numbers."""
    el = timed_steps(w.step, steps, 2, dev, 1)
    link = w.eng.last_transfer()["link_bytes"]
    km = kernel_timing(w, steps, dev)
    algo = w.algo_bytes()
    return {"workload": WORKLOAD_DESC[w.name], "pairs": w.n_pairs, "kernel": w.kernel,
            "value": w.n_pairs * steps / el, "ms_per_step": el / steps * 1e3,
            "kernel_ms": km, "kernel_pairs_per_s": w.n_pairs / (km * 1e-3),
            "roofline_frac": algo / (km * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "d2h_bytes_per_step": link, "d2h_gbs_over_step": link / (el / steps) / 1e9}


def band_sweep(w: Workload, bands, indel: int, steps: int, dev):
    """Config 5's band-width sweep: the same resident pairs at each band (-1 = full DP, the reference).

    band >= 0 is the build's seed-and-extend knob (ungapped seed j*, DP on |(i - j) - (n - j*)| <= band),
    not a reference mode; cells_per_pair counts the DP cells inside the band (full: n * m).  Each point
    gives the step (results to host) and the kernel alone."""
    lens = w.lens()
    n, m = lens[w.a].astype(np.float64), lens[w.b].astype(np.float64)
    out = {"indel": indel, "match": 10, "mismatch": -1, "pairs": w.n_pairs, "points": []}
    for band in bands:
        w.rebind(indel, band)
        el = timed_steps(w.step, steps, 1, dev, 1)
        km = kernel_timing(w, steps, dev)
        cells = float((n * m).mean()) if band < 0 else float(np.minimum(n * m, (2 * band + 1) * n).mean())
        out["points"].append({"band": band, "kernel": w.kernel, "ms_per_step": el / steps * 1e3,
                              "kernel_ms": km, "pairs_per_s": w.n_pairs * steps / el,
                              "cells_per_pair_upper": round(cells, 1),
                              "cells_per_s": w.n_pairs * cells / (km * 1e-3)})
    return out


def sharded_band_sweep(world: int, rank: int, dev, eng, bands, indel: int, steps: int, backend: str):
    """BASELINE configs[4] across the ranks: cfg5's one shared list sharded by Σ n·m, every rank's results
    into rank 0's shared host buffer, at each band (-1 = the full reference DP); max-over-ranks step time."""
    import torch
    import torch.distributed as dist
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    from ovlgraph.sharded import ShardedStep
    reads, _ = dedup_reads(config_reads("cfg5", seed=0))
    out = {"workload": WORKLOAD_DESC["cfg5"], "indel": indel, "match": 10, "mismatch": -1, "points": []}
    for band in bands:
        st = ShardedStep(reads, k=CONFIGS["cfg5"]["k"], engine=eng, dest="host", indel=indel, band=band)
        el = timed_steps(st.step, steps, 1, dev, world)
        t = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        ok = None
        if rank == 0 and band == bands[0]:
            got = st.results()
            ref = eng.score_candidates(10, -1, indel, band)
            ok = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
        out["pairs"] = st.n_pairs
        out["points"].append({"band": band, "kernel": eng.plan(10, -1, indel, band), "ms_per_step": el / steps * 1e3,
                              "pairs_per_s": st.n_pairs * steps / el,
                              **({"matches_single_gpu": ok} if ok is not None else {})})
        st.close()
    return out


def single_process_all_gpus(rank: int, reads, k: int, steps: int, eng):
    """The reference's own shape on the whole node: ONE process, one context over every visible GPU
    (ovl_create over the device list), the same list scored with each GPU storing its
    shard of (score, end) straight into the caller's pinned arrays.  Rank 0 runs it alone while the other
    ranks wait; checked against rank 0's one-GPU engine."""
    import torch
    from ovlgraph import OverlapEngine
    from ovlgraph.hostmem import pinned_empty
    if rank != 0:
        return None
    ids = list(range(torch.cuda.device_count()))
    t0 = time.perf_counter()
    multi = OverlapEngine(devices=ids)
    multi.set_reads(reads)
    n = multi.enumerate_candidates(k)
    setup = time.perf_counter() - t0
    out = (pinned_empty(n), pinned_empty(n))
    for _ in range(3):
        multi.score_candidates(out=out)
    t0 = time.perf_counter()
    for _ in range(steps):
        multi.score_candidates(out=out)
    el = time.perf_counter() - t0
    eng.set_reads(reads)
    eng.enumerate_candidates(k)
    ref = eng.score_candidates()
    ok = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
    multi.close()
    return {"devices": ids, "pairs": n, "ms_per_step": el / steps * 1e3, "pairs_per_s": n * steps / el,
            "setup_s": round(setup, 2), "matches_single_gpu": ok,
            "what": "one process, OverlapEngine(devices=all visible): shards by sum n*m, each GPU's kernels "
                    "store its slice into the caller's pinned arrays (no collective)"}


def multi_gpu(args, world: int, rank: int, dev, backend: str):
    """N > 1: one shared list (cfg4 by default) sharded over the ranks, results to rank 0's host."""
    import torch
    import torch.distributed as dist
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    from ovlgraph.sharded import ShardedStep

    name = args.config or "cfg4"
    cfg = CONFIGS[name]
    t0 = time.perf_counter()
    reads, _ = dedup_reads(config_reads(name, seed=0))  # the same list on every rank
    eng = OverlapEngine(dev.index)
    st = ShardedStep(reads, k=cfg["k"], engine=eng, dest="host")
    t_setup = time.perf_counter() - t0
    n = st.n_pairs
    elapsed = timed_steps(st.step, args.steps, args.warmup, dev, world)
    # the dominant kernel on this rank's shard alone (HIP events on the launch stream)
    stream = torch.cuda.current_stream(dev)
    lo, hi = st.lo, st.hi
    ds = torch.empty(max(1, hi - lo), dtype=torch.int32, device=dev)
    de = torch.empty_like(ds)
    pa, pb, _ = eng.candidates_device()
    launch = lambda: eng.score_device(pa + 4 * lo, pb + 4 * lo, hi - lo, ds.data_ptr(), de.data_ptr(),  # noqa
                                      stream=stream.cuda_stream)
    launch()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        launch()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)
    # parity of the gathered result: rank 0 scores the whole list alone and compares
    ok = 1.0
    if rank == 0:
        sc, en = st.results()
        full = eng.score_candidates()
        ok = float(np.array_equal(sc, full[0]) and np.array_equal(en, full[1]))
    # the RCCL alternative: results gathered into rank 0's HBM (dist.gather), not to its host
    rccl = None
    if not args.no_gather:
        st2 = ShardedStep(reads, k=cfg["k"], engine=eng, dest="rank0")
        el2 = timed_steps(st2.step, max(5, args.steps), 2, dev, world)
        rccl = el2
        st2.close()
    band_sweep_line = None
    if not args.no_extra:
        # BASELINE configs[4] (cfg5 band-width sweep, "4xMI355X"): the same sharded step per band
        band_sweep_line = sharded_band_sweep(world, rank, dev, eng, [8, 16, 32, 64, -1], args.sweep_indel,
                                             args.sweep_steps, backend)
    red = torch.tensor([elapsed, kernel_ms, 0.0 if ok else 1.0, rccl or 0.0, t_setup], dtype=torch.float64,
                       device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(red, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms, bad, rccl_el, t_setup = (float(x) for x in red.tolist())
    lens = np.fromiter((len(r) for r in reads), dtype=np.int64, count=len(reads))
    st.close()
    single = None
    if not args.no_extra:
        single = single_process_all_gpus(rank, reads, cfg["k"], args.steps, eng)
        dist.barrier()
    if rank != 0:
        return None
    algo_per_rank = (n // world) * (2 * int((lens.max() + 3) // 4) + 16)
    achieved = algo_per_rank / (kernel_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": n * args.steps / elapsed, "unit": "overlap-pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": f"{name}: {WORKLOAD_DESC[name]}", "reads": len(reads), "pairs": n,
                   "read_length": cfg["l"],
                   "parallelism": f"pair-sharded x{world}: one process per GPU, one shared device-enumerated "
                                  f"list, shards balanced by sum n*m, each rank's (score, end) DMA'd into rank 0's "
                                  f"shared pinned host buffer",
                   "kernel": eng.plan(), "scoring": {"match": 10, "mismatch": -1, "indel": -2 ** 31, "band": -1}},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel_ms": kernel_ms,
                     "algorithmic_bytes_per_launch": algo_per_rank,
                     "what": "slowest rank's shard kernel (uniform-length estimate of SURVEY §8d bytes)"},
        "gather": {"dest": "rank 0 host (shared memory, per-rank DMA)", "bytes_per_step": 8 * n,
                   "matches_single_gpu": bad == 0.0},
        "setup_s": round(t_setup, 2),
        "cpu_baseline": None,
    }
    if band_sweep_line is not None:
        line["cfg5_band_sweep_sharded"] = band_sweep_line
    if single is not None:
        line["single_process_all_gpus"] = single
    if rccl_el:
        line["rccl_gather_to_rank0_hbm"] = {"ms_per_step": rccl_el / max(5, args.steps) * 1e3,
                                            "pairs_per_s": n * max(5, args.steps) / rccl_el,
                                            "collective": "dist.gather (RCCL send/recv over xGMI)"
                                            if backend == "nccl" else "dist.gather (gloo)"}
    return line


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=sorted(WORKLOAD_DESC),
                    help="workload (default: target at N=1, cfg4 at N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra single-GPU configs and stages")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of all-core CPU-baseline work")
    ap.add_argument("--indel", type=int, default=None, help="indel score (default: the reference's -2**31)")
    ap.add_argument("--band", type=int, default=-1, help="band half-width (-1 = full DP, the reference)")
    ap.add_argument("--band-sweep", default=None,
                    help="comma list of bands (-1 = full) timed on the same workload at --sweep-indel")
    ap.add_argument("--sweep-indel", type=int, default=-2)
    ap.add_argument("--sweep-steps", type=int, default=5)
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the RCCL gather-to-rank-0 timing")
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
        line = multi_gpu(args, world, rank, dev, backend)
        if rank == 0:
            print(json.dumps(line), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return

    name = args.config or "target"
    w = Workload(name, seed=0, dev=dev, indel=args.indel, band=args.band)
    elapsed = timed_steps(w.step, args.steps, args.warmup, dev, 1)
    ms_step = elapsed / args.steps * 1e3
    kernel_ms = kernel_timing(w, max(args.steps, 20), dev)
    algo = w.algo_bytes()
    achieved = algo / (kernel_ms * 1e-3) / 1e9
    value = w.n_pairs * args.steps / elapsed
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "overlap-pairs/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": f"{name}: {WORKLOAD_DESC[name]}",
            "reads": len(w.reads),
            "pairs": w.n_pairs,
            "read_length": w.cfg["l"],
            "step": "ovl_score_candidates: resident reads + device-enumerated list -> kernels storing over the "
                    "link -> (score, end) in pinned host int32 arrays (SURVEY.md §8d, results in host memory; "
                    "packed 2 B/pair chunks expanded by host threads while the next chunk scores, the last "
                    "~20 % stored directly)",
            "parallelism": "1 GPU",
            "kernel": w.kernel,
            "scoring": {"match": 10, "mismatch": -1, "indel": w.indel, "band": w.band},
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": load_traffic(name),
            "kernel_ms": kernel_ms,
            "algorithmic_bytes_per_launch": algo,
            "what": "dominant kernel alone over the whole list (HIP events on its launch stream)",
        },
        "valu_roofline": valu_roofline(name, kernel_ms),
        "kernel_only_pairs_per_s": w.n_pairs / (kernel_ms * 1e-3),
        "step_breakdown": step_breakdown(w, ms_step),
        "occupancy": load_profile(name).get("occupancy"),
        "host_setup_s": {"read_simulation": round(w.t_sim, 3), "upload_pack_enumerate": round(w.t_setup, 4)},
    }
    if not args.no_extra:
        line["host_paths"] = host_paths(w)
        line["candidates"] = candidate_timing(w)
        line["end_to_end"] = end_to_end(w)
        line["local_alignment"] = local_alignment_timing(w.eng)
    if args.band_sweep:
        line["band_sweep"] = band_sweep(w, [int(x) for x in args.band_sweep.split(",")], args.sweep_indel,
                                        args.sweep_steps, dev)
        w.rebind(w.indel if args.indel is None else args.indel, args.band)
    gpu_sc, gpu_en = np.array(w.out[0]), np.array(w.out[1])
    if not args.no_extra:
        extra = {}
        for other in ("cfg2", "cfg3", "cfg4"):
            if other == name:
                continue
            x = Workload(other, seed=0, dev=dev, engine=w.eng, host_list=False)
            extra[other] = config_line(x, 20, dev)
            del x
        line["extra_configs"] = extra
        if name != "cfg5" and not args.band_sweep:
            # BASELINE configs[4]: the cfg5 band-width sweep at indel -2 (gaps can win)
            x = Workload("cfg5", seed=0, dev=dev, engine=w.eng)
            line["cfg5_band_sweep"] = band_sweep(x, [4, 8, 16, 32, 64, -1], args.sweep_indel, 3, dev)
            del x
    if not args.no_cpu_baseline and w.a is not None:
        cb = cpu_baseline(w.reads, w.a, w.b, gpu_sc, gpu_en, args.cpu_budget)
        line["cpu_baseline"] = cb
        line["vs_cpu_baseline"] = {"all_cores_full_dp": value / cb["value"],
                                   "one_core_full_dp": value / cb["one_core"]["value"],
                                   "all_cores_closed_form": value / cb["closed_form"]["value"]}
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
