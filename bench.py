"""Benchmark: overlap-pairs/s of the scoring step (BASELINE.json metric).

A step is one scoring call over the candidate list of one synthetic read
set: the distinct reads and the reference-ordered candidate list (aligners.py:27-57 for
every pair of overlapGraphs.py:43-53) are resident in HBM when the timed region starts
(the list is enumerated on the device, ovl_candidates), and the step ends with every
pair's (score, end) in host memory: the ABI call ``ovl_score_candidates`` runs the
kernels, which store their results over the link into host memory packed (end and
mismatch count, 2 B per pair) and host threads expand them into the caller's pinned
int32 arrays: packed chunks expanded while the next chunk scores, and the last ~20 % of
the pairs stored as int32 straight into the arrays.

    python bench.py [--gpus N --steps K --warmup W --config target]

``--gpus N`` > 1 without a launcher: this process starts ``python -m torch.distributed.run
--nproc-per-node N bench.py ...`` as a CHILD before touching the GPU, waits for it and exits
with its status (the ranks print the line).  Launched by torch.distributed.run (WORLD_SIZE set),
WORLD_SIZE must equal --gpus.

Every N scores the same list (--config, default the north_star target point: PhiX N=50k
l=100 p=0.01 k=5, 1,993,959 candidate pairs), so the N-point curve is strong scaling.
N = 1: one process, one GPU.  N > 1, one process per GPU (north_star: "candidate pairs shard
embarrassingly across the GPUs"): every rank holds the same read set and enumerates the same
list, scores its contiguous shard (balanced by sum n*m) and its kernels store the shard's
(score, end) into rank 0's shared pinned host buffer (ovlgraph.sharded.ShardedStep, a step
fence in shared memory, no collective per step); value = the list's pairs / max-over-ranks
time.  The N > 1 line also carries: the same list scored by rank 0's GPU alone in the same
run (one_gpu_ms_per_step, speedup_vs_one_gpu, matches_one_gpu), rank 0's in-step roofline,
the same shards collected by an RCCL gather into rank 0's HBM (rccl_gather), a read set per
rank (weak_scaling: the reference's joblib shape), BASELINE configs[3] pair-sharded
(cfg4_strong), configs[4]'s band sweep sharded (cfg5_sharded_band_sweep) and one process over
the job's GPUs (single_process_all_gpus).  Rank 0 prints one JSON line.
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
# shader cycles; the uniform sweep's loop mix (59 VALU per two shifts: 34 fast, 25 slow; round 3) averages 3.51.
# The ISA peak is 2 cycles
# per wave64 instruction on a SIMD-32 (MI355X_MICROARCH.md, "Wave scheduling").
VALU_CYCLES_PER_INST = 3.51
ISA_CYCLES_PER_INST = 2.0
SIMD_COUNT = 1024
SHADER_CLOCK_HZ = 2.4e9


def algorithmic_bytes(lens: np.ndarray, a: np.ndarray, b: np.ndarray) -> int:
    """ceil(n/4) + ceil(m/4) 2-bit read bytes + 8 B indices + 8 B (score, end) per pair."""
    q = (lens + 3) // 4
    return int(q[a].sum() + q[b].sum() + 16 * a.shape[0])


def _short_kernel(name: str) -> str:
    """'void ovl::uniform_kernel<4, 0, false, 2, false>(...)' -> 'uniform_kernel<4, 0, false, 2, false>'."""
    name = name.split("(")[0].strip()
    for pre in ("void ", "ovl::"):
        name = name.replace(pre, "")
    return name


def load_profile(workload: str, kernel: str = None):
    """The committed PMC summary (profiles/*pmc*.json, newest round first) for this workload -- and, when
    `kernel` is given, for that kernel (round-3 summaries hold one entry per kernel) -- or {}."""
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
            if d.get("workload") != workload:
                continue
            if "kernels" in d:
                ks = {_short_kernel(k): v for k, v in d["kernels"].items()}
                want = kernel or d.get("headline_kernel")
                if want in ks:
                    return dict(d, **ks[want], kernel=want)
                continue
            if kernel is None or _short_kernel(d.get("kernel", "")) == kernel:
                return d
    return {}


def load_traffic(workload: str, kernel: str = None):
    """HBM bytes per launch of `kernel` from the committed PMC summary for this workload, or None."""
    d = load_profile(workload, kernel)
    return int(d["hbm_bytes_per_launch"]) if d.get("hbm_bytes_per_launch") else None


def shard_traffic(key: str, workload: str, kernel: str, pairs_per_launch: int):
    """(HBM bytes per launch, source) for `kernel` on a shard: the PMC summary of that shard when one is
    committed (profiles/*_pmc.json with workload `key`), else the whole list's per-launch bytes scaled per
    pair (the same kernel over the same reads), else (None, None)."""
    t = load_traffic(key, kernel)
    if t is not None:
        return t, f"pmc ({key})"
    d = load_profile(workload, kernel)
    ppl = (d.get("bench_same_run") or {}).get("pairs_per_launch")
    if d.get("hbm_bytes_per_launch") and ppl:
        return int(d["hbm_bytes_per_launch"] / ppl * pairs_per_launch), \
            f"pmc ({workload}, {ppl} pairs per launch) scaled per pair"
    return None, None


def valu_roofline(workload: str, kernel_ms: float, kernel: str = None):
    """Second bound next to HBM: VALU issue (what the ungapped kernel is limited by), against both the
    measured-mix issue model and the ISA peak (2 cycles per wave64 instruction)."""
    d = load_profile(workload, kernel)
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
        from ovlgraph.engine import encode_reads
        t0 = time.perf_counter()
        raw = config_reads(name, seed=seed)
        self.t_sim = time.perf_counter() - t0
        # the drop-in's per-build fixed cost, stage by stage (overlapGraphs.py:17-53 before the scoring)
        st = {}
        t = time.perf_counter()

        def mark(k):
            nonlocal t
            now = time.perf_counter()
            st[k] = round(now - t, 5)
            t = now
        self.reads, _ = dedup_reads(raw)
        mark("dedup")
        self.eng = engine or OverlapEngine(dev.index)
        mark("engine")
        enc = encode_reads(self.reads)
        mark("encode")
        self.eng.set_reads(self.reads, enc)
        mark("set_reads_upload_pack")
        self.n_pairs = self.eng.enumerate_candidates(self.cfg["k"])
        torch.cuda.synchronize(dev)
        mark("enumerate_device")
        self.indel = INDEL_DEFAULT if indel is None else indel
        self.band = band
        self.kernel = self.eng.plan(10, -1, self.indel, band)
        self.a = self.b = None
        if host_list:
            self.a, self.b = self.eng.candidates_copy(self.n_pairs)
            mark("candidates_to_host")
            self.a, self.b = np.array(self.a), np.array(self.b)
        self.pa, self.pb, _ = self.eng.candidates_device()
        self.ds = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        self.de = torch.empty(self.n_pairs, dtype=torch.int32, device=dev)
        from ovlgraph.hostmem import pinned_empty
        self.out = self.own_out = (pinned_empty(self.n_pairs), pinned_empty(self.n_pairs))
        self.lo, self.hi = 0, self.n_pairs  # the pairs a step scores (a rank's shard at N > 1)
        self.shard = None  # (rank, world) when sharded
        t = time.perf_counter()
        self.step()  # the first scoring call (code objects load, staging and heavy tiles built)
        mark("first_call")
        self.t_stages = st
        self.t_setup = sum(st.values())

    def set_shard(self, rank: int, world: int, lo: int, hi: int, out=None) -> None:
        """Steps score pairs [lo, hi) only (rank `rank`'s shard of `world`), into `out` (full-length arrays,
        e.g. the shared result buffer) or this workload's pinned arrays."""
        self.shard = (rank, world)
        self.lo, self.hi = int(lo), int(hi)
        if out is not None:
            self.out = out

    def refresh_device_list(self) -> None:
        """After something re-enumerated the resident list on this engine (ShardedStep does)."""
        self.pa, self.pb, n = self.eng.candidates_device()
        assert n == self.n_pairs

    @property
    def profile_key(self) -> str:
        """The workload name the committed PMC summaries use (a shard: "<name>/shard<r>of<N>")."""
        return self.name if self.shard is None else f"{self.name}/shard{self.shard[0]}of{self.shard[1]}"

    def close(self) -> None:
        self.eng.close()

    def lens(self) -> np.ndarray:
        return np.fromiter((len(r) for r in self.reads), dtype=np.int64, count=len(self.reads))

    def algo_bytes(self) -> int:
        if self.a is None:
            return int(self.n_pairs) * (2 * int((self.lens().max() + 3) // 4) + 16)
        return algorithmic_bytes(self.lens(), self.a, self.b)

    def step(self) -> None:
        """The metric's step: resident list -> kernels -> (score, end) in pinned host memory (a shard: its
        range of the list into its slice of the arrays)."""
        if self.lo == 0 and self.hi == self.n_pairs:
            self.eng.score_candidates(10, -1, self.indel, self.band, out=self.out)
        elif self.hi > self.lo:
            lo, hi = self.lo, self.hi
            self.eng.score_candidates_range(lo, hi, 10, -1, self.indel, self.band,
                                            out=(self.out[0][lo:hi], self.out[1][lo:hi]))

    def launch(self, stream) -> None:
        """Kernel only (device outputs), on `stream`: the dominant kernel's timing for the roofline."""
        self.eng.score_device(self.pa, self.pb, self.n_pairs, self.ds.data_ptr(), self.de.data_ptr(),
                              10, -1, self.indel, self.band, stream=stream.cuda_stream)

    def rebind(self, indel: int, band: int) -> None:
        self.indel, self.band = indel, band
        self.kernel = self.eng.plan(10, -1, indel, band)


def timed_steps(fn, steps: int, warmup: int, dev, world: int, group=None) -> float:
    """Warmup, then `steps` calls of fn between barriers + synchronize; this rank's seconds.  The engines'
    resident scoring grids are asked to leave before each synchronize (quiesce_all: inside the timed region after
    the last step -- ending the job is part of it), else the synchronize would wait out their idle deadline."""
    import torch
    import torch.distributed as dist
    from ovlgraph.engine import quiesce_all
    for _ in range(warmup):
        fn()
    quiesce_all()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier(group=group)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    quiesce_all()
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
    """``construct_overlap_graph_nx_k`` + ``remove_cycles_from_graph`` (overlapGraphs.py:5-61, 106-130) for this
    workload, stage by stage (not the metric): dedup + encode + upload + device enumeration + scoring with results
    on the host (each stage itemised; the first call and a warm one); the graph as returned (lazy: its dicts are
    built on first use) and the cycle removal on it (CSR from the columns, survivors materialised); then the eager
    forms for comparison: the direct C builder, networkx's ``add_edges_from``, and cycle removal on an eager
    graph."""
    from ovlgraph import overlapGraphs as og
    from ovlgraph.reads import config_reads
    raw = config_reads(w.name, seed=seed)
    cold = {}
    t0 = time.perf_counter()
    og.overlap_edges_k(raw, w.cfg["k"], engine=w.eng, timing=cold)  # first build on this engine since setup
    t_cold = time.perf_counter() - t0
    stages = {}
    t0 = time.perf_counter()
    edges = og.overlap_edges_k(raw, w.cfg["k"], engine=w.eng, timing=stages)
    t1 = time.perf_counter()
    L = edges.to_digraph()  # what construct_overlap_graph_nx_k returns
    t2 = time.perf_counter()
    rc_l = {}
    og.remove_cycles_from_graph(L, timing=rc_l)  # (replay and survivors' dicts overlapped)
    t3 = time.perf_counter()
    n_kept = L.number_of_edges()
    del L
    # the same twice more on fresh lazy graphs: remove_cycles_s is the process's first call (what a user's single
    # graph build pays), remove_cycles_median_s the median of the three (one call's time moves with the box's host
    # by +-10 %); every run is on the line.  (The builder's pooled arenas live only inside its calls, so no call
    # reuses the memory of the one before: csrc/ovl_digraph.c arena_pool.)
    import gc
    runs = [(t3 - t2, rc_l)]
    for _ in range(2):
        gc.collect()
        L = edges.to_digraph()
        rc_r = {}
        tr0 = time.perf_counter()
        og.remove_cycles_from_graph(L, timing=rc_r)
        runs.append((time.perf_counter() - tr0, rc_r))
        assert L.number_of_edges() == n_kept
        del L
    gc.collect()
    t_first, rc_l = runs[0]
    t_med = sorted(runs, key=lambda x: x[0])[1][0]
    # the same with the replay, then the dicts (OVL_CYCLES_STREAM=0), for comparison
    saved = og._STREAM_OFF
    og._STREAM_OFF = True
    try:
        L = edges.to_digraph()
        rc_s = {}
        ts0 = time.perf_counter()
        og.remove_cycles_from_graph(L, timing=rc_s)
        ts1 = time.perf_counter()
        assert L.number_of_edges() == n_kept
        del L
    finally:
        og._STREAM_OFF = saved
    t4 = time.perf_counter()
    G = edges.to_digraph(lazy=False)
    t5 = time.perf_counter()
    G2 = og.assemble_graph(edges.reads, edges.counts, edges.a, edges.b, edges.score, edges.end)
    t6 = time.perf_counter()
    n_e = G.number_of_edges()
    assert n_e == G2.number_of_edges() == edges.n_edges()
    del G2
    rc_e = {}
    t7 = time.perf_counter()
    og.remove_cycles_from_graph(G, timing=rc_e)
    t8 = time.perf_counter()
    assert G.number_of_edges() == n_kept
    return {"reads": len(raw), "pairs": len(edges), "edges": n_e, "edges_removed": n_e - n_kept,
            "dedup_enumerate_score_s": round(t1 - t0, 4),
            "dedup_enumerate_score_first_s": round(t_cold, 4),
            "dedup_enumerate_score_stages_s": {k: round(v, 5) for k, v in stages.items()},
            "dedup_enumerate_score_first_stages_s": {k: round(v, 5) for k, v in cold.items()},
            "construct_s": round(t2 - t0, 4),
            "remove_cycles_s": round(t_first, 4),
            "remove_cycles_median_s": round(t_med, 4),
            "remove_cycles_runs_s": [round(x[0], 4) for x in runs],
            "remove_cycles_stages_s": {k: round(rc_l[k], 4) for k in ("csr", "replay", "remove")},
            "remove_cycles_overlapped": bool(rc_l.get("overlapped")),
            "construct_plus_remove_cycles_s": round(t2 - t0 + t_first, 4),
            "remove_cycles_serial_s": round(ts1 - ts0, 4),
            "remove_cycles_serial_stages_s": {k: round(rc_s[k], 4) for k in ("csr", "replay", "remove")},
            "what": "construct_s: overlap_edges_k + the lazy DiGraph (dicts built on first use); remove_cycles_s: "
                    "on that graph, CSR from the columns, then the replay with the surviving edges' dicts built "
                    "while it runs (stage 'replay' holds both; remove_cycles_serial_s: replay, then the dicts) -- "
                    "the process's first call; remove_cycles_median_s: the median of three calls on fresh lazy "
                    "graphs, remove_cycles_runs_s in call order; construct_plus_remove_cycles_s: both first calls",
            "eager": {"digraph_direct_s": round(t5 - t4, 4), "digraph_networkx_s": round(t6 - t5, 4),
                      "remove_cycles_s": round(t8 - t7, 4),
                      "remove_cycles_stages_s": {k: round(rc_e[k], 4) for k in ("csr", "replay", "remove")}}}


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
                              "cells_per_s": w.n_pairs * cells / (km * 1e-3), "pmc": band_pmc(band)})
    return out


def band_pmc(band: int):
    """The band kernel's counters at this sweep point from the committed PMC profile (tools/gpu_r05_cfg5_pmc.sh,
    tools/cfg5_pmc_summary.py: each counter in its own rocprofv3 pass of the same bench command, so not live):
    valu_isa_frac (VALU pipe issue share at 4 cycles per wave64 instruction), waves_per_simd (mean resident),
    lds_bank_conflict_frac (conflict cycles over LDS-array cycles).  None when the profile lacks the band."""
    src = next((os.path.join("profiles", f"{r}_cfg5_pmc.json") for r in ("r06", "r05")
                if os.path.exists(os.path.join(ROOT, "profiles", f"{r}_cfg5_pmc.json"))),
               os.path.join("profiles", "r05_cfg5_pmc.json"))
    try:
        with open(os.path.join(ROOT, src)) as f:
            ks = json.load(f)["bands"][str(band)]["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    if not ks:
        return None
    k, e = max(ks.items(), key=lambda kv: (kv[1].get("kernel_trace") or {}).get("average_ns", 0.0))
    return {"kernel": k, "valu_isa_frac": e.get("valu_isa_frac"), "waves_per_simd": e.get("waves_per_simd"),
            "lds_bank_conflict_frac": e.get("lds_bank_conflict_frac"),
            "rocprof_kernel_ms": (e.get("kernel_trace") or {}).get("average_ns", 0.0) / 1e6, "source": src}


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
        if rank == 0:
            got = st.results()
            ref = eng.score_candidates(10, -1, indel, band)
            ok = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
        out["pairs"] = st.n_pairs
        if rank == 0:
            print(f"bench.py: sharded band sweep, band {band} done", file=sys.stderr, flush=True)
        out["points"].append({"band": band, "kernel": eng.plan(10, -1, indel, band), "ms_per_step": el / steps * 1e3,
                              "pairs_per_s": st.n_pairs * steps / el,
                              **({"matches_single_gpu": ok} if ok is not None else {})})
        st.close()
    out["what"] = (f"BASELINE configs[4] over {world} ranks: cfg5's one list sharded by sum n*m, each rank's "
                   f"(score, end) into rank 0's shared pinned host buffer; band -1 = the reference's full DP, "
                   f"band >= 0 the seed-and-extend knob (no reference mode); every point checked against rank 0 "
                   f"alone scoring the whole list")
    return out


def single_process_all_gpus(rank: int, world: int, shared: bool, reads, k: int, steps: int, eng):
    """The reference's own shape on the job's GPUs: ONE process, one context over the `world` GPUs of the
    ranks (ovl_create over the device list), the same list scored with each GPU storing its
    shard of (score, end) straight into the caller's pinned arrays.  Rank 0 runs it alone while the other
    ranks wait; checked against rank 0's one-GPU engine.  When ranks share GPUs (a one-GPU rehearsal) the
    context lists GPU 0 `world` times (OVL_SHARE_DEVICES=1: one shard slot each)."""
    from ovlgraph import OverlapEngine
    from ovlgraph.hostmem import pinned_empty
    if rank != 0:
        return None
    ids = [0] * world if shared else list(range(world))
    saved = os.environ.get("OVL_SHARE_DEVICES")
    if shared:
        os.environ["OVL_SHARE_DEVICES"] = "1"
    t0 = time.perf_counter()
    try:
        multi = OverlapEngine(devices=ids)
    finally:
        if shared:
            if saved is None:
                os.environ.pop("OVL_SHARE_DEVICES", None)
            else:
                os.environ["OVL_SHARE_DEVICES"] = saved
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
            "setup_s": round(setup, 2), "matches_single_gpu": ok, "devices_shared": shared,
            "what": "one process, OverlapEngine(devices=[the job's GPUs]): shards by sum n*m, each GPU's kernels "
                    "store its slice into the caller's pinned arrays (no collective)"}


def pair_bytes(lens: np.ndarray, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """SURVEY.md §8d algorithmic bytes of each pair (ceil(n/4) + ceil(m/4) + 16)."""
    q = (lens + 3) // 4
    return q[a] + q[b] + 16


SINKS = {0: "int32 results in HBM (copy-engine transfer after)", 1: "int32 results stored into pinned host memory",
         2: "packed 2 B/pair results stored into pinned host staging (host threads expand)"}


def kernel_name(w, sink: int, pairs: int) -> str:
    """The uniform_kernel instantiation a launch of `pairs` pairs with result sink `sink` runs (ovl_plan
    "ungapped", 2 bit planes, int32 keys; latency mode at <= 32 tiles per CU for device lists, ovl_api.cpp
    kLatTiles)."""
    if w.kernel != "ungapped":
        return f"{w.kernel} kernel"
    lmax = w.eng.info()["lmax"]
    lat = (pairs + 63) // 64 <= 256 * 32
    # (the fifth parameter, IX, is true only for host pair lists read in their encoding)
    return f"uniform_kernel<{(lmax + 31) // 32}, 0, {'true' if lat else 'false'}, {sink}, false>"


# result bytes a launch stores over the host link per pair, by sink (0: HBM outputs, 1: two int32, 2: packed)
LINK_BYTES_PER_PAIR = {0: 0, 1: 8, 2: 2}
# a kernel's stores into pinned host memory, measured on the box (profiles/r02_pcie_write.txt)
LINK_PEAK_GBS = 55.3


def in_step_rooflines(w, ms_per_step: float, reps: int = 7):
    """The kernels that run INSIDE the timed step, each launch timed with HIP events on its stream
    (ovl_set_timing / ovl_last_launches) over `reps` steps: per result sink, the median launch duration,
    pairs and §8d algorithmic bytes per launch (the launch's own pair range), HBM fraction.  Returns
    (roofline of the dominant in-step kernel, per-sink table, step-level roofline)."""
    lens = w.lens()
    cum = np.zeros(w.hi - w.lo + 1, dtype=np.int64)
    np.cumsum(pair_bytes(lens, w.a[w.lo:w.hi], w.b[w.lo:w.hi]), out=cum[1:])
    w.eng.set_timing(True)
    runs = []
    for _ in range(reps):
        w.step()
        runs.append(w.eng.last_launches())
    w.eng.set_timing(False)
    bpp = dict(LINK_BYTES_PER_PAIR)
    by_sink = {}
    for recs in runs:
        off = 0
        for i, r in enumerate(recs):
            lo, hi = off, off + r["pairs"]
            off = hi
            d = by_sink.setdefault(r["sink"], {"ms": [], "pairs": [], "bytes": [], "queued": [], "first": []})
            d["ms"].append(r["ms"])
            d["pairs"].append(hi - lo)
            d["bytes"].append(int(cum[hi] - cum[lo]))
            # a call's first launch starts on an idle stream: its start event also times the command
            # processor's dispatch of the kernel; later launches queue behind the previous one
            (d["first"] if i == 0 else d["queued"]).append(r["ms"])
    table = []
    for sink, d in sorted(by_sink.items()):
        ms_all = float(np.median(d["ms"]))
        ms = float(np.median(d["queued"])) if d["queued"] else ms_all
        pairs = int(np.median(d["pairs"]))
        byts = int(np.median(d["bytes"]))
        launches = len(d["ms"]) / reps
        ach = byts / (ms * 1e-3) / 1e9
        link = int(pairs * bpp.get(sink, 0))
        table.append({"sink": sink, "what": SINKS.get(sink, "?"), "kernel": kernel_name(w, sink, pairs),
                      "link_bytes_per_pair": bpp.get(sink, 0),
                      "link_bytes_per_launch": link, "link_gbs": link / (ms * 1e-3) / 1e9,
                      "link_frac": link / (ms * 1e-3) / 1e9 / LINK_PEAK_GBS,
                      "launches_per_step": launches, "launch_ms": ms, "launch_ms_all": ms_all,
                      "first_launch_ms": float(np.median(d["first"])) if d["first"] else None,
                      "pairs_per_launch": pairs, "algorithmic_bytes_per_launch": byts, "achieved_gbs": ach,
                      "frac": ach / HBM_PEAK_GBS, "ms_per_step": ms_all * launches})
    if not table:  # an empty shard launches nothing
        return None, [], None
    # the dominant in-step kernel: the one that scores most of the step's pairs (the packed chunks); the
    # table beside it has every in-step kernel with its own fraction
    dom = max(table, key=lambda t: t["pairs_per_launch"] * t["launches_per_step"])
    if w.shard is None:
        traffic, tsrc = load_traffic(w.name, dom["kernel"]), "pmc"
    else:
        traffic, tsrc = shard_traffic(w.profile_key, w.name, dom["kernel"], dom["pairs_per_launch"])
    roof = {"bound": "hbm", "achieved": dom["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": dom["frac"], "traffic": traffic, "traffic_source": tsrc, "kernel": dom["kernel"],
            "launch_ms": dom["launch_ms"],
            "pairs_per_launch": dom["pairs_per_launch"],
            "algorithmic_bytes_per_launch": dom["algorithmic_bytes_per_launch"],
            "launches_per_step": dom["launches_per_step"],
            "link": {"bound": "host link", "achieved": dom["link_gbs"], "peak": LINK_PEAK_GBS, "unit": "GB/s",
                     "frac": dom["link_frac"], "bytes_per_launch": dom["link_bytes_per_launch"],
                     "what": "result bytes the launch stores over the PCIe link into host memory / its duration; "
                             "peak: a kernel storing two int32 arrays into pinned host memory "
                             "(profiles/r02_pcie_write.txt)"},
            "what": "the step's dominant kernel (the one scoring most of the step's pairs, inside ms_per_step): "
                    "SURVEY §8d bytes of the pairs one launch scores / its median duration, HIP events on its "
                    "launch stream inside the timed step's own call (ovl_last_launches; launches queued behind "
                    "the call's first, whose start event also times the kernel's dispatch); in_step_kernels lists "
                    "every in-step kernel; traffic: PMC FETCH+WRITE bytes per launch of that kernel "
                    "(profiles/r03_*pmc*.json)"}
    total = int(cum[-1])
    step = {"bound": "hbm", "achieved": total / (ms_per_step * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "algorithmic_bytes_per_step": total,
            "kernels_ms_per_step": sum(t["ms_per_step"] for t in table),
            "what": "SURVEY §8d bytes of the whole list / ms_per_step (kernels, link and host expansion)"}
    step["frac"] = step["achieved"] / HBM_PEAK_GBS
    step["kernels_frac"] = total / (step["kernels_ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS
    return roof, table, step


def abi_one_shot(w, reps: int = 10):
    """SURVEY.md §8(d) literally: the ABI call ``ovl_score_pairs`` with host-resident reads (raw bytes +
    offsets) and a host pair list, results into host int32 arrays -- upload + pack of the reads, the pair
    list over the link, kernels, results back -- at the workload's size; with the pair list in pinned and
    in pageable host memory.  Checked against the resident-list step's results."""
    from ovlgraph.engine import encode_reads
    from ovlgraph.hostmem import pinned_empty
    enc = encode_reads(w.reads)
    out = (pinned_empty(w.n_pairs), pinned_empty(w.n_pairs))
    pa, pb = pinned_empty(w.n_pairs), pinned_empty(w.n_pairs)
    pa[:] = w.a
    pb[:] = w.b
    ga, gb = np.ascontiguousarray(w.a), np.ascontiguousarray(w.b)
    res = {"reads_bytes": int(enc[0].nbytes), "pairs": w.n_pairs}
    ref = (np.array(w.out[0]), np.array(w.out[1]))
    for label, (x, y) in (("pinned_pair_list", (pa, pb)), ("pageable_pair_list", (ga, gb))):
        for _ in range(40):  # (the direct share of compact-list calls settles within ~30 calls, pack_share)
            w.eng.score_pairs(w.reads, x, y, out=out, encoded=enc)
        t0 = time.perf_counter()
        for _ in range(reps):
            w.eng.score_pairs(w.reads, x, y, out=out, encoded=enc)
        dt = (time.perf_counter() - t0) / reps
        ok = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
        res[label] = {"ms_per_call": dt * 1e3, "pairs_per_s": w.n_pairs / dt, "matches_step": ok,
                      "link_bytes": w.eng.last_transfer()["link_bytes"],
                      "reads": "the same read set every call: found resident (compared byte for byte), not uploaded"}
    # every call a read set the device does not hold: calls alternate between the reads and a copy with one base
    # of read 0 changed, so each call uploads and packs (the reference's build over a new read set)
    buf2 = enc[0].copy()
    buf2[0] = ord("C") if buf2[0] != ord("C") else ord("A")
    enc2 = (buf2, enc[1])
    for i in range(10):
        w.eng.score_pairs(w.reads, pa, pb, out=out, encoded=enc if i % 2 == 0 else enc2)
    t0 = time.perf_counter()
    for i in range(reps):
        w.eng.score_pairs(w.reads, pa, pb, out=out, encoded=enc if i % 2 == 0 else enc2)
    dt = (time.perf_counter() - t0) / reps
    w.eng.score_pairs(w.reads, pa, pb, out=out, encoded=enc)
    ok = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
    res["pinned_pair_list_new_reads"] = {"ms_per_call": dt * 1e3, "pairs_per_s": w.n_pairs / dt, "matches_step": ok,
                                         "reads": "a different read set every call (uploaded and packed)"}
    # the call's two halves: ovl_set_reads (upload + pack) and ovl_score_host
    t0 = time.perf_counter()
    for _ in range(reps):
        w.eng.set_reads(w.reads, enc)
    res["set_reads_ms"] = (time.perf_counter() - t0) / reps * 1e3
    w.eng.enumerate_candidates(w.cfg["k"])  # the resident list again (set_reads dropped it)
    res["what"] = ("ovl_score_pairs(seqs, offsets, n_reads, a_idx, b_idx, ...) per call: the reads handed over every "
                   "call (raw bytes + offsets) -- compared byte for byte with the resident set, uploaded and packed "
                   "when they differ (pinned_pair_list_new_reads: every call) --, the pair list read from host "
                   "memory, (score, end) into pinned host arrays; steady state after 40 calls")
    return res


def gather_floats(vals, world: int, dev, backend: str):
    """Every rank's values (a list of floats) on every rank: list of per-rank lists."""
    import torch
    import torch.distributed as dist
    where = dev if backend == "nccl" else "cpu"
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=where)
    rows = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(rows, t)
    return [r.cpu().tolist() for r in rows]


def max_over_ranks(el: float, world: int, dev, backend: str) -> float:
    return max(r[0] for r in gather_floats([el], world, dev, backend))


def per_rank_projection(name: str):
    """The per-rank steps of `name`'s list measured on one GPU (tools/shard_step_ab.py: rank 0's shard of the list
    sharded by sum n*m over N ranks, scored alone; the committed profile named in `source`), and the speed-ups over
    one GPU they project for N ranks on N GPUs -- each rank on its own GPU, link and CPU share, so this prices the
    per-rank step, not the host memory all ranks of one node share.  None when no profile is committed."""
    src = os.path.join("profiles", "r05_cfg4_shard_steps.json" if name == "cfg4" else "r06_shard_steps.json")
    try:
        with open(os.path.join(ROOT, src)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if "runs" in d:  # (round 6: several boxes, resident-grid forms beside the default "pipeline"; the first box)
        d = d["runs"][0]
    ms = {int(r["ranks"]): float(r["median_ms"]) for r in d.get("results", [])
          if r.get("setting", "default") in ("default", "def", "pipeline")}
    if 1 not in ms:
        return None
    return {"source": src, "config": d.get("config"), "ms_per_rank_step": ms,
            "projected_speedup": {n: round(ms[1] / v, 2) for n, v in sorted(ms.items())},
            "projected_efficiency": {n: round(ms[1] / v / n, 2) for n, v in sorted(ms.items())}}


def strong_scaling(name: str, world: int, rank: int, dev, backend: str, steps: int, warmup: int):
    """One read set of `name`, its candidate list sharded by sum n*m over the ranks, every rank's results into
    rank 0's shared pinned host buffer (ShardedStep, dest="host"); then rank 0 alone scores the whole list
    on its GPU (the one-GPU time of the same workload, same run) while the others wait; parity of the
    gathered result against that."""
    import torch.distributed as dist
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    from ovlgraph.sharded import ShardedStep
    t0 = time.perf_counter()
    reads, _ = dedup_reads(config_reads(name, seed=0))  # the same list on every rank
    eng = OverlapEngine(dev.index)
    st = ShardedStep(reads, k=CONFIGS[name]["k"], engine=eng, dest="host")
    setup = time.perf_counter() - t0
    el = timed_steps(st.step, steps, warmup, dev, world)
    el_max = max_over_ranks(el, world, dev, backend)
    one = None
    ok = None
    if rank == 0:
        got = st.results()
        out = (pinned_empty(st.n_pairs), pinned_empty(st.n_pairs))
        one = timed_steps(lambda: eng.score_candidates(out=out), steps, warmup, dev, 1)
        ok = bool(np.array_equal(got[0], out[0]) and np.array_equal(got[1], out[1]))
    dist.barrier()
    st.close()
    eng.close()
    if rank != 0:
        return None
    return {"workload": f"{name}: {WORKLOAD_DESC[name]}", "reads": len(reads), "pairs": st.n_pairs,
            "ms_per_step": el_max / steps * 1e3, "pairs_per_s": st.n_pairs * steps / el_max,
            "one_gpu_ms_per_step": one / steps * 1e3, "one_gpu_pairs_per_s": st.n_pairs * steps / one,
            "speedup_vs_one_gpu": one / el_max, "matches_one_gpu": ok, "setup_s": round(setup, 2),
            "scaling": "strong", "per_rank_projection": per_rank_projection(name),
            "what": "one shared list sharded by sum n*m, each rank's (score, end) into rank 0's shared pinned host "
                    "buffer (step fence in shared memory); one_gpu: rank 0 alone scores the whole list in the "
                    "same run (others idle)"}


GATHER_DESC = ("dest=host: every rank's kernels store its shard's (score, end) over its own GPU's PCIe link "
               "straight into its slice of one pinned host buffer that rank 0 owns (POSIX shared memory, each "
               "rank pins its pages); a step fence of per-rank counters in the buffer's header page orders the "
               "steps (rank 0 returns when every slice has landed; no collective per step), two result slots "
               "(step k into slot k % 2: a rank may score step k while rank 0 still waits for step k - 1); "
               "SURVEY §8e's per-device D2H into pinned host slices")


def sharded_list(name: str, world: int, rank: int, dev, backend: str, args):
    """The N > 1 headline (north_star: candidate pairs sharded across the GPUs): ONE read set of the workload
    (seed args.seed on every rank, so every rank holds the same reads and enumerates the same list), its
    candidate list sharded by sum n*m, every rank's (score, end) into rank 0's shared pinned host buffer.
    Also: rank 0's in-step rooflines on its shard (every rank times its own shard at the same time), the
    whole list scored by rank 0's GPU alone in the same run, parity of the gathered results against that,
    and the same shards gathered into rank 0's HBM by dist.gather (RCCL send/recv over xGMI) instead."""
    import torch.distributed as dist
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.sharded import ShardedStep
    t0 = time.perf_counter()
    w = Workload(name, seed=args.seed, dev=dev)
    st = ShardedStep(w.reads, k=w.cfg["k"], engine=w.eng, dest="host")
    assert st.n_pairs == w.n_pairs
    w.refresh_device_list()
    w.set_shard(rank, world, st.lo, st.hi, out=(st.shared.score, st.shared.end))
    setup = time.perf_counter() - t0
    el = timed_steps(st.step, args.steps, args.warmup, dev, world)
    rows = gather_floats([el, st.hi - st.lo], world, dev, backend)
    el_max = max(r[0] for r in rows)
    # every rank's in-step launches at once (each its own shard, as in the step); rank 0 reports its own
    roof, table, step_roof = in_step_rooflines(w, el / args.steps * 1e3)
    dist.barrier()
    st.step()  # one fenced step: rank 0's buffer holds every slice of it
    one = ok = None
    if rank == 0:
        got = st.results()
        out = (pinned_empty(w.n_pairs), pinned_empty(w.n_pairs))
        one = timed_steps(lambda: w.eng.score_candidates(out=out), args.steps, args.warmup, dev, 1)
        ok = bool(np.array_equal(got[0], out[0]) and np.array_equal(got[1], out[1]))
    dist.barrier()
    w.out = w.own_out  # drop the views of the shared buffer, so that it can be unmapped and unlinked
    st.close()
    # the same shards gathered by a collective into rank 0's HBM (north_star's "RCCL gather"); results end on
    # rank 0's GPU, not in host memory, so this is not the metric's step
    g = ShardedStep(w.reads, k=w.cfg["k"], engine=w.eng, dest="rank0")
    el_g = max_over_ranks(timed_steps(g.step, args.steps, args.warmup, dev, world), world, dev, backend)
    g_ok = None
    if rank == 0:
        got = g.results()
        g_ok = bool(np.array_equal(got[0], out[0]) and np.array_equal(got[1], out[1]))
    g.close()
    w.refresh_device_list()
    res = {"w": w, "el_max": el_max, "pairs_per_rank": [int(r[1]) for r in rows],
           "per_rank_ms_per_step": [r[0] / args.steps * 1e3 for r in rows],
           "roofline": roof, "in_step_kernels": table, "step_roofline": step_roof, "setup_s": round(setup, 2)}
    if rank == 0:
        res.update(one_gpu_ms_per_step=one / args.steps * 1e3, one_gpu_pairs_per_s=w.n_pairs * args.steps / one,
                   speedup_vs_one_gpu=one / el_max, matches_one_gpu=ok,
                   per_rank_projection=per_rank_projection(name),
                   rccl_gather={"dest": "rank0", "backend": backend, "ms_per_step": el_g / args.steps * 1e3,
                                "pairs_per_s": w.n_pairs * args.steps / el_g, "matches_one_gpu": g_ok,
                                "bytes_per_step": g.gather_bytes(),
                                "what": "the same shards scored into each rank's HBM and collected by one "
                                        "dist.gather to rank 0 (RCCL send/recv over xGMI on backend nccl; over "
                                        "gloo when ranks share a GPU); results end in rank 0's HBM, not in host "
                                        "memory, so not the metric's step"})
    return res


def weak_scaling(name: str, world: int, rank: int, dev, backend: str, args):
    """Every rank its own read set of the workload (seed + rank): independent graph builds side by side, the
    reference's joblib shape (experiments.py:537); no data-path collective."""
    w = Workload(name, seed=args.seed + rank, dev=dev)
    el = timed_steps(w.step, args.steps, args.warmup, dev, world)
    rows = gather_floats([el, w.n_pairs, len(w.reads)], world, dev, backend)
    w.close()
    if rank != 0:
        return None
    el_max = max(r[0] for r in rows)
    pairs = [int(r[1]) for r in rows]
    return {"value": sum(pairs) * args.steps / el_max, "unit": "overlap-pairs/s", "scaling": "weak",
            "ms_per_step": el_max / args.steps * 1e3, "pairs": sum(pairs), "pairs_per_rank": pairs,
            "reads_per_rank": [int(r[2]) for r in rows], "seeds": [args.seed + r for r in range(world)],
            "per_rank_ms_per_step": [r[0] / args.steps * 1e3 for r in rows],
            "what": f"x{world} weak: every rank scores its own read set's device-enumerated list into its own "
                    f"pinned host arrays (graph builds side by side, as the reference's joblib workers, "
                    f"experiments.py:537); no data-path collective"}


def multi_line(args, world: int, ident: dict, top: dict, extras: dict) -> dict:
    """Rank 0's N > 1 line: the sharded list at the top, the secondary shapes beside it.  `top` holds the
    measurements of sharded_list (or None-valued placeholders in a dry run)."""
    name = args.config or "target"
    w = top.get("w")
    pairs = w.n_pairs if w is not None else None
    el = top.get("el_max")
    line = {
        "metric": METRIC, "value": pairs * args.steps / el if el else None, "unit": "overlap-pairs/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3 if el else None,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
        "config": {"workload": f"{name}: {WORKLOAD_DESC[name]}", "reads": len(w.reads) if w is not None else None,
                   "pairs": pairs, "pairs_per_rank": top.get("pairs_per_rank"), "seed": args.seed,
                   "read_length": w.cfg["l"] if w is not None else None,
                   "parallelism": f"pair-sharded x{world}: one process per GPU, one read set and its "
                                  f"device-enumerated candidate list on every rank, contiguous shards balanced by "
                                  f"sum n*m, each rank's results into rank 0's shared pinned host buffer",
                   "kernel": w.kernel if w is not None else None,
                   "scoring": {"match": 10, "mismatch": -1, "indel": w.indel if w is not None else None, "band": -1}},
        **ident,
        "gather": {"dest": "host", "fence": "shm", "bytes_per_step": 8 * pairs if pairs else None,
                   "what": GATHER_DESC},
        "one_gpu_ms_per_step": top.get("one_gpu_ms_per_step"),
        "one_gpu_pairs_per_s": top.get("one_gpu_pairs_per_s"),
        "speedup_vs_one_gpu": top.get("speedup_vs_one_gpu"),
        "matches_one_gpu": top.get("matches_one_gpu"),
        "per_rank_projection": top.get("per_rank_projection"),
        "per_rank_ms_per_step": top.get("per_rank_ms_per_step"),
        "roofline": top.get("roofline"),
        "in_step_kernels": top.get("in_step_kernels"),
        "step_roofline": top.get("step_roofline"),
        "rccl_gather": top.get("rccl_gather"),
        "setup_s": top.get("setup_s"),
        "cpu_baseline": None,
        "cpu_baseline_note": "the CPU baseline runs on rank 0 at N = 1 only (bench contract); see the N = 1 line",
    }
    if line["roofline"] is not None:
        line["roofline"]["what"] = "rank 0's shard: " + line["roofline"]["what"]
    line.update(extras)
    return line


def extra_plan(args, world: int):
    """The secondary N > 1 measurements this run makes, in order (empty with --no-extra)."""
    if args.no_extra:
        return []
    name = args.config or "target"
    plan = ["weak_scaling"]
    if name != "cfg4":
        plan.append("cfg4_strong")  # BASELINE configs[3]: 8x pair-sharded
    if name != "cfg5":
        plan.append("cfg5_sharded_band_sweep")  # BASELINE configs[4]: the band sweep across the ranks (4x)
    plan.append("single_process_all_gpus")  # the reference's own shape: one process over the job's GPUs
    return plan


SHARDED_SWEEP_BANDS = [4, 8, 16, 32, 64, -1]


class Heartbeat:
    """Rank 0's progress on stderr while the N > 1 stages run: a line when a stage ends and, from a daemon thread,
    one every `every` seconds naming the stage still running, so a long stage never reads as a hung run (a
    harness ends a command that writes nothing for 3 minutes)."""

    def __init__(self, rank: int, every: float = 30.0):
        import threading
        self.rank, self.every, self.t0 = rank, every, time.perf_counter()
        self.stage = "setup"
        self._stop = threading.Event()
        self._thread = None
        if rank == 0 and every > 0:
            self._thread = threading.Thread(target=self._beat, daemon=True)
            self._thread.start()

    def _beat(self):
        while not self._stop.wait(self.every):
            print(f"bench.py: {self.stage} still running at {time.perf_counter() - self.t0:.1f} s", file=sys.stderr,
                  flush=True)

    def start(self, stage: str):
        self.stage = stage

    def done(self, what: str):
        if self.rank == 0:
            print(f"bench.py: {what} done at {time.perf_counter() - self.t0:.1f} s", file=sys.stderr, flush=True)

    def close(self):
        self._stop.set()


def run_extras(plan, run_stage, budget_s: float, elapsed_max, hb: Heartbeat) -> dict:
    """The secondary N > 1 stages in order, each under the run's time budget: a stage starts only while the
    slowest rank's elapsed time (elapsed_max(): the same value on every rank, so every rank takes the same
    decision and no collective is left waiting) is below budget_s; the others are recorded as skipped."""
    extras = {}
    for item in plan:
        spent = elapsed_max()
        if spent >= budget_s:
            extras[item] = {"skipped": f"the N > 1 stages' time budget ({budget_s:.0f} s) was spent "
                                       f"({spent:.1f} s) before this stage"}
            hb.done(f"{item} skipped,")
            continue
        hb.start(item)
        extras[item] = run_stage(item)
        hb.done(item)
    return extras


def multi_gpu(args, world: int, rank: int, dev, backend: str, shared: bool):
    """N > 1: the workload's one list sharded over the ranks (the line's value), then the secondary shapes."""
    import torch
    import torch.distributed as dist
    name = args.config or "target"
    ident = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
             "devices_visible": torch.cuda.device_count(), "devices_shared": shared,
             "rank0_numa_node": int(os.environ["OVL_BENCH_NUMA_NODE"]) if os.environ.get("OVL_BENCH_NUMA_NODE") else None}
    if shared:
        ident["note"] = ("more ranks than visible GPUs: ranks share devices (flow rehearsal, gloo barriers) -- "
                         "not a scaling number")
    hb = Heartbeat(rank)
    hb.start("sharded list")
    top = sharded_list(name, world, rank, dev, backend, args)
    hb.done("sharded list")
    w = top["w"]

    def run_stage(item):
        if item == "weak_scaling":
            r = weak_scaling(name, world, rank, dev, backend, args)
        elif item == "cfg4_strong":
            r = strong_scaling("cfg4", world, rank, dev, backend, max(5, args.steps // 2), 2)
        elif item == "cfg5_sharded_band_sweep":
            r = sharded_band_sweep(world, rank, dev, w.eng, SHARDED_SWEEP_BANDS, args.sweep_indel, 3, backend)
        else:
            r = single_process_all_gpus(rank, world, shared, w.reads, w.cfg["k"], args.steps, w.eng)
        dist.barrier()
        return r

    extras = run_extras(extra_plan(args, world), run_stage, args.extra_budget,
                        lambda: max_over_ranks(time.perf_counter() - hb.t0, world, dev, backend), hb)
    hb.close()
    line = multi_line(args, world, ident, top, extras) if rank == 0 else None
    w.close()
    return line


def gpu_numa_node(dev) -> int:
    """The NUMA node the GPU's PCIe link hangs off (sysfs), or -1."""
    import torch
    pr = torch.cuda.get_device_properties(dev)
    path = "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
    try:
        with open(path) as fh:
            return int(fh.read().strip())
    except (OSError, ValueError):
        return -1


def bind_to_gpu_node(dev):
    """One process per GPU on a 2-socket host (4 GPUs per socket on the MI355X nodes): run this rank's threads
    on its GPU's NUMA node, so its pinned result arrays, staging and host-pool threads are socket-local -- N
    ranks each write ~16 MB of results per step into host memory, and remote-socket traffic would cross the
    inter-socket link.  Returns the node, or None when unknown or not allowed."""
    node = gpu_numa_node(dev)
    if node < 0:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            spec = fh.read().strip()
        cpus = set()
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return node
    except (OSError, ValueError):
        return None


def spawn_ranks(n: int) -> int:
    """--gpus N > 1 without a launcher: run torch.distributed.run with N ranks of this script as a child
    process (never an exec: nothing here has touched the GPU) and return its exit status."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=sorted(WORKLOAD_DESC),
                    help="workload at every N (default: the north_star target point)")
    ap.add_argument("--seed", type=int, default=0,
                    help="read-set seed (the secondary weak-scaling field: rank r uses seed + r)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the extra configs and stages")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="leave the CPU affinity alone (default: each process on its GPU's NUMA node)")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of all-core CPU-baseline work")
    ap.add_argument("--indel", type=int, default=None, help="indel score (default: the reference's -2**31)")
    ap.add_argument("--band", type=int, default=-1, help="band half-width (-1 = full DP, the reference)")
    ap.add_argument("--band-sweep", default=None,
                    help="comma list of bands (-1 = full) timed on the same workload at --sweep-indel")
    ap.add_argument("--sweep-indel", type=int, default=-2)
    ap.add_argument("--sweep-steps", type=int, default=5)
    # launcher checks without a GPU (tests/test_bench_launch.py): ranks join a gloo group, rank 0 prints the
    # identity line, and --dry-run-fail-rank R makes rank R exit with status 3
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    # the N > 1 code path at world size 1 (torch.distributed over RCCL with one rank): a one-GPU box runs the
    # multi-process line's collectives, gathers and sharded step for real (tests/test_gpu_bench_dist.py)
    ap.add_argument("--dist-path", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--dry-run-stage-s", type=float, default=0.0, help=argparse.SUPPRESS)  # each stage sleeps this
    ap.add_argument("--extra-budget", type=float, default=240.0,
                    help="seconds after which the N > 1 run starts no further secondary stage")
    ap.add_argument("--heartbeat", type=float, default=30.0, help=argparse.SUPPRESS)
    # profiling aid at N = 1: time only shard R of N of the list (what rank R scores at N ranks), so rocprofv3 and
    # PMC passes on a one-GPU box see a rank's launches (tools/gpu_r04_shard_profile.sh)
    ap.add_argument("--shard", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    return args


def launch_plan(gpus: int, env) -> str:
    """What this process does: "spawn" (start gpus ranks as a child launcher), "rank" (one rank of a
    launched job), "single" (N = 1), or an error message when --gpus and WORLD_SIZE disagree."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 else "single"
    try:
        w = int(ws)
    except ValueError:
        return f"error: WORLD_SIZE={ws!r} is not an integer"
    if w != gpus:
        return f"error: --gpus {gpus} but WORLD_SIZE={w} (launch N ranks with --gpus N)"
    return "rank" if w > 1 else "single"


def dry_run(args) -> int:
    """The launch path alone (no GPU): join the process group over gloo and print the line rank 0 would print,
    built by the same code (multi_line) with every measurement left null, so the launcher tests see which
    fields and secondary shapes a run at this N carries."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    if rank == args.dry_run_fail_rank:
        return 3
    if world > 1:
        dist.barrier()
    # the stages' budget and heartbeat as a real run takes them (each stage sleeps --dry-run-stage-s instead)
    hb = Heartbeat(rank, args.heartbeat)

    def elapsed_max():
        if world == 1:
            return time.perf_counter() - hb.t0
        import torch
        t = torch.tensor([time.perf_counter() - hb.t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def run_stage(item):
        time.sleep(args.dry_run_stage_s)
        if world > 1:
            dist.barrier()
        return None

    extras = run_extras(extra_plan(args, world), run_stage, args.extra_budget, elapsed_max, hb)
    hb.close()
    if rank == 0:
        ident = {"world_size": dist.get_world_size() if world > 1 else 1,
                 "backend": dist.get_backend() if world > 1 else None}
        line = multi_line(args, world, ident, {}, extras)
        line["dry_run"] = True
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main() -> int:
    args = parse_args()
    plan = launch_plan(args.gpus, os.environ)
    if plan.startswith("error"):
        print(f"bench.py: {plan}", file=sys.stderr)
        return 2
    if plan == "spawn":
        return spawn_ranks(args.gpus)
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = torch.cuda.device_count()  # (does not initialise the GPU)
    shared = world > max(1, n_dev)
    # one process per GPU; ranks beyond the visible devices (flow rehearsal on a 1-GPU box) share them, and
    # RCCL refuses two ranks on one GPU, so those run gloo
    local = local % max(1, n_dev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("OVL_BENCH_BACKEND") or ("gloo" if shared else "nccl")  # nccl = RCCL on ROCm
    numa = None
    # (N = 1 too: on the 2-socket box the step's host side -- expansion threads, pinned arrays -- runs on whichever
    # socket the scheduler picks; bound, 0.140-0.149 ms against 0.138-0.169 unbound, tools/gpu_r04_numa.sh)
    if not shared and not args.no_numa_bind:
        numa = bind_to_gpu_node(dev)  # before the engine, its host pool and any pinned allocation
    os.environ["OVL_BENCH_NUMA_NODE"] = "" if numa is None else str(numa)
    if world > 1 or args.dist_path:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        line = multi_gpu(args, world, rank, dev, backend, shared)
        if rank == 0:
            print(json.dumps(line), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return 0

    name = args.config or "target"
    w = Workload(name, seed=args.seed, dev=dev, indel=args.indel, band=args.band)
    if args.shard:
        r, n = (int(x) for x in args.shard.split("/"))
        cuts = w.eng.candidate_shards(n)
        w.set_shard(r, n, cuts[r], cuts[r + 1])
    elapsed = timed_steps(w.step, args.steps, args.warmup, dev, 1)
    ms_step = elapsed / args.steps * 1e3
    roof, table, step_roof = in_step_rooflines(w, ms_step)
    if args.shard:
        print(json.dumps({"shard": args.shard, "workload": w.profile_key, "pairs": w.hi - w.lo,
                          "ms_per_step": ms_step, "pairs_per_s": (w.hi - w.lo) * args.steps / elapsed,
                          "roofline": roof, "in_step_kernels": table, "step_roofline": step_roof}), flush=True)
        return 0
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
            "seed": args.seed,
            "step": "ovl_score_candidates: resident reads + device-enumerated list -> kernels storing over the "
                    "link -> (score, end) in pinned host int32 arrays (SURVEY.md §8d, results in host memory; "
                    "packed 2 B/pair chunks expanded by host threads while the next chunk scores, the last "
                    "~20 % stored directly)",
            "parallelism": "1 GPU",
            "host_numa_node": int(os.environ["OVL_BENCH_NUMA_NODE"]) if os.environ.get("OVL_BENCH_NUMA_NODE") else None,
            "kernel": w.kernel,
            "scoring": {"match": 10, "mismatch": -1, "indel": w.indel, "band": w.band},
        },
        "roofline": roof,
        "in_step_kernels": table,
        "step_roofline": step_roof,
        "kernel_only_roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(name, kernel_name(w, 0, w.n_pairs)), "kernel_ms": kernel_ms,
            "algorithmic_bytes_per_launch": algo, "kernel": kernel_name(w, 0, w.n_pairs),
            "what": "the same list through the kernel with HBM outputs alone (not in the step; HIP events on its "
                    "launch stream)"},
        "valu_roofline": valu_roofline(name, kernel_ms, kernel_name(w, 0, w.n_pairs)),
        "kernel_only_pairs_per_s": w.n_pairs / (kernel_ms * 1e-3),
        "step_breakdown": step_breakdown(w, ms_step),
        "occupancy": load_profile(name, kernel_name(w, 0, w.n_pairs)).get("occupancy"),
        "host_setup_s": dict(w.t_stages, read_simulation=round(w.t_sim, 4)),
    }
    if not args.no_extra:
        line["abi_one_shot"] = abi_one_shot(w)
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
        # "share": the threads the port ran on (cpu_baseline.cores: OMP_NUM_THREADS, else the affinity mask -- the
        # box's 16-CPU share, not the machine's cores)
        line["vs_cpu_baseline"] = {"share_threads": cb["cores"],
                                   "share_threads_full_dp": value / cb["value"],
                                   "one_core_full_dp": value / cb["one_core"]["value"],
                                   "share_threads_closed_form": value / cb["closed_form"]["value"]}
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
