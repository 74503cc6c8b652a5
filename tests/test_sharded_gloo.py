"""N>1 path on CPU: world_size-2 gloo ranks shard the pair list and gather results in order."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ovlgraph.sharded import shard_bounds


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            cost = np.random.default_rng(n + w).integers(1, 100, size=n)
            c = [shard_bounds(n, w, r, cost) for r in range(w)]
            assert c[0][0] == 0 and c[-1][1] == n
            assert all(c[i][1] == c[i + 1][0] and c[i][0] <= c[i][1] for i in range(w - 1))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "genome-assembly-using-overlap-graphs_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist
    import oracle
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    from ovlgraph.sharded import score_pairs_sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    reads = simulate_reads(read_genome_from_fasta(), 60, 600, 0.02, seed=11)
    distinct, _ = dedup_reads(reads)
    a, b = enumerate_candidates(distinct, 3)
    sc, en = score_pairs_sharded(distinct, a, b, local_scorer=lambda r, x, y: oracle.batch_ungapped(r, x, y))
    # the repeated-step form bench.py times at N > 1: setup once, step twice, gather in reference order
    from ovlgraph.sharded import ShardedStep
    st = ShardedStep(distinct, a, b, local_scorer=lambda r, x, y: oracle.batch_ungapped(r, x, y))
    st.step()
    st.step()
    sc2, en2 = st.results()
    assert st.gather_bytes() == world * 2 * st.width * 4
    if rank == 0:
        q.put((a, b, sc, en, distinct, sc2, en2))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_single_process(oracle_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    a, b, sc, en, distinct, sc2, en2 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref_sc, ref_en = oracle_mod.batch_dp(distinct, a, b)
    assert len(a) > 100
    np.testing.assert_array_equal(sc, ref_sc)
    np.testing.assert_array_equal(en, ref_en)
    np.testing.assert_array_equal(sc2, ref_sc)
    np.testing.assert_array_equal(en2, ref_en)
