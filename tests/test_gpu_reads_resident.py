"""ovl_set_reads keeps a read set that is already resident (same offsets, and the same 128-bit digest of its bytes)
instead of uploading and packing it again; any difference -- one base, a moved read boundary, another read count,
the same bytes at another address -- must reach the device.  Each case is checked against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _reads(rng, n, lo=20, hi=120):
    return ["".join(rng.choice(list("ACGT"), size=int(rng.integers(lo, hi)))) for _ in range(n)]


def test_resident_reads_follow_every_change(oracle_mod):
    from ovlgraph import OverlapEngine
    from ovlgraph.engine import encode_reads
    rng = np.random.default_rng(3)
    reads = _reads(rng, 300)
    a = rng.integers(0, len(reads), 5000, dtype=np.int32)
    b = rng.integers(0, len(reads), 5000, dtype=np.int32)

    def check(eng, rs, enc=None, x=a, y=b):
        sc, en = eng.score_pairs(rs, x, y, encoded=enc)
        es, ee = oracle_mod.batch_dp(rs, x, y)
        np.testing.assert_array_equal(sc, es)
        np.testing.assert_array_equal(en, ee)

    with OverlapEngine(0) as eng:
        check(eng, reads)
        check(eng, reads)                                 # resident: same content
        buf, offs = encode_reads(reads)
        check(eng, reads, (buf.copy(), offs.copy()))      # same content at other addresses
        changed = list(reads)
        r = changed[7]
        changed[7] = r[:5] + ("A" if r[5] != "A" else "C") + r[6:]
        check(eng, changed)                               # one base
        check(eng, reads)                                 # and back
        moved = list(reads)
        moved[10], moved[11] = moved[10] + moved[11][:3], moved[11][3:]  # same bytes, one boundary moved
        check(eng, moved)
        check(eng, reads)
        keep = (a < len(reads) - 1) & (b < len(reads) - 1)
        check(eng, reads[:-1], x=a[keep], y=b[keep])      # one read fewer: a different set
        check(eng, reads)
        # the resident list goes with every set_reads, uploaded or kept
        eng.candidates(5)
        eng.set_reads(reads)
        with pytest.raises(Exception):
            eng.score_candidates()


def test_resident_reads_digest_over_parts(oracle_mod):
    """A read set of ~0.7 MB (the digest runs in 256 KiB parts on the host pool, 256-byte blocks of 32 lanes, then
    a tail): one base changed in each part -- at the start of the set, in the middle part's lane blocks, in the
    last bytes (the tail) -- reaches the device every time, and the unchanged set stays resident."""
    from ovlgraph import OverlapEngine
    rng = np.random.default_rng(11)
    reads = _reads(rng, 6000, 100, 130)
    total = sum(len(r) for r in reads)
    assert total > 2 * (1 << 18)
    starts = np.cumsum([0] + [len(r) for r in reads])

    def read_at(byte):
        return int(np.searchsorted(starts, byte, side="right") - 1)

    with OverlapEngine(0) as eng:
        for byte in (3, (1 << 18) + 5000, total - 2):
            i = read_at(byte)
            others = rng.integers(0, len(reads), 400, dtype=np.int32)
            a = np.concatenate([np.full(400, i, np.int32), others])
            b = np.concatenate([others, np.full(400, i, np.int32)])
            changed = list(reads)
            r = changed[i]
            k = byte - starts[i]
            changed[i] = r[:k] + ("A" if r[k] != "A" else "G") + r[k + 1:]
            want = [oracle_mod.batch_dp(rs, a, b) for rs in (reads, changed)]
            # (the change must show in some pair's result, or the check below could not see a stale set)
            assert not (np.array_equal(want[0][0], want[1][0]) and np.array_equal(want[0][1], want[1][1]))
            for rs, (es, ee) in zip((reads, changed, reads), want + want[:1]):
                sc, en = eng.score_pairs(rs, a, b)
                np.testing.assert_array_equal(sc, es, err_msg=f"byte {byte}")
                np.testing.assert_array_equal(en, ee, err_msg=f"byte {byte}")
