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
