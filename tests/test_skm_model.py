"""The NumPy model of the super-k-mer routing (tests/skm_model.py) on CPU: the packed stream
format both ways, strand symmetry of the canonical-minimizer owner (a k-mer and its reverse
complement have one owner, so the owners' counts are exact), and the super-k-mers covering every
valid window exactly once."""
import numpy as np

import skm_model as sm

COMP = str.maketrans("ACGT", "TGCA")


def _seqs(n, rng, lo=1, hi=200):
    return ["".join("ACGT"[x] for x in rng.integers(0, 4, int(rng.integers(lo, hi)))) for _ in range(n)]


def test_pack_roundtrip():
    rng = np.random.default_rng(1)
    seqs = _seqs(300, rng)
    pk, bk = sm.pack(seqs)
    assert sm.unpack(pk, bk) == seqs
    assert len(pk) == len(bk) == (sum(len(s) + 1 for s in seqs) + 31) // 32


def test_owner_is_strand_symmetric():
    rng = np.random.default_rng(2)
    for k, G in ((31, 8), (51, 3), (127, 5), (9, 4)):
        for s in _seqs(20, rng, k, 3 * k):
            rc = s.translate(COMP)[::-1]
            a = sm.window_owners(sm.CODE[np.frombuffer(s.encode(), np.uint8)], k, G)
            b = sm.window_owners(sm.CODE[np.frombuffer(rc.encode(), np.uint8)], k, G)
            assert (a == b[::-1]).all() and (a >= 0).all() and (a < G).all()


def test_owners_are_balanced():
    """Every owner gets about 1/G of the windows (the minimizer value is mixed before it picks an
    owner: its raw value, a minimum of many hashes, is small)."""
    rng = np.random.default_rng(4)
    seq = "".join("ACGT"[x] for x in rng.integers(0, 4, 200_000))
    for k, G in ((31, 3), (51, 8)):
        own = sm.window_owners(sm.CODE[np.frombuffer(seq.encode(), np.uint8)], k, G)
        share = np.bincount(own, minlength=G) / len(own)
        assert share.min() > 0.5 / G and share.max() < 1.5 / G, share


def test_superkmers_cover_every_window_once():
    rng = np.random.default_rng(3)
    seqs = _seqs(200, rng, 10, 400)
    seqs[0] = seqs[0][:50] + "N" + seqs[0][50:]
    for k, G in ((31, 4), (51, 2), (15, 7)):
        routed = sm.route(seqs, k, G)
        got = sorted(s[i:i + k] for part in routed for s in part for i in range(len(s) - k + 1))
        want = sorted(s[i:i + k] for s in seqs for i in range(len(s) - k + 1) if "N" not in s[i:i + k])
        assert got == want
        for o, part in enumerate(routed):  # every window of an owner's super-k-mers is the owner's
            for s in part:
                assert (sm.window_owners(sm.CODE[np.frombuffer(s.encode(), np.uint8)], k, G) == o).all()
