"""GPU: Kaarme's compact representation built from the counted table.

kc_compact writes the reference's 8-byte slot words (kmer.hpp:103-149) plus a secondary
array of chain-start keys; every k-mer must come back, with its count, from
  * the device reconstruction (kc_compact_dump: the reference fixtures' sorted output),
  * the reference's own walk restated in Python (compact_model.reconstruct, from
    kmer_hash_table.cpp:3848-4058) over the copied slot words, and
  * lookups by key through the compact words alone (kc_compact_lookup).
"""
import subprocess

import numpy as np
import pytest

from compact_model import reconstruct
from conftest import GEN, load_cases, oracle_count, sorted_digest_file, sorted_digest_lines
import kaarme_amd as ka

pytestmark = pytest.mark.gpu

def _args(case):
    a = case["args"]
    return (int(a[a.index("-m") + 1]) if "-m" in a else 2), (int(a[a.index("-a") + 1]) if "-a" in a else 2)


CASES = [c for c in load_cases()["cases"] if "-b" not in c["args"] and _args(c)[0] != 0]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['input']}-k{c['k']}-" + "".join(a.strip("-") for a in c["args"]))
def test_compact_golden(case, golden_input):
    """Counted table -> compact words -> reconstructed k-mers = the reference's output."""
    path = golden_input(case["input"])
    mode, a = _args(case)
    args = case["args"]
    slots = int(args[args.index("-s") + 1]) if "-s" in args else 0
    kc, st = ka.count_file(path, case["k"], mode=mode, min_abundance=a, table_slots=max(slots, 1 << 16))
    with kc:
        info = kc.compact()
        assert info["kmers"] == st["distinct"]
        recs, max_hops, mean_hops = kc.compact_dump()
        lines = sorted(f"{s} {c}" for s, c in ka.decode_records(recs, case["k"]))
        assert sorted_digest_lines(lines) == (case["sorted_sha256"], case["lines"])
        assert max_hops <= max(0, case["k"] - 2)


@pytest.mark.parametrize("k", [5, 15, 21, 31, 32, 33, 51, 63, 64, 95, 127, 200, 255, 300, 479])
def test_compact_reference_walk_and_lookup(tmp_path, k):
    """Synthetic reads (errors, both strands): the slot words walked by the reference's
    algorithm (Python restatement) give the dumped k-mers; lookups by key give the counts,
    absent keys 0; chain starts are a small fraction; walks stay within k - 2 hops."""
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "3000", str(max(150, k + 100)), "40000", "-e", "0.002"], check=True)
    kc, st = ka.count_file(str(fa), k, mode=2, min_abundance=1, table_slots=1 << 20)
    with kc:
        full = kc.dump()
        info = kc.compact(0.85)
        assert info["kmers"] == st["distinct"] == len(full) > 0
        assert info["slots"] >= info["kmers"] / 0.85
        recs, max_hops, mean_hops = kc.compact_dump()
        assert max_hops <= max(0, k - 2)
        got = {tuple(r[:-1]): int(r[-1]) for r in recs.tolist()}
        want = {tuple(r[:-1]): int(r[-1]) for r in full.tolist()}
        assert got == want
        if k >= 21:  # neighbours share their minimizer: most k-mers have a predecessor
            assert info["chain_starts"] < 0.25 * info["kmers"], info
        # the reference's walk over the copied words
        words, second = kc.compact_read(info)
        occ = np.nonzero(words & np.uint64(1))[0]
        rng = np.random.default_rng(k)
        strings = {s: c for s, c in ka.decode_records(full, k)}
        for slot in rng.choice(occ, size=min(400, occ.size), replace=False):
            s, hops = reconstruct(words, second, int(slot), k, max_hops=max(0, k - 2))
            assert strings[s] == (int(words[slot]) >> 12) & 16383
        # lookups: every key, then keys that are not in the table
        assert (kc.compact_lookup(full[:, :-1]) == full[:, -1].astype(np.uint32)).all()
        absent = full[:200, :-1].copy()
        absent[:, -1] ^= np.uint64(1)  # flip the last character's low bit
        expect = np.array([want.get(tuple(r), 0) for r in absent.tolist()], dtype=np.uint32)
        assert (kc.compact_lookup(absent) == expect).all()


def test_compact_saturated_counts_and_homopolymers(tmp_path):
    """Poly-A runs (AAA...A is its own predecessor) and counts past 16383 (saturated)."""
    fa = tmp_path / "polya.fasta"
    with open(fa, "w") as f:
        f.write(">a\n" + "A" * 20000 + "\n>b\n" + "ACGT" * 50 + "T" * 300 + "\n")
    k = 31
    kc, st = ka.count_file(str(fa), k, mode=2, min_abundance=1, table_slots=1 << 16)
    with kc:
        full = kc.dump()
        kc.compact()
        recs, max_hops, _ = kc.compact_dump()
        assert sorted(map(tuple, recs.tolist())) == sorted(map(tuple, full.tolist()))
        out = tmp_path / "oracle.txt"
        oracle_count(str(fa), k, ["-m", "2", "-a", "1"], out)
        lines = [f"{s} {c}" for s, c in ka.decode_records(recs, k)]
        assert sorted_digest_lines(lines) == sorted_digest_file(out)
        assert int(kc.compact_lookup(np.zeros((1, 1), dtype=np.uint64))[0]) == 16383  # AAAA...A


def test_compact_needs_kaarme_counts(tmp_path):
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "100", "150", "4000"], check=True)
    kc, _ = ka.count_file(str(fa), 31, mode=0, min_abundance=1, table_slots=1 << 16)
    with kc:
        with pytest.raises(ka.KcError, match="14 bits"):
            kc.compact()
