"""CPU: pin the C oracle (oracle/kc_oracle_core.h) against the reference.

* every golden case (outputs of the reference CLI, tests/golden/cases.json);
* XXH64 golden vectors from the vendored xxHash v0.8.2;
* when the reference binary was built here (oracle/_ref/kaarme), a live comparison
  on inputs that are not part of the fixtures.
"""
import json
import os
import subprocess

import pytest

from conftest import (GOLDEN, ORACLE, ORACLE_DIR, REF_BIN, GEN, load_cases, oracle_count, sorted_digest_file,
                      text_digest)

DIGEST = os.path.join(ORACLE_DIR, "_ref", "kc_digest")

CASES = load_cases()["cases"]


def _case_id(c):
    return f"{c['input']}-k{c['k']}-" + "".join(a.strip("-") for a in c["args"])


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_oracle_matches_reference_fixture(case, golden_input, tmp_path):
    path = golden_input(case["input"])
    out = tmp_path / "o.txt"
    st = oracle_count(path, case["k"], case["args"], out)
    dig, n = sorted_digest_file(out)
    assert n == case["lines"]
    assert dig == case["sorted_sha256"]
    if case["distinct"] is not None and "-b" not in case["args"]:
        assert st["distinct"] == case["distinct"]


def test_xxh64_vectors():
    with open(os.path.join(GOLDEN, "xxh64.json")) as f:
        vec = json.load(f)["vectors"]
    by_seed = {}
    for v in vec:
        by_seed.setdefault(v["seed"], []).append(v)
    for seed, vs in by_seed.items():
        out = subprocess.run([ORACLE, "xxh64", str(seed)] + [str(v["value"]) for v in vs],
                             capture_output=True, text=True, check=True).stdout.split()
        assert [int(x) for x in out] == [v["xxh64"] for v in vs]


def test_rk_root_is_strand_symmetric():
    """RollingHasherDual F/B mod 2^54 (hash_functions.cpp:102-192): root(x) == root(revcomp(x))."""
    comp = str.maketrans("ACGT", "TGCA")
    for s in ["ACGTTGCAAGGCTTAACGT", "A" * 31, "ACGT" * 20 + "A"]:
        r1 = subprocess.run([ORACLE, "root", str(len(s)), s], capture_output=True, text=True).stdout.split()
        rc = s.translate(comp)[::-1]
        r2 = subprocess.run([ORACLE, "root", str(len(s)), rc], capture_output=True, text=True).stdout.split()
        assert r1[0] == r2[1] and r1[1] == r2[0] and r1[2] == r2[2]


@pytest.mark.skipif(not os.path.exists(REF_BIN), reason="reference binary not built (needs /root/reference)")
@pytest.mark.parametrize("k,args", [
    (27, ["-a", "1", "-s", "500000"]),
    (45, ["-m", "0", "-a", "1", "-s", "500000"]),
    (23, ["-b", "-u", "60000", "-a", "1"]),
    (77, ["-m", "1", "-a", "2", "-s", "500000"]),
])
def test_oracle_matches_live_reference(k, args, tmp_path):
    inp = tmp_path / "live.fasta"
    subprocess.run([GEN, str(inp), "700", "120", "20000", "-s", "1234", "-w", "50", "-n", "0.003", "-e", "0.01"],
                   check=True)
    ro = tmp_path / "ref.txt"
    subprocess.run([REF_BIN, str(inp), str(k), "-t", "3", "-o", str(ro)] + args, check=True, capture_output=True)
    oo = tmp_path / "or.txt"
    oracle_count(str(inp), k, args, oo)
    assert sorted_digest_file(ro) == sorted_digest_file(oo)


def test_bloom_model_xxh64_matches_golden_vectors():
    """The test-side XXH64 of tests/bloom_model.py (used to predict device Bloom
    positions) against the vendored xxHash v0.8.2 vectors."""
    import json
    import bloom_model as bm
    from conftest import GOLDEN
    vec = json.load(open(os.path.join(GOLDEN, "xxh64.json")))["vectors"]
    assert all(bm.xxh64_u64(v["value"], v["seed"]) == v["xxh64"] for v in vec)


def _digest_json(args):
    return json.loads(subprocess.run([DIGEST] + args, capture_output=True, text=True, check=True).stdout)


def _same(a, b):
    return all(a[key] == b[key] for key in ("lines", "count_sum", "hash_sum", "hash_xor"))


# the whole-job digests of tests/golden/fullsize.json (C4, C5) come from `kc_digest count`: it must give
# the digest of the reference's output on every golden case it can restate (no Bloom filter, or a >= 2,
# where the reference's Bloom output equals the unfiltered count)
DIGEST_CASES = [c for c in CASES if "-b" not in c["args"] or int(c["args"][c["args"].index("-a") + 1]) >= 2]


@pytest.mark.parametrize("case", DIGEST_CASES, ids=_case_id)
def test_partitioned_digest_matches_reference_output(case, golden_input, tmp_path):
    path = golden_input(case["input"])
    args = case["args"]
    out = tmp_path / "o.txt"
    oracle_count(path, case["k"], args, out)  # sorted-equal to the reference's output (test above)
    want = text_digest(str(out))
    assert want["lines"] == case["lines"]
    assert _same(_digest_json(["lines", str(out)]) if out.exists() else want, want)
    m = args[args.index("-m") + 1] if "-m" in args else "2"
    a = args[args.index("-a") + 1] if "-a" in args else "2"
    got = _digest_json(["count", path, str(case["k"]), "-m", m, "-a", a, "-p", "3", "-j", "2"])
    assert _same(got, want), (got, want)


def test_digest_is_order_independent(tmp_path):
    p = tmp_path / "o.txt"
    lines = [b"ACGT 3\n", b"CCCA 1\n", b"AAAA 16383\n"]
    p.write_bytes(b"".join(lines))
    q = tmp_path / "r.txt"
    q.write_bytes(b"".join(reversed(lines)))
    assert _same(_digest_json(["lines", str(p)]), _digest_json(["lines", str(q)]))
    assert _same(_digest_json(["lines", str(p)]), text_digest(str(p)))


def test_fullsize_digests_are_consistent():
    """Every full-size fixture with a digest: the digest's lines / count sum are the case's (for the
    reference-run cases these come from the reference's own output), and --ref runs agree."""
    doc = json.load(open(os.path.join(GOLDEN, "fullsize.json")))
    for name, c in doc["cases"].items():
        d = c.get("digest")
        if not d:
            continue
        assert (d["lines"], d["count_sum"]) == (c["lines"], c["count_sum"]), name
        if c.get("ref_digest"):
            assert _same(c["ref_digest"], d), name
