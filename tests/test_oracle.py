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

from conftest import (GOLDEN, ORACLE, REF_BIN, GEN, load_cases, oracle_count, sorted_digest_file)

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
