"""GPU: the Bloom filter's hashing and positions, pinned bit for bit.

Bloom results for -a >= 2 do not depend on the hash (the filter only gates), so the
golden cases cannot catch a wrong device hash or a wrong position count.  These tests
read the device filter itself (kc_bloom_read) after inserting one k-mer:
  * device XXH64 (kc_xxh64, the function of the reference layout) == the vendored
    xxHash v0.8.2 golden vectors (tests/golden/xxh64.json);
  * pass 1 sets exactly the ceil(hf) filter-1 positions of the k-mer (main.cpp:417),
    a second occurrence the same positions of filter 2 (insertion_process,
    double_bloomfilter.hpp:371-413), in both layouts, fpr 0.01 / 0.001 / 0.05;
  * the pass-2 gate tests exactly the trunc(hf) filter-2 positions
    (parallel_parser.hpp:2397,2436-2441): clearing position trunc(hf) (past the gate)
    keeps the k-mer, clearing any gate position drops it.
The expected positions come from tests/bloom_model.py (the reference's formulas for
its layout; the engine's block formulas for the blocked one).
"""
import json
import os
import random

import pytest

import bloom_model as bm
import kaarme_amd as ka
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_device_xxh64_matches_golden_vectors():
    vec = json.load(open(os.path.join(GOLDEN, "xxh64.json")))["vectors"]
    got = ka.xxh64_device([v["value"] for v in vec], [v["seed"] for v in vec])
    assert got == [v["xxh64"] for v in vec]
    # and on the roots the passes feed it (values < 2^54), against the model
    rng = random.Random(1)
    vals = [rng.getrandbits(54) for _ in range(500)]
    seeds = [bm.SEEDS[i % 10] for i in range(500)]
    assert ka.xxh64_device(vals, seeds) == [bm.xxh64_u64(v, s) for v, s in zip(vals, seeds)]


@pytest.fixture(params=["blocked", "reference"])
def layout(request, monkeypatch):
    if request.param == "reference":
        monkeypatch.setenv("KC_BLOOM_LAYOUT", "reference")
    else:
        monkeypatch.delenv("KC_BLOOM_LAYOUT", raising=False)
    return request.param


@pytest.fixture(params=["direct", "partitioned"])
def bloom_path(request, monkeypatch):
    monkeypatch.setenv("KC_INSERT_PATH", request.param)
    return request.param


def _counter(k, fpr, U=20000):
    return ka.KmerCounter(ka.Config(k=k, mode=2, bf_enable=True, est_unique=U, fpr=fpr, min_abundance=1,
                                    batch_bytes=1 << 20))


@pytest.mark.parametrize("k", [31, 51])
@pytest.mark.parametrize("fpr", [0.01, 0.001, 0.05])
def test_pass1_sets_ceil_hf_positions(k, fpr, layout, bloom_path):
    rng = random.Random(k * 1000 + int(fpr * 1000))
    kmer = "".join(rng.choice("ACGT") for _ in range(k))
    bits, nh, ng = bm.sizes(20000, fpr)
    with _counter(k, fpr) as kc:
        info = kc.bloom_info()
        assert (info["bits"], info["nh"], info["nh_gate"], info["layout"]) == (bits, nh, ng, layout)
        kc.bloom_chunk((kmer + "\n").encode(), ka.FMT_PLAIN)
        f1, f2 = bm.positions(kmer, bits, nh, layout)
        assert bm.set_bits(kc.bloom_read()) == set(f1)
        kc.bloom_chunk((kmer + "\n").encode(), ka.FMT_PLAIN)  # second occurrence: filter 2
        assert bm.set_bits(kc.bloom_read()) == set(f1) | set(f2)


@pytest.mark.parametrize("fpr", [0.01, 0.001, 0.05])
def test_pass2_gate_tests_trunc_hf_positions(fpr, layout, bloom_path):
    k = 31
    rng = random.Random(int(fpr * 10000))
    kmer = "".join(rng.choice("ACGT") for _ in range(k))
    bits, nh, ng = bm.sizes(20000, fpr)
    f1, f2 = bm.positions(kmer, bits, nh, layout)
    # clear one filter-2 position: j = ng is past the gate (kept), j < ng is tested (dropped)
    for j in sorted({ng, 0, ng - 1}):
        if j >= nh:
            continue
        with _counter(k, fpr) as kc:
            for _ in range(2):
                kc.bloom_chunk((kmer + "\n").encode(), ka.FMT_PLAIN)
            kc.bloom_finalize()
            words = kc.bloom_read()
            w, b = f2[j]
            words[w] &= ~(1 << b) & 0xFFFFFFFF
            kc.bloom_write(words)
            set_now = bm.set_bits(words)
            passes = all(p in set_now for p in f2[:ng])  # the gate: positions j < trunc(hf)
            kc.count_chunk((kmer + "\n").encode(), ka.FMT_PLAIN)
            kc.finish()
            assert kc.lines() == ([f"{min(kmer, bm_rc(kmer))} 1"] if passes else []), (j, nh, ng)


def bm_rc(s):
    return "".join({"A": "T", "C": "G", "G": "C", "T": "A"}[c] for c in reversed(s))
