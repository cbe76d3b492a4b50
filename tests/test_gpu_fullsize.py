"""Reference parity at the benchmarked configurations (BASELINE.md's
parity rule): bench.py's own job -- the device image generated in HBM, one staging batch,
the bench's table geometry, and for C3 the counting pass from the Bloom pass's kept level-2
partitions -- against the reference CLI's output on the same input
(tests/golden/fullsize.json, made by tests/golden/make_fullsize.py from oracle/_ref/kaarme).

Compared: SHA-256 of the byte-sorted output text (kaarme_amd.digest from kc_dump records),
its line count and the sum of its counts; the image's SHA-256 against the file kc_gen wrote
for the reference.  The CPU test pins the digest helper against Python's own sort.
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO

sys.path.insert(0, REPO)

FULLSIZE = os.path.join(GOLDEN, "fullsize.json")


def _fixture():
    with open(FULLSIZE) as f:
        return json.load(f)


def _bench_args(config, share=0):
    import bench
    base = argparse.Namespace(config=config, reads=None, read_len=None, genome=None, k=None, slots=None,
                              unique=None, batch_mib=0, err=0.001, seed=42, share=share, s_table=False)
    return bench, bench.resolve(base, config)


# fixture name -> (bench preset, --share): the strong presets' rank-0 shares at 8 GPUs
SHARES = {"C4S": ("C4", 8), "C5S": ("C5", 8)}


@pytest.mark.parametrize("n", [0, 1, 7, 1000])
@pytest.mark.parametrize("k", [5, 31, 51, 95])
def test_digest_helper_matches_sorted_text(k, n):
    from kaarme_amd import words_for_k
    from kaarme_amd.digest import sorted_text_digest, _text_numpy
    W = words_for_k(k)
    rng = np.random.default_rng(k * 1000 + n)
    keys = set()
    while len(keys) < n:
        keys.add(int(rng.integers(0, 1 << 62)) | (int(rng.integers(0, 1 << 62)) << 62))
    recs = np.zeros((n, W + 1), dtype=np.uint64)
    lines = []
    for i, x in enumerate(sorted(keys)):
        x &= (1 << (2 * k)) - 1
        c = int(rng.choice([1, 2, 9, 10, 99, 100, 16383, 65535]))
        for w in range(W):
            recs[i, W - 1 - w] = (x >> (64 * w)) & ((1 << 64) - 1)
        recs[i, W] = c
        s = "".join("ACGT"[(x >> (2 * (k - 1 - j))) & 3] for j in range(k))
        lines.append(f"{s} {c}\n".encode())
    # de-duplicate keys that collided after the mask, as a counter's output would be
    _, first = np.unique(recs[:, :W], axis=0, return_index=True)
    recs = recs[np.sort(first)]
    lines = [lines[i] for i in np.sort(first)]
    rng.shuffle(recs)
    want = b"".join(sorted(lines))
    if len(recs):
        assert _text_numpy(recs, k, W).tobytes() == want
    d = sorted_text_digest(recs, k)
    assert d["sorted_sha256"] == hashlib.sha256(want).hexdigest()
    assert d["lines"] == len(lines)
    assert d["count_sum"] == sum(int(l.split()[1]) for l in lines)


def test_fixture_cases_match_bench_presets():
    """Every full-size fixture is a bench workload (bench.fixture_case finds it)."""
    doc = _fixture()
    for name, c in doc["cases"].items():
        config, share = SHARES.get(name, (name, 0))
        bench, args = _bench_args(config, share)
        if share:
            inp = doc["inputs"][c["input"]]
            fx = bench.fixture_case(args, share, inp["first"], inp["count"])
        else:
            fx = bench.fixture_case(args)
        assert fx is not None and fx["name"] == name, name
        assert fx["sorted_sha256"] == c["sorted_sha256"]
        # the whole strong jobs are found at every world size (bench.py's N > 1 parity)
        assert bool(c.get("whole_job")) == (name in ("C4", "C5")), name


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("config", ["C2", "C3", "C2S"])
def test_bench_job_equals_reference_output(config):
    import torch
    import kaarme_amd as ka
    from kaarme_amd.digest import sorted_text_digest
    doc = _fixture()
    if config not in doc["cases"]:
        pytest.skip(f"no {config} fixture")
    bench, args = _bench_args(config)
    env = {"torch": torch, "ka": ka, "lib": ka.load_library(), "dist": None, "rank": 0, "world": 1, "local": 0}
    torch.cuda.set_device(0)
    job = bench.setup_job(args, env)
    fx = job.fixture
    assert fx is not None and fx["name"] == config
    try:
        img = job.image.cpu().numpy()
        assert hashlib.sha256(memoryview(img)).hexdigest() == fx["input_sha256"], "device image != kc_gen file"
        del img
        # two steps on one context: the first job is a cold context's, the
        # second the one bench.py times (after kc_reset); both must equal the reference
        for step in range(2):
            job.step()
            st = job.counter.finish()
            assert st["windows"] == job.windows_expected
            assert st["chunks"] == len(job.chunks)
            assert st["part_fallbacks"] == 0
            if args.unique:  # the bench path: the counting pass from the kept level-2 partitions
                assert st["reused_passes"] == 1 and st["reuse_level"] == 2, (step, st)
            got = sorted_text_digest(job.counter.dump(), args.k)
            assert got["lines"] == fx["lines"], step
            assert got["count_sum"] == fx["count_sum"], step
            assert got["sorted_sha256"] == fx["sorted_sha256"], step
            if fx["distinct"] is not None and not args.unique:
                assert st["distinct"] == fx["distinct"]
            if fx.get("digest"):  # the order-independent digest of the same output (make_digests.py)
                assert ka.same_digest(job.counter.output_digest(), fx["digest"]), step
    finally:
        job.counter.close()
        del job
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["C4S", "C5S"])
def test_bench_share_equals_reference_output(name):
    """rank 0's share of the strong presets at 8 GPUs (bench.py --config C4|C5
    --share 8: 12.5 M x 150 bp at k = 51; 125 k x 10 kbp at k = 127), its local table sized from the
    distinct estimate, against the reference CLI's output on the same reads (make_fullsize.py)."""
    import torch
    import kaarme_amd as ka
    from kaarme_amd.digest import sorted_text_digest
    doc = _fixture()
    if name not in doc["cases"]:
        pytest.skip(f"no {name} fixture")
    config, share = SHARES[name]
    bench, args = _bench_args(config, share)
    env = {"torch": torch, "ka": ka, "lib": ka.load_library(), "dist": None, "rank": 0, "world": 1, "local": 0}
    torch.cuda.set_device(0)
    job = bench.setup_job(args, env)
    fx = job.fixture
    assert fx is not None and fx["name"] == name
    try:
        img = job.image.cpu().numpy()
        assert hashlib.sha256(memoryview(img)).hexdigest() == fx["input_sha256"], "device image != kc_gen file"
        del img
        job.step()
        st = job.counter.finish()
        assert st["windows"] == job.windows_expected
        assert st["distinct"] == fx["distinct"]
        got = sorted_text_digest(job.counter.dump(), args.k)
        assert (got["lines"], got["count_sum"]) == (fx["lines"], fx["count_sum"])
        assert got["sorted_sha256"] == fx["sorted_sha256"]
        if fx.get("digest"):
            assert ka.same_digest(job.counter.output_digest(), fx["digest"])
    finally:
        job.counter.close()
        del job
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["C4", "C5"])
def test_whole_strong_job_on_one_gpu(name):
    """the whole C4 (100 M x 150 bp, k = 51, -s 2.6e9) and C5 (1 M x 10 kbp,
    k = 127, -s 3.6e9) jobs on one GPU -- bench.py's N = 1 point of the strong-scaling curve, many
    staging batches into one table -- against the whole-job digest of tests/golden/fullsize.json (the
    pinned CPU restatement, partitioned: make_digests.py; no reference run covers these sizes here).
    Two steps on one context, as bench.py times them."""
    import torch
    import kaarme_amd as ka
    doc = _fixture()
    if name not in doc["cases"]:
        pytest.skip(f"no {name} fixture")
    bench, args = _bench_args(name)
    env = {"torch": torch, "ka": ka, "lib": ka.load_library(), "dist": None, "rank": 0, "world": 1, "local": 0}
    torch.cuda.set_device(0)
    job = bench.setup_job(args, env)
    fx = job.fixture
    assert fx is not None and fx["name"] == name and fx.get("whole_job")
    try:
        for step in range(2):
            job.step()
            st = job.counter.finish()
            assert st["windows"] == job.windows_expected == fx["count_sum"]
            assert st["distinct"] == fx["distinct"], step
            assert ka.same_digest(job.counter.output_digest(), fx["digest"]), step
    finally:
        job.counter.close()
        del job
        torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_device_writer_at_full_size(tmp_path):
    """the writer's bytes at full size -- kc_write of the C2 job (86.5 M lines,
    device formatting + pinned copy-out) sorted and hashed against the reference's output digest
    (the records' digest is test_bench_job_equals_reference_output's)."""
    import subprocess
    import torch
    import kaarme_amd as ka
    doc = _fixture()
    bench, args = _bench_args("C2")
    env = {"torch": torch, "ka": ka, "lib": ka.load_library(), "dist": None, "rank": 0, "world": 1, "local": 0}
    torch.cuda.set_device(0)
    job = bench.setup_job(args, env)
    fx = job.fixture
    try:
        job.step()
        job.counter.finish()
        out = tmp_path / "c2.txt"
        job.counter.write(str(out))
        p = subprocess.Popen(["sort", "-S", "12G", "--parallel=16", "-T", str(tmp_path), str(out)],
                             stdout=subprocess.PIPE, env=dict(os.environ, LC_ALL="C"))
        h = hashlib.sha256()
        lines = 0
        for b in iter(lambda: p.stdout.read(1 << 24), b""):
            h.update(b)
            lines += b.count(b"\n")
        assert p.wait() == 0
        assert lines == fx["lines"] == doc["cases"]["C2"]["lines"]
        assert h.hexdigest() == fx["sorted_sha256"]
    finally:
        job.counter.close()
        del job
        torch.cuda.empty_cache()
