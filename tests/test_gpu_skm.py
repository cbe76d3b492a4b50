"""Super-k-mer routing (kc_route_superkmers_device, kc_skm.hip) and counting of packed streams
(kc_count_packed_device / kc_bloom_packed_device): the multi-GPU exchange's device half, checked
on one GPU against the NumPy model (tests/skm_model.py) and the oracle.

For every owner o the device's stream must hold exactly the windows the model assigns to o (the
oracle's counts over the device's super-k-mers = its counts over the model's), every window of the
input exactly once over all owners, and counting the owners' streams on the device must give the
oracle's counts of the whole input (combined output digests)."""
import os

import numpy as np
import pytest

from conftest import GEN, oracle_count, text_digest
import kaarme_amd as ka
import skm_model as sm

pytestmark = pytest.mark.gpu


def _input(tmp_path, n=6000, L=150, G=300_000, seed=9, err=0.002):
    import subprocess
    p = tmp_path / "reads.fasta"
    subprocess.run([GEN, str(p), str(n), str(L), str(G), "-s", str(seed), "-e", str(err)], check=True)
    host = open(p, "rb").read()
    seqs = [l for l in host.decode().splitlines() if l and not l.startswith(">")]
    return p, host, seqs


def _route(host, k, G, cap_scale=1.3, batch=None):
    import torch
    img = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 200_000)
    cfg = ka.Config(k=k, mode=2, min_abundance=1, table_slots=1 << 20, batch_bytes=batch or 0)
    with ka.KmerCounter(cfg) as kc:
        need, wins = kc.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, G)
        cap = int(max(need) * cap_scale) + 2
        pk = torch.zeros(G * cap + 2, dtype=torch.int64, device="cuda")
        bk = torch.zeros(G * cap + 2, dtype=torch.int32, device="cuda")
        words, wins2 = kc.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, G, pk.data_ptr(),
                                                  bk.data_ptr(), cap)
        torch.cuda.synchronize()
    assert words == need and wins2 == wins
    pkh = pk.cpu().numpy().view(np.uint64)
    bkh = bk.cpu().numpy().view(np.uint32)
    return [(pkh[o * cap:o * cap + words[o]], bkh[o * cap:o * cap + words[o]]) for o in range(G)], wins, (pk, bk, cap,
                                                                                                           words)


@pytest.mark.parametrize("k,G", [(31, 1), (31, 3), (51, 8), (127, 5), (21, 3), (15, 4), (9, 2)])
def test_superkmers_match_the_model(k, G, tmp_path):
    path, host, seqs = _input(tmp_path)
    streams, wins, _ = _route(host, k, G, batch=256 << 10)  # (several staging batches)
    model = sm.route(seqs, k, G)
    total = 0
    for o in range(G):
        got = sm.unpack(*streams[o])
        assert all(len(s) >= k for s in got)
        w = sum(len(s) - k + 1 for s in got)
        assert w == wins[o] == sum(len(s) - k + 1 for s in model[o]), o
        total += w
        if not got:
            continue
        # the same windows: the oracle's counts over the device's and the model's super-k-mers
        a, b = tmp_path / f"dev{o}.txt", tmp_path / f"mod{o}.txt"
        a.write_text("".join(s + "\n" for s in got))
        b.write_text("".join(s + "\n" for s in model[o]))
        oa, ob = tmp_path / f"dev{o}.out", tmp_path / f"mod{o}.out"
        oracle_count(str(a), k, ["-a", "1"], oa)
        oracle_count(str(b), k, ["-a", "1"], ob)
        assert text_digest(str(oa)) == text_digest(str(ob)), o
    assert total == sum(max(0, len(s) - k + 1) for s in seqs)


@pytest.mark.parametrize("k,G", [(31, 4), (51, 3), (127, 2)])
def test_owners_count_the_whole_job(k, G, tmp_path):
    """Each owner counts its stream (kc_count_packed_device, in several batches with the deferred
    level 3); the owners' digests combined equal the oracle's digest of the whole input."""
    path, host, seqs = _input(tmp_path, n=8000)
    _, wins, (pk, bk, cap, words) = _route(host, k, G)
    exp = tmp_path / "exp.txt"
    oracle_count(str(path), k, ["-a", "1"], exp)
    parts = []
    for o in range(G):
        cfg = ka.Config(k=k, mode=2, min_abundance=1, table_slots=2_000_000, batch_bytes=64 << 10)
        with ka.KmerCounter(cfg) as kc:
            kc.count_packed_device(pk.data_ptr() + o * cap * 8, bk.data_ptr() + o * cap * 4, words[o], wins[o])
            st = kc.finish()
            assert st["windows"] == wins[o]
            parts.append(kc.output_digest())
    assert ka.same_digest(ka.combine_digests(parts), text_digest(str(exp)))


def test_packed_bloom_job_on_one_owner(tmp_path):
    """An owner's Bloom job over its received stream (kc_bloom_packed_device, kc_bloom_finalize,
    kc_count_packed_device): k-mers seen twice or more are the oracle's exactly and a count-1 line
    is a true singleton."""
    path, host, seqs = _input(tmp_path, n=8000)
    k = 51
    _, wins, (pk, bk, cap, words) = _route(host, k, 1)
    cfg = ka.Config(k=k, mode=2, min_abundance=1, bf_enable=True, est_unique=1_000_000, batch_bytes=64 << 10)
    with ka.KmerCounter(cfg) as kc:
        kc.bloom_packed_device(pk.data_ptr(), bk.data_ptr(), words[0], wins[0])
        kc.bloom_finalize()
        kc.count_packed_device(pk.data_ptr(), bk.data_ptr(), words[0], wins[0])
        lines = kc.lines()
    out = tmp_path / "oracle.txt"
    oracle_count(str(path), k, ["-a", "1"], out)
    exact = dict(l.split() for l in open(out).read().splitlines())
    assert sorted(l for l in lines if int(l.split()[1]) >= 2) == sorted(f"{a} {c}" for a, c in exact.items()
                                                                        if int(c) >= 2)
    assert all(exact.get(l.split()[0]) == "1" for l in lines if l.endswith(" 1"))


def test_route_overflow_reports_the_sizes(tmp_path):
    import torch
    path, host, seqs = _input(tmp_path, n=2000)
    img = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    chunks = ka.plan_chunks(host, 31, ka.FMT_FASTA)
    with ka.KmerCounter(ka.Config(k=31, mode=2, table_slots=1 << 20)) as kc:
        need, _ = kc.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, 2)
        pk = torch.zeros(2 * 64 + 2, dtype=torch.int64, device="cuda")
        bk = torch.zeros(2 * 64 + 2, dtype=torch.int32, device="cuda")
        with pytest.raises(ka.KcError, match="too small") as ei:
            kc.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, 2, pk.data_ptr(), bk.data_ptr(), 64)
        assert ei.value.words == need

