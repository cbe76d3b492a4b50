"""GPU: the sharded counting path (kc_route_device -> exchange -> kc_insert_keys_device).

One GPU, G emulated ranks: each rank is its own engine (own table) and counts its own
slice of the reads; the all-to-all is emulated in-process by slicing the owner groups.
The per-rank outputs must be disjoint and their union must equal the oracle's count of
the whole input (bit-exact sorted output).  The same ranks over RCCL are what bench.py
runs at N > 1; tests/test_sharded.py covers the collective itself over gloo.
"""
import subprocess

import pytest
import torch

from conftest import GEN, oracle_count, sorted_digest_file, sorted_digest_lines
import kaarme_amd as ka
from kaarme_amd.sharded import DeviceEngine

pytestmark = pytest.mark.gpu


def _image(path):
    data = open(path, "rb").read()
    return data, torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()


@pytest.mark.parametrize("k,mode,G,path", [(31, 2, 2, "direct"), (31, 2, 3, "partitioned"),
                                            (21, 0, 4, "partitioned"), (51, 2, 2, "direct"),
                                            (51, 0, 3, "partitioned"), (95, 1, 2, "partitioned")])
def test_emulated_ranks_union(tmp_path, monkeypatch, k, mode, G, path):
    monkeypatch.setenv("KC_INSERT_PATH", path)
    n_reads = 30000
    per = n_reads // G
    images = []
    for r in range(G):
        fa = tmp_path / f"r{r}.fasta"
        cnt = per if r < G - 1 else n_reads - per * (G - 1)
        subprocess.run([GEN, str(fa), str(n_reads), "150", "200000", "--first", str(r * per), "--count", str(cnt)],
                       check=True)
        images.append(_image(str(fa)))
    whole = tmp_path / "all.fasta"
    with open(whole, "wb") as f:
        for data, _ in images:
            f.write(data)
    engines = [DeviceEngine(ka.Config(k=k, mode=mode, table_slots=400000, min_abundance=1,
                                      batch_bytes=max(len(d) for d, _ in images) * 2 + (1 << 20)))
               for _ in range(G)]
    W = engines[0].W
    stream = torch.cuda.current_stream().cuda_stream
    routed = []
    for r, (data, img) in enumerate(images):
        chunks = ka.plan_chunks(data, k, ka.FMT_FASTA, chunk_size=256 * 1024)
        buf, counts = engines[r].route(img.data_ptr(), chunks, ka.FMT_FASTA, G, stream)
        torch.cuda.synchronize()
        assert sum(counts) == engines[r].kc.finish()["windows"]
        keys = buf[: sum(counts) * W].view(-1, W)
        assert int((keys[:, 0] == 0).sum()) == 0, "table key word 0 is never 0"
        routed.append((buf.clone(), counts))
    for d in range(G):  # emulated all-to-all: rank d receives group d of every source, in rank order
        parts = []
        for buf, counts in routed:
            lo = sum(counts[:d]) * W
            parts.append(buf[lo:lo + counts[d] * W])
        recv = torch.cat(parts)
        n = recv.numel() // W
        engines[d].insert(recv, n, stream)
        torch.cuda.synchronize()
        assert engines[d].kc.finish()["inserted"] == n
    shard_lines = [set(e.kc.lines()) for e in engines]
    kmers = [set(l.rsplit(" ", 1)[0] for l in s) for s in shard_lines]
    for a in range(G):
        for b in range(a + 1, G):
            assert not (kmers[a] & kmers[b]), "a k-mer has two owners"
        assert kmers[a], "empty shard"
    union = set().union(*shard_lines)
    out = tmp_path / "oracle.txt"
    oracle_count(str(whole), k, ["-m", str(mode), "-a", "1"], out)
    assert sorted_digest_lines(union) == sorted_digest_file(out)


@pytest.mark.parametrize("path", ["direct", "partitioned"])
def test_insert_rejects_non_table_keys(monkeypatch, path):
    """Word 0 == 0 marks an empty slot and is never a table key: such keys are skipped
    (no hang, no corrupted slot) and kc_finish reports them."""
    monkeypatch.setenv("KC_INSERT_PATH", path)
    e = DeviceEngine(ka.Config(k=51, mode=0, table_slots=100000, min_abundance=1))
    keys = torch.zeros(2 * 5000, dtype=torch.int64, device="cuda")
    keys[::4] = 12345  # every other key (word 0 of even keys) is a valid table key
    e.insert(keys, 5000, torch.cuda.current_stream().cuda_stream)
    with pytest.raises(ka.KcError, match="not table keys"):
        e.kc.finish()


@pytest.mark.parametrize("merge", ["runs", "general", "shuffled", "runs_gaps"])
@pytest.mark.parametrize("path", ["direct", "partitioned"])
@pytest.mark.parametrize("k,mode,G", [(31, 2, 2), (31, 0, 3), (51, 2, 4), (63, 1, 2), (127, 0, 2)])
def test_preaggregated_merge_union(tmp_path, monkeypatch, k, mode, G, path, merge):
    """Pre-aggregated sharding (ShardedCounter's path): each emulated rank counts its own
    reads locally, routes its table as {key, count} records by owner, and every owner adds
    the records it receives; the owners' outputs are disjoint and their union is the
    oracle's count of the whole input (transforms applied to the merged counts).
    merge: runs = the region-sorted groups in one level-3 pass (kc_insert_counts_runs_device),
    general = the partitioned merge insert, shuffled = runs on unsorted groups (the device
    check sends them to the general insert)."""
    monkeypatch.setenv("KC_INSERT_PATH", path)  # local counting and the merge insert
    n_reads = 20000
    per = n_reads // G
    images = []
    for r in range(G):
        fa = tmp_path / f"r{r}.fasta"
        cnt = per if r < G - 1 else n_reads - per * (G - 1)
        # a small genome: every k-mer occurs on several ranks, so the merge adds counts
        subprocess.run([GEN, str(fa), str(n_reads), "150", "20000", "--first", str(r * per), "--count", str(cnt)],
                       check=True)
        images.append(_image(str(fa)))
    whole = tmp_path / "all.fasta"
    with open(whole, "wb") as f:
        for data, _ in images:
            f.write(data)
    engines = [DeviceEngine(ka.Config(k=k, mode=mode, table_slots=400000, min_abundance=1)) for _ in range(G)]
    W = engines[0].W
    stream = torch.cuda.current_stream().cuda_stream
    routed = []
    for r, (data, img) in enumerate(images):
        engines[r].reset()
        engines[r].count(img.data_ptr(), ka.plan_chunks(data, k, ka.FMT_FASTA, chunk_size=128 * 1024), ka.FMT_FASTA,
                         stream)
        recs, counts = engines[r].route_table(G, stream)
        torch.cuda.synchronize()
        assert sum(counts) == engines[r].kc.finish()["distinct"]
        routed.append((recs[: sum(counts) * (W + 1)].clone(), counts))
    for d in range(G):
        parts = []
        for recs, counts in routed:
            lo = sum(counts[:d]) * (W + 1)
            parts.append(recs[lo:lo + counts[d] * (W + 1)])
        if merge == "shuffled":
            parts = [p.view(-1, W + 1)[torch.randperm(p.numel() // (W + 1), device=p.device)].reshape(-1)
                     for p in parts]
        if merge == "runs_gaps":  # empty groups before, between and after the senders' groups
            empty = parts[0][:0]
            parts = [empty] + [x for p in parts for x in (p, empty)]
        recv = torch.cat(parts)
        gc = [p.numel() // (W + 1) for p in parts] if merge != "general" else None
        engines[d].insert_counts(recv, recv.numel() // (W + 1), stream, group_counts=gc)
        torch.cuda.synchronize()
        assert engines[d].owner_table().finish()["inserted"] == int(recv.view(-1, W + 1)[:, W].sum())
    shard_lines = [set(e.owner_table().lines()) for e in engines]
    kmers = [set(l.rsplit(" ", 1)[0] for l in s) for s in shard_lines]
    for a in range(G):
        for b in range(a + 1, G):
            assert not (kmers[a] & kmers[b]), "a k-mer has two owners"
    union = set().union(*shard_lines)
    out = tmp_path / "oracle.txt"
    oracle_count(str(whole), k, ["-m", str(mode), "-a", "1"], out)
    assert sorted_digest_lines(union) == sorted_digest_file(out)


@pytest.mark.parametrize("k,mode,G", [(31, 2, 2), (51, 0, 3)])
def test_two_merges_route_only_new_counts(tmp_path, k, mode, G):
    """A job that merges twice (count, merge, count more, merge): after routing, the local
    table is cleared (kc_clear_table) but keeps its window counters, so the second merge
    routes only what was counted after the first and the owners' union is still exact."""
    n_reads = 12000
    per = n_reads // G
    images = []
    for r in range(G):
        fa = tmp_path / f"r{r}.fasta"
        cnt = per if r < G - 1 else n_reads - per * (G - 1)
        subprocess.run([GEN, str(fa), str(n_reads), "150", "20000", "--first", str(r * per), "--count", str(cnt)],
                       check=True)
        images.append(_image(str(fa)))
    whole = tmp_path / "all.fasta"
    with open(whole, "wb") as f:
        for data, _ in images:
            f.write(data)
    engines = [DeviceEngine(ka.Config(k=k, mode=mode, table_slots=400000, min_abundance=1)) for _ in range(G)]
    W = engines[0].W
    stream = torch.cuda.current_stream().cuda_stream
    plans = [ka.plan_chunks(data, k, ka.FMT_FASTA, chunk_size=64 * 1024) for data, _ in images]
    per_windows = [len(data.split(b"\n")) // 2 * (150 - k + 1) for data, _ in images]
    for e in engines:
        e.reset()
    for phase in range(2):
        routed = []
        for r, (data, img) in enumerate(images):
            ch = plans[r]
            half = ch[: len(ch) // 2] if phase == 0 else ch[len(ch) // 2:]
            engines[r].count(img.data_ptr(), half, ka.FMT_FASTA, stream)
            recs, counts = engines[r].route_table(G, stream)
            engines[r].clear_local()
            torch.cuda.synchronize()
            routed.append((recs[: sum(counts) * (W + 1)].clone(), counts))
        for d in range(G):
            recv = torch.cat([recs[sum(c[:d]) * (W + 1):(sum(c[:d]) + c[d]) * (W + 1)] for recs, c in routed])
            engines[d].insert_counts(recv, recv.numel() // (W + 1), stream)
            torch.cuda.synchronize()
    for r in range(G):  # the cleared local tables kept their window counters
        assert engines[r].kc.finish()["windows"] == per_windows[r]
    union = set().union(*[set(e.owner_table().lines()) for e in engines])
    out = tmp_path / "oracle.txt"
    oracle_count(str(whole), k, ["-m", str(mode), "-a", "1"], out)
    assert sorted_digest_lines(union) == sorted_digest_file(out)
