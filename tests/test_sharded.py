"""Multi-rank sharding on CPU: world_size 2 over gloo.

The pre-aggregated exchange of kaarme_amd.sharded (local counts -> owner-grouped
{key, count} records -> one all-to-all of counts and one of records -> merge at the
owner) runs unchanged; the HIP engine is replaced by a NumPy engine that tokenizes
PLAIN lines, canonicalises, splits keys into W words and owns keys by a hash of the key.
The union of the owner tables must equal a single-process count and the owners must be
disjoint.  The sharded Bloom filter (ShardedCounter.bloom_finalize: all-to-all of filter
slices, merge, all-gather) runs over gloo with a NumPy double Bloom filter of the blocked
layout: every k-mer with count >= 2 must get its exact count, and a count-1 k-mer may pass
the gate only as a true singleton.
"""
import collections
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "canonical-k-mer-hash-table_amd"))

from kaarme_amd import Config  # noqa: E402
from kaarme_amd.sharded import ShardedCounter, exchange  # noqa: E402

COMP = str.maketrans("ACGT", "TGCA")
CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def canonical_windows(seq, k):
    """Canonical k-mers of every all-ACGT window (kmer_factory.cpp semantics)."""
    out = []
    run = 0
    for i, ch in enumerate(seq):
        run = run + 1 if ch in CODE else 0
        if run >= k:
            w = seq[i - k + 1:i + 1]
            rc = w.translate(COMP)[::-1]
            out.append(min(w, rc))
    return out


def to_words(kmer, W):
    v = 0
    for ch in kmer:
        v = (v << 2) | CODE[ch]
    return [(v >> (64 * (W - 1 - j))) & ((1 << 64) - 1) for j in range(W)]


def from_words(words, k):
    v = 0
    for w in words:
        v = (v << 64) | (int(w) & ((1 << 64) - 1))
    return "".join("ACGT"[(v >> (2 * (k - 1 - i))) & 3] for i in range(k))


def owner(words, parts):
    h = 0
    for w in words:
        h = (h * 0x9E3779B97F4A7C15 + w + 1) & ((1 << 64) - 1)
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & ((1 << 64) - 1)
    h ^= h >> 33
    return ((h & 0xFFFFFFFF) * parts) >> 32


class _Table:
    def __init__(self):
        self.table = collections.Counter()

    def sync(self):
        pass

    def finish(self):
        return {"windows": sum(self.table.values()), "distinct": len(self.table)}

    def output_digest(self):
        """kc_output_digest of this table's lines (T(c) = c mod 65536, -m 0; a = 1)."""
        from conftest import lines_digest
        return lines_digest(f"{km} {c & 0xFFFF}" for km, c in self.table.items())


def bloom_positions(words, nblocks, nh):
    """Blocked-layout model: one 16-word block per k-mer, position j = a 5-bit field of
    its hash in word j mod 8 of each filter half (kc_common.h block_insert's shape)."""
    h = 0
    for w in words:
        h = (h * 0xC2B2AE3D27D4EB4F + w + 7) & ((1 << 64) - 1)
    h ^= h >> 29
    h = (h * 0x9E3779B97F4A7C15) & ((1 << 64) - 1)
    blk = (h >> 40) % nblocks
    return [(blk * 16 + (j & 7), (h >> (5 * j)) & 31) for j in range(nh)]


class NumpyEngine:
    """Stand-in for sharded.DeviceEngine: same count / route_table / insert_counts contract
    on CPU tensors (records: W key words + 1 count word), and the owner-sharded Bloom contract
    (bloom = the ungated local count / bloom_records / owner_bloom_finalize / count_records)."""

    NBLOCKS, NH, NH_GATE = 40, 7, 6

    def __init__(self, k, lines, bf=False):
        self.k = k
        self.W = 2 * k // 64 + 1
        self.lines = lines
        self.kc = _Table()      # local
        self.owner = _Table()
        self.bf = bf
        self.filter = np.zeros(16 * self.NBLOCKS, dtype=np.uint32)  # the owner's filter
        self.new_in_second = 0

    def _has(self, pos, half):
        return all((int(self.filter[w + half]) >> b) & 1 for w, b in pos)

    def _insert(self, words):
        """insertion_process (double_bloomfilter.hpp:371-413) on the blocked-layout model."""
        pos = bloom_positions(words, self.NBLOCKS, self.NH)
        if self._has(pos, 8):
            return
        second = self._has(pos, 0)  # filter 1 complete: the second sighting goes to filter 2
        for w, b in pos:
            self.filter[w + (8 if second else 0)] |= np.uint32(1 << b)
        self.new_in_second += second

    def _rows(self, recs, n):
        return recs[: n * (self.W + 1)].numpy().view(np.uint64).reshape(n, self.W + 1)

    def bloom(self, dev_ptr, chunks, fmt, stream=0):  # the rank's ungated local count
        for off, ln, _ in chunks:
            for line in self.lines[off:off + ln]:
                self.kc.table.update(canonical_windows(line, self.k))

    def bloom_records(self, recs, n, stream=0):
        # the senders' records of one k-mer summed (DeviceEngine._distinct_records), then the
        # k-mers seen at least twice (inserted twice) before the singletons (once)
        agg = collections.Counter()
        for row in self._rows(recs, n):
            agg[tuple(int(x) for x in row[:self.W])] += int(row[self.W])
        self._uniq = agg
        for ws, c in agg.items():
            if c >= 2:
                self._insert(list(ws))
                self._insert(list(ws))
        for ws, c in agg.items():
            if c == 1:
                self._insert(list(ws))

    def owner_bloom_finalize(self):
        return self.new_in_second

    def count_records(self, recs, n, stream=0):
        for ws, c in self._uniq.items():
            if self._has(bloom_positions(list(ws), self.NBLOCKS, self.NH)[: self.NH_GATE], 8):
                self.owner.table[from_words(np.array(ws, dtype=np.uint64), self.k)] += c

    def count(self, dev_ptr, chunks, fmt, stream=0):
        for off, ln, _ in chunks:
            for line in self.lines[off:off + ln]:
                self.kc.table.update(canonical_windows(line, self.k))

    def route_table(self, parts, stream=0):
        groups = [[] for _ in range(parts)]
        for km, c in self.kc.table.items():
            ws = to_words(km, self.W)
            groups[owner(ws, parts)].extend(ws + [c])
        flat = [w for g in groups for w in g]
        arr = np.array(flat, dtype=np.uint64).view(np.int64)
        return torch.from_numpy(arr.copy()), [len(g) // (self.W + 1) for g in groups]

    def insert_counts(self, recs, n, stream=0, group_counts=None):
        rows = recs[: n * (self.W + 1)].numpy().view(np.uint64).reshape(n, self.W + 1)
        for row in rows:
            self.owner.table[from_words(row[:self.W], self.k)] += int(row[self.W])

    def clear_local(self):
        self.kc.table.clear()

    def owner_table(self):
        return self.owner

    # -- super-k-mer exchange (DeviceEngine.skm_route / count_packed / bloom_packed): the host
    # router of tests/skm_model.py, the device stream format both ways
    def skm_route(self, dev_ptr, chunks, fmt, parts, stream=0):
        import skm_model as sm
        seqs = [line for off, ln, _ in chunks for line in self.lines[off:off + ln]]
        routed = sm.route(seqs, self.k, parts)
        pks, bks, words, wins = [], [], [], []
        for o in range(parts):
            pk, bk = sm.pack(routed[o]) if routed[o] else (np.zeros(0, np.uint64), np.zeros(0, np.uint32))
            if len(pk) % 2:
                pk = np.concatenate([pk, np.zeros(1, np.uint64)])
                bk = np.concatenate([bk, np.full(1, 0xFFFFFFFF, np.uint32)])
            pks.append(pk)
            bks.append(bk)
            words.append(len(pk))
            wins.append(sum(len(x) - self.k + 1 for x in routed[o]))
        pk = np.concatenate(pks) if pks else np.zeros(0, np.uint64)
        bk = np.concatenate(bks) if bks else np.zeros(0, np.uint32)
        return (torch.from_numpy(pk.view(np.int64).copy()), torch.from_numpy(bk.view(np.int64).copy()), words, wins)

    def _packed_kmers(self, pk, bk, n):
        import skm_model as sm
        seqs = sm.unpack(pk[:n].numpy().view(np.uint64), bk[:n].numpy().view(np.uint32))
        return [km for x in seqs for km in canonical_windows(x, self.k)]

    def count_packed(self, pk, bk, n, windows, stream=0):
        kms = self._packed_kmers(pk, bk, n)
        assert len(kms) == windows
        if self.bf:  # behind the owner's gate
            kms = [km for km in kms
                   if self._has(bloom_positions(to_words(km, self.W), self.NBLOCKS, self.NH)[: self.NH_GATE], 8)]
        self.owner.table.update(kms)

    def bloom_packed(self, pk, bk, n, windows, stream=0):
        for km in self._packed_kmers(pk, bk, n):
            self._insert(to_words(km, self.W))

    def reset(self):
        self.kc.table.clear()
        self.owner.table.clear()
        self.filter[:] = 0
        self.new_in_second = 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_reads(n, L, seed):
    rng = np.random.default_rng(seed)
    genome = "".join(rng.choice(list("ACGT"), 400))
    reads = []
    for i in range(n):
        p = int(rng.integers(0, len(genome) - L))
        r = genome[p:p + L]
        if rng.random() < 0.5:
            r = r.translate(COMP)[::-1]
        if i % 7 == 0:
            q = int(rng.integers(0, L))
            r = r[:q] + "N" + r[q + 1:]
        reads.append(r)
    return reads


def _worker(rank, world, port, k, reads, outdir, rounds):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = NumpyEngine(k, reads)
        sc = ShardedCounter(Config(k=k, mode=0), dist, engine=eng)
        sc.reset()
        # rank r counts a contiguous slice of the reads, in several batches
        per = (len(reads) + world - 1) // world
        lo, hi = rank * per, min(len(reads), (rank + 1) * per)
        step = max(1, (hi - lo + rounds - 1) // rounds)
        batches = list(range(lo, hi, step))
        half = len(batches) // 2
        for b in batches[:half]:
            sc.count_device(0, [(b, min(step, hi - b), 0)], 2)
        sc.sync()                  # a first merge mid-job (every rank calls it)
        for b in batches[half:]:
            sc.count_device(0, [(b, min(step, hi - b), 0)], 2)
        sc.count_device(0, [], 2)  # an empty batch changes nothing
        sc.sync()                  # the second merge routes only what came after the first
        sc.sync()                  # nothing pending: no third exchange
        with open(os.path.join(outdir, f"shard{rank}.json"), "w") as f:
            json.dump(dict(eng.owner.table), f)
        # the whole job's output digest: the owners' digests gathered and combined (bench.py's N > 1
        # parity record)
        with open(os.path.join(outdir, f"digest{rank}.json"), "w") as f:
            json.dump(sc.output_digest(), f)
    finally:
        dist.destroy_process_group()


def _skm_worker(rank, world, port, k, reads, outdir, bf):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = NumpyEngine(k, reads, bf=bf)
        cfg = Config(k=k, mode=2, bf_enable=bf, est_unique=1000) if bf else Config(k=k, mode=0)
        sc = ShardedCounter(cfg, dist, engine=eng, exchange="superkmers")
        per = (len(reads) + world - 1) // world
        lo, hi = rank * per, min(len(reads), (rank + 1) * per)
        out = {}
        for job in range(2):  # two jobs on one counter, as bench.py's steps
            sc.reset()
            if bf:
                sc.bloom_device(0, [(lo, hi - lo, 0)], 2)
                out["nis"] = sc.bloom_finalize()
            sc.count_device(0, [(lo, hi - lo, 0)], 2)
            sc.sync()
            st = sc.finish()
            out["windows"] = st["windows"]
            out["owner"] = dict(eng.owner.table)
            if not bf:
                out["digest"] = sc.output_digest()
        out["sent"] = sc.xstats["bytes_sent"]
        with open(os.path.join(outdir, f"shard{rank}.json"), "w") as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,world,bf", [(21, 2, False), (33, 3, False), (51, 2, True)])
def test_sharded_superkmers(tmp_path, k, world, bf):
    """The super-k-mer exchange: every rank routes its reads' super-k-mers to
    their canonical-minimizer owners (two all-to-alls of packed words) and each owner counts what it
    receives -- no local table.  The owners are disjoint, their union is the single-process count
    (and, with the Bloom filter, exact for every k-mer seen twice, count-1 only for true singletons),
    each rank reports its own input's windows, and the combined digest is the whole job's."""
    reads = make_reads(60, 90, seed=k + world)
    mp.spawn(_skm_worker, args=(world, _free_port(), k, reads, str(tmp_path), bf), nprocs=world, join=True)
    shards = [json.load(open(tmp_path / f"shard{r}.json")) for r in range(world)]
    truth = collections.Counter(km for r in reads for km in canonical_windows(r, k))
    union = collections.Counter()
    for a in range(world):
        for b in range(a + 1, world):
            assert not (set(shards[a]["owner"]) & set(shards[b]["owner"]))
        union.update(shards[a]["owner"])
    per = (len(reads) + world - 1) // world
    for r in range(world):
        assert shards[r]["windows"] == sum(len(canonical_windows(x, k)) for x in reads[r * per:(r + 1) * per])
    assert any(s["sent"] > 0 for s in shards)
    if bf:
        assert {km: c for km, c in union.items() if truth[km] >= 2} == {km: c for km, c in truth.items() if c >= 2}
        assert all(truth[km] == 1 == c for km, c in union.items() if truth[km] < 2)
        assert all(s["nis"] == shards[0]["nis"] for s in shards)
    else:
        assert union == truth
        from conftest import lines_digest
        want = lines_digest(f"{km} {c & 0xFFFF}" for km, c in truth.items())
        assert all(s["digest"] == want for s in shards)


@pytest.mark.parametrize("k", [5, 21, 33, 51])
def test_sharded_union_equals_single(tmp_path, k):
    reads = make_reads(60, 90, seed=k)
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), k, reads, str(tmp_path), 3), nprocs=world, join=True)
    shards = [json.load(open(tmp_path / f"shard{r}.json")) for r in range(world)]
    assert not (set(shards[0]) & set(shards[1])), "a k-mer was counted by two owners"
    union = collections.Counter()
    for s in shards:
        union.update(s)
    truth = collections.Counter(km for r in reads for km in canonical_windows(r, k))
    assert union == truth
    assert all(len(s) > 0 for s in shards)
    from conftest import lines_digest
    want = lines_digest(f"{km} {c & 0xFFFF}" for km, c in truth.items())
    for r in range(world):
        assert json.load(open(tmp_path / f"digest{r}.json")) == want


def _bloom_worker(rank, world, port, k, reads, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = NumpyEngine(k, reads, bf=True)
        sc = ShardedCounter(Config(k=k, mode=2, bf_enable=True, est_unique=1000), dist, engine=eng)
        per = (len(reads) + world - 1) // world
        lo, hi = rank * per, min(len(reads), (rank + 1) * per)
        sc.bloom_device(0, [(lo, hi - lo, 0)], 2)
        nis = sc.bloom_finalize()
        sc.count_device(0, [(lo, hi - lo, 0)], 2)
        sc.sync()
        with open(os.path.join(outdir, f"shard{rank}.json"), "w") as f:
            json.dump({"owner": dict(eng.owner.table), "nis": nis, "own_nis": eng.new_in_second}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,world", [(21, 2), (33, 3)])
def test_sharded_bloom(tmp_path, k, world):
    """Owner-sharded Bloom filter: every rank counts its reads ungated, the records
    go to their owners, each owner runs the Bloom pass over its records (twice for a count >= 2)
    and counts them behind its own filter: each k-mer seen twice anywhere (also once on each of
    two ranks) keeps its exact count, the owners are disjoint, and every rank returns the same
    new_in_second, the sum of the owners' counters."""
    reads = make_reads(40, 70, seed=k)
    mp.spawn(_bloom_worker, args=(world, _free_port(), k, reads, str(tmp_path)), nprocs=world, join=True)
    shards = [json.load(open(tmp_path / f"shard{r}.json")) for r in range(world)]
    assert all(s["nis"] == shards[0]["nis"] > 0 for s in shards)
    assert shards[0]["nis"] == sum(s["own_nis"] for s in shards)
    union = collections.Counter()
    for a in range(world):
        for b in range(a + 1, world):
            assert not (set(shards[a]["owner"]) & set(shards[b]["owner"]))
        union.update(shards[a]["owner"])
    truth = collections.Counter(km for r in reads for km in canonical_windows(r, k))
    per = (len(reads) + world - 1) // world
    ranks_of = collections.defaultdict(set)
    for i, r in enumerate(reads):
        for km in canonical_windows(r, k):
            ranks_of[km].add(i // per)
    assert any(truth[km] == 2 and len(ranks_of[km]) == 2 for km in truth), "no k-mer split over two ranks"
    assert {km: c for km, c in union.items() if truth[km] >= 2} == {km: c for km, c in truth.items() if c >= 2}
    assert all(truth[km] == 1 == c for km, c in union.items() if truth[km] < 2)


class _ShortDelivery:
    """torch.distributed proxy whose item all-to-alls lose the last received word."""

    def __getattr__(self, name):
        return getattr(dist, name)

    @staticmethod
    def all_to_all_single(out, inp, output_split_sizes=None, input_split_sizes=None, group=None):
        dist.all_to_all_single(out, inp, output_split_sizes=output_split_sizes, input_split_sizes=input_split_sizes,
                               group=group)
        if output_split_sizes is not None and out.numel():
            out[-1] = 0


def _corrupt_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = torch.arange(1, 1 + 2 * 6, dtype=torch.int64)
        try:
            exchange(_ShortDelivery(), keys, [3, 3], 2)
            msg = "no error"
        except RuntimeError as e:
            msg = str(e)
        with open(os.path.join(outdir, f"c{rank}.txt"), "w") as f:
            f.write(msg)
    finally:
        dist.destroy_process_group()


def test_exchange_detects_short_delivery(tmp_path):
    """A collective that delivers less than was sent raises on the receiving rank."""
    mp.spawn(_corrupt_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert "corrupt data from rank 1" in open(tmp_path / f"c{r}.txt").read()


def _exchange_worker(rank, world, port, outdir, chunk):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = 3
        # rank r sends (r+1)*(d+1) keys to rank d; key words encode (src, dst, i, j)
        counts = [(rank + 1) * (d + 1) for d in range(world)]
        rows = [[rank * 1000000 + d * 10000 + i * 10 + j for j in range(W)] for d in range(world)
                for i in range(counts[d])]
        keys = torch.tensor(sum(rows, []) + [-1] * 7, dtype=torch.int64)  # slack past the groups
        out, n = exchange(dist, keys, counts, W, chunk_words=chunk)
        got = out[: n * W].view(n, W).tolist()
        with open(os.path.join(outdir, f"x{rank}.json"), "w") as f:
            json.dump({"n": n, "rows": got}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chunk", [1 << 24, 5, 3])
def test_exchange_splits(tmp_path, chunk):
    """One all-to-all, or rounds of at most `chunk` words per peer: same result."""
    world = 3
    mp.spawn(_exchange_worker, args=(world, _free_port(), str(tmp_path), chunk), nprocs=world, join=True)
    for d in range(world):
        r = json.load(open(tmp_path / f"x{d}.json"))
        want = [[s * 1000000 + d * 10000 + i * 10 + j for j in range(3)] for s in range(world)
                for i in range((s + 1) * (d + 1))]
        assert r["n"] == len(want)
        assert r["rows"] == want


def test_batch_groups():
    from kaarme_amd.sharded import batch_groups
    chunks = [(0, 4096, 0), (4096, 1, 0), (5000, 0, 0), (6000, 8192, 0), (20000, 100, 1)]
    assert batch_groups(chunks, 3 * 4096) == [[(0, 4096, 0), (4096, 1, 0)], [(6000, 8192, 0), (20000, 100, 1)]]
    g = batch_groups(chunks, 3 * 4096)
    assert [c for grp in g for c in grp] == [c for c in chunks if c[1]]
    for grp in g:
        assert sum((c[1] + 4095) // 4096 * 4096 for c in grp) <= 3 * 4096
    with pytest.raises(ValueError):
        batch_groups([(0, 5 * 4096, 0)], 4 * 4096)
