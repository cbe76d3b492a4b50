"""Hash-prefix owner sharding of the counting table across GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, over xGMI).

Pre-aggregated exchange (`ShardedCounter`):
  1. every rank counts its own input into a private *local* table with the full
     single-GPU pipeline (kc_count_device);
  2. at the end of the job (`sync`/`merge`), `kc_route_table_device` writes the local
     table's occupied slots as records {table key, raw count}, grouped by owner shard
     (owner = a bit field of the table key, independent of the table's region/bucket
     bits), and ONE all-to-all exchanges them (counts first, then the records);
  3. every rank adds what it received into its *owner* table (kc_insert_counts_device).
Every canonical k-mer has exactly one owner, so the union of the owner tables is the
exact global count, and the output is the concatenation of the per-rank outputs.  The
exchange moves one record per distinct k-mer of each rank instead of one key per window
(86 M records instead of 1.2 G keys for C2), which keeps xGMI off the critical path.
The count transforms (mod 65536 / min(c, 16383)) apply to the merged counts.

The per-window alternative (kc_route_device + kc_insert_keys_device: route every
window's key to its owner, no local table) stays in the C ABI and is exercised by
tests/test_gpu_sharded.py.

Bloom prefilter (-b, main.cpp:395-461 / parallel_parser.hpp:2680-2974), sharded by the same
owner as the table: each rank holds the filter of the k-mers it owns, sized for
its 1/world share of -u, so one filter's worth of bits is spread over the ranks.
  1. `bloom_device`: every rank counts its own input, ungated, into its local table;
  2. `bloom_finalize` (collective): the local tables' {key, count} records go to their owners
     in one all-to-all; each owner runs Bloom pass 1 over what it received
     (kc_bloom_records_device: insertion_process once per record, twice for a record of
     count >= 2), sizes its table from its new_in_second (2 x, main.cpp:454), and counts the
     same records behind its gate (kc_count_records_device).  A k-mer seen twice in the whole
     input -- twice on one rank, or once on each of two -- sets its filter-2 bits at its owner,
     and a k-mer seen once meets one filter holding exactly the insertions one GPU's filter
     would hold for it, so the owners gate as the reference's single filter does;
  3. `count_device` over the same input then only confirms it (the owners counted it).
new_in_second is the sum of the owners' counters (all-reduce).

The exchange logic (:func:`exchange`) is backend-agnostic torch code: the CPU tests run
it over ``gloo`` with a NumPy engine, the GPU path over RCCL with the HIP engine.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

from . import Config, KmerCounter, words_for_k


# Largest message per (peer, all-to-all) in int64 words (KC_EXCHANGE_CHUNK_MB overrides it;
# 0 = one all-to-all).  An early multi-GPU run saw RCCL (the ROCm torch wheel's) return only
# part of a 1.4 GB single-peer all_to_all_single.  No cause was found in the code: split sizes
# are int64 in Python and size_t from c10d's computeLengthsAndOffsets through
# all2all_single_unequal_split to ncclAllToAllv / ncclSend / ncclRecv (torch/csrc/cuda/nccl.h,
# rccl.h), and 1.4 GB is below every 32-bit byte count; the run's record was not kept and one
# GPU cannot host two RCCL ranks, so the observation is unconfirmed.  Big exchanges therefore
# go in rounds of at most this many words per peer, and every exchange checks per-peer sums of
# what arrived (`verify`) so that a short or corrupt delivery raises instead of miscounting.
EXCHANGE_CHUNK_WORDS = 1 << 25  # 256 MB: a C2 rank's records to each of 8 peers (~173 MB) in one round


def chunk_words_default() -> int:
    import os

    mb = os.environ.get("KC_EXCHANGE_CHUNK_MB")
    if mb is None:
        return EXCHANGE_CHUNK_WORDS
    return (int(mb) << 20) // 8 or (1 << 62)


def exchange(dist, keys, counts: Sequence[int], W: int, group=None, chunk_words: int = 0,
             with_counts: bool = False, verify: bool = True, extra: int = 0):
    """All-to-all of owner-grouped items of W int64 words each.  keys: int64 tensor
    holding sum(counts)*W words (group d = the items for rank d, in rank order).
    Returns (received items, n received[, items received from each rank]); the items
    from rank s follow those of s-1.  verify: the senders' per-group word sums travel
    beside the items and must equal the sums of the groups received (else RuntimeError).
    extra: words of slack after the received items (readable, unspecified)."""
    import torch

    chunk_words = chunk_words or chunk_words_default()
    dev = keys.device
    world = len(counts)
    if world == 1:  # nothing leaves the rank
        if extra and keys.numel() < int(counts[0]) * W + extra:
            keys = torch.cat([keys[: int(counts[0]) * W], keys.new_zeros(extra)])
        return (keys, int(counts[0]), [int(counts[0])]) if with_counts else (keys, int(counts[0]))
    if _host_staged(dist, group, keys):
        # gloo moves host tensors only: the items cross through host memory (tests with several
        # ranks on one GPU; RCCL moves device memory directly)
        res = exchange(dist, keys.cpu(), counts, W, group, chunk_words, True, verify, extra)
        out = res[0].to(dev)
        return (out, res[1], res[2]) if with_counts else (out, res[1])
    sw = [int(c) * W for c in counts]
    so = [sum(sw[:d]) for d in range(world)]

    def group_sums(t, offs, lens):  # wrapping int64 sums: equal on both sides for equal words
        return torch.stack([t[o: o + n].sum() if n else t.new_zeros(()) for o, n in zip(offs, lens)])

    # the header per destination d: [count_d] or [count_d, sum of group d]
    send_head = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev).view(world, 1)
    if verify:
        send_head = torch.cat([send_head, group_sums(keys, so, sw).view(world, 1)], dim=1)
    send_head = send_head.contiguous().view(-1)
    recv_head = torch.empty_like(send_head)
    dist.all_to_all_single(recv_head, send_head, group=group)
    rh = recv_head.view(world, -1).cpu().tolist()
    recv = [int(r[0]) for r in rh]
    total = sum(recv)
    out = torch.empty(max(1, total * W + extra), dtype=torch.int64, device=dev)
    rw = [r * W for r in recv]
    ro = [sum(rw[:d]) for d in range(world)]
    big = torch.tensor([max(sw + rw + [0])], dtype=torch.int64, device=dev)
    dist.all_reduce(big, op=dist.ReduceOp.MAX, group=group)
    rounds = max(1, -(-int(big.item()) // chunk_words))
    if rounds == 1:
        dist.all_to_all_single(out[: total * W], keys[: sum(sw)], output_split_sizes=rw, input_split_sizes=sw,
                               group=group)
    else:
        for r in range(rounds):
            lo = r * chunk_words
            sin = [min(max(sw[d] - lo, 0), chunk_words) for d in range(world)]
            rin = [min(max(rw[d] - lo, 0), chunk_words) for d in range(world)]
            send = torch.cat([keys[so[d] + lo: so[d] + lo + sin[d]] for d in range(world)])
            got = torch.empty(max(1, sum(rin)), dtype=torch.int64, device=dev)
            dist.all_to_all_single(got[: sum(rin)], send, output_split_sizes=rin, input_split_sizes=sin,
                                   group=group)
            pos = 0
            for d in range(world):
                if rin[d]:
                    out[ro[d] + lo: ro[d] + lo + rin[d]].copy_(got[pos: pos + rin[d]])
                pos += rin[d]
    if verify:
        got = group_sums(out, ro, rw).tolist()
        for s in range(world):
            if got[s] != int(rh[s][1]):
                raise RuntimeError(f"all-to-all delivered corrupt data from rank {s}: {rw[s]} words, "
                                   f"sum {got[s]} != the sender's {int(rh[s][1])} ({rounds} round(s) of "
                                   f"<= {chunk_words} words per peer)")
    return (out, total, recv) if with_counts else (out, total)


def _gather_into_tensor(dist, group) -> bool:
    return hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo"


def _host_staged(dist, group, t) -> bool:
    """Device tensors over gloo (which collects host tensors only) go through host memory."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _on_stream(device: str, stream: int):
    """Context that makes the caller's HIP stream torch's current stream, so the collectives
    (which torch orders after its current stream) follow the kc_* work queued on `stream` and
    the kc_* calls queued after them follow the collectives.  NULL stream / CPU: no-op."""
    import contextlib

    if device != "cuda" or not stream:
        return contextlib.nullcontext()
    import torch

    return torch.cuda.stream(torch.cuda.ExternalStream(stream))


def owner_share(slots: int, world: int) -> int:
    """Slots of one owner's table for a job whose whole table is `slots`: the 1/world share
    plus 8 sigma of the binomial spread of hash-split keys."""
    share = -(-slots // world)
    return share if world == 1 else share + 8 * int(share ** 0.5) + 64


TILE = 4096
DEFAULT_BATCH = 256 << 20  # kc_api.cpp kDefaultBatch


def batch_groups(chunks, batch_bytes: int):
    """Split a chunk table into groups that each fit one staging batch (kc_api.cpp:
    chunks are placed at 4 KiB-aligned offsets of a batch_bytes stage)."""
    cap = (batch_bytes or DEFAULT_BATCH) // TILE * TILE
    groups, cur, used = [], [], 0
    for c in chunks:
        need = (c[1] + TILE - 1) // TILE * TILE
        if c[1] == 0:
            continue
        if need > cap:
            raise ValueError("chunk larger than the staging batch")
        if cur and used + need > cap:
            groups.append(cur)
            cur, used = [], 0
        cur.append(c)
        used += need
    if cur:
        groups.append(cur)
    return groups


class DeviceEngine:
    """The HIP engine of one rank: a local table counting the rank's input and an owner
    table holding the merged counts of the k-mers this rank owns.  superkmers: no local table --
    a routing context (tokenizer + kc_route_superkmers_device) and the owner table, which counts
    the super-k-mer streams the rank receives (kc_count_packed_device)."""

    def __init__(self, cfg: Config, local_slots: int = 0, world: int = 1, superkmers: bool = False):
        import dataclasses

        self.cfg = cfg  # the owner table: this rank's share of -s
        self.world = world
        self.superkmers = superkmers
        self._skm_cap = 0
        self._spk = self._sbk = None
        if superkmers:
            # (the routing context's own table is a stub: it never counts)
            self.kc = KmerCounter(dataclasses.replace(cfg, bf_enable=False, table_slots=1 << 16))
            self.same_geometry = False
            self.owner = None
            self._agg = None
            self._agg_slots = 0
            self._uniq, self._nuniq = None, 0
            self.W = words_for_k(cfg.k)
            self.device = "cuda"
            self._buf = None
            self._rec = None
            return
        # the local table must hold every distinct k-mer of this rank's input, which the
        # owner share does not bound (a rank sees ~all k-mers of the genome at low
        # per-rank coverage): local_slots, e.g. min(-s total, this rank's windows).  With the
        # Bloom filter the local count is ungated (the owners gate): it holds every distinct
        # k-mer of the rank's input -- local_slots when given (e.g. bench.py's distinct estimate;
        # -u overstates it ~8x for C3), else -u
        if cfg.bf_enable:
            local = dataclasses.replace(cfg, bf_enable=False,
                                        table_slots=local_slots or max(cfg.est_unique, cfg.table_slots))
        else:
            local = dataclasses.replace(cfg, table_slots=max(cfg.table_slots, local_slots))
            # the owner table takes the same size: the records a rank receives are then region-sorted
            # groups merged by one level-3 pass (kc_insert_counts_runs_device), with no partition
            # buffers beside the two tables (a local table larger than the owner's share is the
            # strong presets' case: C4 at 8 ranks 567 M local vs 406 M owner slots)
            self.cfg = cfg = dataclasses.replace(cfg, table_slots=local.table_slots)
        self.kc = KmerCounter(local)    # local table (also used by the per-window route path)
        if world > 1:  # its level-3 passes keep the per-owner counts the merge's route needs
            self.kc.route_hint(world)
        # every rank's local table has the owner table's geometry: the records a rank
        # receives are region-sorted groups, merged in one pass (kc_insert_counts_runs_device)
        self.same_geometry = local.table_slots == cfg.table_slots
        self.owner = None               # created on first use
        self._agg = None                # sharded Bloom: the owner's aggregation table
        self._agg_slots = 0
        self._uniq, self._nuniq = None, 0
        self.W = words_for_k(cfg.k)
        self.device = "cuda"
        self._buf = None
        self._rec = None

    # -- per-window routing (no local table)
    def route(self, dev_ptr: int, chunks, fmt: int, parts: int, stream: int = 0):
        import torch

        cap = sum((ln + 4095) // 4096 * 4096 for _, ln, _ in chunks) + len(chunks) + 64
        if self._buf is None or self._buf.numel() < cap * self.W:
            self._buf = torch.empty(cap * self.W, dtype=torch.int64, device="cuda")
        counts = self.kc.route_device(dev_ptr, chunks, fmt, parts, self._buf.data_ptr(), cap, stream)
        return self._buf, counts

    def insert(self, keys, n: int, stream: int = 0):
        self.kc.insert_keys_device(keys.data_ptr(), n, stream)

    # -- pre-aggregated path
    def count(self, dev_ptr: int, chunks, fmt: int, stream: int = 0):
        self.kc.count_device(dev_ptr, chunks, fmt, stream)

    def route_table(self, parts: int, stream: int = 0):
        import torch

        from . import KcError

        R = self.W + 1
        if self._rec is not None:
            try:  # the usual case: the buffer of the previous merge is large enough
                return self._rec, self.kc.route_table_device(parts, self._rec.data_ptr(), self._rec.numel() // R,
                                                             stream)
            except KcError:
                pass
        counts = self.kc.route_table_device(parts, 0, 0, stream)  # record counts per owner
        need = max(1, sum(counts)) * R
        self._rec = torch.empty(need + need // 4, dtype=torch.int64, device="cuda")
        return self._rec, self.kc.route_table_device(parts, self._rec.data_ptr(), self._rec.numel() // R, stream)

    def clear_local(self):
        """The local table was routed to its owners: empty it (its counters stay)."""
        self.kc.clear_table()

    def owner_table(self) -> KmerCounter:
        if self.owner is None:
            import dataclasses

            cfg = self.cfg
            if cfg.bf_enable:  # the owner's filter: its 1/world share of -u
                cfg = dataclasses.replace(cfg, est_unique=max(1, -(-cfg.est_unique // self.world)))
            self.owner = KmerCounter(cfg)
        return self.owner

    def insert_counts(self, recs, n: int, stream: int = 0, group_counts=None):
        if group_counts is not None and self.same_geometry and 0 < len(group_counts) <= 64:
            self.owner_table().insert_counts_runs_device(recs.data_ptr(), group_counts, stream)
        else:
            self.owner_table().insert_counts_device(recs.data_ptr(), n, stream)

    # -- super-k-mer exchange (kc_route_superkmers_device / kc_count_packed_device)
    def _skm_alloc(self, parts: int, need: int):
        import torch

        cap = (int(need * 1.1) + 64) // 2 * 2
        self._spk = torch.empty(parts * cap + 2, dtype=torch.int64, device="cuda")
        self._sbk = torch.empty(parts * cap + 2, dtype=torch.int32, device="cuda")
        self._skm_cap = cap

    def skm_route(self, dev_ptr: int, chunks, fmt: int, parts: int, stream: int = 0):
        """The image's super-k-mers per owner, as contiguous send buffers in rank order: (pk words
        int64, bk words as int64 pairs, words per owner (even: an odd group gets a pad word of
        breaks), windows per owner).  The regions are sized by a dry run the first time and grow
        when a route reports them too small."""
        import torch

        from . import KcError

        for attempt in range(2):
            if self._skm_cap == 0:
                need, _ = self.kc.route_superkmers_device(dev_ptr, chunks, fmt, parts, stream=stream)
                self._skm_alloc(parts, max(need))
            try:
                words, wins = self.kc.route_superkmers_device(dev_ptr, chunks, fmt, parts, self._spk.data_ptr(),
                                                              self._sbk.data_ptr(), self._skm_cap, stream=stream)
                break
            except KcError as e:
                if attempt or getattr(e, "words", None) is None:
                    raise
                self._skm_alloc(parts, max(e.words))
        cap = self._skm_cap
        pks, bks, even = [], [], []
        for o in range(parts):
            n = int(words[o])
            pks.append(self._spk[o * cap: o * cap + n])
            bks.append(self._sbk[o * cap: o * cap + n])
            if n % 2:  # (a pad word: no symbol, every position a break)
                pks.append(self._spk.new_zeros(1))
                bks.append(self._sbk.new_full((1,), -1))
            even.append(n + n % 2)
        return torch.cat(pks), torch.cat(bks).view(torch.int64), even, [int(w) for w in wins]

    def count_packed(self, pk, bk, n_words: int, windows: int, stream: int = 0):
        self.owner_table().count_packed_device(pk.data_ptr(), bk.data_ptr(), n_words, windows, stream)

    def bloom_packed(self, pk, bk, n_words: int, windows: int, stream: int = 0):
        self.owner_table().bloom_packed_device(pk.data_ptr(), bk.data_ptr(), n_words, windows, stream)

    # -- owner-sharded Bloom filter: the rank's ungated local count, then the owner's two
    # passes over the {key, count} records it receives
    def bloom(self, dev_ptr: int, chunks, fmt: int, stream: int = 0):
        self.kc.count_device(dev_ptr, chunks, fmt, stream)

    def _distinct_records(self, recs, n: int, stream: int = 0):
        """The received records with every key once (the senders' records of one k-mer summed):
        kc_bloom_records_device takes distinct keys.  An aggregation table (kc_insert_counts_device)
        read back as records (kc_route_table_device, one part)."""
        import dataclasses

        import torch

        need = max(1 << 16, n)
        if self._agg is None or self._agg_slots < need:
            if self._agg is not None:
                self._agg.close()
            self._agg_slots = need + need // 4
            self._agg = KmerCounter(dataclasses.replace(self.cfg, bf_enable=False, table_slots=self._agg_slots))
        else:
            self._agg.clear_table()
        self._agg.insert_counts_device(recs.data_ptr(), n, stream)
        R = self.W + 1
        out = torch.empty(max(1, n) * R, dtype=torch.int64, device="cuda")
        m = self._agg.route_table_device(1, out.data_ptr(), max(1, n), stream)[0]
        return out, m

    def bloom_records(self, recs, n: int, stream: int = 0):
        self._uniq, self._nuniq = self._distinct_records(recs, n, stream)
        self.owner_table().bloom_records_device(self._uniq.data_ptr(), self._nuniq, stream)

    def owner_bloom_finalize(self) -> int:
        return self.owner_table().bloom_finalize()

    def count_records(self, recs, n: int, stream: int = 0):
        """(the distinct records of the preceding bloom_records)"""
        self.owner_table().count_records_device(self._uniq.data_ptr(), self._nuniq, stream)
        self._uniq = None

    def reset(self):
        self.kc.reset()
        if self.owner is not None:
            self.owner.reset()

    def close(self):
        self.kc.close()
        if self.owner is not None:
            self.owner.close()
        if self._agg is not None:
            self._agg.close()


class ShardedCounter:
    """KmerCounter-compatible front end whose table is sharded over the process group."""

    def __init__(self, cfg: Config, dist, engine=None, group=None, local_slots: int = 0, exchange: str = "records"):
        """cfg.table_slots = this rank's owner share of -s, also the local table's size
        unless local_slots is larger.  local_slots must bound the distinct k-mers of this
        rank's own input: when each rank holds a small share of a large genome (strong
        scaling, e.g. C4), pass min(-s total, this rank's windows).
        exchange: "records" (every rank counts its input locally; the table's {key, count} records
        go to their owners at the merge) or "superkmers" (every counting / Bloom pass routes the
        input's super-k-mers to their canonical-minimizer owners, which count them: no local table;
        collective per pass)."""
        if exchange not in ("records", "superkmers"):
            raise ValueError(f"exchange must be 'records' or 'superkmers', not {exchange!r}")
        self.cfg = cfg
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.W = words_for_k(cfg.k)
        self.mode = exchange
        if engine is None:
            engine = DeviceEngine(cfg, local_slots, self.world, superkmers=exchange == "superkmers")
        self.engine = engine
        self._in_windows = 0  # super-k-mers: the windows this rank routed (its input's)
        self._skm_recv = None  # super-k-mers: the Bloom pass's received streams (its counting pass reuses them)
        self.device = getattr(self.engine, "device", "cpu")
        self._pending = False
        self._stream = 0
        self._inflight = []
        self._bloom_input = None  # the Bloom pass's (image, chunks, format): the owners count it
        self._counted = False
        # exchange traffic of the merges (xGMI bytes reported beside HBM bytes)
        # with profile(True) the merge's phases are timed too (route / exchange / owner insert; the
        # insert waits for its kernels, which the step's end would wait for anyway)
        self.xstats = {"bytes_sent": 0, "bytes_recv": 0, "exchange_s": 0.0, "route_s": 0.0, "insert_s": 0.0,
                       "merges": 0}
        self._profiling = False

    def _skm_exchange(self, dev_ptr: int, chunks, fmt: int, stream: int):
        """Route this rank's image as super-k-mers and exchange them (two all-to-alls: the pk words
        and the bk words; the windows per owner beside them): (pk, bk int32, words, windows) received."""
        import time

        import torch

        with _on_stream(self.device, stream):
            tr = time.perf_counter()
            spk, sbk, words, wins = self.engine.skm_route(dev_ptr, chunks, fmt, self.world, stream)
            self.xstats["route_s"] += time.perf_counter() - tr
            self._in_windows += sum(wins)
            t0 = time.perf_counter()
            rpk, n, per_rank = exchange(self.dist, spk, words, 1, self.group, with_counts=True, extra=2)
            rbk, n2 = exchange(self.dist, sbk, [w // 2 for w in words], 1, self.group, extra=1)
            if 2 * n2 != n:
                raise RuntimeError(f"super-k-mer exchange: {n} pk words but {2 * n2} bk words received")
            if self.world > 1:
                dev = "cpu" if self.dist.get_backend(self.group) == "gloo" else spk.device
                wt = torch.tensor(wins, dtype=torch.int64, device=dev)
                rt = torch.empty_like(wt)
                self.dist.all_to_all_single(rt, wt, group=self.group)
                windows = int(rt.sum().item())
            else:
                windows = sum(wins)
            self.xstats["exchange_s"] += time.perf_counter() - t0
            self.xstats["bytes_sent"] += sum(w for d, w in enumerate(words) if d != self.rank) * 12
            self.xstats["bytes_recv"] += sum(w for d, w in enumerate(per_rank) if d != self.rank) * 12
            self.xstats["merges"] += 1
        return rpk, rbk.view(torch.int32), n, windows

    def _skm_count(self, recv, stream: int):
        import time

        pk, bk, n, windows = recv
        with _on_stream(self.device, stream):
            ti = time.perf_counter()
            self.engine.count_packed(pk, bk, n, windows, stream)
            if self._profiling and self.device == "cuda":
                import torch

                torch.cuda.synchronize()
                self.xstats["insert_s"] += time.perf_counter() - ti
        self._inflight = [pk, bk]  # the receive buffers must outlive the count

    # the counting pass over a device image (chunks from kaarme_amd.plan_chunks): local
    def count_device(self, dev_ptr: int, chunks: List[Tuple[int, int, int]], fmt: int, stream: int = 0):
        if self.mode == "superkmers":  # (collective)
            if self.cfg.bf_enable:
                if self._skm_recv is None or self._bloom_input != (dev_ptr, tuple(map(tuple, chunks)), fmt):
                    raise ValueError("a sharded Bloom job counts the input of its Bloom pass (bloom_device, "
                                     "bloom_finalize, count_device over the same image and chunks)")
                self._skm_count(self._skm_recv, stream)
                self._skm_recv = None
            else:
                self._skm_count(self._skm_exchange(dev_ptr, chunks, fmt, stream), stream)
            self._stream = stream
            return
        if self.cfg.bf_enable:
            # the owners counted the Bloom pass's input behind their gates (bloom_finalize): the
            # counting pass must present that input again (the reference reads the file twice)
            if not self._counted or self._bloom_input != (dev_ptr, tuple(map(tuple, chunks)), fmt):
                raise ValueError("a sharded Bloom job counts the input of its Bloom pass (bloom_device, "
                                 "bloom_finalize, count_device over the same image and chunks)")
            self._counted = False
            return
        self.engine.count(dev_ptr, chunks, fmt, stream)
        self._pending = True
        self._stream = stream

    def merge(self, stream: int = 0):
        """Route the local table's records to their owners (one all-to-all) and add them
        into the owner tables.  Collective: every rank calls it the same number of times."""
        import time

        if self._local_owner():
            # one rank owns every k-mer: its local table is its owner table, no record moves
            # (the route, the region check and the runs insert were 2.9 ms of
            # an 18.3 ms C2 step at one rank)
            self.xstats["merges"] += 1
            self._pending = False
            return
        with _on_stream(self.device, stream):
            tr = time.perf_counter()
            recs, counts = self.engine.route_table(self.world, stream)  # (the counts come back to the host)
            self.xstats["route_s"] += time.perf_counter() - tr
            # the records hold the local counts now: a later merge must route only what is
            # counted after this one
            self.engine.clear_local()
            t0 = time.perf_counter()
            recv, n, per_rank = exchange(self.dist, recs, counts, self.W + 1, self.group, with_counts=True)
            rec_bytes = (self.W + 1) * 8
            self.xstats["bytes_sent"] += sum(c for d, c in enumerate(counts) if d != self.rank) * rec_bytes
            self.xstats["bytes_recv"] += sum(c for d, c in enumerate(per_rank) if d != self.rank) * rec_bytes
            self.xstats["exchange_s"] += time.perf_counter() - t0  # (route synced before, the sums check after)
            self.xstats["merges"] += 1
            ti = time.perf_counter()
            self.engine.insert_counts(recv, n, stream, group_counts=per_rank)
            if self._profiling and self.device == "cuda":
                import torch

                torch.cuda.synchronize()
                self.xstats["insert_s"] += time.perf_counter() - ti
        self._inflight = [recv]  # the receive buffer must outlive the insert
        self._pending = False

    # the Bloom pass over a device image: this rank's ungated local count (super-k-mers: the owners'
    # Bloom pass 1 over the streams they receive, collective)
    def bloom_device(self, dev_ptr: int, chunks: List[Tuple[int, int, int]], fmt: int, stream: int = 0):
        if not self.cfg.bf_enable:
            raise ValueError("bloom_device needs Config(bf_enable=True)")
        if self.mode == "superkmers":
            recv = self._skm_exchange(dev_ptr, chunks, fmt, stream)
            pk, bk, n, windows = recv
            with _on_stream(self.device, stream):
                self.engine.bloom_packed(pk, bk, n, windows, stream)
            self._skm_recv = recv
            self._bloom_input = (dev_ptr, tuple(map(tuple, chunks)), fmt)
            self._stream = stream
            return
        self.engine.bloom(dev_ptr, chunks, fmt, stream)
        self._bloom_input = (dev_ptr, tuple(map(tuple, chunks)), fmt)
        self._stream = stream

    def bloom_finalize(self, stream: int = None) -> int:
        """End of the Bloom pass (collective): the local tables' records to their owners, the
        owners' Bloom pass over them, their tables sized (2 x their new_in_second) and the same
        records counted behind their gates.  Returns new_in_second summed over the owners."""
        import time

        import torch

        stream = self._stream if stream is None else stream
        if self.mode == "superkmers":  # every owner holds all occurrences of its k-mers: its own pass 1
            with _on_stream(self.device, stream):
                nis = self.engine.owner_bloom_finalize()
                tot = torch.tensor([int(nis)], dtype=torch.int64, device=self.device if self.device == "cuda" else "cpu")
                if self.world > 1:
                    self.dist.all_reduce(tot, group=self.group)
            self._pending = False
            return int(tot.item())
        with _on_stream(self.device, stream):
            recs, counts = self.engine.route_table(self.world, stream)
            self.engine.clear_local()
            t0 = time.perf_counter()
            recv, n, per_rank = exchange(self.dist, recs, counts, self.W + 1, self.group, with_counts=True)
            rec_bytes = (self.W + 1) * 8
            self.xstats["bytes_sent"] += sum(c for d, c in enumerate(counts) if d != self.rank) * rec_bytes
            self.xstats["bytes_recv"] += sum(c for d, c in enumerate(per_rank) if d != self.rank) * rec_bytes
            self.xstats["exchange_s"] += time.perf_counter() - t0
            self.xstats["merges"] += 1
            self.engine.bloom_records(recv, n, stream)
            nis = self.engine.owner_bloom_finalize()
            self.engine.count_records(recv, n, stream)
            tot = torch.tensor([int(nis)], dtype=torch.int64, device=self.device if self.device == "cuda" else "cpu")
            if self.world > 1:
                self.dist.all_reduce(tot, group=self.group)
        self._inflight = [recv]  # the receive buffer must outlive the owner's passes
        self._counted = True
        self._pending = False
        return int(tot.item())

    @property
    def kc(self) -> KmerCounter:
        """The owner table (this rank's share of the merged counts)."""
        if self._local_owner():
            return self.engine.kc
        return self.engine.owner_table()

    def _local_owner(self) -> bool:
        """One rank, no Bloom filter: the local table is the owner table (merge moves nothing)."""
        return self.world == 1 and not self.cfg.bf_enable and self.mode == "records"

    def reset(self):
        self.engine.reset()
        self._pending = False
        self._inflight = []
        self._bloom_input = None
        self._counted = False
        self._in_windows = 0
        self._skm_recv = None

    def sync(self):
        """Completes the job: the (collective) merge if counts are pending, then waits."""
        if self._pending:
            self.merge(self._stream)
        self.engine.kc.sync()
        if not self._local_owner():
            self.kc.sync()
        self._inflight = []

    def profile(self, enable: bool = True):
        self._profiling = enable
        self.engine.kc.profile(enable)
        if not self._local_owner():
            self.kc.profile(enable)

    def timing(self) -> dict:
        """Local counting batches (+ the table routing) plus the merge insert (count_ms); super-k-mers:
        the owner's batches (the routing passes are not timed)."""
        a = self.engine.kc.timing()
        if self._local_owner():
            return dict(a)
        if self.mode == "superkmers":
            return dict(self.kc.timing())
        b = self.kc.timing()
        out = dict(a)
        out["count_ms"] = a["count_ms"] + b["count_ms"]
        return out

    def finish(self) -> dict:
        """Stats of the owner table; windows / chunks / bytes are this rank's input."""
        self.sync()
        if self.mode == "superkmers":  # (no local table: the windows are the ones this rank routed)
            st = dict(self.kc.finish())
            st["owner_windows"] = st["windows"]
            st["windows"] = self._in_windows
            st["local_distinct"] = 0
            return st
        local = self.engine.kc.finish()
        own = local if self._local_owner() else self.kc.finish()
        st = dict(own)
        keys = ("windows", "chunks", "bytes", "reused_passes")
        if not self.cfg.bf_enable:  # (with the filter, the owner's Bloom counters are its own)
            keys += ("bf_windows", "bf_bits", "new_in_first", "new_in_second", "failed_in_first")
        for key in keys:
            st[key] = local[key]
        if self.cfg.bf_enable:
            st["bf_windows"] = local["windows"]  # the ungated local count saw every window
        st["local_distinct"] = local["distinct"]
        return st

    def close(self):
        """Free the rank's device tables (the counter is unusable afterwards)."""
        self._inflight = []
        close = getattr(self.engine, "close", None)
        if close:
            close()

    def output_digest(self, combine: bool = True) -> dict:
        """Digest of this rank's output (its owner table, kc_output_digest) or, with combine
        (collective), of the whole job's: the owners' digests add up (their k-mers are disjoint),
        gathered over the group.  The whole job's output is the concatenation of the owners'
        outputs, so this is the digest a single table of the whole input would give."""
        from . import combine_digests, digest_dict

        self.sync()
        d = self.kc.output_digest()
        if not combine or self.world == 1:
            return d
        import torch

        vals = [d["lines"], d["count_sum"], int(d["hash_sum"], 16), int(d["hash_xor"], 16)]
        dev = "cuda" if self.device == "cuda" and self.dist.get_backend(self.group) != "gloo" else "cpu"
        t = torch.tensor([v - (1 << 64) if v >= (1 << 63) else v for v in vals], dtype=torch.int64, device=dev)
        got = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(got, t, group=self.group)
        return combine_digests(digest_dict(*[int(v) & (2**64 - 1) for v in g.tolist()]) for g in got)

    def dump(self):
        return self.kc.dump()

    def lines(self):
        return self.kc.lines()

    def write(self, path: str):
        self.kc.write(path)
