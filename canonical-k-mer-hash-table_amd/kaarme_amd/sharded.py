"""Hash-prefix owner sharding of the counting table across GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, over xGMI).
Per batch every rank
  1. tokenizes its own input and routes the table keys of its windows to their owner
     shard (``kc_route_device``: keys grouped by owner, owner = a bit field of the
     engine's bijective table key, independent of the table's region/bucket bits);
  2. exchanges the groups with ONE all-to-all (counts first, then the keys);
  3. inserts what it received into its private table (``kc_insert_keys_device``).
Every canonical k-mer has exactly one owner, so the union of the per-shard tables is
the exact global count and the output is the concatenation of the per-shard dumps.

The exchange logic (:func:`exchange`) is backend-agnostic torch code: the CPU tests run
it over ``gloo`` with a NumPy engine, the GPU path over RCCL with the HIP engine.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

from . import Config, KmerCounter, words_for_k


def exchange(dist, keys, counts: Sequence[int], W: int, group=None):
    """All-to-all of owner-grouped keys.  keys: int64 tensor holding sum(counts)*W words
    (group d = the keys for rank d, in rank order).  Returns (received keys, n received)."""
    import torch

    dev = keys.device
    send_counts = torch.tensor(list(counts), dtype=torch.int64, device=dev)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    recv = [int(x) for x in recv_counts.cpu().tolist()]
    total = sum(recv)
    out = torch.empty(max(1, total * W), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out[: total * W], keys[: sum(counts) * W],
                           output_split_sizes=[r * W for r in recv],
                           input_split_sizes=[c * W for c in counts], group=group)
    return out, total


class DeviceEngine:
    """The HIP engine of one rank: routes device images, inserts received keys."""

    def __init__(self, cfg: Config):
        self.cfg = cfg
        self.kc = KmerCounter(cfg)
        self.W = words_for_k(cfg.k)
        self._buf = None

    def route(self, dev_ptr: int, chunks, fmt: int, parts: int, stream: int = 0):
        import torch

        cap = sum((ln + 4095) // 4096 * 4096 for _, ln, _ in chunks) + len(chunks) + 64
        if self._buf is None or self._buf.numel() < cap * self.W:
            self._buf = torch.empty(cap * self.W, dtype=torch.int64, device="cuda")
        counts = self.kc.route_device(dev_ptr, chunks, fmt, parts, self._buf.data_ptr(), cap, stream)
        return self._buf, counts

    def insert(self, keys, n: int, stream: int = 0):
        self.kc.insert_keys_device(keys.data_ptr(), n, stream)


class ShardedCounter:
    """KmerCounter-compatible front end whose table is sharded over the process group."""

    def __init__(self, cfg: Config, dist, engine=None, group=None):
        self.cfg = cfg
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.W = words_for_k(cfg.k)
        self.engine = engine if engine is not None else DeviceEngine(cfg)
        self._inflight = []

    # the counting pass over a device image (chunks from kaarme_amd.plan_chunks)
    def count_device(self, dev_ptr: int, chunks: List[Tuple[int, int, int]], fmt: int, stream: int = 0):
        keys, counts = self.engine.route(dev_ptr, chunks, fmt, self.world, stream)
        recv, n = exchange(self.dist, keys, counts, self.W, self.group)
        self.engine.insert(recv, n, stream)
        self._inflight = [recv]  # keep the receive buffer alive until the insert completed

    # delegation to the local shard
    @property
    def kc(self) -> KmerCounter:
        return self.engine.kc

    def reset(self):
        self.kc.reset()

    def sync(self):
        self.kc.sync()
        self._inflight = []

    def profile(self, enable: bool = True):
        self.kc.profile(enable)

    def timing(self) -> dict:
        return self.kc.timing()

    def finish(self) -> dict:
        return self.kc.finish()

    def dump(self):
        return self.kc.dump()

    def lines(self):
        return self.kc.lines()
