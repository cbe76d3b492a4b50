"""Digest of a counting result in the reference's parity form:
SHA-256 of the byte-sorted output text "<CANONICAL_KMER> <T(c)>\\n", its line count and the sum
of its counts -- what `LC_ALL=C sort out.kaarme_counts | sha256sum` gives for the reference's
output (kmer_hash_table.cpp:4318-4524), computed from kc_dump records without writing a file.

The records are sorted by key on the device (torch, when a GPU is present; numpy otherwise):
every line starts with a k-character k-mer over A < C < G < T and the k-mers are distinct, so
byte order of the lines is the numeric order of the 2-bit keys.  Used by bench.py (parity of
the timed configuration against tests/golden/fullsize.json) and the tests.
"""
from __future__ import annotations

import hashlib

import numpy as np

from . import words_for_k

_SIGN = -(1 << 63)


def _torch_device():
    try:
        import torch
        if torch.cuda.is_available():
            return torch, torch.device("cuda")
    except ImportError:
        pass
    return None, None


def sorted_text_digest(records: np.ndarray, k: int, min_abundance: int = 1) -> dict:
    """records: (n, W+1) uint64 (kc_dump layout: key words, most significant first, then T(c))."""
    W = words_for_k(k)
    recs = np.ascontiguousarray(records, dtype=np.uint64).reshape(-1, W + 1)
    if min_abundance > 1:
        recs = recs[recs[:, W] >= np.uint64(min_abundance)]
    n = recs.shape[0]
    if n == 0:
        return {"sorted_sha256": hashlib.sha256(b"").hexdigest(), "lines": 0, "count_sum": 0}
    torch, dev = _torch_device()
    h = hashlib.sha256()
    if torch is not None:
        for piece in _text_torch(torch, dev, recs, k, W):
            h.update(memoryview(piece))
    else:
        h.update(memoryview(_text_numpy(recs, k, W)))
    counts = recs[:, W]
    return {"sorted_sha256": h.hexdigest(), "lines": int(n), "count_sum": int(counts.sum(dtype=np.uint64))}


ROWS = 1 << 23  # lines formatted per device piece (boolean indexing of > 2^31 elements fails on ROCm)


def _text_torch(torch, dev, recs, k, W):
    """The sorted text in pieces of ROWS lines (host uint8 arrays)."""
    r_all = torch.from_numpy(recs.view(np.int64)).to(dev)
    perm = torch.arange(r_all.shape[0], device=dev)
    for w in reversed(range(W)):  # stable LSD passes: word W-1 first, word 0 last
        key = r_all[perm, w] ^ _SIGN  # unsigned order as signed order
        perm = perm[torch.sort(key, stable=True).indices]
    for lo in range(0, r_all.shape[0], ROWS):
        yield _lines_torch(torch, dev, r_all[perm[lo:lo + ROWS]], k, W)


def _lines_torch(torch, dev, r, k, W):
    n = r.shape[0]
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    line = torch.empty((n, k + 7), dtype=torch.uint8, device=dev)
    for j in range(k):
        bit = 2 * (k - 1 - j)
        line[:, j] = lut[(r[:, W - 1 - bit // 64] >> (bit % 64)) & 3]
    line[:, k] = ord(" ")
    c = r[:, W]
    nd = 1 + (c >= 10).long() + (c >= 100).long() + (c >= 1000).long() + (c >= 10000).long()
    for t in range(6):  # column k+1+t: digit t of the count, then '\n'
        p = torch.clamp(nd - 1 - t, min=0)
        digit = (c // (10 ** p)) % 10 + ord("0")
        col = torch.where(t < nd, digit, torch.full_like(c, ord("\n")))
        line[:, k + 1 + t] = col.to(torch.uint8)
    keep = torch.arange(k + 7, device=dev).unsqueeze(0) <= (k + 1 + nd).unsqueeze(1)
    return line[keep].cpu().numpy()


def _text_numpy(recs, k, W):
    order = np.lexsort(tuple(recs[:, w] for w in reversed(range(W))))
    r = recs[order]
    n = r.shape[0]
    lut = np.frombuffer(b"ACGT", dtype=np.uint8)
    line = np.empty((n, k + 7), dtype=np.uint8)
    for j in range(k):
        bit = 2 * (k - 1 - j)
        line[:, j] = lut[(r[:, W - 1 - bit // 64] >> np.uint64(bit % 64)) & np.uint64(3)]
    line[:, k] = ord(" ")
    c = r[:, W].astype(np.int64)
    nd = 1 + (c >= 10) + (c >= 100) + (c >= 1000) + (c >= 10000)
    for t in range(6):
        p = np.maximum(nd - 1 - t, 0)
        digit = (c // (10 ** p)) % 10 + ord("0")
        line[:, k + 1 + t] = np.where(t < nd, digit, ord("\n")).astype(np.uint8)
    keep = np.arange(k + 7)[None, :] <= (k + 1 + nd)[:, None]
    return line[keep]
