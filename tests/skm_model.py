"""NumPy model of the super-k-mer routing (canonical-k-mer-hash-table_amd/csrc/kc_skm.hip), test
infrastructure: the canonical-minimizer owner of every window of a sequence, the packed symbol
stream format (kc_internal.h PackedView) both ways, and a host router that produces the same
per-owner streams the device kernel does (up to the order of the super-k-mers).

owner(window) = fmix32(min over its k - m + 1 m-mers of h(canonical m-mer)) * G >> 32, with
h(x) = fmix32(lo32(x) ^ hi32(x) * SKM_FOLD ^ SKM_SEED32) (0xFFFFFFFF -> 0xFFFFFFFE), m = min(15, k) by default (the
minimum of many uniform hashes is small: mixed again before it picks an owner).
"""
import numpy as np

SKM_SEED32 = 0x4C957F2D
SKM_FOLD = 0x9E3779B1
BROKEN = 0xFFFFFFFF
DEFAULT_M = 15

CODE = np.full(256, 4, dtype=np.uint8)
for _i, _c in enumerate("ACGT"):
    CODE[ord(_c)] = _i
    CODE[ord(_c.lower())] = _i


def mmer_hashes(codes, m):
    """h(canonical m-mer) of the m-mer ending at every position q >= m - 1 (index q - m + 1);
    BROKEN where the m-mer holds a non-ACGT symbol."""
    codes = np.asarray(codes, dtype=np.uint8)
    if len(codes) < m:
        return np.zeros(0, dtype=np.uint64)
    win = np.lib.stride_tricks.sliding_window_view(codes, m)
    bad = (win > 3).any(axis=1)
    c = np.where(win > 3, 0, win).astype(np.uint64)
    sh = (2 * np.arange(m - 1, -1, -1)).astype(np.uint64)
    fwd = (c << sh).sum(axis=1, dtype=np.uint64)
    rc = ((np.uint64(3) - c[:, ::-1]) << sh).sum(axis=1, dtype=np.uint64)
    canon = np.minimum(fwd, rc)
    m32 = np.uint64(0xFFFFFFFF)
    x = (canon & m32) ^ (((canon >> np.uint64(32)) * np.uint64(SKM_FOLD)) & m32) ^ np.uint64(SKM_SEED32)
    h = fmix32(x)
    h = np.where(h == BROKEN, BROKEN - 1, h)
    return np.where(bad, BROKEN, h).astype(np.uint64)


def fmix32(h):
    h = h.astype(np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def window_owners(codes, k, G, m=0):
    """Owner of the window ending at every position p >= k - 1 (index p - k + 1), -1 if invalid."""
    m = m or min(DEFAULT_M, k)
    h = mmer_hashes(codes, m)
    w = k - m + 1
    if len(h) < w:
        return np.zeros(0, dtype=np.int64)
    hw = np.lib.stride_tricks.sliding_window_view(h, w)
    mn, mx = hw.min(axis=1), hw.max(axis=1)
    own = ((fmix32(mn ^ np.uint64(0x9E3779B9)) * np.uint64(G)) >> np.uint64(32)).astype(np.int64)
    return np.where(mx == BROKEN, -1, own)


def superkmers(codes, k, G, m=0):
    """(owner, first window end p, run length r) of every super-k-mer of a sequence."""
    own = window_owners(codes, k, G, m)
    out = []
    i = 0
    while i < len(own):
        if own[i] < 0:
            i += 1
            continue
        j = i + 1
        while j < len(own) and own[j] == own[i]:
            j += 1
        out.append((int(own[i]), i + k - 1, j - i))
        i = j
    return out


def pack(seqs):
    """Sequences -> (pk uint64 words, bk uint32 words): each sequence preceded by a break symbol,
    the last word's padding breaks (the device stream format)."""
    syms, brk = [], []
    for s in seqs:
        c = CODE[np.frombuffer(s.encode(), dtype=np.uint8)]
        syms.append(np.concatenate([[0], np.where(c > 3, 0, c)]).astype(np.uint64))
        brk.append(np.concatenate([[1], (c > 3).astype(np.uint32)]).astype(np.uint32))
    sy = np.concatenate(syms) if syms else np.zeros(0, np.uint64)
    br = np.concatenate(brk) if brk else np.zeros(0, np.uint32)
    n = (len(sy) + 31) // 32
    pad = n * 32 - len(sy)
    sy = np.concatenate([sy, np.zeros(pad, np.uint64)]).reshape(n, 32)
    br = np.concatenate([br, np.ones(pad, np.uint32)]).reshape(n, 32)
    pk = (sy << (62 - 2 * np.arange(32, dtype=np.uint64))).sum(axis=1, dtype=np.uint64)
    bk = (br << (31 - np.arange(32, dtype=np.uint32))).sum(axis=1, dtype=np.uint64).astype(np.uint32)
    return pk, bk


def unpack(pk, bk):
    """(pk, bk) -> the maximal break-free symbol runs as ACGT strings."""
    pk = np.asarray(pk, dtype=np.uint64)
    bk = np.asarray(bk, dtype=np.uint32)
    j = np.arange(32, dtype=np.uint64)
    sy = ((pk[:, None] >> (np.uint64(62) - 2 * j)) & np.uint64(3)).astype(np.uint8).ravel()
    br = ((bk[:, None].astype(np.uint64) >> (np.uint64(31) - j)) & np.uint64(1)).astype(bool).ravel()
    letters = np.frombuffer(b"ACGT", dtype=np.uint8)[sy]
    letters = np.where(br, ord("\n"), letters).astype(np.uint8)
    return [s for s in letters.tobytes().decode().split("\n") if s]


def route(seqs, k, G, m=0):
    """Host router: per owner the list of super-k-mer strings of the sequences."""
    out = [[] for _ in range(G)]
    for s in seqs:
        c = CODE[np.frombuffer(s.encode(), dtype=np.uint8)]
        for o, p, r in superkmers(c, k, G, m):
            out[o].append(s[p - k + 1:p + r])
    return out
