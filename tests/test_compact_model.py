"""CPU: the compaction rule of kc_compact_impl.h restated in Python over a small k-mer set,
walked back by the reference's reconstruction (compact_model.reconstruct, restated from
kmer_hash_table.cpp:3848-4058): every k-mer is rebuilt, within k - 2 hops."""
import collections
import random

import pytest

from compact_model import reconstruct

COMP = str.maketrans("ACGT", "TGCA")
CODE = {"A": 0, "C": 1, "G": 2, "T": 3}
M64 = (1 << 64) - 1


def rc(s):
    return s.translate(COMP)[::-1]


def canon(s):
    return min(s, rc(s))


def fmix64(x):
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & M64
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & M64
    x ^= x >> 33
    return x


def enc(s):
    v = 0
    for ch in s:
        v = (v << 2) | CODE[ch]
    return v


def minimizer_forward(K, m):
    """True if the smallest-hash canonical m-mer reads forward in K (kc_compact_impl.h)."""
    best, ori = None, True
    for i in range(len(K) - m + 1):
        f, r = enc(K[i:i + m]), enc(rc(K[i:i + m]))
        h = fmix64(min(f, r) ^ 0x632BE59BD9B4E019)
        if best is None or h < best:
            best, ori = h, f < r
    return ori


def minimizer_len(k):
    return 15 if k >= 15 else (k if k & 1 else k - 1)


def to_words(s, W):
    v = enc(s)
    return [(v >> (64 * (W - 1 - j))) & M64 for j in range(W)]


def build(kmers, k):
    """{canonical k-mer: count} -> (slot words, secondary keys, slot of each k-mer)."""
    m = minimizer_len(k)
    W = k // 32 + 1
    order = sorted(kmers)
    random.Random(k).shuffle(order)   # slot order is irrelevant to the walk
    slot = {K: i for i, K in enumerate(order)}
    words, second = [0] * len(order), []
    for K in order:
        ox = minimizer_forward(K, m)
        X = K if ox else rc(K)
        w = 1 | (min(kmers[K], 16383) << 12) | (CODE[K[-1]] << 8) | (CODE[K[0]] << 10) | (16 if ox else 0)
        for c in "ACGT":
            P = c + X[:-1]
            pc = P <= rc(P)
            KP = canon(P)
            if KP in slot and minimizer_forward(KP, m) == pc:
                w |= 2 | (32 if pc else 0) | (slot[KP] << 26)
                break
        else:
            w |= len(second) << 26
            second.append(to_words(K, W))
        words[slot[K]] = w
    return words, second, slot


@pytest.mark.parametrize("k", [1, 2, 3, 5, 9, 16, 21, 31, 33, 40])
def test_compaction_rule_reconstructs(k):
    rng = random.Random(100 + k)
    genome = "".join(rng.choice("ACGT") for _ in range(600)) + "A" * 80 + "CA" * 40
    kmers = collections.Counter()
    for _ in range(60):
        p = rng.randrange(0, len(genome) - 100)
        r = genome[p:p + 100]
        if rng.random() < 0.5:
            r = rc(r)
        if rng.random() < 0.3:  # a substitution error
            q = rng.randrange(len(r))
            r = r[:q] + rng.choice("ACGT".replace(r[q], "")) + r[q + 1:]
        for i in range(len(r) - k + 1):
            kmers[canon(r[i:i + k])] += 1
    words, second, slot = build(kmers, k)
    for K, i in slot.items():
        s, hops = reconstruct(words, second, i, k, max_hops=max(0, k - 2))
        assert s == K
        assert (words[i] >> 12) & 16383 == kmers[K]
    if k >= 21:
        assert len(second) < 0.35 * len(kmers)
