"""Test-side model of the Bloom filter bit positions (checker only).

* reference layout (KC_BLOOM_LAYOUT=reference): the reference's positions
  h_j = XXH64(&root, 8, seed_j) & (bits - 1) (calculate_hashes, double_bloomfilter.hpp:
  276-281, seeds :434-444), root = min(F, B) of RollingHasherDual mod 2^54
  (hash_functions.cpp:102-192); filter-1 bit of h at 2h, filter-2 bit at 2h + 1
  (MyAtomicBitArrayFT, mybitarray.hpp:30-125), stored LSB-first in u32 words.
* blocked layout (the engine's default, kc_count_impl.h): one 64-byte block per k-mer
  picked by the table key (kc_common.h to_tkey), position j = a 5-bit field of one
  multiply-fold of it, in word j mod 8 of each filter half.
* sizes: main.cpp:402-418 (bits), ceil(hf) pass-1 positions (main.cpp:417), trunc(hf)
  pass-2 gate positions (the double passed as uint64_t, parallel_parser.hpp:2397).
"""
import math

M64 = (1 << 64) - 1
M54 = (1 << 54) - 1
SEEDS = [2411, 3253, 1061, 1129, 2269, 7309, 3491, 8237, 6359, 8779]
CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def xxh64_u64(v, seed):
    """XXH64 of one 8-byte little-endian value (xxHash spec, input length 8)."""
    P1, P2, P3, P4, P5 = (0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9, 0x85EBCA77C2B2AE63,
                          0x27D4EB2F165667C5)
    h = (seed + P5 + 8) & M64
    k1 = (rotl((v * P2) & M64, 31) * P1) & M64
    h ^= k1
    h = (rotl(h, 27) * P1 + P4) & M64
    h ^= h >> 33
    h = (h * P2) & M64
    h ^= h >> 29
    h = (h * P3) & M64
    h ^= h >> 32
    return h


def sizes(U, fpr):
    bits_min = (-U * math.log(fpr)) / (math.log(2) ** 2)
    hf = bits_min / U * math.log(2)
    b = 2
    while b < int(bits_min):
        b *= 2
    return b, math.ceil(hf), int(hf)


def root(kmer):
    k = len(kmer)
    F = B = 0
    for i, ch in enumerate(kmer):
        c = CODE[ch]
        F = (F + c * pow(5, k - 1 - i, 1 << 54)) & M54
        B = (B + (3 - c) * pow(5, i, 1 << 54)) & M54
    return min(F, B)


def canonical_words(kmer):
    k = len(kmer)
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    rc = "".join(comp[c] for c in reversed(kmer))
    s = min(kmer, rc)  # lexicographic = numeric with A<C<G<T (kmer_factory.cpp:219-233)
    v = 0
    for ch in s:
        v = (v << 2) | CODE[ch]
    W = k // 32 + 1
    return [(v >> (64 * (W - 1 - i))) & M64 for i in range(W)]


def fmix64(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def table_key0(kmer):
    """Word 0 of the table key (kc_common.h to_tkey): W = 1: tmix(key0 ^ MIX_C); W >= 2:
    tmix(last word ^ g(the other words)), a zero argument standing as TK_ZERO."""
    w = canonical_words(kmer)
    if len(w) == 1:
        x = w[0] ^ 0x9E3779B97F4A7C15
    else:
        g = 0
        for i in range(len(w) - 1):
            g = fmix64(g ^ w[i] ^ ((0x243F6A8885A308D3 * (i + 1)) & M64))
        x = (w[-1] ^ g) or 0x6A09E667F3BCC909
    y = (x * 0x9E3779B97F4A7C15) & M64
    return y ^ (y >> 32)


def positions(kmer, bits, n, layout):
    """[(word, bit)] of filter 1 and of filter 2 for positions j < n."""
    if layout == "reference":
        r = root(kmer)
        f1, f2 = [], []
        for j in range(n):
            h = xxh64_u64(r, SEEDS[j]) & (bits - 1)
            f1.append(((2 * h) >> 5, (2 * h) & 31))
            f2.append(((2 * h + 1) >> 5, (2 * h + 1) & 31))
        return f1, f2
    t0 = table_key0(kmer)
    nblocks = max(1, bits // 256)
    blk = (t0 >> 32) >> (32 - (nblocks.bit_length() - 1))
    x = ((t0 ^ 0xD6E8FEB86659FD93) * 0xBF58476D1CE4E5B9) & M64
    h = x ^ (x >> 31)
    f1, f2 = [], []
    for j in range(n):
        b = ((h & 0xFFFFFFFF) >> (5 * j)) & 31 if j < 6 else ((h >> 32) >> (5 * (j - 6))) & 31
        f1.append((blk * 16 + (j & 7), b))
        f2.append((blk * 16 + 8 + (j & 7), b))
    return f1, f2


def set_bits(words):
    """{(word, bit)} of every set bit of a u32 array."""
    out = set()
    for i in [int(x) for x in (words != 0).nonzero()[0]]:
        w = int(words[i])
        for b in range(32):
            if (w >> b) & 1:
                out.add((i, b))
    return out
