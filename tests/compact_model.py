"""Test-side restatement of Kaarme's compact k-mer representation (checker only).

Slot word (OneCharacterAndPointerKMerAtomicVariable, kmer.hpp:103-149; accessors
kmer.cpp:610-714): bit 0 occupied, 1 predecessor exists, 4 self canonical during
insertion, 5 predecessor canonical during insertion, 8-9 right character, 10-11 left
character, 12-25 count, 26-63 predecessor slot (or the secondary-array index of a chain
start).  `reconstruct` follows reconstruct_kmer_in_slot (kmer_hash_table.cpp:3848-4058)
step by step: L/R = leftmost/rightmost untaken position, Lc/Rc = the current chain k-mer's
ends in the frame, pir = "process in reverse"; the eight flag cases of :3925-3998; the
secondary-array fill of :4005-4038 (get_secondary_array_char = character b of the start's key).
"""

ACGT = "ACGT"


def key_char(words, k, j):
    """Character j (0 = leftmost) of a canonical key given as W big-endian u64 words."""
    W = len(words)
    pos = 2 * (k - 1 - j)
    return (int(words[W - 1 - pos // 64]) >> (pos % 64)) & 3


def reconstruct(words, second, slot, k, max_hops=None):
    """The k-mer string of `slot`, and the number of predecessor hops taken."""
    chars = [4] * k
    L, R, Lc, Rc = 0, k - 1, 0, k - 1
    pir = False
    pos = slot
    hops = 0
    start = False
    while True:
        w = int(words[pos])
        assert w & 1, "walk reached an unoccupied slot"
        if not (w >> 1) & 1:
            start = True
            break
        left, right = (w >> 10) & 3, (w >> 8) & 3
        if L == Lc:
            chars[L] = 3 - right if pir else left
            L += 1
            if L > R:
                break
        if R == Rc:
            chars[R] = 3 - left if pir else right
            R -= 1
            if L > R:
                break
        self_c, pred_c = (w >> 4) & 1, (w >> 5) & 1
        if self_c:
            if pred_c:
                d, flip = (+1, False) if pir else (-1, False)   # T T T / T T F
            else:
                d, flip = (+1, True) if pir else (-1, True)     # T F T / T F F
        else:
            if pred_c:
                d, flip = (-1, True) if pir else (+1, True)     # F T T / F T F
            else:
                d, flip = (-1, False) if pir else (+1, False)   # F F T / F F F
        Lc += d
        Rc += d
        if flip:
            pir = not pir
        pos = w >> 26
        hops += 1
        if max_hops is not None:
            assert hops <= max_hops, "walk too long"
    if start:
        sidx = int(words[pos]) >> 26
        key = second[sidx]
        Ls = L - Lc
        if not pir:
            a, b = L, Ls
            while a <= R:
                chars[a] = key_char(key, k, b)
                a += 1
                b += 1
        else:
            a, b = L, k - Ls - 1
            while a <= R:
                chars[a] = 3 - key_char(key, k, b)
                a += 1
                b -= 1
    return "".join(ACGT[c] for c in chars), hops
