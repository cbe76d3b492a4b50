"""Deterministic edge-case FASTA / plain generator for parity fixtures.

Exercises the reference tokenizer's corners (parallel_parser.hpp:1373-1465,
1322-1372): headers that contain ACGT letters and extra '>' characters, '>' inside
sequence lines, lower case, 'N', '\\r', empty lines, wrapped and unwrapped records,
empty records, and long poly-A runs (count saturation at 16383 for -m 1/2, uint16
wrap for -m 0).  Counter-based (splitmix64 over (seed, record, field, index)) and
vectorised with numpy, so the bytes never depend on the Python version.

    python make_edge.py OUT SEED N_RECORDS [--hdr-max H] [--seq-max L] [--polya P] [--plain]
"""
import argparse

import numpy as np

U = np.uint64


def mix(x):
    x = (x + U(0x9E3779B97F4A7C15))
    x = (x ^ (x >> U(30))) * U(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> U(27))) * U(0x94D049BB133111EB)
    return x ^ (x >> U(31))


def rnd(seed, rec, field, idx):
    """uint64 array of randoms for index array idx."""
    with np.errstate(over="ignore"):
        base = mix(U(seed) ^ (U(rec) * U(0xD1342543DE82EF95)) ^ (U(field) << U(56)))
        return mix(base + np.asarray(idx, dtype=np.uint64))


def make(out, seed, n, hdr_max=300, seq_max=800, polya=0.002, plain=False):
    hdr_alpha = np.frombuffer(b"ACGTacgtxyz >", dtype=np.uint8)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    parts = []
    one = np.arange(1, dtype=np.uint64)
    for i in range(n):
        with np.errstate(over="ignore"):
            r0 = rnd(seed, i, 0, np.arange(8, dtype=np.uint64))
        if not plain:
            hl = int(r0[0] % U(hdr_max + 1))
            h = hdr_alpha[(rnd(seed, i, 1, np.arange(hl, dtype=np.uint64)) % U(len(hdr_alpha))).astype(np.int64)]
            parts.append(b">" + h.tobytes() + b"\n")
        L = int(r0[1] % U(seq_max + 1))
        idx = np.arange(L, dtype=np.uint64)
        c = acgt[(rnd(seed, i, 2, idx) % U(4)).astype(np.int64)].copy()
        q = rnd(seed, i, 3, idx).astype(np.float64) / 2.0 ** 64
        low = (q >= 0.003) & (q < 0.006)
        c[low] = c[low] + 32
        if not plain:
            c[(q >= 0.0065) & (q < 0.007)] = ord(">")
        c[(q >= 0.006) & (q < 0.0065)] = ord("\r")
        c[q < 0.003] = ord("N")
        s = c.tobytes()
        w = [0, 60, 61, 7, 1000][int(r0[2] % U(5))] if not plain else 0
        if w:
            s = b"\n".join(s[j:j + w] for j in range(0, len(s), w))
        parts.append(s + b"\n")
        if r0[3] / 2.0 ** 64 < 0.05:
            parts.append(b"\n")
        if r0[4] / 2.0 ** 64 < polya:
            parts.append(b"A" * 70000 + b"\n")
    data = b"".join(parts)
    if plain:
        data = data.lstrip(b"\n\rNn")
        if not data or data[:1] not in b"ACGTacgt":
            data = b"A" + data
    with open(out, "wb") as f:
        f.write(data)
    return len(data)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("seed", type=int)
    ap.add_argument("n", type=int)
    ap.add_argument("--hdr-max", type=int, default=300)
    ap.add_argument("--seq-max", type=int, default=800)
    ap.add_argument("--polya", type=float, default=0.002)
    ap.add_argument("--plain", action="store_true")
    a = ap.parse_args()
    print(make(a.out, a.seed, a.n, a.hdr_max, a.seq_max, a.polya, a.plain))
