"""Regenerates the golden parity fixtures under tests/golden/ FROM THE REFERENCE.

Run in the build container (needs /root/reference):
    make -C oracle ref oracle && make -C canonical-k-mer-hash-table_amd
    python tests/golden/make_golden.py [--append]
(--append: keep the cases already in cases.json and run the reference only for new ones)

What it writes (all data, no reference source):
  * small inputs (*.fasta / *.txt, committed) made by our generators
    (canonical-k-mer-hash-table_amd/bin/kc_gen, tests/golden/make_edge.py);
  * recipes for the >10 MiB multi-chunk inputs (regenerated at test time, their
    SHA-256 pinned);
  * cases.json: for every (input, k, options) the SHA-256 and line count of the
    byte-sorted output of the reference CLI oracle/_ref/kaarme run with -t 3
    (one worker thread: deterministic even with the Bloom filter and -a 1),
    plus the reference's "Main array slots used" (distinct k-mers) for -m 1/2;
  * xxh64.json: XXH64(&v, 8, seed) golden vectors from the vendored xxHash v0.8.2
    (oracle/_ref/libxxh.so) for the Bloom seeds of double_bloomfilter.hpp:434-444.
"""
import ctypes
import hashlib
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "kaarme")
XXH = os.path.join(REPO, "oracle", "_ref", "libxxh.so")
GEN = os.path.join(REPO, "canonical-k-mer-hash-table_amd", "bin", "kc_gen")
sys.path.insert(0, HERE)
import make_edge  # noqa: E402

# name -> recipe.  "commit": file is stored in tests/golden.
INPUTS = {
    "reads_w60.fasta": {"gen": ["1000", "150", "30000", "-s", "42", "-e", "0.002", "-w", "60", "-n", "0.002"],
                        "commit": True},
    "reads.txt": {"gen": ["1000", "150", "30000", "-s", "7", "-n", "0.002", "--plain"], "commit": True},
    "long.fasta": {"gen": ["40", "5000", "20000", "-s", "5", "-e", "0.01"], "commit": True},
    "edge.fasta": {"edge": [11, 300, 300, 800, 0.02, False], "commit": True},
    # long reads with few errors: k-mers of k >= 256 seen twice or more
    "long_lo.fasta": {"gen": ["60", "6000", "20000", "-s", "6", "-e", "0.0005"], "commit": False},
    "edge.txt": {"edge": [3, 200, 0, 800, 0.02, True], "commit": True},
    "big_edge.fasta": {"edge": [7, 16000, 2000, 400, 0.002, False], "commit": False},
    "big_reads.fasta": {"gen": ["150000", "150", "2000000", "-s", "9", "-e", "0.002", "-w", "60"],
                        "commit": False},
    # skew: 5 % poly-A/T reads, 3 % (CA)n reads, a 300-bp repeat in 300 copies of the genome
    "skew.fasta": {"gen": ["20000", "150", "300000", "-s", "11", "-e", "0.001", "--homo", "0.05", "--dinuc", "0.03",
                           "--repeat", "300", "300"], "commit": False},
    "big_skew.fasta": {"gen": ["100000", "150", "1000000", "-s", "12", "-e", "0.001", "--homo", "0.05",
                               "--dinuc", "0.03", "--repeat", "300", "1000"], "commit": False},
}

CASES = [
    ("reads_w60.fasta", 31, ["-m", "2", "-a", "1", "-s", "1000000"]),
    ("reads_w60.fasta", 51, ["-m", "0", "-a", "2", "-s", "1000000"]),
    ("reads_w60.fasta", 33, ["-m", "1", "-a", "1", "-s", "1000000"]),
    # -m 1 -b: the Bloom pass runs, then the filter is ignored (main.cpp:482-489)
    ("reads_w60.fasta", 33, ["-m", "1", "-b", "-u", "100000", "-a", "1"]),
    ("reads_w60.fasta", 33, ["-m", "1", "-b", "-u", "100000", "-a", "2"]),
    ("reads_w60.fasta", 17, ["-b", "-u", "100000", "-a", "1"]),
    ("reads_w60.fasta", 51, ["-b", "-u", "100000", "-f", "0.05", "-a", "2"]),
    ("reads_w60.fasta", 1, ["-a", "1", "-s", "100"]),
    ("reads_w60.fasta", 5, ["-m", "0", "-a", "1", "-s", "10000"]),
    ("reads_w60.fasta", 63, ["-a", "1", "-s", "1000000"]),
    ("reads_w60.fasta", 95, ["-a", "1", "-s", "1000000"]),
    ("reads_w60.fasta", 127, ["-a", "1", "-s", "1000000"]),
    ("reads.txt", 31, ["-a", "1", "-s", "1000000"]),
    ("reads.txt", 21, ["-m", "0", "-b", "-u", "50000", "-a", "1"]),
    ("long.fasta", 127, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 100, ["-a", "2", "-s", "1000000"]),
    ("edge.fasta", 25, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("edge.fasta", 31, ["-a", "1", "-s", "1000000"]),
    ("edge.fasta", 31, ["-m", "1", "-a", "3", "-s", "1000000"]),
    ("edge.fasta", 40, ["-a", "1", "-s", "1000000"]),
    ("edge.txt", 31, ["-a", "1", "-s", "1000000"]),
    ("edge.txt", 15, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("big_edge.fasta", 31, ["-a", "1", "-s", "8000000"]),
    ("big_edge.fasta", 51, ["-m", "0", "-a", "1", "-s", "8000000"]),
    ("big_reads.fasta", 31, ["-a", "2", "-s", "8000000"]),
    ("big_reads.fasta", 55, ["-b", "-u", "3000000", "-a", "2"]),
    # k >= 128: keys of five to eight 64-bit words (kmer_factory.cpp:33 sizes the blocks by k)
    ("reads_w60.fasta", 129, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 129, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("long.fasta", 131, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 131, ["-b", "-u", "300000", "-a", "2"]),
    ("long.fasta", 200, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 200, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("long.fasta", 200, ["-b", "-u", "300000", "-a", "2"]),
    ("long.fasta", 255, ["-a", "2", "-s", "1000000"]),
    ("long.fasta", 255, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("long.fasta", 255, ["-b", "-u", "300000", "-f", "0.05", "-a", "2"]),
    ("edge.fasta", 140, ["-a", "1", "-s", "1000000"]),
    # k = 256..479: keys of nine to fifteen words (one slot per 128-byte bucket)
    ("long.fasta", 257, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 300, ["-a", "1", "-s", "1000000"]),
    ("long.fasta", 300, ["-m", "0", "-a", "1", "-s", "1000000"]),
    ("long.fasta", 421, ["-m", "1", "-a", "1", "-s", "1000000"]),
    ("long_lo.fasta", 289, ["-a", "2", "-s", "1000000"]),
    ("long_lo.fasta", 383, ["-b", "-u", "300000", "-a", "2"]),
    ("long_lo.fasta", 479, ["-a", "2", "-s", "1000000"]),
    ("long_lo.fasta", 479, ["-m", "0", "-a", "3", "-s", "1000000"]),
    ("long_lo.fasta", 479, ["-m", "0", "-b", "-u", "300000", "-a", "1"]),
    ("big_edge.fasta", 161, ["-a", "1", "-s", "8000000"]),
    # skew (hot keys: homopolymers, dinucleotide repeats, a high-copy repeat)
    ("skew.fasta", 31, ["-a", "1", "-s", "4000000"]),
    ("skew.fasta", 25, ["-m", "0", "-a", "1", "-s", "4000000"]),
    ("skew.fasta", 51, ["-a", "2", "-s", "4000000"]),
    ("skew.fasta", 31, ["-b", "-u", "3000000", "-a", "2"]),
    ("big_skew.fasta", 31, ["-a", "2", "-s", "16000000"]),
    ("big_skew.fasta", 63, ["-b", "-u", "12000000", "-a", "2"]),
]

XXH_SEEDS = [2411, 3253, 1061, 1129, 2269, 7309, 3491, 8237, 6359, 8779, 0]
XXH_VALUES = [0, 1, 2, 3, 5, 1234567, (1 << 54) - 1, 1 << 53, 0xDEADBEEFCAFEBABE, (1 << 64) - 1,
              9007199254740881, 17592186044416 + 31]


def build_input(name, dest_dir):
    path = os.path.join(dest_dir, name)
    r = INPUTS[name]
    if "gen" in r:
        subprocess.run([GEN, path] + r["gen"], check=True)
    else:
        seed, n, hdr, seq, polya, plain = r["edge"]
        make_edge.make(path, seed, n, hdr, seq, polya, plain)
    return path


def sha256_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def sorted_digest(path):
    with open(path, "rb") as f:
        lines = f.read().splitlines(keepends=True)
    lines.sort()
    return hashlib.sha256(b"".join(lines)).hexdigest(), len(lines)


def main():
    tmp = os.environ.get("TMPDIR", "/tmp")
    work = os.path.join(tmp, "kc_golden")
    os.makedirs(work, exist_ok=True)
    inputs = {}
    for name, r in INPUTS.items():
        path = build_input(name, HERE if r["commit"] else work)
        inputs[name] = {"sha256": sha256_file(path), "bytes": os.path.getsize(path), "commit": r["commit"]}
        inputs[name].update({k: v for k, v in r.items() if k in ("gen", "edge")})
    old = {}
    if "--append" in sys.argv[1:]:
        with open(os.path.join(HERE, "cases.json")) as f:
            prev = json.load(f)
        for c in prev["cases"]:
            if prev["inputs"][c["input"]]["sha256"] == inputs[c["input"]]["sha256"]:
                old[(c["input"], c["k"], tuple(c["args"]))] = c
    cases = []
    for name, k, args in CASES:
        if (name, k, tuple(args)) in old:
            cases.append(old[(name, k, tuple(args))])
            continue
        src = os.path.join(HERE if INPUTS[name]["commit"] else work, name)
        out = os.path.join(work, "ref.out")
        if os.path.exists(out):
            os.remove(out)
        p = subprocess.run([REF, src, str(k), "-t", "3", "-o", out] + args, capture_output=True, text=True)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        dig, n = sorted_digest(out) if os.path.exists(out) else (hashlib.sha256(b"").hexdigest(), 0)
        m = re.search(r"Main array slots used (\d+)", p.stdout)
        cases.append({"input": name, "k": k, "args": args, "sorted_sha256": dig, "lines": n,
                      "distinct": int(m.group(1)) if m else None})
        print(name, k, args, n, flush=True)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/make_golden.py from oracle/_ref/kaarme (-t 3)",
                   "inputs": inputs, "cases": cases}, f, indent=1)
    lib = ctypes.CDLL(XXH)
    lib.XXH64.restype = ctypes.c_uint64
    lib.XXH64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    vec = []
    for s in XXH_SEEDS:
        for v in XXH_VALUES:
            x = ctypes.c_uint64(v)
            vec.append({"seed": s, "value": v, "xxh64": lib.XXH64(ctypes.byref(x), 8, s)})
    with open(os.path.join(HERE, "xxh64.json"), "w") as f:
        json.dump({"generated_by": "tests/golden/make_golden.py from vendored xxHash v0.8.2", "vectors": vec},
                  f, indent=0)


if __name__ == "__main__":
    main()
