"""Full-size reference parity fixtures: the bench's own C2 / C3 / C2S inputs through the
reference CLI (oracle/_ref/kaarme), one digest per case -> tests/golden/fullsize.json.

Run in the build container (needs oracle/_ref/kaarme, built from /root/reference by
`make -C oracle ref`, and canonical-k-mer-hash-table_amd/bin/kc_gen):
    python tests/golden/make_fullsize.py [CASE ...]

Inputs: kc_gen seed 42, 10 M x 150 bp reads, genome 50 Mbp, 0.1 % substitutions --
byte-identical to the image bench.py generates in HBM (kc_synth_device, the device twin of
kc_gen; tests/test_gpu_fullsize.py checks the image's SHA-256 against `input_sha256`).

Per case: SHA-256 of the byte-sorted output (BASELINE.md's parity rule: the reference's line
order is nondeterministic), its line count, the sum of its counts, and the
reference's own timer lines (Time used to build hash table / bloom filter k-mers,
parallel_parser.hpp:1544-1550,2966-2972) with the thread count used.  The outputs themselves
(3 GB per case) are not kept.  Without the Bloom filter the reference output does not depend
on the thread count; with it, k-mers seen at least twice are exact and the cases use -a 2
(SURVEY 8a A18).
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "kaarme")
GEN = os.path.join(REPO, "canonical-k-mer-hash-table_amd", "bin", "kc_gen")
OUT_JSON = os.path.join(HERE, "fullsize.json")

C2_INPUT = {"reads": 10_000_000, "read_len": 150, "genome": 50_000_000, "seed": 42, "err": 0.001}
C2S_INPUT = dict(C2_INPUT, skew=[0.05, 0.03, 300, 10_000])
# rank 0's share of the strong presets at 8 GPUs (bench.py --config C4|C5 --share 8): reads
# [first, first + count) of the whole job's generator
C4S_INPUT = {"reads": 100_000_000, "read_len": 150, "genome": 500_000_000, "seed": 42, "err": 0.001,
             "first": 0, "count": 12_500_000}
C5S_INPUT = {"reads": 1_000_000, "read_len": 10_000, "genome": 500_000_000, "seed": 42, "err": 0.001,
             "first": 0, "count": 125_000}

CASES = {
    "C2": {"input": C2_INPUT, "k": 31, "args": ["-m", "2", "-s", "200000000", "-a", "1"]},
    "C3": {"input": C2_INPUT, "k": 51, "args": ["-m", "2", "-b", "-u", "400000000", "-a", "2"]},
    "C2S": {"input": C2S_INPUT, "k": 31, "args": ["-m", "2", "-s", "200000000", "-a", "1"]},
    # the shares' tables are sized from a distinct-count estimate on the GPU; -s only has to hold
    # the share's distinct k-mers for the reference (515.7 M / 590.1 M), the counts do not depend on it
    "C4S": {"input": C4S_INPUT, "k": 51, "share": 8, "args": ["-m", "2", "-s", "700000000", "-a", "1"]},
    "C5S": {"input": C5S_INPUT, "k": 127, "share": 8, "args": ["-m", "2", "-s", "760000000", "-a", "1"]},
}

INPUT_NAMES = {"C2": C2_INPUT, "C2S": C2S_INPUT, "C4S": C4S_INPUT, "C5S": C5S_INPUT}


def gen_args(inp):
    a = [str(inp["reads"]), str(inp["read_len"]), str(inp["genome"]), "-s", str(inp["seed"]), "-e", str(inp["err"])]
    if "skew" in inp:
        h, d, rl, rc = inp["skew"]
        a += ["--homo", str(h), "--dinuc", str(d), "--repeat", str(rl), str(rc)]
    if "first" in inp:
        a += ["--first", str(inp["first"]), "--count", str(inp["count"])]
    return a


def sha256_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def partsort_tool(tmp):
    """tests/golden/partsort.c built into the scratch directory (fixture tooling only)."""
    exe = os.path.join(tmp, "partsort")
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(HERE, "partsort.c")], check=True)
    return exe


def run_sorted_stats(cmd, tmp):
    """Runs the reference with -o a FIFO, streams its output into 64 buckets by the first three
    characters (partsort), then sorts the buckets one by one: SHA-256 of the byte-sorted output,
    its lines and the sum of its counts without ever holding the whole file (C5S: ~78 GB).
    Returns (completed reference process, digest, lines, count sum) or the process alone on failure."""
    env = dict(os.environ, LC_ALL="C")
    fifo = os.path.join(tmp, "ref.fifo")
    parts = os.path.join(tmp, "parts")
    if os.path.exists(fifo):
        os.remove(fifo)
    os.mkfifo(fifo)
    os.makedirs(parts, exist_ok=True)
    for name in os.listdir(parts):
        os.remove(os.path.join(parts, name))
    ps = subprocess.Popen([partsort_tool(tmp), fifo, parts], stdout=subprocess.PIPE, text=True)
    p = subprocess.run(cmd + ["-o", fifo], capture_output=True, text=True)
    if p.returncode != 0:
        # the reader may still wait on a FIFO the reference never opened
        try:
            with open(fifo, "wb"):
                pass
        except OSError:
            pass
    out, _ = ps.communicate()
    os.remove(fifo)
    if p.returncode != 0:
        return p, None, None, None
    assert ps.returncode == 0, "partsort failed"
    lines, total = (int(x) for x in out.split())
    h = hashlib.sha256()
    seen = 0
    for name in sorted(os.listdir(parts)):  # "AAA" < ... < "TTT" < "zzz": byte order of the buckets
        path = os.path.join(parts, name)
        if os.path.getsize(path):
            q = subprocess.Popen(["sort", "-S", "8G", "--parallel=8", "-T", tmp, path], stdout=subprocess.PIPE,
                                 env=env)
            for b in iter(lambda: q.stdout.read(1 << 24), b""):
                h.update(b)
                seen += b.count(b"\n")
            assert q.wait() == 0
        os.remove(path)
    assert seen == lines
    return p, h.hexdigest(), lines, total


def main():
    tmp = os.environ.get("KC_FULLSIZE_TMP", "/tmp/kc_fullsize")
    os.makedirs(tmp, exist_ok=True)
    threads = int(os.environ.get("KC_REF_THREADS", "10"))
    names = sys.argv[1:] or list(CASES)
    doc = {"generated_by": "tests/golden/make_fullsize.py from oracle/_ref/kaarme", "inputs": {}, "cases": {}}
    if os.path.exists(OUT_JSON):
        with open(OUT_JSON) as f:
            doc = json.load(f)
    for name in names:
        c = CASES[name]
        iname = next(n for n, v in INPUT_NAMES.items() if v is c["input"])
        fa = os.path.join(tmp, iname + ".fasta")
        if not os.path.exists(fa):
            subprocess.run([GEN, fa] + gen_args(c["input"]), check=True)
        doc["inputs"][iname] = dict(c["input"], sha256=sha256_file(fa), bytes=os.path.getsize(fa))
        # the reference's worker threads occasionally crash it (a reference-side race, also seen
        # on the GPU box): up to three attempts, the failed exit codes recorded
        failed = []
        for _ in range(3):
            t0 = time.time()
            p, dig, n, total = run_sorted_stats([REF, fa, str(c["k"]), "-t", str(threads)] + c["args"], tmp)
            wall = time.time() - t0
            if p.returncode == 0:
                break
            failed.append(p.returncode)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        timers = {m.group(1): int(m.group(2)) for m in re.finditer(r"Time used to ([a-z -]+?): (\d+) microseconds",
                                                                    p.stdout)}
        m = re.search(r"Main array slots used (\d+)", p.stdout)
        doc["cases"][name] = {"input": iname, "k": c["k"], "args": c["args"], "sorted_sha256": dig, "lines": n,
                              **({"share": c["share"]} if "share" in c else {}),
                              "count_sum": total, "distinct": int(m.group(1)) if m else None,
                              "ref_threads": threads, "ref_timers_us": timers, "ref_wall_s": round(wall, 1),
                              "ref_failed_exit_codes": failed}
        print(name, doc["cases"][name], flush=True)
        with open(OUT_JSON, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
