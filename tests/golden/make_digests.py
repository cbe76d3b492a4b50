"""Order-independent output digests for the full-size fixtures (tests/golden/fullsize.json).

The digest of a job's output (oracle/kc_digest.c, the engine's kc_output_digest): lines, the sum
of T(c), and the sum mod 2^64 and XOR of XXH64 over every output line.  It does not depend on line
order and adds up over disjoint line sets, so the owners of a sharded job can combine theirs
(bench.py all-reduces them) and a whole job too large to sort is still checked line for line.

Run in the build container:
    python tests/golden/make_digests.py [--ref] [CASE ...]

Per case, `digest` = `kc_digest count` on the case's input: the pinned CPU restatement
(oracle/kc_oracle_core.h: the reference chunking, tokenizer, canonical keys, count transform),
partitioned by key hash so that C4 / C5 (10 G windows, ~1.2-1.6 G distinct k-mers) fit this
container.  For the cases whose reference output was digested by make_fullsize.py the restatement
is pinned by that case's `sorted_sha256` at the same time (tests/test_oracle.py runs kc_digest
against kc_oracle on every golden case); with --ref the reference itself runs again
(oracle/_ref/kaarme -o FIFO | kc_digest lines) and `ref_digest` must equal `digest`.

New cases: the whole jobs of the strong presets, which no reference run covers
in this container's time (C4S alone, 1/8 of C4, took the reference 5385 s of table build at -t 8):
  C4: 100 M x 150 bp, k = 51, -m 2 -s 2600000000 -a 1 (the kc_gen seed-42 generator, genome 500 Mbp)
  C5: 1 M x 10 kbp, k = 127, -m 2 -s 3600000000 -a 1
Their `digest` is the restatement's ("source" says so); `sorted_sha256` is null.
"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_fullsize as mf  # noqa: E402

REPO = mf.REPO
DIGEST = os.path.join(REPO, "oracle", "_ref", "kc_digest")

C4_INPUT = {"reads": 100_000_000, "read_len": 150, "genome": 500_000_000, "seed": 42, "err": 0.001}
C5_INPUT = {"reads": 1_000_000, "read_len": 10_000, "genome": 500_000_000, "seed": 42, "err": 0.001}
WHOLE = {
    "C4": {"input": C4_INPUT, "k": 51, "args": ["-m", "2", "-s", "2600000000", "-a", "1"], "parts": 24},
    "C5": {"input": C5_INPUT, "k": 127, "args": ["-m", "2", "-s", "3600000000", "-a", "1"], "parts": 40},
}
INPUTS = dict(mf.INPUT_NAMES, C4=C4_INPUT, C5=C5_INPUT)


def opt(args, name, default):
    return args[args.index(name) + 1] if name in args else default


def restatement_digest(fa, k, args, parts, threads):
    cmd = [DIGEST, "count", fa, str(k), "-m", opt(args, "-m", "2"), "-a", opt(args, "-a", "2"), "-p", str(parts),
           "-j", str(threads)]
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, check=True)
    d = json.loads(p.stdout)
    d["seconds"] = round(time.time() - t0, 1)
    d["source"] = ("oracle/_ref/kc_digest count: the CPU restatement (oracle/kc_oracle_core.h) partitioned by key "
                   f"hash ({parts} parts, {threads} threads)")
    return d


def reference_digest(fa, k, args, threads, tmp):
    """The reference CLI writing into a FIFO that kc_digest lines reads."""
    fifo = os.path.join(tmp, "dig.fifo")
    if os.path.exists(fifo):
        os.remove(fifo)
    os.mkfifo(fifo)
    rd = subprocess.Popen([DIGEST, "lines", fifo], stdout=subprocess.PIPE, text=True)
    t0 = time.time()
    p = subprocess.run([mf.REF, fa, str(k), "-t", str(threads)] + args + ["-o", fifo], capture_output=True, text=True)
    if p.returncode != 0:
        try:
            with open(fifo, "wb"):
                pass
        except OSError:
            pass
    out, _ = rd.communicate()
    os.remove(fifo)
    assert p.returncode == 0, p.stdout[-1000:] + p.stderr[-1000:]
    d = json.loads(out)
    d["seconds"] = round(time.time() - t0, 1)
    d["source"] = f"oracle/_ref/kaarme -t {threads} -o FIFO | oracle/_ref/kc_digest lines"
    return d


def main():
    argv = sys.argv[1:]
    ref = "--ref" in argv
    names = [a for a in argv if not a.startswith("--")]
    tmp = os.environ.get("KC_FULLSIZE_TMP", "/tmp/kc_fullsize")
    os.makedirs(tmp, exist_ok=True)
    threads = int(os.environ.get("KC_DIGEST_THREADS", "8"))
    with open(mf.OUT_JSON) as f:
        doc = json.load(f)
    names = names or list(doc["cases"]) + list(WHOLE)
    for name in names:
        if name in WHOLE:
            c = WHOLE[name]
            iname = name
        else:
            c = dict(doc["cases"][name])
            iname = c["input"]
        fa = os.path.join(tmp, iname + ".fasta")
        if not os.path.exists(fa):
            subprocess.run([mf.GEN, fa] + mf.gen_args(INPUTS[iname]), check=True)
        if iname not in doc["inputs"]:
            doc["inputs"][iname] = dict(INPUTS[iname], sha256=mf.sha256_file(fa), bytes=os.path.getsize(fa))
        parts = c.get("parts") or (8 if c["k"] <= 63 else 16)
        d = restatement_digest(fa, c["k"], c["args"], parts, threads)
        print(name, "restatement", d, flush=True)
        if name in WHOLE:
            case = {"input": iname, "k": c["k"], "args": c["args"], "whole_job": True, "sorted_sha256": None,
                    "lines": d["lines"], "count_sum": d["count_sum"], "distinct": d["distinct"]}
            doc["cases"][name] = case
        case = doc["cases"][name]
        assert (d["lines"], d["count_sum"]) == (case["lines"], case["count_sum"]), (name, d, case)
        case["digest"] = {key: d[key] for key in ("lines", "count_sum", "hash_sum", "hash_xor", "source", "seconds")}
        if ref and name not in WHOLE:
            r = reference_digest(fa, c["k"], c["args"], int(os.environ.get("KC_REF_THREADS", "10")), tmp)
            print(name, "reference", r, flush=True)
            case["ref_digest"] = r
            assert all(r[key] == d[key] for key in ("lines", "count_sum", "hash_sum", "hash_xor")), (name, r, d)
        with open(mf.OUT_JSON, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
