#!/usr/bin/env python3
"""bench.py -- canonical k-mer counting throughput on MI355X.

Metric (BASELINE.json): canonical k-mers/s inserted (+ achieved HBM GB/s).
Workload (--config, BASELINE.md CPU-baseline plan; SURVEY.md 8d generator: uniform
genome, 50 % reverse complement, 0.1 % substitutions, single-line FASTA):
  C2 (default, BASELINE.json configs[1]): 10M x 150 bp reads per GPU, k=31, -m 2 -s 200000000
  C3: 10M x 150 bp per GPU, k=51, -m 2 -b -u 400000000 (Bloom pass + gated counting pass)
  C4: 100M x 150 bp over the GPUs, k=51, -m 2 -s 2600000000 (split over the shards)
  C5: 1M x 10 kbp over the GPUs, k=127 (4-word keys), -m 2 -s 3600000000 (split)

One step = one full counting job over the resident input: table re-initialised
(kc_reset, the table constructor), [Bloom pass,] reference chunking of the FASTA image,
gather into the chunk stage, tokenize, canonicalise + insert every window.  The FASTA
image is generated directly in HBM before timing (inputs resident, as the contract asks).

N > 1 (torch.distributed over RCCL; default --config C4, strong scaling, with a C2 weak-scaling
record): every rank counts its own slice into a local table, whose {key, count} records go to
their hash-prefix owner in one all-to-all per job (kaarme_amd/sharded.py) and are merged there;
the owners' order-independent output digests combine into the whole job's parity record.

Extra JSON keys: roofline (the counting pass vs 8 TB/s HBM; traffic from the committed
PMC summary profiles/pmc_traffic.json when it matches the workload), cpu_baseline (the
reference CLI oracle/_ref/kaarme on a bounded sample of the same workload, rank 0, N=1).
"""
import argparse
import ctypes
import json
import math
import os
import re
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "canonical-k-mer-hash-table_amd")
sys.path.insert(0, PKG)

METRIC = "k-mers/s inserted (canonical) + achieved HBM GB/s, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


PRESETS = {
    # BASELINE.md CPU-baseline plan (SURVEY.md 8d generator).  "weak": every rank counts
    # its own `reads`; "strong": the `reads` and the -s capacity are split over the ranks.
    "C2": dict(reads=10_000_000, read_len=150, genome=50_000_000, k=31, slots=200_000_000, unique=0, scale="weak"),
    "C3": dict(reads=10_000_000, read_len=150, genome=50_000_000, k=51, slots=0, unique=400_000_000, scale="weak"),
    "C4": dict(reads=100_000_000, read_len=150, genome=500_000_000, k=51, slots=2_600_000_000, unique=0,
               scale="strong"),
    "C5": dict(reads=1_000_000, read_len=10_000, genome=500_000_000, k=127, slots=3_600_000_000, unique=0,
               scale="strong"),
    # C2 with hot keys: 5 % poly-A/T reads, 3 % (CA)n reads and a 300-bp
    # repeat in 10^4 copies of the genome (kc_synth.h skew options)
    "C2S": dict(reads=10_000_000, read_len=150, genome=50_000_000, k=31, slots=200_000_000, unique=0, scale="weak",
                skew=(0.05, 0.03, 300, 10_000)),
}


def table_args(slots, unique):
    return ["-b", "-u", str(unique)] if unique else ["-s", str(slots)]


def cpu_baseline(args):
    """Time the reference CLI (or, if it was not built, the C oracle) on a bounded sample."""
    ref = os.path.join(REPO, "oracle", "_ref", "kaarme")
    orc = os.path.join(REPO, "oracle", "_ref", "kc_oracle")
    gen = os.path.join(PKG, "bin", "kc_gen")
    if not os.path.exists(gen):
        return None
    kind = "reference" if os.path.exists(ref) else ("port" if os.path.exists(orc) else None)
    if kind is None:
        return None
    # about 150 M bases (10-30 s of reference work on a 16-core share), from a genome scaled with
    # the sample so that its coverage is the workload's (a 1 M-read sample of the
    # 50 Mbp genome is a 3x-coverage input, a different workload for the reference's chains)
    n = max(1, args.cpu_sample_bases // args.read_len)
    if kind == "port":
        n = max(1, n // 20)
    n = min(n, args.reads)
    genome = max(10 * args.read_len, round(args.genome * n / args.reads))
    # The box gives one GPU's job a 16-core share of a larger host (OMP_NUM_THREADS is set to
    # it; the affinity mask still lists every CPU).  -t = share + 2: share hashing workers plus
    # the IO thread (main.cpp:383).
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(3, min(args.cpu_threads or share + 2, 64))
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        fa = os.path.join(td, "sample.fasta")
        sk = PRESETS[args.config].get("skew")
        skew_args = (["--homo", str(sk[0]), "--dinuc", str(sk[1]), "--repeat", str(sk[2]), str(sk[3])] if sk else [])
        subprocess.run([gen, fa, str(n), str(args.read_len), str(genome), "-s", str(args.seed),
                        "-e", str(args.err)] + skew_args, check=True)
        with open(fa, "rb") as f:  # pre-warm the page cache
            while f.read(1 << 24):
                pass
        windows = n * (args.read_len - args.k + 1)
        # distinct <= windows: never ask the reference for more slots than the sample can fill
        slots = min(args.slots, int(windows * 1.3) + 1000) if args.slots else 0
        # -b -u: the estimate scaled to the sample (the filter is sized for the reads counted)
        unique = max(1000, args.unique * n // max(1, args.reads)) if args.unique else 0
        targs = table_args(slots, unique)
        # -a: the workload's output threshold (the reference fixture's: C2 1, C3 2), so both the
        # reference and the drop-in CLI write their output and time it
        amin = str(fixture_case(args)["min_abundance"]) if fixture_case(args) else "2"
        out_txt = os.path.join(td, "ref_out.txt")
        write_s = None
        if kind == "reference":
            cmd = [ref, fa, str(args.k), "-m", "2", "-t", str(threads), "-a", amin, "-o", out_txt] + targs
            # args.cpu_runs runs (3), the median reported with min / max (one run on
            # a 16-core share of a busy host moved -22 % / +47 % between rounds).  The reference's
            # worker threads occasionally crash it (seen once in ~10 runs on the box: killed before
            # its timers): a failed run is retried once, its exit code kept in failed_exit_codes
            failures, runs = [], []
            while len(runs) < args.cpu_runs and len(failures) <= args.cpu_runs:
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=1800)
                m = re.search(r"Time used to build hash table: (\d+) microseconds", p.stdout)
                mb = re.search(r"Time used to bloom filter k-mers: (\d+) microseconds", p.stdout)
                if p.returncode == 0 and m:
                    mw = re.search(r"Time used to write k-mers in a file: (\d+) microseconds", p.stdout)
                    runs.append(((int(m.group(1)) + (int(mb.group(1)) if mb else 0)) / 1e6,
                                 int(mw.group(1)) / 1e6 if mw else None))
                    continue
                failures.append(p.returncode)
                log(f"cpu baseline run failed (exit {p.returncode}):", p.stdout[-300:], p.stderr[-300:])
            if not runs:
                return None
            ordered = sorted(runs)
            secs, write_s = ordered[len(ordered) // 2]
            run_secs = [round(r[0], 3) for r in runs]
            out_bytes = os.path.getsize(out_txt) if os.path.exists(out_txt) else None
            cores = threads - 2  # t-2 hashing workers (+ 1 mostly idle IO thread, main.cpp:383)
            e2e = cli_e2e(fa, [str(args.k), "-m", "2", "-t", str(threads), "-a", amin] + targs, windows)
        else:
            t0 = time.perf_counter()
            subprocess.run([orc, "count", fa, str(args.k), "-a", "0"] + targs, check=True, capture_output=True)
            secs = time.perf_counter() - t0
            cores = 1
    if kind != "reference":
        failures, run_secs, write_s = [], [round(secs, 3)], None
        e2e = None
        out_bytes = None
    rec = {"value": windows / secs, "unit": "k-mers/s", "cores": cores, "kind": kind, "e2e": e2e,
            "runs_s": run_secs, "statistic": f"median of {len(run_secs)} run(s)",
            "min": windows / max(run_secs), "max": windows / min(run_secs),
            "write_s": write_s, "output_bytes": out_bytes,
            "attempts": len(run_secs) + len(failures), "failed_exit_codes": failures, "cpu_model": cpu_model(),
            "nproc": os.cpu_count(), "core_share": share,
            "coverage": round(n * args.read_len / genome, 2),
            "workload_coverage": round(args.reads * args.read_len / args.genome, 2),
            "sample": f"{n} reads of the same generator on a {genome}-base genome (the workload's coverage; "
                      f"{windows} windows, k={args.k}, -m 2 {' '.join(targs)} -t {threads} -a {amin if kind == 'reference' else 0}, "
                      f"{secs:.2f} s counting time{' incl. the Bloom pass' if args.unique else ''} (median); write_s = "
                      f"its 'Time used to write k-mers in a file')"}
    # the reference on the whole workload on the same host (its own timers; the full-size tables
    # miss the caches the samples' tables fit): profiles/r03_ref_fullsize_box.txt
    full = FULLSIZE_REF.get(args.config)
    if full:
        rec["fullsize"] = dict(full, source="profiles/r03_ref_fullsize_box.txt (oracle/_ref/kaarme -t 18 on the "
                                            "bench's full-size input, AMD EPYC 9575F 16-core share)")
    return rec


# the reference CLI on the full-size C2 / C3 inputs on the GPU box's 16-core share (its own timers)
FULLSIZE_REF = {
    "C2": {"value": 1.2e9 / 176.187355, "unit": "k-mers/s", "build_s": 176.187, "write_s": 59.446},
    "C3": {"value": 1.0e9 / (54.0524 + 323.708936), "unit": "k-mers/s", "bloom_s": 54.052, "build_s": 323.709,
           "write_s": 31.586},
}


def run_cli(fasta, cli_args, out, extra=()):
    """The drop-in CLI bin/kaarme on a file: (seconds by its own "Time used to build hash table" (+ Bloom)
    lines, write seconds, process wall, stdout) or None when it failed."""
    cli = os.path.join(PKG, "bin", "kaarme")
    if not os.path.exists(cli):
        return None
    t0 = time.perf_counter()
    p = subprocess.run([cli, fasta] + list(cli_args) + ["-o", out] + list(extra), capture_output=True, text=True,
                       timeout=900)
    wall = time.perf_counter() - t0
    m = re.search(r"Time used to build hash table: (\d+) microseconds", p.stdout)
    mb = re.search(r"Time used to bloom filter k-mers: (\d+) microseconds", p.stdout)
    if p.returncode != 0 or not m:
        log("drop-in CLI run failed:", p.stdout[-300:], p.stderr[-300:])
        return None
    mw = re.search(r"Time used to write k-mers in a file: (\d+) microseconds", p.stdout)
    return ((int(m.group(1)) + (int(mb.group(1)) if mb else 0)) / 1e6, int(mw.group(1)) / 1e6 if mw else None, wall,
            p.stdout)


def cli_e2e(fasta, cli_args, windows):
    """The drop-in CLI (file -> HBM -> counts) on the CPU-baseline sample, timed by the same
    "Time used to build hash table" (+ Bloom) lines as the reference: file read included.
    build_s is that timed build (after the CLI's untimed warm-up pass); process_wall_s the whole
    process (HIP start-up, warm-up, write); no_warmup the same run without the warm-up."""
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        r = run_cli(fasta, cli_args, os.path.join(td, "o.txt"))
        r0 = run_cli(fasta, cli_args, os.path.join(td, "o0.txt"), ["--no-warmup"])
    if r is None:
        return None
    secs, write_s, wall, out = r
    return {"value": windows / secs, "unit": "k-mers/s", "build_s": round(secs, 4), "process_wall_s": round(wall, 3),
            "write_s": write_s,
            "no_warmup": {"build_s": round(r0[0], 4), "value": windows / r0[0],
                          "process_wall_s": round(r0[2], 3)} if r0 else None,
            "path": "drop-in CLI bin/kaarme on the same sample file: page-cached file -> HBM (pread into pinned "
                    "slices; after an untimed one-read warm-up pass) -> passes; build_s = the reference's own timer "
                    "lines (the timed build), process_wall_s = the whole process",
            "input_path": "device image" if "Input path: device image" in out else "host chunks"}


def cli_fullsize(job, args):
    """The drop-in CLI on the whole workload: the job's image written to a file in
    TMPDIR (page-cached), bin/kaarme with the fixture's options, its own timer lines, and the output
    file's order-independent digest (oracle/_ref/kc_digest lines, the checker) against the
    reference's (tests/golden/fullsize.json)."""
    fx = job.fixture
    dig = os.path.join(REPO, "oracle", "_ref", "kc_digest")
    if fx is None or not fx.get("digest"):
        return None
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        fa = os.path.join(td, "input.fasta")
        with open(fa, "wb") as f:
            f.write(memoryview(job.image.cpu().numpy()))
        with open(fa, "rb") as f:  # page-cached, as the sample's
            while f.read(1 << 24):
                pass
        out = os.path.join(td, "out.txt")
        share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        cli_args = [str(args.k)] + fx["args"] + ["-t", str(max(3, min(share + 2, 64)))]
        # a whole strong job's text (C4: ~60 GB) is digested on the device instead of written
        # (--digest-only: kc_output_digest, the digest the fixture holds)
        big = fx.get("whole_job", False)
        r = run_cli(fa, cli_args, out, ["--digest-only"] if big else ())
        if r is None:
            return {"error": "CLI failed"}
        secs, write_s, wall, stdout = r
        rec = {"value": job.windows_expected / secs, "unit": "k-mers/s", "build_s": round(secs, 4),
               "write_s": write_s, "process_wall_s": round(wall, 3), "input_bytes": job.nbytes,
               "args": " ".join(cli_args),
               "input_path": "device image" if "Input path: device image" in stdout else "host chunks",
               "path": "bin/kaarme on the whole workload's FASTA (page-cached file in TMPDIR): the reference's timer "
                       "lines include reading the file (parallel_parser.hpp:1230-1299,1544-1550)"}
        m = re.search(r"Output digest: (\{.*\})", stdout)
        if big and m:
            import kaarme_amd as ka
            got = json.loads(m.group(1))
            rec["parity"] = {"match": ka.same_digest(got, fx["digest"]), "digest": got,
                             "reference_case": f"tests/golden/fullsize.json {fx['name']}",
                             "checker": "the CLI's --digest-only (kc_output_digest on the device) against the "
                                        "fixture's whole-job digest"}
            rec["sized_from_estimate"] = "Device table sized from the distinct estimate" in stdout
            rec["path"] += "; --digest-only: the output digest instead of the file (write_s = its time)"
        elif os.path.exists(dig):
            t0 = time.perf_counter()
            p = subprocess.run([dig, "lines", out], capture_output=True, text=True)
            if p.returncode == 0:
                import kaarme_amd as ka
                got = json.loads(p.stdout)
                rec["parity"] = {"match": ka.same_digest(got, fx["digest"]), "digest": got,
                                 "reference_case": f"tests/golden/fullsize.json {fx['name']}",
                                 "checker": "oracle/_ref/kc_digest lines (XXH64 per output line)",
                                 "digest_s": round(time.perf_counter() - t0, 2)}
    return rec


def host_chunks_record(job, args, batch_mib=256, reps=3):
    """The C-ABI path INTEGRATION.md section 2 tells a maintainer to bind: the
    whole job through kc_count_chunk, one call per reference chunk (~10 MiB) straight from host
    memory (a pageable array holding the file's bytes), the library's pinned double-buffered
    stage (batch_mib MiB batches: the copy of batch i+1 overlaps the counting of batch i) and
    H2D copies included, timed from the first call to kc_finish; the best of `reps` jobs after one
    untimed job (pinned-stage allocation, kernel loading), digested against the fixture."""
    import ctypes as C
    import kaarme_amd as ka
    fx = job.fixture
    host = job.image.cpu().numpy()
    base = host.ctypes.data
    cfg = ka.Config(k=args.k, mode=2, table_slots=job.slots, min_abundance=fx["min_abundance"] if fx else 2,
                    batch_bytes=batch_mib << 20)
    kc = ka.KmerCounter(cfg)
    try:
        times = []
        for rep in range(reps + 1):
            kc.reset()
            t0 = time.perf_counter()
            for off, ln, bh in job.chunks:
                kc._chk(kc.lib.kc_count_chunk(kc._ctx, C.c_void_p(base + off), ln, ka.FMT_FASTA, int(bh)),
                        "kc_count_chunk")
            st = kc.finish()
            if rep:
                times.append(time.perf_counter() - t0)
        secs = min(times)
        rec = {"value": st["windows"] / secs, "unit": "k-mers/s", "seconds": round(secs, 4),
               "runs_s": [round(t, 4) for t in times], "statistic": f"best of {reps} after one untimed job",
               "chunks": len(job.chunks), "batch_mib": batch_mib, "windows": st["windows"],
               "path": "kc_count_chunk per reference chunk from pageable host memory -> the library's pinned "
                       "double-buffered stage -> H2D -> tokenize + count (PCIe-inclusive; the C ABI's host-chunk "
                       "entry point, include/kc_api.h, INTEGRATION.md section 2)"}
        if fx is not None and fx.get("digest"):
            got = kc.output_digest()
            rec["parity"] = {"match": ka.same_digest(got, fx["digest"]), "digest": got,
                             "reference_case": f"tests/golden/fullsize.json {fx['name']}"}
        return rec
    finally:
        kc.close()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def kernel_source_digest():
    """SHA-256 (16 hex) of the engine's kernel and host sources: what a PMC summary was measured with
    (the drop-in CLI's kc_cli.cpp is not part of the library bench.py runs)."""
    import hashlib
    h = hashlib.sha256()
    src = os.path.join(PKG, "csrc")
    for name in sorted(os.listdir(src)):
        if name == "kc_cli.cpp":
            continue
        with open(os.path.join(src, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def load_traffic(workload):
    """(HBM bytes per roofline launch, entry) of this workload from the committed rocprofv3 PMC
    summary profiles/pmc_traffic.json, if any."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get("workloads", {}).get(workload)
        if e:
            return e.get("bytes_per_launch"), e
    except (OSError, ValueError):
        pass
    return None, None


def resolve(args, name):
    """args with the preset's values for every workload option left unset."""
    r = argparse.Namespace(**vars(args))
    r.config = name
    preset = PRESETS[name]
    for key in ("reads", "read_len", "genome", "k", "slots", "unique"):
        if getattr(r, key) is None or name != args.config:
            setattr(r, key, preset[key])
    if r.unique:
        r.slots = 0
    return r


def same_image(a, b):
    pa, pb = PRESETS[a.config], PRESETS[b.config]
    return (a.reads, a.read_len, a.genome, pa["scale"], pa.get("skew")) == (b.reads, b.read_len, b.genome, pb["scale"],
                                                                           pb.get("skew"))


FIXTURES = os.path.join(REPO, "tests", "golden", "fullsize.json")


def fixture_case(args, share=0, first=0, count=None):
    """The tests/golden/fullsize.json case (reference output digest, tests/golden/make_fullsize.py)
    whose input and options are this workload's at one GPU, or None.  share: rank 0's share of
    a strong preset (--share G): reads [first, first + count) of the whole job, whose local
    table is sized from the distinct estimate (the reference case's -s only has to hold them)."""
    try:
        with open(FIXTURES) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    preset = PRESETS[args.config]
    for name, c in doc.get("cases", {}).items():
        inp = doc["inputs"][c["input"]]
        skew = inp.get("skew")
        same_in = ((inp["reads"], inp["read_len"], inp["genome"], inp["seed"], inp["err"]) ==
                   (args.reads, args.read_len, args.genome, args.seed, args.err)
                   and (list(skew) if skew else None) == (list(preset["skew"]) if preset.get("skew") else None))
        if share:
            same_in = same_in and (inp.get("first"), inp.get("count"), c.get("share")) == (first, count, share)
        elif "first" in inp:
            continue
        a = c["args"]
        opt = table_args(args.slots, args.unique)
        # a share's reference case sizes -s for the share alone (its -s is not the run's); its Bloom
        # filter on / off must still be the run's
        same_tbl = a[2:-2] == opt or (share and ("-b" in a) == bool(args.unique))
        if same_in and c["k"] == args.k and a[:2] == ["-m", "2"] and same_tbl:
            return dict(c, name=name, min_abundance=int(a[-1]), input_sha256=inp["sha256"])
    return None


def gpu_free(torch, args, world):
    """Free HBM this rank may plan with: all of it, or its 1/world share when --rehearse-one-gpu
    puts every rank on one GPU (the ranks size their buffers concurrently)."""
    free, _ = torch.cuda.mem_get_info()
    return free // world if getattr(args, "rehearse_one_gpu", False) else free


def setup_job(args, env, image=None):
    """The counting job one bench step runs: the device image (generated in HBM unless given),
    the reference chunk table, the counter with the bench's table and staging geometry, and
    step() = one full counting job.  tests/test_gpu_fullsize.py runs the same object."""
    torch, ka, lib, dist = env["torch"], env["ka"], env["lib"], env["dist"]
    rank, world, local = env["rank"], env["world"], env["local"]
    preset = PRESETS[args.config]
    L, k = args.read_len, args.k
    W = ka.words_for_k(k)
    strong = preset["scale"] == "strong"
    # --share G (one GPU, strong presets): rank 0's share of a G-rank job -- its reads and its
    # local table -- counted without the exchange (the per-rank half of a sharded step)
    share = args.share if strong and world == 1 and not dist and args.share > 1 else 0
    ranks = share or world
    if strong:  # this rank's share of the reads and of the table capacity
        first = args.reads * rank // ranks
        N = args.reads * (rank + 1) // ranks - first
        slots = -(-args.slots // ranks) if args.slots else 0
    else:
        first, N, slots = rank * args.reads, args.reads, args.slots
    stream = torch.cuda.current_stream()
    nbytes = lib.kc_synth_bytes(first, N, L, 0)
    sk = preset.get("skew")
    if image is None:
        image = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        if sk:
            skew = ka.kc_synth_skew(sk[0], sk[1], sk[2], sk[3])
            rc = lib.kc_synth_skew_device(image.data_ptr(), first, N, args.seed, args.genome, L, 0, args.err, 0.0,
                                          ctypes.byref(skew), stream.cuda_stream)
        else:
            rc = lib.kc_synth_device(image.data_ptr(), first, N, args.seed, args.genome, L, 0, args.err, 0.0,
                                     stream.cuda_stream)
        assert rc == 0, "kc_synth_device failed"
        torch.cuda.synchronize()
    assert image.numel() == nbytes
    # the reference chunk table: the planner reads the bytes around chunk ends from HBM
    chunks = ka.plan_chunks_device(image.data_ptr(), nbytes, k, ka.FMT_FASTA)
    if args.batch_mib:
        cap = args.batch_mib << 20
    else:
        # as large as HBM allows beside the table: kc_api.cpp ensure_part_geo keeps two level
        # buffers of ~1.25 x 8W bytes per staged byte (segment slack) plus the skew list (an
        # eighth of the windows as {W words, count} records), ~21 W + 3 bytes per staged byte.
        # The table is 1.25 x -s slots in 128-byte buckets of 16 // (W + 1) slots (-b: sized
        # from 2 x new_in_second, bounded here by 2 x -u).  The earlier table-blind rule
        # (0.45 x free / (28 W + 4)) stays as a floor: every recorded configuration ran with it
        # (C5 at full size takes the exact layout, whose buffers need less).  Batches stay
        # within the 2 GiB measured on the device (C4 at full size: 2.06 GB).
        free = gpu_free(torch, args, world)
        want = 1.25 * (slots if slots else 2 * (args.unique or 0))
        table = int(want / (16 // (W + 1))) * 128
        fit = int(0.85 * max(0, free - nbytes - table)) // (21 * W + 3)
        cap = min(max(fit, int(0.45 * (free - nbytes)) // (28 * W + 4)), 1 << 31)
    batch = min((nbytes + len(chunks) * 4096 + (1 << 20)) // 4096 * 4096, cap // 4096 * 4096)
    windows_expected = N * (L - k + 1)
    estimate = None
    # (strong presets on one GPU too, unless --s-table: the job's table is then sized from the
    # estimate -- C4 holds 1.0 G distinct k-mers in a -s 2.6e9 table, C5 1.5 G in -s 3.6e9, which as
    # 25 % headroom over -s take 83 / 192 GB of HBM for 35 / 86 GB of need)
    est_table = strong and not dist and not share and not args.s_table
    # N > 1: the exchange.  "superkmers": each rank routes its reads' super-k-mers
    # to their canonical-minimizer owners, which count them (no local table, no estimate); "records":
    # each rank counts locally and its table's {key, count} records go to their owners.  auto: super-
    # k-mers for the strong presets and Bloom jobs (C4 / 8 ranks: ~1.3 B per window against ~10 B of
    # records), records for a weak job without the filter (C2: each rank's reads cover the genome 30x,
    # so its 86 M distinct k-mers x 16 B undercut 1.2 G windows of super-k-mers)
    xmode = getattr(args, "exchange", "auto")
    if xmode == "auto":
        xmode = "superkmers" if (strong or args.unique) else "records"
    skm = bool(dist) and world > 1 and xmode == "superkmers"
    #  on one GPU the whole job's estimate runs inside the timed step: the
    # counter is created with -s and every step sizes its table from the estimate (kc_size_table)
    if not skm and ((strong and (share or (dist and world > 1))) or (dist and args.unique)):
        # (sharded Bloom jobs too: the rank's ungated local count holds all its distinct k-mers)
        # a rank's local table holds its own input's distinct k-mers, which its 1/G share of -s
        # does not bound: sized from a HyperLogLog estimate of them (kc_estimate_distinct_device,
        # once per job before the timed steps), 1.1 x the estimate (x 1.25 buckets: load <= 0.73)
        torch.cuda.synchronize()
        e0 = time.perf_counter()
        probe = ka.KmerCounter(ka.Config(k=k, mode=2, table_slots=1 << 16, batch_bytes=batch, device=local))
        est = probe.estimate_distinct_device(image.data_ptr(), chunks, ka.FMT_FASTA, stream.cuda_stream)
        probe.close()
        local_slots = min(windows_expected, int(1.1 * est) + (1 << 20))
        if dist and world > 1:
            # one size for every rank's local (and owner) table: the groups a rank receives are then
            # sorted by its own table's regions, and merge in one level-3 pass (sharded.DeviceEngine)
            t = torch.tensor([local_slots], dtype=torch.int64, device=coll_device(dist))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            local_slots = int(t.item())
        estimate = {"distinct_estimate": int(est), "local_slots": local_slots,
                    "ms": round((time.perf_counter() - e0) * 1e3, 1),
                    "method": "HyperLogLog, 2^14 registers (~0.8 % std. error); local table = 1.1 x estimate"}
    if skm and not args.batch_mib:
        # a rank holds its owner table (its 1/G share of -s, or of 2 x -u with the filter) and the
        # super-k-mer buffers (sent, a contiguous copy, received: ~0.5 B per image byte each)
        from kaarme_amd.sharded import owner_share
        osl = owner_share(slots or 2 * (args.unique or 0), world) if (slots or args.unique) else windows_expected
        per_table = int(1.25 * osl / (16 // (W + 1))) * 128
        free = gpu_free(torch, args, world)
        fit = int(0.85 * max(0, free - per_table - 2 * nbytes)) // (21 * W + 3)
        batch = min(batch, max(64 << 20, min(fit, 1 << 31)) // 4096 * 4096)
    elif dist and world > 1 and not args.batch_mib:
        # a rank also holds its owner table (the local table's geometry, sharded.DeviceEngine) and
        # the merge's record buffers (send x 1.25 + receive: W + 1 words per distinct k-mer of its
        # input) beside the local count's partition buffers: the batch takes what is left
        lsl = estimate["local_slots"] if estimate else min(slots or windows_expected, windows_expected)
        per_table = int(1.25 * (lsl if estimate else max(slots or 0, lsl)) / (16 // (W + 1))) * 128
        recs = int(2.25 * lsl * (W + 1) * 8)
        free = gpu_free(torch, args, world)  # (the image is already allocated)
        fit = int(0.85 * max(0, free - 2 * per_table - recs)) // (21 * W + 3)
        batch = min(batch, max(64 << 20, min(fit, 1 << 31)) // 4096 * 4096)
    tbl =" ".join(["-m", "2"] + table_args(slots, args.unique))
    workload = (f"{args.config}: synthetic {N} x {L} bp reads/GPU, k={k}, {tbl}" if not strong else
                f"{args.config}: synthetic {args.reads} x {L} bp reads over {world} GPU(s), k={k}, {tbl} per GPU")
    if est_table:
        workload += (" (device table sized from the distinct estimate, 1.1 x HLL, not 1.25 x -s; the estimate runs "
                     "inside every timed step)")
    if share:
        workload = (f"{args.config} share 1/{share}: synthetic {N} x {L} bp reads (rank 0 of {args.reads} over "
                    f"{share} GPUs), k={k}, -m 2, local table from the distinct estimate, no exchange")
    if sk:
        workload += (f", skew: {sk[0]:.0%} poly-A/T reads, {sk[1]:.0%} (CA)n reads, a {sk[2]}-bp repeat x "
                     f"{sk[3]} in the genome")
    # -a only selects output lines (it does not change counting): the reference fixture's -a when
    # this workload has one, so the parity digest covers the same lines
    # the whole job's reference digest: one GPU, a share, or a strong preset over all ranks (each
    # rank's owner table digests its k-mers; parity_record combines them).  A weak job over N > 1
    # ranks counts N x the preset's reads, which no fixture covers.
    fx = fixture_case(args, share, first, N) if (world == 1 or strong) else None
    # (N > 1 strong: the owner table takes the local table's estimate-sized geometry, not the 1/G share
    # of -s -- the largest rank's distinct k-mers bound an owner's, about the job's 1/G, from above)
    tslots = slots
    if share or (dist and world > 1 and strong and estimate):
        tslots = estimate["local_slots"] if share else min(slots, estimate["local_slots"])
    if skm and slots:  # (every rank owns ~1/G of the distinct k-mers: its share of -s, + 8 sigma)
        from kaarme_amd.sharded import owner_share
        tslots = owner_share(slots, world)
    cfg = ka.Config(k=k, mode=2, table_slots=tslots,
                    min_abundance=fx["min_abundance"] if fx else 2, batch_bytes=batch,
                    device=local, bf_enable=bool(args.unique), est_unique=args.unique)
    if dist:
        from kaarme_amd.sharded import ShardedCounter
        local_slots = 0
        if strong or args.unique:
            local_slots = estimate["local_slots"] if estimate else min(args.slots or 0, windows_expected)
        counter = ShardedCounter(cfg, dist, local_slots=local_slots, exchange=xmode)
    else:
        counter = ka.KmerCounter(cfg)

    est_log = []  # (estimate, slots, seconds) of every step that sized its table from the estimate

    def step():
        counter.reset()
        if est_table:
            # the whole job's distinct estimate (tokenizer + k_hll over every batch; the call waits
            # for it) and the table sized from it, inside the step the line times
            e0 = time.perf_counter()
            est = counter.estimate_distinct_device(image.data_ptr(), chunks, ka.FMT_FASTA, stream.cuda_stream)
            tab = min(windows_expected, int(1.1 * est) + (1 << 20))
            counter.size_table(tab)
            est_log.append((est, tab, time.perf_counter() - e0))
        if args.unique:  # Bloom pass, table sized 2 * new_in_second, counting pass behind the gate
            counter.bloom_device(image.data_ptr(), chunks, ka.FMT_FASTA, stream.cuda_stream)
            counter.bloom_finalize()
        counter.count_device(image.data_ptr(), chunks, ka.FMT_FASTA, stream.cuda_stream)
        counter.sync()

    return argparse.Namespace(counter=counter, image=image, chunks=chunks, step=step, N=N, first=first, nbytes=nbytes,
                              slots=slots, strong=strong, windows_expected=windows_expected, tbl=tbl,
                              workload=workload, fixture=fx, stream=stream, estimate=estimate, share=share,
                              est_log=est_log, exchange=xmode if dist else None)


def parity_record(job, k, dist=None):
    """The timed job's output against the reference's (tests/golden/fullsize.json), after the timed
    steps: the order-independent output digest (kc_output_digest: lines, sum of T(c), sum and XOR
    of XXH64 per line; on N ranks the owners' digests combined, an all-gather) against the case's
    `digest`, and on one GPU also the SHA-256 of the sorted output text from kc_dump when the case
    has the reference's sorted digest and its text stays below ~30 GB."""
    fx = job.fixture
    import kaarme_amd as ka
    t0 = time.perf_counter()
    if fx is None:  # (no reference case for this input: the digest alone, e.g. to compare N = 1 with N > 1)
        return {"reference_case": None, "digest": job.counter.output_digest(), "match": None,
                "digest_s": round(time.perf_counter() - t0, 2)}
    rec = {"reference_case": f"tests/golden/fullsize.json {fx['name']}: " + (
        f"oracle/_ref/kaarme {' '.join(fx['args'])} on the same input" if fx.get("sorted_sha256") else
        f"{' '.join(fx['args'])}, digest of the pinned CPU restatement (whole job)")}
    ok = True
    want = fx.get("digest")
    if want:
        got = job.counter.output_digest()
        ok = ok and ka.same_digest(got, want)
        rec["digest"] = got
        rec["digest_source"] = want.get("source")
    if fx.get("sorted_sha256") and not dist and fx["lines"] * (k + 8) < 30e9:
        from kaarme_amd.digest import sorted_text_digest
        got = sorted_text_digest(job.counter.dump(), k)
        ok = ok and (got["sorted_sha256"], got["lines"], got["count_sum"]) == (fx["sorted_sha256"], fx["lines"],
                                                                                 fx["count_sum"])
        rec.update(sorted_sha256=got["sorted_sha256"], lines=got["lines"], count_sum=got["count_sum"])
    elif not want:
        return None
    rec["match"] = ok
    rec["digest_s"] = round(time.perf_counter() - t0, 2)
    return rec


def writer_record(job, verify):
    """The output writer at full size (kmer_hash_table.cpp:4318-4524): kc_write of
    the timed job's table (device formatting, double-buffered copy-out, file writes) timed to a
    file in TMPDIR; with verify, the SHA-256 of the byte-sorted file against the reference's output
    digest (tests/golden/fullsize.json) -- the bytes the writer produced, not the records."""
    import hashlib
    fx = job.fixture
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        path = os.path.join(td, "out.txt")
        t0 = time.perf_counter()
        job.counter.write(path)
        secs = time.perf_counter() - t0
        size = os.path.getsize(path)
        rec = {"seconds": round(secs, 3), "bytes": size, "gbs": round(size / secs / 1e9, 2),
               "path": "kc_write: k_text_bytes + k_text on the device, pinned double-buffered copy-out, fwrite "
                       "to TMPDIR (page cache)"}
        if fx is not None:
            # the reference CLI writing the same job's output on the GPU box's 16-core share (its own
            # "Time used to write k-mers in a file", profiles/r03_ref_fullsize_box.txt)
            ref_w = {"C2": 59.446, "C3": 31.586}.get(fx["name"])
            if ref_w:
                rec["reference_write_s"] = ref_w
                rec["reference_write_source"] = "profiles/r03_ref_fullsize_box.txt (oracle/_ref/kaarme -t 18)"
        if verify and fx is not None:
            t1 = time.perf_counter()
            env = dict(os.environ, LC_ALL="C")
            p = subprocess.Popen(["sort", "-S", "12G", "--parallel=16", "-T", td, path], stdout=subprocess.PIPE,
                                 env=env)
            h = hashlib.sha256()
            lines = 0
            for b in iter(lambda: p.stdout.read(1 << 24), b""):
                h.update(b)
                lines += b.count(b"\n")
            ok = p.wait() == 0
            rec["parity"] = {"match": ok and h.hexdigest() == fx["sorted_sha256"] and lines == fx["lines"],
                             "sorted_sha256": h.hexdigest(), "lines": lines,
                             "reference_case": f"tests/golden/fullsize.json {fx['name']}",
                             "digest_s": round(time.perf_counter() - t1, 2)}
    return rec


def run_workload(args, env, image=None):
    """Times one workload (warmup + steps of a full counting job) and returns its JSON record
    plus the device image (reusable by a workload with the same generator parameters)."""
    torch, ka, dist = env["torch"], env["ka"], env["dist"]
    rank, world = env["rank"], env["world"]
    job = setup_job(args, env, image)
    counter, image, chunks, step = job.counter, job.image, job.chunks, job.step
    N, nbytes, strong, workload, tbl = job.N, job.nbytes, job.strong, job.workload, job.tbl
    windows_expected = job.windows_expected
    L, k = args.read_len, args.k
    if rank == 0:  # progress on stderr (a long setup / digest is not a hang)
        log(f"{args.config}: job ready ({nbytes} image bytes, {len(chunks)} chunks); warmup")
    for _ in range(args.warmup):
        step()
    counter.profile(True)
    counter.timing()  # drop warmup events
    if dist:
        counter.xstats = {key: 0 for key in counter.xstats}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    counter.profile(False)
    tm = counter.timing()
    xgmi = None
    if dist and world > 1:  # the merge's exchange, per rank and step, beside the HBM figures
        xs = counter.xstats
        t = torch.tensor([xs["bytes_sent"], xs["exchange_s"], xs.get("route_s", 0.0), xs.get("insert_s", 0.0)],
                         dtype=torch.float64, device=coll_device(dist))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sent, xsec, rsec, isec = (float(v) for v in t.tolist())
        xgmi = {"sent_bytes_per_step_per_rank": int(sent / args.steps),
                "exchange_ms_per_step": round(xsec / args.steps * 1e3, 3),
                "gbs_per_rank": round(sent / max(xsec, 1e-9) / 1e9, 2), "peak_gbs_per_gpu": 7 * 153,
                "route_ms_per_step": round(rsec / args.steps * 1e3, 3),
                "owner_insert_ms_per_step": round(isec / args.steps * 1e3, 3), "exchange": job.exchange,
                "note": "max over ranks; the all-to-all of {key, count} records incl. its count/sum headers; "
                        "route = the local table as owner-grouped records (host waits for its counts), "
                        "owner insert = the received records into the owner table (waited for)"}
        if job.exchange == "superkmers":
            # bytes per rank of the super-k-mer exchange at G ranks, from this run's bytes per window: a run
            # of r windows costs k + r symbols (12 bytes per 32); runs of one owner merge consecutive
            # super-k-mers, r_G = r_1 G / (G - 1), so r_1 follows from this run's r_world; every rank sends
            # (G - 1) / G of its 1/G of the job's windows
            bpw = sent / args.steps / max(1, windows_expected) * world / max(1, world - 1)
            spw = bpw / (12 / 32)
            r1 = k / max(spw - 1, 1e-6) * (world - 1) / world
            total_w = args.reads * (L - k + 1) if strong else windows_expected * world

            def bpw_at(G):
                r = r1 * G / (G - 1)
                return (k + r) / r * 12 / 32

            xgmi["bytes_per_window_sent"] = round(bpw, 4)
            xgmi["superkmer_windows_per_run"] = round(r1, 2)
            xgmi["model_sent_bytes_per_rank"] = {str(G): int(total_w / G * bpw_at(G) * (G - 1) / G) for G in (2, 4, 8)}
            xgmi["records_design_bytes_per_rank"] = "~10.8 GB at G = 8 for C4 (DESIGN 4; round 5's exchange)"
            xgmi["note"] = ("max over ranks; two all-to-alls (packed symbol words, break words) of the canonical-"
                            "minimizer super-k-mers + their count/sum headers; route = tokenizer + k_skm_route + the "
                            "send buffers; owner insert = kc_count_packed_device of the received streams (waited "
                            "for); model = the job's windows / G x the bytes per window at G (superkmer_windows_per_run, runs of one owner "
                            "merging G / (G - 1) super-k-mers) x (G - 1) / G")
    st = counter.finish()  # raises on table overflow
    if rank == 0:
        log(f"{args.config}: {args.steps} steps in {elapsed:.3f} s; parity / writer records")
    parity = parity_record(job, k, dist) if args.verify else None
    # (the text writer and its sorted-file digest for outputs up to ~8 GB: C2 / C3; a strong
    # share's 30 GB of text would take minutes to sort)
    writer = writer_record(job, args.verify) if (args.writer and not dist and job.fixture is not None and
                                                 job.fixture["lines"] * (k + 8) < 8e9) else None
    compact = None
    if not dist and args.compact:  # the Kaarme slot words built from this table
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        try:
            info = counter.compact()
        except ka.KcError as e:  # (the compact words need HBM beside the table: none left by C5's)
            info = {"error": str(e)}
        c1 = time.perf_counter()
        n = max(1, info.get("kmers", 0))
        compact = {"error": info["error"]} if "error" in info else {"build_ms": round((c1 - c0) * 1e3, 2), "kmers": info["kmers"],
                   "chain_starts": info["chain_starts"], "bytes_per_kmer": round(info["bytes"] / n, 2),
                   "table_bytes_per_kmer": round(info["table_bytes"] / n, 2),
                   "note": "kc_compact after the timed steps (not in value): 8-byte slot words at load 0.8 + "
                           "chain-start keys, vs the full-key table sized by -s"}
    counter.close()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device(dist))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    windows_step = st["windows"]
    assert windows_step == windows_expected, (windows_step, windows_expected)
    total_windows = windows_step * args.steps
    if dist:
        t = torch.tensor([total_windows], dtype=torch.float64, device=coll_device(dist))
        dist.all_reduce(t)
        total_windows = float(t.item())
    value = total_windows / elapsed

    # --- roofline of the counting pass: A = sym_B + (1+u)*K + 8 bytes per
    # window (K = 8*ceil(2k/64) key bytes, u = distinct/windows, 8 = count read + write),
    # times the windows of one launch (one staged batch), over the pass's event time.
    K = 8 * math.ceil(2 * k / 64)
    u = st["distinct"] / max(1, windows_step)
    launches = max(1, tm["launches"])
    per_step = launches / args.steps
    sym_per_launch = nbytes / per_step
    win_per_launch = windows_step / per_step
    bytes_per_launch = sym_per_launch + win_per_launch * ((1 + u) * K + 8)
    # the roofline window is the tokenizer + the counting pass of a batch (the
    # input bytes sym_B are read by the tokenizer, so its time is inside the window that A counts)
    count_ms = (tm["tokenize_ms"] + tm["count_ms"]) / launches
    if job.est_log:
        # the strong presets' distinct estimate (tokenizer + k_hll, whose tokenized batches the counting
        # pass reads) is part of every batch's window: its wall time per batch (host waits included)
        timed = job.est_log[-args.steps:]
        count_ms += sum(x[2] for x in timed) / len(timed) * 1e3 / per_step
    units_per_step = per_step
    if args.unique:
        # Bloom configs: the unit is one Bloom pass + one counting pass over
        # the same batch: a second sym_B, ceil(hf) 8-byte filter-word RMWs (pass 1) and
        # trunc(hf) 4-byte tests (pass 2) per window, the table term for the windows that
        # pass the gate
        hf = -math.log(0.01) / math.log(2)  # -f 0.01 (the Config default)
        nh, nh_gate = math.ceil(hf), int(hf)
        p_gate = st["inserted"] / max(1, windows_step)
        pairs = max(1, launches // 2)
        bytes_rmw = (2 * nbytes / args.steps + windows_step * (8 * nh + 4 * nh_gate)
                     + windows_step * p_gate * ((1 + u) * K + 8)) * args.steps / pairs
        count_ms = (tm["tokenize_ms"] + tm["count_ms"]) / pairs
        units_per_step = pairs / args.steps
        filter_rmw = windows_step * (8 * nh + 4 * nh_gate) * args.steps / pairs
        # the headline fraction leaves out SURVEY 8d's per-window filter-word
        # RMWs, which the blocked filter never performs (k_b3 sweeps each 64 KiB filter region
        # once per pass); the RMW-priced figure stays beside it (with_filter_rmw)
        bytes_per_launch = bytes_rmw - filter_rmw
    achieved = bytes_per_launch / (count_ms * 1e-3) / 1e9
    traffic, tentry = load_traffic(workload)
    traffic_stale = bool(tentry) and tentry.get("source_sha") != kernel_source_digest()
    if dist:
        kname = "tokenizer + local count pass + merge insert of the received {key, count} records"
    elif args.unique:
        kname = ("tokenizer + Bloom pass 1 (k_p1 -> k_p2f -> k_b3: LDS-resident filter regions, whole table keys "
                 "in fine hash-prefix bins) + counting pass from the kept partitions (k_p3 with the gate at level "
                 "3; kc_stats.reused_passes), one of each per batch")
    else:
        kname = ("tokenizer (k_tile_summary_m, tile scan, k_emit) + count pass: k_p1 (segmented scatter), k_p2f, "
                 "k_p3 (partitioned insert)")
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": kname,
                "kernel_ms": round(count_ms, 4), "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "window": "tokenizer + counting pass (HIP events on the pass's stream)" + (
                    "; + the distinct estimate (tokenizer + k_hll, wall time per batch) whose tokenized batches the "
                    "counting pass reads" if job.est_log else "")}
    if args.unique:
        roofline["with_filter_rmw"] = {"achieved": round(bytes_rmw / (count_ms * 1e-3) / 1e9, 2),
                                       "frac": round(bytes_rmw / (count_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                                       "algorithmic_bytes_per_launch": int(bytes_rmw),
                                       "note": "SURVEY 8d's A with ceil(hf) 8-byte filter RMWs + trunc(hf) 4-byte "
                                               "tests per window (not performed by the blocked filter)"}
    if traffic:
        # the bytes this design moves (rocprofv3 PMC, profiles/pmc_traffic.json) over the same time;
        # stale = measured with other kernel sources than these (the entry's source_sha)
        roofline["traffic_gbs"] = round(traffic / (count_ms * 1e-3) / 1e9, 2)
        roofline["traffic_frac"] = round(traffic / (count_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        roofline["traffic_source"] = {"stale": traffic_stale, "source_sha": tentry.get("source_sha"),
                                      "commit": tentry.get("commit")}
    step_ms = elapsed / args.steps * 1e3
    out = {
        "metric": METRIC, "value": value, "unit": "k-mers/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_ms, "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic (seeded generator, SURVEY.md 8d)",
        "config": {"workload": workload, "reads_per_gpu": N, "read_len": L, "k": k, "genome": args.genome,
                   "table": tbl, "batches_per_step": per_step,
                   "parallelism": f"hash-prefix shard x{world}" if dist else "single"},
        "roofline": roofline,
        "hbm_gbs_step": round(bytes_per_launch * units_per_step / (step_ms * 1e-3) / 1e9, 2),
        "kernel_ms": {"gather": round(tm["gather_ms"] / launches, 4), "tokenize": round(tm["tokenize_ms"] / launches, 4),
                      "count": round(tm["count_ms"] / (max(1, launches // 2) if args.unique else launches), 4)},
        "image_bytes": nbytes, "stage_bytes": sum(c[1] for c in chunks),
        "windows_per_step_per_gpu": windows_step, "distinct_per_gpu": st["distinct"], "table_slots": st["table_slots"],
        "skew_lists": {"spilled_keys": st["spilled"], "heavy_records": st["heavy_records"],
                       "batches_redone": st["part_fallbacks"]},
        "cpu_baseline": None,
    }
    if parity:
        out["parity"] = parity
    if compact:
        out["compact"] = compact
    if writer:
        out["writer"] = writer
    if xgmi:
        out["xgmi"] = xgmi
    if job.estimate:
        out["local_table"] = job.estimate
    if job.est_log:
        timed = job.est_log[-args.steps:]
        e, tab, _ = timed[-1]
        out["local_table"] = {"distinct_estimate": int(e), "local_slots": tab, "in_timed_step": True,
                              "ms": round(sum(x[2] for x in timed) / len(timed) * 1e3, 2),
                              "method": "HyperLogLog, 2^14 registers (~0.8 % std. error) over the whole image "
                                        "(kc_estimate_distinct_device), then kc_size_table(1.1 x estimate), in "
                                        "every timed step (ms = its mean share of ms_per_step)"}
    if job.share:
        out["config"]["parallelism"] = f"one rank's share of hash-prefix shard x{job.share} (no exchange)"
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not job.share:
        out["cpu_baseline"] = cpu_baseline(args)
    if world == 1 and not dist and args.cli_fullsize and not job.share and args.config in ("C2", "C3", "C4", "C5"):
        out["cli_fullsize"] = cli_fullsize(job, args)
    if world == 1 and not dist and args.host_chunks and not job.share and args.config == "C2":
        out["c_abi_host_chunks"] = host_chunks_record(job, args)
    return out, image


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_gpus():
    """GPUs the rank processes can use, counted without initialising HIP in this process (VERDICT r4
    item 1, ADVICE r4: torch.cuda.device_count() may fall back to hipGetDeviceCount): the device
    lists of ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set (ROCm
    applies them in that order, so the smallest count bounds), else the GPU nodes of the kfd
    topology (sysfs; a node with gpu_id 0 is a CPU).  None when neither tells."""
    counts = []
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            counts.append(len([x for x in v.split(",") if x.strip()]))
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(base)
    except OSError:
        nodes = None
    if nodes is not None:
        n = 0
        for d in nodes:
            try:
                with open(os.path.join(base, d, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                pass
        counts.append(n)
    return min(counts) if counts else None


def coll_device(dist):
    """Where the line's own collectives keep their tensors: the GPU over RCCL, the host over gloo
    (--rehearse-one-gpu)."""
    return "cpu" if dist.get_backend() == "gloo" else "cuda"


def launch_ranks(n, cpu_only):
    """Starts `n` rank processes of this same command line (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment, as torch.distributed.run would set
    them) and waits for them.  The launcher itself never touches the GPU (it does not import torch:
    visible_gpus reads the environment and sysfs); the ranks are children, not an exec.  Rank 0
    prints the JSON line on the inherited stdout.  Returns the exit code (the first nonzero rank's;
    a failed rank stops the others)."""
    if not cpu_only and "--rehearse-one-gpu" not in sys.argv:
        have = visible_gpus()
        if have is not None and have < n:
            log(f"error: --gpus {n} but {have} GPU(s) visible")
            return 2
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                log(f"rank {procs.index(p)} exited with {c}: stopping the other ranks")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def launch_check(args):
    """--launch-only: join the process group (gloo on CPU) and report how many ranks joined."""
    import torch
    import torch.distributed as dist
    dist.init_process_group(args.backend)
    t = torch.ones(1)
    dist.all_reduce(t)
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "k-mers/s", "n_gpus": world,
                          "ranks_joined": int(t.item()), "launch_only": True, "backend": args.backend}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, choices=sorted(PRESETS),
                    help="BASELINE.md workload (default: C2 on one GPU, C4 -- the multi-GPU config BASELINE.json "
                         "names, strong scaling -- on N > 1)")
    ap.add_argument("--reads", type=int, default=None, help="reads (per GPU for weak, total for strong presets)")
    ap.add_argument("--read-len", type=int, default=None)
    ap.add_argument("--genome", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--slots", type=int, default=None, help="-s (total for strong presets)")
    ap.add_argument("--unique", type=int, default=None, help="-b -u U (Bloom filter) instead of -s")
    ap.add_argument("--batch-mib", type=int, default=0, help="staging batch (0 = the whole image if HBM allows)")
    ap.add_argument("--err", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-sample-bases", type=int, default=150_000_000)
    ap.add_argument("--cpu-threads", type=int, default=0, help="-t of the reference (0 = core share + 2)")
    ap.add_argument("--cpu-runs", type=int, default=3, help="reference runs on the sample (the median is reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-compact", dest="compact", action="store_false",
                    help="skip the compact-representation figure (kc_compact after the timed steps)")
    ap.add_argument("--secondary", default="C3",
                    help="at N=1 with the default C2: also time this workload (the north star's k=51 Bloom "
                         "config) and attach it as a second record ('none' = skip)")
    ap.add_argument("--secondary-cpu-sample-bases", type=int, default=50_000_000)
    ap.add_argument("--tertiary", default="C4",
                    help="at N=1 with the default C2: also time this workload on the one GPU ('c4' record: the "
                         "whole C4 job, the N=1 point of the strong-scaling curve the N > 1 lines time; 'none' = "
                         "skip)")
    ap.add_argument("--quaternary", default="C5",
                    help="at N=1 with the default C2: also time this workload on the one GPU ('c5' record: the "
                         "whole long-read C5 job; 'none' = skip)")
    ap.add_argument("--tertiary-cpu-sample-bases", type=int, default=50_000_000)
    ap.add_argument("--multi-secondary", default="C2",
                    help="at N > 1 with the default C4: also time this weak-scaling workload ('none' = skip)")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="skip the parity digest against the reference's output (tests/golden/fullsize.json)")
    ap.add_argument("--no-cli-fullsize", dest="cli_fullsize", action="store_false",
                    help="skip the drop-in CLI on the whole workload's file (cli_fullsize record; C2 / C3 / C4 / C5)")
    ap.add_argument("--no-host-chunks", dest="host_chunks", action="store_false",
                    help="skip the C-ABI host-chunk record (kc_count_chunk over the C2 job's chunks from host memory)")
    ap.add_argument("--no-writer", dest="writer", action="store_false",
                    help="skip writing the timed job's output with kc_write (timed, and digested with --verify)")
    ap.add_argument("--share", type=int, default=0,
                    help="strong presets on one GPU: time rank 0's share of a G-rank job (its reads, its local "
                         "table sized from the distinct estimate; no exchange)")
    ap.add_argument("--s-table", action="store_true",
                    help="strong presets on one GPU: size the table from -s (1.25 x) instead of the distinct estimate")
    ap.add_argument("--exchange", default="auto", choices=("auto", "records", "superkmers"),
                    help="N > 1: the sharded exchange (auto: super-k-mers for strong presets and Bloom jobs, "
                         "records for weak ones)")
    ap.add_argument("--force-sharded", action="store_true",
                    help="use the sharded (RCCL) path even at one rank (testing)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend of the ranks (nccl = RCCL; gloo only with --launch-only)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 on a one-GPU box: every rank on cuda:0, gloo instead of RCCL (the exchange goes "
                         "through host memory) -- runs the multi-GPU line's code path end to end (testing)")
    ap.add_argument("--launch-only", action="store_true",
                    help="start the ranks, join the process group and print the line without any GPU work "
                         "(tests the N-rank launch on CPU)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher starts its own N rank processes
        # (before anything here touches the GPU) instead of timing one GPU
        sys.exit(launch_ranks(args.gpus, args.launch_only))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world_env}")
        sys.exit(2)
    if args.launch_only:
        sys.exit(launch_check(args))
    # stdout carries exactly one JSON line: libraries (RCCL prints a version banner at
    # communicator init) write to fd 1 too, so fd 1 becomes stderr and the JSON goes to a
    # private copy of the original stdout
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1 or args.force_sharded:
        import torch.distributed as dist
        for key, val in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(key, val)
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import kaarme_amd as ka

    env = {"torch": torch, "ka": ka, "lib": ka.load_library(), "dist": dist, "rank": rank, "world": world,
           "local": local}
    if args.config is None:
        args.config = "C4" if world > 1 else "C2"
    primary = resolve(args, args.config)
    out, image = run_workload(primary, env)
    keep = ("value", "unit", "ms_per_step", "scaling", "config", "roofline", "kernel_ms", "windows_per_step_per_gpu",
            "distinct_per_gpu", "table_slots", "cpu_baseline", "parity", "compact", "writer", "xgmi", "local_table",
            "cli_fullsize")
    extra = []
    if world == 1 and not dist and args.config == "C2":
        if args.secondary != "none":
            extra.append((args.secondary, dict(cpu_sample_bases=args.secondary_cpu_sample_bases)))
        if args.tertiary != "none":
            # (C4 -- the north star's "150 bp reads at k=51" -- with its own CPU
            # baseline, the reference on a sample at C4's 30x coverage; no compact figure)
            extra.append((args.tertiary, dict(cpu_sample_bases=args.tertiary_cpu_sample_bases, compact=False)))
        if args.quaternary != "none":
            extra.append((args.quaternary, dict(no_cpu_baseline=True, compact=False)))
    elif world > 1 and args.config == "C4" and args.multi_secondary != "none":
        extra.append((args.multi_secondary, {}))
    for name, over in extra:
        sec = resolve(args, name)
        for key, val in over.items():
            setattr(sec, key, val)
        if not same_image(primary, sec):
            image = None
            torch.cuda.empty_cache()
        rec, image = run_workload(sec, env, image)
        out[sec.config.lower()] = {key: rec[key] for key in keep if key in rec}
    del image
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
