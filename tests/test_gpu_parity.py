"""GPU parity: the MI355X path through the C ABI against the reference fixtures and
the oracle.  Integer work, so everything is bit-exact on sorted output.

Bloom-filter runs with -a 1 are nondeterministic in the reference itself once more
than one worker runs: for those the GPU must reproduce every
k-mer with count >= 2 exactly and may only emit count-1 k-mers that truly occur once.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import CLI, GEN, load_cases, oracle_count, sorted_digest_file, sorted_digest_lines, text_digest
import kaarme_amd as ka

pytestmark = pytest.mark.gpu

CASES = load_cases()["cases"]


def _case_id(c):
    return f"{c['input']}-k{c['k']}-" + "".join(a.strip("-") for a in c["args"])


def parse_ref_args(args):
    o = {"mode": 2, "min_abundance": 2, "table_slots": 0, "bf_enable": False, "est_unique": 0, "fpr": 0.01}
    i = 0
    while i < len(args):
        a = args[i]
        if a == "-b":
            o["bf_enable"] = True
            i += 1
            continue
        v = args[i + 1]
        key = {"-m": "mode", "-a": "min_abundance", "-s": "table_slots", "-u": "est_unique", "-f": "fpr"}[a]
        o[key] = float(v) if key == "fpr" else int(v)
        i += 2
    return o


def lines_of(kc):
    return kc.lines()


def bf_singleton_check(lines, path, k, mode, tmp_path):
    """BF with -a 1: counts >= 2 exact, count-1 lines must be true singletons."""
    full = tmp_path / "nobf.txt"
    oracle_count(path, k, ["-m", str(mode), "-a", "1"], full)
    truth = dict(l.rsplit(" ", 1) for l in open(full).read().splitlines())
    got = dict(l.rsplit(" ", 1) for l in lines)
    solid_truth = {s: c for s, c in truth.items() if int(c) >= 2}
    solid_got = {s: c for s, c in got.items() if int(c) >= 2}
    assert solid_got == solid_truth
    for s, c in got.items():
        if c == "1":
            assert truth.get(s) == "1", s


@pytest.fixture(params=["direct", "partitioned", "exact"])
def insert_path(request, monkeypatch):
    """Every insert path must give the reference's result (KC_INSERT_PATH forces one):
    direct = device-scope atomics, partitioned = single-pass segmented scatters,
    exact = the histogram-offset scatters (the segmented path's fallback)."""
    monkeypatch.setenv("KC_INSERT_PATH", request.param)
    return request.param


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_golden_case_host_chunks(case, golden_input, tmp_path, insert_path):
    check_golden_case(case, golden_input, tmp_path)


@pytest.mark.parametrize("case", [c for c in CASES if "-b" in c["args"]], ids=_case_id)
def test_golden_bloom_cases_reference_layout(case, golden_input, tmp_path, monkeypatch):
    """The Bloom filter with the reference's bit positions (one XXH64 per hash function,
    KC_BLOOM_LAYOUT=reference) instead of the default one-line-per-k-mer blocked layout:
    same results (the filter only gates; counts >= 2 are exact either way)."""
    monkeypatch.setenv("KC_BLOOM_LAYOUT", "reference")
    check_golden_case(case, golden_input, tmp_path)


def check_golden_case(case, golden_input, tmp_path):
    path = golden_input(case["input"])
    o = parse_ref_args(case["args"])
    kc, st = ka.count_file(path, case["k"], mode=o["mode"], min_abundance=o["min_abundance"],
                           table_slots=max(o["table_slots"], 1 << 16), bf_enable=o["bf_enable"],
                           est_unique=o["est_unique"], fpr=o["fpr"])
    with kc:
        lines = lines_of(kc)
        # -m 1 -b runs the Bloom pass and then ignores the filter (main.cpp:482-489): exact
        if o["bf_enable"] and o["min_abundance"] == 1 and o["mode"] != 1:
            bf_singleton_check(lines, path, case["k"], o["mode"], tmp_path)
        else:
            assert sorted_digest_lines(lines) == (case["sorted_sha256"], case["lines"])
        if case["distinct"] is not None and not o["bf_enable"]:
            assert st["distinct"] == case["distinct"]
        # the device text formatter (kc_write) gives the same lines as the records
        out = tmp_path / "out.txt"
        kc.write(str(out))
        assert sorted(open(out).read().splitlines()) == sorted(lines)
        # the order-independent digest (kc_output_digest, the whole-job parity of bench.py's N > 1
        # lines) is the written text's
        assert kc.output_digest() == text_digest(str(out))


@pytest.mark.parametrize("name,k,args", [
    ("reads_w60.fasta", 31, ["-a", "1"]),
    ("edge.fasta", 25, ["-m", "0", "-a", "1"]),
    ("long.fasta", 127, ["-a", "1"]),
    ("big_edge.fasta", 31, ["-a", "1"]),
])
def test_device_image_path_and_small_batches(name, k, args, golden_input, tmp_path, insert_path):
    """kc_count_device over a device-resident image with the reference chunk table,
    with a staging batch far smaller than the input (many batches, chunk splits)."""
    torch = pytest.importorskip("torch")
    path = golden_input(name)
    image = open(path, "rb").read()
    fmt = ka.detect_format(path, image[0])
    o = parse_ref_args(args)
    exp = tmp_path / "exp.txt"
    oracle_count(path, k, args, exp)
    for chunk_size, batch in [(0, 0), (5000, 1 << 16), (100003, 1 << 20)]:
        chunks = ka.plan_chunks(image, k, fmt, chunk_size)
        dev = torch.frombuffer(bytearray(image), dtype=torch.uint8).cuda()
        with ka.KmerCounter(ka.Config(k=k, mode=o["mode"], min_abundance=o["min_abundance"],
                                      table_slots=1 << 22, batch_bytes=batch)) as kc:
            kc.count_device(dev.data_ptr(), chunks, fmt, torch.cuda.current_stream().cuda_stream)
            kc.finish()
            # chunking other than the reference's 10 MiB changes nothing on these inputs
            # except where a header is cut (then the oracle is re-run with the same chunking)
            if chunk_size:
                exp2 = tmp_path / f"exp_{chunk_size}.txt"
                oracle_count(path, k, args + ["-c", str(chunk_size)], exp2)
                want = sorted_digest_file(exp2)
            else:
                want = sorted_digest_file(exp)
            assert sorted_digest_lines(kc.lines()) == want, (chunk_size, batch)


def test_synth_device_matches_cpu_generator(tmp_path):
    torch = pytest.importorskip("torch")
    lib = ka.load_library()
    for (first, n, L, w, e, nr) in [(0, 3000, 150, 0, 0.001, 0.0), (977, 1500, 151, 60, 0.01, 0.002),
                                    (0, 20, 10000, 0, 0.001, 0.0)]:
        nbytes = lib.kc_synth_bytes(first, n, L, w)
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        rc = lib.kc_synth_device(buf.data_ptr(), first, n, 42, 200000, L, w, e, nr,
                                 torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        p = tmp_path / "c.fa"
        subprocess.run([GEN, str(p), str(first + n), str(L), "200000", "-s", "42", "-e", str(e), "-n", str(nr),
                        "--first", str(first), "--count", str(n)] + (["-w", str(w)] if w else []), check=True)
        assert bytes(buf.cpu().numpy()) == open(p, "rb").read()


@pytest.mark.parametrize("case", [c for c in CASES if c["input"] in ("reads_w60.fasta", "edge.fasta", "big_reads.fasta")
                                  and not ("-b" in c["args"] and "1" == c["args"][c["args"].index("-a") + 1]
                                           and parse_ref_args(c["args"])["mode"] != 1)],
                         ids=_case_id)
@pytest.mark.parametrize("cli_path", ["device", "host"])
def test_cli_end_to_end(case, cli_path, golden_input, tmp_path):
    """The drop-in CLI: the input read into HBM by parallel pinned slices and counted from
    there (device; Bloom jobs count from the Bloom pass's partitions), or staged as host
    chunks (--host-chunks)."""
    path = golden_input(case["input"])
    out = tmp_path / "out.kaarme_counts"
    extra = ["--host-chunks"] if cli_path == "host" else []
    r = subprocess.run([CLI, path, str(case["k"]), "-t", "3", "-o", str(out)] + case["args"] + extra,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert sorted_digest_file(out) == (case["sorted_sha256"], case["lines"])
    assert "Time used to build hash table" in r.stdout
    assert ("Input path: device image" in r.stdout) == (cli_path == "device")


@pytest.mark.parametrize("name,k,args", [("reads_w60.fasta", 31, ["-m", "2", "-a", "1", "-s", "1000000"]),
                                         ("reads.txt", 31, ["-a", "1", "-s", "1000000"]),
                                         ("big_reads.fasta", 31, ["-a", "2", "-s", "8000000"])])
@pytest.mark.parametrize("members", [1, 3, "bgzf"])
def test_cli_gzip_input_is_counted_whole(name, k, args, members, golden_input, tmp_path):
    """gzip input (an extension): the reference reads only part of a
    compressed file; the drop-in CLI decompresses every member of the
    stream and must give the uncompressed file's fixture (big_reads.fasta: > 10 MiB, so
    the decompressed image spans several chunks)."""
    import gzip

    case = next(c for c in CASES if c["input"] == name and c["k"] == k and c["args"] == args)
    raw = open(golden_input(name), "rb").read()
    gz = tmp_path / (name + ".gz")
    if members == "bgzf":  # blocked gzip: members inflated in parallel (kc_cli.cpp gunzip_bgzf)
        from test_host import _bgzf

        gz.write_bytes(_bgzf(raw))
    else:
        cuts = [len(raw) * i // members for i in range(members + 1)]
        with open(gz, "wb") as f:  # concatenated members split at arbitrary bytes
            for a, b in zip(cuts, cuts[1:]):
                f.write(gzip.compress(raw[a:b], compresslevel=1))
    out = tmp_path / "out.kaarme_counts"
    r = subprocess.run([CLI, str(gz), str(k), "-t", "3", "-o", str(out)] + args, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "gzip compressed:          yes" in r.stdout
    assert sorted_digest_file(out) == (case["sorted_sha256"], case["lines"])


def test_cli_default_output_name(golden_input, tmp_path):
    path = golden_input("reads.txt")
    r = subprocess.run([CLI, path, "31", "-s", "100000", "-a", "1"], capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "reads.kaarme_counts").exists()
    r = subprocess.run([CLI, path, "31", "-s", "100000", "-a", "0", "-o", "none.txt"], capture_output=True,
                       text=True, cwd=tmp_path)
    assert r.returncode == 0 and not (tmp_path / "none.txt").exists()  # -a 0 writes nothing


def test_table_full_is_an_error(golden_input, insert_path):
    path = golden_input("reads_w60.fasta")
    with pytest.raises(ka.KcError) as e:
        ka.count_file(path, 31, table_slots=64, min_abundance=1)
    assert e.value.code == -3


def test_counts_sum_to_windows_at_scale(insert_path):
    """Size-independent properties on a larger device-generated input (no N's):
    windows == N*(L-k+1); sum of counts == windows; counting the input twice doubles
    every count; distinct k-mers equal the dumped records at -a 1."""
    torch = pytest.importorskip("torch")
    lib = ka.load_library()
    N, L, G, k = 400_000, 150, 5_000_000, 31
    nbytes = lib.kc_synth_bytes(0, N, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, N, 42, G, L, 0, 0.001, 0.0, 0) == 0
    torch.cuda.synchronize()
    host = bytes(img.cpu().numpy())
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA)
    with ka.KmerCounter(ka.Config(k=k, min_abundance=1, table_slots=30_000_000)) as kc:
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        assert st["windows"] == N * (L - k + 1)
        rec = kc.dump()
        assert rec.shape[0] == st["distinct"]
        assert int(rec[:, -1].sum()) == st["windows"]
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.finish()
        rec2 = kc.dump()
        a = rec[np.lexsort(rec[:, :-1].T[::-1])]
        b = rec2[np.lexsort(rec2[:, :-1].T[::-1])]
        assert np.array_equal(a[:, :-1], b[:, :-1])
        assert np.array_equal(2 * a[:, -1], b[:, -1])


@pytest.mark.parametrize("name,k,args", [("reads_w60.fasta", 31, ["-a", "1", "-s", "1000000"]),
                                         ("reads_w60.fasta", 51, ["-m", "0", "-a", "2", "-s", "1000000"]),
                                         ("long.fasta", 127, ["-a", "1", "-s", "1000000"]),
                                         ("long.fasta", 200, ["-a", "1", "-s", "1000000"])])
@pytest.mark.parametrize("spill", ["list", "full"])
@pytest.mark.parametrize("src", ["host", "device"])
def test_segment_overflow_spills_or_falls_back(name, k, args, spill, src, golden_input, tmp_path, monkeypatch):
    """Tiny forced segment capacities overflow.  spill=list: the keys past a segment's end
    go to the spill list and are inserted through the exact levels after level 3;
    spill=full: the spill list is too small too, so the device redoes the whole batch on
    the exact layout (behind the overflow gate).  Either way the result is the reference's.
    src=device: a device image, whose batch tail the host launches after reading the
    overflow flag and the skew-list length (kc_api.cpp tail_needed)."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_SEG_CAP", "8")
    monkeypatch.setenv("KC_SPILL_CAP", "64" if spill == "full" else str(1 << 24))
    path = golden_input(name)
    o = parse_ref_args(args)
    cfg = ka.Config(k=k, mode=o["mode"], min_abundance=o["min_abundance"], table_slots=o["table_slots"],
                    batch_bytes=64 << 20)
    data = open(path, "rb").read()
    with ka.KmerCounter(cfg) as kc:
        chunks = ka.plan_chunks(data, k, ka.FMT_FASTA)
        if src == "device":
            import torch
            img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
            kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        else:
            for off, ln, bh in chunks:
                kc.count_chunk(data[off:off + ln], ka.FMT_FASTA, bool(bh))
        st = kc.finish()
        if spill == "full":
            assert st["part_fallbacks"] >= 1
        else:
            assert st["part_fallbacks"] == 0 and st["spilled"] > 0
        lines = kc.lines()
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, args, out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


@pytest.mark.parametrize("piece", [0, 1 << 17])
def test_device_text_writer_at_scale(piece, monkeypatch, tmp_path):
    """kc_write formats on the device in pieces (KC_TEXT_PIECE forces small ones, so the
    double-buffered copy-out runs many times): one line per distinct k-mer, the counts
    sum to the windows, and the lines equal the decoded records."""
    torch = pytest.importorskip("torch")
    if piece:
        monkeypatch.setenv("KC_TEXT_PIECE", str(piece))
    lib = ka.load_library()
    N, L, G = 20_000, 150, 1_000_000
    nbytes = lib.kc_synth_bytes(0, N, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, N, 7, G, L, 0, 0.01, 0.001, 0) == 0
    torch.cuda.synchronize()
    host = bytes(img.cpu().numpy())
    for k, mode in ((31, 2), (51, 0), (100, 2)):
        chunks = ka.plan_chunks(host, k, ka.FMT_FASTA)
        with ka.KmerCounter(ka.Config(k=k, mode=mode, min_abundance=1, table_slots=8_000_000)) as kc:
            kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            st = kc.finish()
            out = tmp_path / f"w{k}.txt"
            kc.write(str(out))
            text = open(out).read().splitlines()
            assert len(text) == st["distinct"]
            assert sum(int(l.rsplit(" ", 1)[1]) for l in text) == st["windows"]
            assert sorted(text) == kc.lines()


@pytest.mark.parametrize("k", [5, 31, 51])
def test_fastq_equals_plain_sequence_lines(k, tmp_path):
    """FASTQ input (an extension: the reference rejects it) counts exactly the k-mers of
    its sequence lines: the same as the plain one-sequence-per-line file, which the
    oracle (pinned by the golden fixtures) counts.  Host chunks with small chunk sizes,
    the device-image path, and the CLI."""
    torch = pytest.importorskip("torch")
    from test_host import make_fastq
    fq, pl = make_fastq(4000)
    fqp, plp = tmp_path / "r.fastq", tmp_path / "r.txt"
    fqp.write_bytes(fq)
    plp.write_bytes(pl)
    exp = tmp_path / "exp.txt"
    oracle_count(str(plp), k, ["-a", "1"], exp)
    want = sorted_digest_file(exp)
    kc, st = ka.count_file(str(fqp), k, min_abundance=1, table_slots=1 << 22, chunk_size=5000)
    with kc:
        assert sorted_digest_lines(kc.lines()) == want
    chunks = ka.plan_chunks(fq, k, ka.FMT_FASTQ, 20000)
    dev = torch.frombuffer(bytearray(fq), dtype=torch.uint8).cuda()
    with ka.KmerCounter(ka.Config(k=k, min_abundance=1, table_slots=1 << 22, batch_bytes=1 << 16)) as kc:
        kc.count_device(dev.data_ptr(), chunks, ka.FMT_FASTQ, torch.cuda.current_stream().cuda_stream)
        kc.finish()
        assert sorted_digest_lines(kc.lines()) == want
    out = tmp_path / "cli.txt"
    r = subprocess.run([CLI, str(fqp), str(k), "-t", "3", "-a", "1", "-s", "4000000", "-o", str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert sorted_digest_file(out) == want


@pytest.mark.parametrize("k,fpr", [(31, 0.01), (51, 0.01), (51, 0.001), (95, 0.05)])
def test_bloom_at_scale_equals_exact_solid_kmers(k, fpr, insert_path):
    """Bloom filter (-b, blocked layout) on a larger device-generated input: pass 1 runs
    the partitioned LDS filter (k_b3) or the direct one, pass 2 gates at level 3 (or in
    the direct kernel).  The filter only gates, so every k-mer seen >= 2 times has its
    exact count (the same records as counting without the filter at -a 2), every
    window is seen by both passes, and at most the windows are inserted."""
    torch = pytest.importorskip("torch")
    lib = ka.load_library()
    N, L, G = 300_000, 150, 3_000_000
    nbytes = lib.kc_synth_bytes(0, N, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, N, 11, G, L, 0, 0.002, 0.0, 0) == 0
    torch.cuda.synchronize()
    host = bytes(img.cpu().numpy())
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA)
    with ka.KmerCounter(ka.Config(k=k, min_abundance=2, table_slots=20_000_000)) as kc:
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.finish()
        want = kc.dump()
    # fpr 0.001: ceil(hf) = 10 positions, two per filter word for j >= 8 (repeats counted once)
    with ka.KmerCounter(ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000,
                                  fpr=fpr)) as kc:
        kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        n2 = kc.bloom_finalize()
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        got = kc.dump()
    windows = N * (L - k + 1)
    assert st["windows"] == windows and st["bf_windows"] == windows
    assert st["inserted"] <= windows and n2 > 0
    # the counting pass started from the Bloom pass's level-1 partition (same image, same
    # chunks, one batch) on the segmented path; the direct and exact paths do not keep it
    assert st["reused_passes"] == (1 if insert_path == "partitioned" else 0)
    a = want[np.lexsort(want[:, :-1].T[::-1])]
    b = got[np.lexsort(got[:, :-1].T[::-1])]
    assert np.array_equal(a, b)


def _bloom_job_device(torch, img, chunks, k, count_img=None, count_chunks=None, batch_bytes=0, est_unique=4_000_000):
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=est_unique, fpr=0.01, batch_bytes=batch_bytes)
    with ka.KmerCounter(cfg) as kc:
        kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.bloom_finalize()
        ci = img if count_img is None else count_img
        kc.count_device(ci.data_ptr(), chunks if count_chunks is None else count_chunks, ka.FMT_FASTA)
        st = kc.finish()
        got = kc.dump()
    return st, got[np.lexsort(got[:, :-1].T[::-1])]


@pytest.mark.parametrize("change", ["none", "small_u", "bytes", "chunks", "batches"])
def test_level1_reuse_only_on_the_same_input(change, monkeypatch):
    """Partition reuse (kc_api.cpp): the counting pass starts from the Bloom pass's window
    partitions only for the same image, chunk table and bytes in one batch -- from level 2
    when the table's regions are unions of the fine bins (none), from level 1 when the table
    outgrew the bins sized from -u (small_u).  Bytes changed after the Bloom pass
    (checksum), a different chunk table, or a Bloom pass of several batches run the ordinary
    counting pass; every variant equals the run with reuse off."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    lib = ka.load_library()
    N, L, G, k = 200_000, 150, 2_000_000, 51
    nbytes = lib.kc_synth_bytes(0, N, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, N, 5, G, L, 0, 0.002, 0.0, 0) == 0
    torch.cuda.synchronize()
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    count_img, count_chunks, bb = None, None, 0
    if change == "chunks":
        count_chunks = chunks[: max(1, len(chunks) - 1)]
    elif change == "batches":
        bb = 16 << 20  # (a chunk is up to 10 MiB: several batches)
    def run():
        if change == "bytes":  # same pointer and chunks, bytes changed between the passes
            img2 = img.clone()
            st, got = None, None
            cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=4_000_000, fpr=0.01)
            with ka.KmerCounter(cfg) as kc:
                kc.bloom_device(img2.data_ptr(), chunks, ka.FMT_FASTA)
                kc.bloom_finalize()
                torch.cuda.synchronize()
                seg = img2[1000:1600]
                seg[seg == ord("A")] = ord("C")  # the image changes between the passes
                torch.cuda.synchronize()
                kc.count_device(img2.data_ptr(), chunks, ka.FMT_FASTA)
                st = kc.finish()
                got = kc.dump()
            return st, got[np.lexsort(got[:, :-1].T[::-1])]
        return _bloom_job_device(torch, img, chunks, k, count_img, count_chunks, bb,
                                 est_unique=1_000_000 if change == "small_u" else 4_000_000)
    st, got = run()
    assert st["reused_passes"] == (1 if change in ("none", "small_u") else 0)
    monkeypatch.setenv("KC_REUSE", "0")
    st0, want = run()
    assert st0["reused_passes"] == 0
    assert np.array_equal(got, want)
    # (inserted may differ by count-1 k-mers: which first sightings pass the gate depends on
    # the order of the Bloom insertions, nondeterministic in the reference too)
    assert st["windows"] == st0["windows"] and st["inserted"] <= st["windows"]


@pytest.mark.parametrize("case", [c for c in CASES if c["input"] == "skew.fasta" and "-b" in c["args"]][:1],
                         ids=_case_id)
def test_level1_reuse_declined_on_skewed_input(case, golden_input):
    """Hot keys put heavy records into the Bloom pass's skew list: its partition is not the
    whole input, so the counting pass runs in full (and matches the reference)."""
    torch = pytest.importorskip("torch")
    path = golden_input(case["input"])
    o = parse_ref_args(case["args"])
    image = open(path, "rb").read()
    chunks = ka.plan_chunks(image, case["k"], ka.FMT_FASTA)
    dev = torch.frombuffer(bytearray(image), dtype=torch.uint8).cuda()
    cfg = ka.Config(k=case["k"], mode=o["mode"], min_abundance=o["min_abundance"], bf_enable=True,
                    est_unique=o["est_unique"], fpr=o["fpr"])
    with ka.KmerCounter(cfg) as kc:
        kc.bloom_device(dev.data_ptr(), chunks, ka.FMT_FASTA)
        kc.bloom_finalize()
        kc.count_device(dev.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        lines = kc.lines()
    assert st["reused_passes"] == 0
    assert sorted_digest_lines(lines) == (case["sorted_sha256"], case["lines"])


@pytest.mark.parametrize("spill", ["list", "full"])
@pytest.mark.parametrize("src", ["host", "device"])
def test_bloom_segment_overflow_spills_or_falls_back(spill, src, golden_input, tmp_path, monkeypatch):
    """Forced tiny segments in the partitioned Bloom pass and the gated count pass: spilled
    keys go through the exact levels (spill=list), or both passes are redone on the exact
    layout (spill=full); the result is still the reference's (src=device: host-launched
    batch tails, and no partition reuse after a spill)."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_SEG_CAP", "8")
    monkeypatch.setenv("KC_SPILL_CAP", "64" if spill == "full" else str(1 << 24))
    path = golden_input("reads_w60.fasta")
    args = ["-b", "-u", "200000", "-a", "2"]
    if src == "device":
        import torch
        data = open(path, "rb").read()
        img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        chunks = ka.plan_chunks(data, 31, ka.FMT_FASTA)
        kc = ka.KmerCounter(ka.Config(k=31, min_abundance=2, bf_enable=True, est_unique=200000, fpr=0.01))
        kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.bloom_finalize()
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        assert st["reused_passes"] == 0
    else:
        kc, st = ka.count_file(path, 31, min_abundance=2, bf_enable=True, est_unique=200000, fpr=0.01)
    with kc:
        if spill == "full":
            assert st["part_fallbacks"] >= 2
        else:
            assert st["part_fallbacks"] == 0 and st["spilled"] > 0
        lines = kc.lines()
    out = tmp_path / "oracle.txt"
    oracle_count(path, 31, args, out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


def _job(kc, path, k):
    image = open(path, "rb").read()
    fmt = ka.detect_format(path, image[0])
    chunks = ka.plan_chunks(image, k, fmt)
    for off, ln, bh in chunks:
        kc.bloom_chunk(image[off:off + ln], fmt, bool(bh))
    kc.bloom_finalize()
    for off, ln, bh in chunks:
        kc.count_chunk(image[off:off + ln], fmt, bool(bh))
    kc.finish()
    return kc.lines()


def test_bloom_context_reused_for_a_larger_job(golden_input, tmp_path, insert_path):
    """One Bloom context, two jobs: a small input, kc_reset, then a much larger one.  The
    second table (2 * new_in_second slots) has more regions and more level-1 bins than
    the first, so every partition array must follow the new geometry (the
    level-1 histograms kept their first size)."""
    big = [c for c in CASES if c["input"] == "big_reads.fasta" and "-b" in c["args"]][0]
    o = parse_ref_args(big["args"])
    small = golden_input("reads_w60.fasta")
    with ka.KmerCounter(ka.Config(k=big["k"], mode=2, bf_enable=True, est_unique=o["est_unique"],
                                  min_abundance=o["min_abundance"], batch_bytes=64 << 20)) as kc:
        got = _job(kc, small, big["k"])
        exp = tmp_path / "exp.txt"
        oracle_count(small, big["k"], ["-a", str(o["min_abundance"])], exp)
        assert got == sorted(open(exp).read().splitlines())
        kc.reset()
        lines = _job(kc, golden_input("big_reads.fasta"), big["k"])
        assert sorted_digest_lines(lines) == (big["sorted_sha256"], big["lines"])
        kc.reset()  # and back to a small job on the grown buffers
        assert _job(kc, small, big["k"]) == got


@pytest.mark.parametrize("case", [c for c in CASES if "skew" in c["input"]], ids=_case_id)
@pytest.mark.parametrize("seg", ["default", "tiny"])
def test_skewed_input_uses_the_skew_lists(case, seg, golden_input, tmp_path, monkeypatch):
    """Hot keys (poly-A/T and (CA)n reads, a 300-bp repeat in hundreds of copies, reference
    fixtures): the partitioned path collapses repeated windows into heavy {key, count}
    records and spills what overflows a segment, without redoing the batch; with tiny
    forced segments (seg=tiny) most keys take the spill list."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    if seg == "tiny":
        monkeypatch.setenv("KC_SEG_CAP", "8")
        monkeypatch.setenv("KC_SPILL_CAP", str(1 << 25))
    path = golden_input(case["input"])
    o = parse_ref_args(case["args"])
    kc, st = ka.count_file(path, case["k"], mode=o["mode"], min_abundance=o["min_abundance"],
                           table_slots=max(o["table_slots"], 1 << 16), bf_enable=o["bf_enable"],
                           est_unique=o["est_unique"], fpr=o["fpr"])
    with kc:
        lines = kc.lines()
    assert sorted_digest_lines(lines) == (case["sorted_sha256"], case["lines"])
    # big_skew carries its repeat in 30 % of the genome: what overflows the segments may pass
    # the spill list's capacity (an eighth of the windows), and then the batch is redone
    if case["input"] == "skew.fasta":
        assert st["part_fallbacks"] == 0
    assert st["heavy_records"] > 0 or st["part_fallbacks"] > 0  # the homopolymer reads (a redone batch: none)
    if seg == "tiny":
        assert st["spilled"] > 0


@pytest.mark.parametrize("k,slots", [(51, 1_250_000_000), (127, 1_250_000_000), (51, 567_000_000),
                                     (33, 567_000_000)])
def test_big_table_geometry(tmp_path, k, slots):
    """Tables of the strong presets' size (-s 1.25e9 per GPU; 5.67e8 = the C4 share's
    estimate-sized local table) choose partition geometries whose level-1 and level-2 LDS
    arrays fit (wide keys: more regions per coarse bin, level 2 at half its workgroup; level-1
    runs under 8 keys per tile: fewer, wider coarse bins, 271 x 1024 for 5.67e8); a small input
    through the device path gives the oracle's counts."""
    torch = pytest.importorskip("torch")
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "20000", "300", "100000"], check=True)
    data = open(fa, "rb").read()
    img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=slots)) as kc:
        kc.count_device(img.data_ptr(), ka.plan_chunks(data, k, ka.FMT_FASTA), ka.FMT_FASTA)
        st = kc.finish()
        assert st["part_fallbacks"] == 0
        lines = kc.lines()
    out = tmp_path / "oracle.txt"
    oracle_count(str(fa), k, ["-m", "2", "-a", "1"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


@pytest.mark.parametrize("slots", [200_000_000, 1_250_000_000])
@pytest.mark.parametrize("k,seg", [(31, "default"), (25, "tiny"), (15, "default")])
def test_six_byte_level2_records(tmp_path, k, seg, slots, monkeypatch):
    """One-word keys in tables of >= 2^16 regions (C2's -s 2e8 rounds up to exactly 2^16; -s 1.25e9
    gives 381 952, not a power of two) move 6-byte level-2 records (kc_count_impl.h StoreRec6:
    32 low bits + the offset of the top half inside its region's range).  With tiny segments the
    keys past their segment's end take the skew list beside them."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    if seg == "tiny":
        monkeypatch.setenv("KC_SEG_CAP", "64")
        monkeypatch.setenv("KC_SPILL_CAP", str(1 << 24))
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "30000", "150", "200000", "-s", "5", "-n", "0.001"], check=True)
    data = open(fa, "rb").read()
    img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=slots)) as kc:
        kc.count_device(img.data_ptr(), ka.plan_chunks(data, k, ka.FMT_FASTA), ka.FMT_FASTA)
        st = kc.finish()
        assert st["part_fallbacks"] == 0
        assert st["table_slots"] >= 65536 * 4096
        if seg == "tiny":
            assert st["spilled"] > 0
        lines = kc.lines()
    out = tmp_path / "oracle.txt"
    oracle_count(str(fa), k, ["-m", "2", "-a", "1"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


@pytest.mark.parametrize("slots", [2_000_000, 300_000_000])
@pytest.mark.parametrize("k,seg", [(33, "default"), (51, "default"), (51, "tiny"), (55, "default")])
def test_twelve_byte_table_records(tmp_path, k, seg, slots, monkeypatch):
    """Two-word keys in the counting pass's own geometry (not a power of two: -s 2e6 gives 977
    regions, -s 3e8 146 485) move 12-byte level records (kc_count_impl.h Rec12, R12_REG: x
    recovered from x mod 2^xb and the bin's lowest x) where the bins are narrow enough: k = 33 at
    both levels; k = 51 at level 2 (and level 1 of the big table); k = 55 at level 2 of the big
    table only.  Compared with the oracle."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    if seg == "tiny":
        monkeypatch.setenv("KC_SEG_CAP", "64")
        monkeypatch.setenv("KC_SPILL_CAP", str(1 << 24))
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "30000", "150", "200000", "-s", "7", "-n", "0.001"], check=True)
    data = open(fa, "rb").read()
    img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=slots)) as kc:
        kc.count_device(img.data_ptr(), ka.plan_chunks(data, k, ka.FMT_FASTA), ka.FMT_FASTA)
        st = kc.finish()
        assert st["part_fallbacks"] == 0
        if seg == "tiny" and slots < 10 ** 8:  # (146 485 regions leave every segment short)
            assert st["spilled"] > 0
        got = sorted_digest_lines(kc.lines())
    out = tmp_path / "oracle.txt"
    oracle_count(str(fa), k, ["-m", "2", "-a", "1"], out)
    assert got == sorted_digest_file(out)


@pytest.mark.parametrize("k", [15, 31, 51, 127])
def test_distinct_estimate(tmp_path, k):
    """kc_estimate_distinct_device (HyperLogLog, 2^14 registers, ~0.8 % standard error) against
    the exact distinct count of the same image; it counts nothing (the table stays empty)."""
    torch = pytest.importorskip("torch")
    fa = tmp_path / "r.fasta"
    subprocess.run([GEN, str(fa), "60000", "150", "2000000", "-s", "11", "-n", "0.002"], check=True)
    data = open(fa, "rb").read()
    img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    chunks = ka.plan_chunks(data, k, ka.FMT_FASTA)
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=1 << 24)) as kc:
        est = kc.estimate_distinct_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        est_small = kc.estimate_distinct_device(img.data_ptr(), chunks[:1], ka.FMT_FASTA)
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        assert st["windows"] > 0
        exact = st["distinct"]
    assert abs(est - exact) / exact < 0.04, (est, exact)
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=1 << 24)) as kc:
        kc.count_device(img.data_ptr(), chunks[:1], ka.FMT_FASTA)
        exact_small = kc.finish()["distinct"]
    assert abs(est_small - exact_small) / exact_small < 0.04, (est_small, exact_small)


@pytest.mark.parametrize("name,k", [("reads_w60.fasta", 31), ("edge.fasta", 25), ("long.fasta", 127),
                                    ("big_edge.fasta", 51), ("skew.fasta", 31)])
@pytest.mark.parametrize("chunk_size", [0, 5000, 65537, 100003])
def test_device_chunk_planner_equals_host(name, k, chunk_size, golden_input):
    """kc_plan_chunks_device (the planner reading 64 KiB pages around chunk ends from HBM, used by
    bench.py instead of copying the image to the host) gives kc_plan_chunks' chunk table."""
    torch = pytest.importorskip("torch")
    path = golden_input(name)
    image = open(path, "rb").read()
    fmt = ka.detect_format(path, image[0])
    dev = torch.frombuffer(bytearray(image), dtype=torch.uint8).cuda()
    assert ka.plan_chunks_device(dev.data_ptr(), len(image), k, fmt, chunk_size) == \
        ka.plan_chunks(image, k, fmt, chunk_size)


@pytest.mark.parametrize("chunk_size", [0, 4096, 70000])
def test_device_chunk_planner_fastq_and_plain(chunk_size, tmp_path):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(chunk_size)
    seqs = ["".join("ACGT"[x] for x in rng.integers(0, 4, size=int(rng.integers(20, 300)))) for _ in range(3000)]
    fq = "".join(f"@r{i}\n{s}\n+\n{'@' * len(s)}\n" for i, s in enumerate(seqs)).encode()
    plain = "".join(s + "\n" for s in seqs).encode()
    for data, fmt in ((fq, ka.FMT_FASTQ), (plain, ka.FMT_PLAIN)):
        dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        assert ka.plan_chunks_device(dev.data_ptr(), len(data), 31, fmt, chunk_size) == \
            ka.plan_chunks(data, 31, fmt, chunk_size)


def test_cli_overlapped_upload_equals_one_pass(tmp_path):
    """A -s job on an input of >= 512 MiB counts the image's first half while the second half
    uploads (two counting passes into one table, kc_cli.cpp): the output equals the single-pass
    library run's over the same bytes (digest of every line), and the CLI says it split."""
    import torch
    n, L = 4_000_000, 150  # 0.64 GB of FASTA
    p = tmp_path / "big.fasta"
    subprocess.run([GEN, str(p), str(n), str(L), "5000000", "-s", "7", "-e", "0.001"], check=True)
    out = tmp_path / "out.txt"
    r = subprocess.run([CLI, str(p), "31", "-m", "2", "-s", "60000000", "-a", "1", "-t", "3", "-o", str(out), "--phases"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "overlapped upload" in r.stderr, r.stderr[-2000:]
    host = open(p, "rb").read()
    img = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    chunks = ka.plan_chunks(host, 31, ka.FMT_FASTA)
    with ka.KmerCounter(ka.Config(k=31, mode=2, min_abundance=1, table_slots=60_000_000)) as kc:
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.finish()
        want = kc.output_digest()
    assert ka.same_digest(text_digest(str(out)), want)


@pytest.mark.parametrize("sizing", ["estimate", "auto"])
def test_cli_table_sized_from_estimate(sizing, tmp_path):
    """the CLI sizes a large -s job's table from the input's distinct estimate
    (kc_estimate_distinct_device + kc_size_table inside its timer; auto: when the -s table would pass
    16 GiB) and --digest-only prints the output digest; both equal the oracle's output."""
    n, L = 200_000, 150
    p = tmp_path / "reads.fasta"
    subprocess.run([GEN, str(p), str(n), str(L), "2000000", "-s", "11", "-e", "0.001"], check=True)
    out = tmp_path / "out.txt"
    # auto: an -s whose 25 %-headroom table is > 16 GiB (k = 51: 5 slots per 128-byte bucket)
    s = "4000000" if sizing == "estimate" else "800000000"
    r = subprocess.run([CLI, str(p), "51", "-m", "2", "-s", s, "-a", "1", "-t", "3", "-o", str(out),
                        "--table-sizing", sizing], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sized from the distinct estimate" in r.stdout, r.stdout[-2000:]
    exp = tmp_path / "exp.txt"
    oracle_count(str(p), 51, ["-a", "1"], exp)
    assert ka.same_digest(text_digest(str(out)), text_digest(str(exp)))
    r2 = subprocess.run([CLI, str(p), "51", "-m", "2", "-s", s, "-a", "1", "-t", "3", "-o", str(out),
                         "--table-sizing", sizing, "--digest-only"], capture_output=True, text=True)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    import json
    import re
    got = json.loads(re.search(r"Output digest: (\{.*\})", r2.stdout).group(1))
    assert ka.same_digest(got, text_digest(str(exp)))


def test_size_table_from_estimate(tmp_path):
    """kc_size_table: a job's table sized from its distinct estimate instead of -s (two jobs on one
    context, as bench.py's C4 / C5 steps), the counts equal the oracle's; refused once the job has
    counted and for a Bloom job."""
    import torch
    n, L = 20_000, 150
    p = tmp_path / "reads.fasta"
    subprocess.run([GEN, str(p), str(n), str(L), "400000", "-s", "3", "-e", "0.002"], check=True)
    host = open(p, "rb").read()
    img = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    k = 51
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 300_000)
    exp = tmp_path / "exp.txt"
    oracle_count(str(p), k, ["-a", "1"], exp)
    want = text_digest(str(exp))
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=400_000_000,
                                  batch_bytes=1 << 20)) as kc:
        big = None
        for _ in range(2):
            kc.reset()
            est = kc.estimate_distinct_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            assert abs(est - want["lines"]) < 0.05 * want["lines"], (est, want["lines"])
            kc.size_table(int(1.1 * est) + 4096)
            kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            st = kc.finish()
            assert st["table_slots"] < 400_000_000 // 100
            assert ka.same_digest(kc.output_digest(), want)
            with pytest.raises(ka.KcError, match="counted already"):
                kc.size_table(1 << 20)
        kc.reset()
        kc.size_table(0)  # back to -s
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        big = kc.finish()
        assert big["table_slots"] >= 400_000_000
        assert ka.same_digest(kc.output_digest(), want)
    with ka.KmerCounter(ka.Config(k=k, mode=2, bf_enable=True, est_unique=100_000)) as kb:
        with pytest.raises(ka.KcError, match="Bloom"):
            kb.size_table(1 << 20)
