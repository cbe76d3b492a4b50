"""CPU: the C-ABI library loads and exports the boundary; host logic of the engine
(reference chunking, format detection, CLI option semantics, generator sizes) --
nothing here launches a kernel."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import CLI, GEN, LIB, ORACLE, REPO, golden_input  # noqa: F401
import kaarme_amd as ka

HEADER = os.path.join(REPO, "include", "kc_api.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(kc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 15
    lib = ctypes.CDLL(LIB)
    for s in syms:
        assert hasattr(lib, s), s
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in nm.splitlines() if l.strip())
    assert set(syms) <= exported
    assert set(ka.EXPORTS) == set(syms)


def oracle_chunks(path, k, chunk):
    out = subprocess.run([ORACLE, "chunks", path, str(k), "-c", str(chunk)], capture_output=True, text=True,
                         check=True).stdout.split()
    return [tuple(int(x) for x in out[i:i + 3]) for i in range(0, len(out), 3)]


@pytest.mark.parametrize("name", ["reads_w60.fasta", "edge.fasta", "edge.txt", "long.fasta"])
@pytest.mark.parametrize("k", [1, 2, 31, 51, 127])
def test_plan_chunks_matches_oracle_small_chunks(name, k, golden_input):
    """read_chunk_from_file's overlap / fake-symbol / broken_header logic at many
    boundaries (tiny chunk sizes put boundaries inside headers and wrapped lines)."""
    path = golden_input(name)
    image = open(path, "rb").read()
    fmt = ka.detect_format(path, image[0])
    for chunk in (k + 1, 97, 1000, 4093, 65536):
        if chunk <= k:
            continue
        got = ka.plan_chunks(image, k, fmt, chunk)
        assert got == oracle_chunks(path, k, chunk), (chunk,)


def test_plan_chunks_big_input_has_broken_headers(golden_input):
    path = golden_input("big_edge.fasta")
    image = open(path, "rb").read()
    got = ka.plan_chunks(image, 31, ka.FMT_FASTA)
    assert got == oracle_chunks(path, 31, 10 << 20)
    assert len(got) >= 3 and any(bh for _, _, bh in got)


def test_synth_bytes_matches_cpu_generator(tmp_path):
    lib = ka.load_library()
    for (n, L, w) in [(1000, 150, 0), (37, 5000, 60), (12345, 100, 0), (1, 31, 7)]:
        p = tmp_path / "g.fa"
        args = [GEN, str(p), str(n), str(L), str(max(L, 20000))] + (["-w", str(w)] if w else [])
        subprocess.run(args, check=True)
        assert lib.kc_synth_bytes(0, n, L, w) == os.path.getsize(p)
    # a slice [first, first+count) has the bytes of its records
    full = tmp_path / "full.fa"
    part = tmp_path / "part.fa"
    subprocess.run([GEN, str(full), "2000", "150", "50000"], check=True)
    subprocess.run([GEN, str(part), "2000", "150", "50000", "--first", "990", "--count", "20"], check=True)
    data = open(full, "rb").read()
    off = lib.kc_synth_bytes(0, 990, 150, 0)
    assert data[off:off + os.path.getsize(part)] == open(part, "rb").read()


def test_detect_format():
    assert ka.detect_format("x.fasta", ord(">")) == ka.FMT_FASTA
    assert ka.detect_format("x.fa", ord(">")) == ka.FMT_FASTA
    assert ka.detect_format("x.fq", ord("@")) == ka.FMT_FASTQ
    assert ka.detect_format("x.txt", ord("a")) == ka.FMT_PLAIN
    with pytest.raises(ValueError):
        ka.detect_format("x.fasta", ord("A"))
    with pytest.raises(ValueError):
        ka.detect_format("x.txt", ord(">"))


def run_cli(*args, cwd=None):
    return subprocess.run([CLI] + [str(a) for a in args], capture_output=True, text=True, cwd=cwd)


def test_cli_option_semantics(golden_input, tmp_path):
    """CLI11 semantics of main.cpp:127-156 (exit codes = CLI11 ExitCodes)."""
    fa = golden_input("reads_w60.fasta")
    assert run_cli(fa, 31).returncode == 106                         # neither -s nor -u
    assert run_cli(fa, 31, "-s", 10, "-u", 10, "-b").returncode == 106  # both
    assert run_cli(fa, 31, "-u", 1000).returncode == 107             # -u needs -b
    assert run_cli(fa, 31, "-s", 1000, "-b").returncode in (106, 107)  # -b needs -u
    assert run_cli(fa, 31, "-s", 1000, "-f", 0.1).returncode == 107  # -f needs -b
    assert run_cli(fa, 31, "-b", "-u", "4e8").returncode == 104      # integers only
    assert run_cli(fa, 31, "-s", 1000, "-t", 2).returncode == 105    # -t in 3..64
    assert run_cli(fa, 31, "-s", 1000, "-m", 3).returncode == 105    # -m in 0..2
    assert run_cli(fa, 0, "-s", 1000).returncode == 105              # KLEN > 0
    assert run_cli(tmp_path / "missing.fa", 31, "-s", 1000).returncode == 105
    assert run_cli(fa).returncode == 106
    assert run_cli("-h").returncode == 0
    # k above KC_MAX_K (fifteen key words) is refused with a message (INTEGRATION.md Differences)
    r = run_cli(fa, 480, "-s", 1000, "-o", tmp_path / "big_k.txt")
    assert r.returncode == 1 and "above 479" in r.stderr and not (tmp_path / "big_k.txt").exists()


def test_cli_format_checks(tmp_path):
    bad = tmp_path / "bad.fasta"
    bad.write_bytes(b"ACGT\n")
    r = run_cli(bad, 5, "-s", 100)
    assert r.returncode == 1 and "ill-formed" in r.stderr
    fq = tmp_path / "r.fq"
    fq.write_bytes(b"ACGT\n")  # FASTQ must start with '@' (FASTQ input is an extension, test_gpu_parity)
    r = run_cli(fq, 3, "-s", 100, "-o", tmp_path / "out.txt")
    assert r.returncode == 1 and "ill-formed" in r.stderr
    assert not (tmp_path / "out.txt").exists()


def test_cli_gzip_format_checks(tmp_path):
    """gzip input: the format comes from the name without its .gz suffix and the first
    decompressed byte; a truncated stream is an error, never a silently shorter input."""
    import gzip
    good = gzip.compress(b">r0\n" + b"ACGTTGCA" * 5000 + b"\n")
    bad = tmp_path / "bad.txt.gz"
    bad.write_bytes(gzip.compress(b">r0\nACGT\n"))  # plain text must not start with '>'
    r = run_cli(bad, 5, "-s", 100)
    assert r.returncode == 1 and "ill-formed" in r.stderr
    cut = tmp_path / "cut.fasta.gz"
    cut.write_bytes(good[: len(good) // 2])
    r = run_cli(cut, 5, "-s", 100, "-o", tmp_path / "out.txt")
    assert r.returncode == 1 and "corrupt or truncated" in r.stderr
    assert not (tmp_path / "out.txt").exists()


def make_fastq(n, seed=5, maxlen=300):
    """4-line FASTQ records with N's, lowercase, and quality lines that begin with '@'
    or '+' (the cases a naive record finder gets wrong); returns (fastq, plain) bytes,
    plain = the sequence lines only (what the FASTQ counts must equal)."""
    import random
    rng = random.Random(seed)
    fq, pl = [], []
    for i in range(n):
        L = rng.randint(0, maxlen)
        seq = "".join(rng.choice("ACGTACGTACGTacgtN") for _ in range(L))
        qual = "".join(rng.choice("@+!#IJ") for _ in range(L))
        fq.append(f"@read{i} x\n{seq}\n+{'' if i % 2 else 'read' + str(i)}\n{qual}\n")
        pl.append(seq + "\n")
    return "".join(fq).encode(), "".join(pl).encode()


def test_fastq_chunks_are_whole_records():
    fq, _ = make_fastq(3000)
    for cs in (0, 997, 4096, 100003):
        ch = ka.plan_chunks(fq, 31, ka.FMT_FASTQ, cs)
        assert ch[0][0] == 0 and sum(ln for _, ln, _ in ch) == len(fq)
        pos = 0
        for off, ln, bh in ch:
            assert off == pos and bh == 0
            assert fq[off:off + 1] == b"@" and fq[off:off + ln].count(b"\n") % 4 == 0
            pos = off + ln


def test_committed_traffic_book_covers_the_bench_workloads():
    """bench.py's roofline.traffic comes from profiles/pmc_traffic.json, keyed by the
    workload string of each bench line: every committed v11 bench line must find its entry."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for name in ("c2", "c3", "c4s", "c5s"):
        line = json.load(open(os.path.join(root, "profiles", f"r01_v11_bench_{name}.json")))
        got, entry = bench.load_traffic(line["config"]["workload"])
        assert got and got > line["roofline"]["algorithmic_bytes_per_launch"] * 0.5, name
        assert entry["bytes_per_launch"] == got


def _bgzf(data, block=60000):
    """BGZF (bgzip's blocked gzip): members of <= 64 KiB with their size in a 'BC' extra field,
    ending with the empty EOF member."""
    import struct
    import zlib

    out = bytearray()
    for chunk in [data[i:i + block] for i in range(0, len(data), block)] + [b""]:
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        cd = c.compress(chunk) + c.flush()
        bsize = 18 + len(cd) + 8
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 6) + b"BC"
        out += struct.pack("<HH", 2, bsize - 1) + cd + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    return bytes(out)


def test_cli_gunzip_bgzf_parallel_and_streams(golden_input, tmp_path):
    """gzip input (an extension): BGZF members inflate in parallel into their slots;
    other gzip files (one or several members) go through one zlib stream; a corrupt member fails."""
    import gzip

    data = open(golden_input("reads_w60.fasta"), "rb").read() * 3
    bz = _bgzf(data)
    assert gzip.decompress(bz) == data  # the writer above makes valid gzip
    src = tmp_path / "r.fasta.gz"
    src.write_bytes(bz)
    out = tmp_path / "out.bin"
    r = run_cli(src, 31, "-s", 1000, "--gunzip-to", out)
    assert r.returncode == 0 and "BGZF, parallel" in r.stdout, r.stderr
    assert out.read_bytes() == data
    # plain multi-member gzip: one stream
    mm = tmp_path / "m.fasta.gz"
    mm.write_bytes(gzip.compress(data[:100000]) + gzip.compress(data[100000:]))
    r = run_cli(mm, 31, "-s", 1000, "--gunzip-to", out)
    assert r.returncode == 0 and "BGZF" not in r.stdout and out.read_bytes() == data
    # a corrupt BGZF member (a byte of the second member's deflate data flipped)
    bad = bytearray(bz)
    second = bz.index(b"\x1f\x8b\x08\x04", 1)
    bad[second + 40] ^= 0xFF
    badp = tmp_path / "bad.fasta.gz"
    badp.write_bytes(bytes(bad))
    r = run_cli(badp, 31, "-s", 1000, "--gunzip-to", out)
    assert r.returncode == 1 and "corrupt" in r.stderr
    # a forged ISIZE: the first member claims 4 GiB -- rejected as corrupt, not
    # allocated (BGZF members hold at most 64 KiB)
    forged = bytearray(bz)
    first_end = bz.index(b"\x1f\x8b\x08\x04", 1)
    forged[first_end - 4:first_end] = (0xFFFFFFF0).to_bytes(4, "little")
    fp = tmp_path / "forged.fasta.gz"
    fp.write_bytes(bytes(forged))
    r = run_cli(fp, 31, "-s", 1000, "--gunzip-to", out)
    assert r.returncode == 1 and "corrupt" in r.stderr, (r.returncode, r.stderr[-500:])
