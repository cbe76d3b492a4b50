"""Deferred level 3: a counting pass over an image of several staging batches
keeps the level-2 segments of a group of batches in HBM and inserts them with one level-3 pass
(one sweep of the table per group instead of per batch; kc_api.cpp plan_deferral / run_deferred).
Results must equal the oracle's (the reference's restatement) and the undeferred pass's, for every
key width and record format, for groups that do not divide the batch count, and when a batch of a
group needs its tail (a skew list, or segments that overflow and send the batch to the exact
pipeline)."""
import pytest

from conftest import oracle_count, sorted_digest_file, sorted_digest_lines, text_digest
import kaarme_amd as ka

pytestmark = pytest.mark.gpu


def _image(tmp_path, n=12_000, L=150, G=400_000, seed=5):
    import torch
    lib = ka.load_library()
    nbytes = lib.kc_synth_bytes(0, n, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, n, seed, G, L, 0, 0.01, 0.001, 0) == 0
    torch.cuda.synchronize()
    host = bytes(img.cpu().numpy())
    path = tmp_path / "img.fasta"
    path.write_bytes(host)
    return img, host, str(path)


def _count(img, host, k, slots, batch, mode=2):
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 200_000)
    with ka.KmerCounter(ka.Config(k=k, mode=mode, min_abundance=1, table_slots=slots, batch_bytes=batch)) as kc:
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        return kc.lines(), st, kc.output_digest()


# (k, table slots): one-word keys in a >= 2^16-region table take 6-byte level-2 records, two-word
# keys 12-byte records, k = 127 whole 32-byte keys; 1.4 G two-word slots (a 35 GB table of 525 coarse
# bins, as the whole C4 job's) run the 1024-thread level 1 (kc_internal.h p1_wide)
@pytest.mark.parametrize("k,slots", [(31, 40_000_000), (31, 2_000_000), (51, 6_000_000), (127, 3_000_000),
                                     (51, 1_400_000_000)])
@pytest.mark.parametrize("group", ["auto", "2"])
def test_deferred_level3_equals_oracle(k, slots, group, tmp_path, monkeypatch):
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    if group != "auto":
        monkeypatch.setenv("KC_DEFER", group)  # 5 batches: groups of 2, 2, 1
    img, host, path = _image(tmp_path)
    lines, st, dig = _count(img, host, k, slots, 400 << 10)
    nb = -(-len(host) // (400 << 10))
    assert st["deferred_level3"] >= 1
    assert st["deferred_level3"] < nb, (st["deferred_level3"], nb)
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, ["-a", "1", "-c", "200000"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)
    assert dig == text_digest(str(out))
    monkeypatch.setenv("KC_DEFER", "0")
    lines0, st0, _ = _count(img, host, k, slots, 400 << 10)
    assert st0["deferred_level3"] == 0
    assert lines0 == lines
    assert st0["distinct"] == st["distinct"] and st0["windows"] == st["windows"]


@pytest.mark.parametrize("k", [31, 51])
@pytest.mark.parametrize("spill", ["list", "full"])
def test_deferred_level3_with_batch_tails(k, spill, tmp_path, monkeypatch):
    """Tiny forced segment capacities: every batch leaves a skew list (list) or overflows its
    segments and is redone on the exact layout (full); the waiting batches of its group are inserted
    first, then the batch's tail runs."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_SEG_CAP", "8")
    monkeypatch.setenv("KC_SPILL_CAP", "64" if spill == "full" else str(1 << 24))
    img, host, path = _image(tmp_path, n=6000)
    lines, st, _ = _count(img, host, k, 4_000_000, 300 << 10)
    nb = -(-len(host) // (300 << 10))
    if spill == "full":
        assert st["part_fallbacks"] >= 1
    else:
        assert st["spilled"] > 0
        # a skew list does not end a group: its batches append to one list, inserted after the
        # group's level 3
        assert st["deferred_level3"] < nb, (st["deferred_level3"], nb)
    assert st["deferred_level3"] >= 1
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, ["-a", "1", "-c", "200000"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


@pytest.mark.parametrize("k", [31, 51])
def test_deferred_group_overflow_after_earlier_skew_lists(k, tmp_path, monkeypatch):
    """The group's skew list holds its earlier batches' entries when a later batch overflows it: those
    entries are inserted after the group's level 3 and the overflowing batch is redone on the exact
    layout (run_deferred).  The list's capacity is 1.5 batches' worth of entries, so the second batch
    of a group overflows it."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_SEG_CAP", "8")
    monkeypatch.setenv("KC_DEFER", "3")
    img, host, path = _image(tmp_path, n=6000)
    nb = -(-len(host) // (300 << 10))
    monkeypatch.setenv("KC_SPILL_CAP", str(1 << 24))
    _, st0, _ = _count(img, host, k, 4_000_000, 300 << 10)
    per_batch = (st0["spilled"] + st0["heavy_records"]) / nb
    assert per_batch > 100
    monkeypatch.setenv("KC_SPILL_CAP", str(int(per_batch * 1.5)))
    lines, st, _ = _count(img, host, k, 4_000_000, 300 << 10)
    assert st["part_fallbacks"] >= 1
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, ["-a", "1", "-c", "200000"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)


def test_deferred_level3_twice_on_one_context(tmp_path, monkeypatch):
    """Two jobs on one context (kc_reset between them), as bench.py times them: the second job's
    groups start from an empty slot set."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_DEFER", "3")
    img, host, path = _image(tmp_path)
    k = 51
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 200_000)
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, ["-a", "1", "-c", "200000"], out)
    groups = []
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=6_000_000, batch_bytes=400 << 10)) as kc:
        for _ in range(2):
            kc.reset()
            kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            st = kc.finish()
            groups.append(st["deferred_level3"])
            assert kc.output_digest() == text_digest(str(out))
    assert groups[0] == groups[1] >= 2  # (groups of 3 batches: the same groups in both jobs)


@pytest.mark.parametrize("k", [31, 51, 127])
def test_deferred_level3_behind_the_bloom_gate(k, tmp_path, monkeypatch):
    """A Bloom job (-b, mode 2 with the gate at level 3) whose counting pass spans several staging
    batches defers its level 3 behind the gate: the k-mers seen twice or more are the
    oracle's exactly (the filter only gates) and a count-1 line is a true singleton, with and without
    the deferral."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_DEFER", "2")
    img, host, path = _image(tmp_path)
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 200_000)

    def job():
        cfg = ka.Config(k=k, mode=2, min_abundance=1, bf_enable=True, est_unique=2_000_000, fpr=0.01,
                        batch_bytes=400 << 10)
        with ka.KmerCounter(cfg) as kc:
            kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            kc.bloom_finalize()
            kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
            return kc.lines(), kc.finish()

    lines, st = job()
    assert st["deferred_level3"] >= 1
    out = tmp_path / "oracle.txt"
    oracle_count(path, k, ["-a", "1", "-c", "200000"], out)
    exact = dict(l.split() for l in open(out).read().splitlines())
    want2 = sorted(f"{km} {c}" for km, c in exact.items() if int(c) >= 2)
    monkeypatch.setenv("KC_DEFER", "0")
    lines0, st0 = job()
    assert st0["deferred_level3"] == 0
    # (Bloom pass 1 is order-dependent for false positives, as the reference's insertion_process with
    # several workers: the singletons that pass the gate may differ between two jobs, so each job is
    # checked on its own)
    for got in (lines, lines0):
        assert sorted(l for l in got if int(l.rsplit(" ", 1)[1]) >= 2) == want2
        assert all(exact.get(l.split()[0]) == "1" for l in got if l.endswith(" 1"))


def test_failed_pass_leaves_no_deferred_group(tmp_path, monkeypatch):
    """a counting pass whose later chunk does not fit a staging batch fails before it
    counts anything (the chunks are checked first), and the context stays usable: host chunks counted
    next on the same context give the oracle's counts for exactly those bytes."""
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_DEFER", "2")
    img, host, path = _image(tmp_path)
    k = 31
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA, 200_000)
    bad = list(chunks)
    off, _, bh = bad[-1]
    bad[-1] = (off, 2 << 20, bh)  # larger than the 400 KiB stage (the bytes are never read)
    with ka.KmerCounter(ka.Config(k=k, mode=2, min_abundance=1, table_slots=4_000_000,
                                  batch_bytes=400 << 10)) as kc:
        with pytest.raises(ka.KcError, match="larger than the staging batch"):
            kc.count_device(img.data_ptr(), bad, ka.FMT_FASTA)
        first = host[chunks[0][0]:chunks[0][0] + chunks[0][1]]
        kc.count_chunk(first, ka.FMT_FASTA, bool(chunks[0][2]))
        st = kc.finish()
        assert st["deferred_level3"] == 0
        lines = kc.lines()
    part = tmp_path / "first.fasta"
    part.write_bytes(first)
    out = tmp_path / "oracle.txt"
    oracle_count(str(part), k, ["-a", "1"], out)
    assert sorted_digest_lines(lines) == sorted_digest_file(out)
