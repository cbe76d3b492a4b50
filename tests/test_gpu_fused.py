"""The fused Bloom + counting pass (kc_api.cpp run_batch, kc_count_impl.h
k_bf3 / k_bprobe): a one-batch Bloom pass over a device image counts its kept level-2 keys
behind the gate in the same workgroup that built the region's filter blocks, into a table
sized from a sample of the kept bins; the counting pass only confirms the input (checksum).

The fused pass is opt-in (KC_FUSE=1; it measured slower than the two kernels it fuses).
The filter only gates: every k-mer seen at least twice has its exact count,
so the fused job's records at -a 2 equal the records of the same job with the fused pass off
(KC_FUSE=0: k_b3, then the gated k_p3 from the kept partitions), and those of counting without
the filter.  Every way of leaving the fused pass's table unused (other bytes, other chunks,
host chunks, reading the table before the counting pass, a region the probe underestimated)
must give the reference's result too.
"""
import numpy as np
import pytest

import kaarme_amd as ka

pytestmark = pytest.mark.gpu


def _image(torch, N, L, G, seed, err=0.002):
    lib = ka.load_library()
    nbytes = lib.kc_synth_bytes(0, N, L, 0)
    img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert lib.kc_synth_device(img.data_ptr(), 0, N, seed, G, L, 0, err, 0.0, 0) == 0
    torch.cuda.synchronize()
    return img


def _sorted(recs):
    return recs[np.lexsort(recs[:, :-1].T[::-1])]


def _bloom_job(kc, img, chunks, count_img=None):
    kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
    kc.bloom_finalize()
    kc.count_device((img if count_img is None else count_img).data_ptr(), chunks, ka.FMT_FASTA)
    st = kc.finish()
    return st, _sorted(kc.dump())


def _exact_solid(img, chunks, k):
    with ka.KmerCounter(ka.Config(k=k, min_abundance=2, table_slots=40_000_000)) as kc:
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.finish()
        return _sorted(kc.dump())


@pytest.fixture
def partitioned(monkeypatch):
    monkeypatch.setenv("KC_INSERT_PATH", "partitioned")
    monkeypatch.setenv("KC_FUSE", "1")  # (opt-in: kc_api.cpp fuse_enabled)


@pytest.mark.parametrize("k,fpr", [(31, 0.01), (51, 0.01), (51, 0.001), (95, 0.05), (127, 0.01)])
def test_fused_equals_unfused_and_exact(k, fpr, partitioned, monkeypatch):
    torch = pytest.importorskip("torch")
    N, L, G = 300_000, 150, 3_000_000
    img = _image(torch, N, L, G, 11)
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    want = _exact_solid(img, chunks, k)
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=fpr)
    with ka.KmerCounter(cfg) as kc:
        st, got = _bloom_job(kc, img, chunks)
    windows = N * (L - k + 1)
    assert st["windows"] == windows and st["bf_windows"] == windows
    assert st["reused_passes"] == 1 and st["reuse_level"] == 3, st
    assert 0 < st["inserted"] <= windows
    assert np.array_equal(got, want)
    monkeypatch.setenv("KC_FUSE", "0")
    with ka.KmerCounter(cfg) as kc:
        st0, got0 = _bloom_job(kc, img, chunks)
    assert st0["reuse_level"] in (1, 2) and st0["reused_passes"] == 1
    assert np.array_equal(got0, want)
    assert st["windows"] == st0["windows"]


def test_fused_region_overflow_falls_back(partitioned, monkeypatch):
    """KC_FUSE_R forces fewer table regions than the gated keys need: regions overflow, the
    fused table is dropped at kc_bloom_finalize and the counting pass runs from the kept
    level 2 into the reference-sized table."""
    torch = pytest.importorskip("torch")
    k = 51
    img = _image(torch, 300_000, 150, 3_000_000, 12)
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    want = _exact_solid(img, chunks, k)
    # -u 8e6: 2^19 filter blocks, 8192 fine bins; 512 regions (the fewest the fused kernel takes:
    # 1024 blocks each) hold 1.3 M slots for ~2.6 M k-mers that pass the gate
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=0.01)
    monkeypatch.setenv("KC_FUSE_R", "512")
    with ka.KmerCounter(cfg) as kc:
        st, got = _bloom_job(kc, img, chunks)
    assert st["reuse_level"] != 3, st
    assert np.array_equal(got, want)


@pytest.mark.parametrize("how", ["bytes", "other_image", "chunks", "host_chunks", "dump_first", "second_bloom_batch"])
def test_fused_table_dropped_when_not_confirmed(how, partitioned, monkeypatch):
    """The fused pass's table stands only for a counting pass over the same bytes and chunk
    table; otherwise (and when the table is read before the counting pass) it is dropped and
    the ordinary counting pass runs: the same records as the job with partition reuse off."""
    torch = pytest.importorskip("torch")
    k = 31
    img = _image(torch, 200_000, 150, 2_000_000, 13)
    host = bytes(img.cpu().numpy())
    chunks = ka.plan_chunks(host, k, ka.FMT_FASTA)
    assert len(chunks) > 1
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=4_000_000, fpr=0.01)

    def run():
        work = img.clone()
        with ka.KmerCounter(cfg) as kc:
            kc.bloom_device(work.data_ptr(), chunks, ka.FMT_FASTA)
            if how == "second_bloom_batch":  # the filter changes after the fused pass ran
                kc.bloom_device(work.data_ptr(), chunks, ka.FMT_FASTA)
            kc.bloom_finalize()
            count_img, count_chunks = work, chunks
            if how == "bytes":  # same pointer and chunks, bytes changed between the passes
                torch.cuda.synchronize()
                seg = work[5000:9000]
                seg[seg == ord("A")] = ord("C")
                torch.cuda.synchronize()
            elif how == "other_image":
                count_img = work.clone()
            elif how == "chunks":
                count_chunks = chunks[:-1]
            if how == "dump_first":
                assert len(kc.dump()) == 0  # nothing is counted before the counting pass
            if how == "host_chunks":
                for off, ln, bh in chunks:
                    kc.count_chunk(host[off:off + ln], ka.FMT_FASTA, bool(bh))
            else:
                kc.count_device(count_img.data_ptr(), count_chunks, ka.FMT_FASTA)
            st = kc.finish()
            return st, _sorted(kc.dump())

    st, got = run()
    assert st["reused_passes"] == 0, st  # (a copy of the same bytes is another input to the ABI)
    monkeypatch.setenv("KC_REUSE", "0")
    st0, want = run()
    assert np.array_equal(got, want)
    assert st["windows"] == st0["windows"]


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_one_context_small_big_small_jobs(partitioned, monkeypatch, fuse):
    """one Bloom context, device-image jobs of growing and shrinking size with
    kc_reset between them (kc_reset applies the fine geometry the last kc_bloom_finalize
    learned): each job counts from its own fused pass (reuse_level 3) or, by default, from the
    Bloom pass's kept partitions (level 2 or 1), the table follows each job's size, and every
    job equals the exact solid records."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("KC_FUSE", fuse)
    k = 51
    small = _image(torch, 50_000, 150, 500_000, 21)
    big = _image(torch, 400_000, 150, 4_000_000, 22)
    cs = ka.plan_chunks(bytes(small.cpu().numpy()), k, ka.FMT_FASTA)
    cb = ka.plan_chunks(bytes(big.cpu().numpy()), k, ka.FMT_FASTA)
    ws, wb = _exact_solid(small, cs, k), _exact_solid(big, cb, k)
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=0.01)
    with ka.KmerCounter(cfg) as kc:
        slots = []
        for img, ch, want in ((small, cs, ws), (big, cb, wb), (small, cs, ws), (big, cb, wb)):
            st, got = _bloom_job(kc, img, ch)
            assert st["reuse_level"] in ((3,) if fuse == "1" else (1, 2)) and st["reused_passes"] == 1, st
            assert np.array_equal(got, want)
            slots.append(st["table_slots"])
            kc.reset()
    assert slots[1] > slots[0] and slots[2] == slots[0] and slots[3] == slots[1]


def test_fused_two_steps_one_context(partitioned):
    """bench.py's C3 step twice on one context: the second job, after
    kc_reset, gives the same records as the first."""
    torch = pytest.importorskip("torch")
    k = 51
    img = _image(torch, 300_000, 150, 3_000_000, 23)
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=0.01)
    with ka.KmerCounter(cfg) as kc:
        st1, a = _bloom_job(kc, img, chunks)
        kc.reset()
        st2, b = _bloom_job(kc, img, chunks)
    assert st1["reuse_level"] == st2["reuse_level"] == 3
    assert np.array_equal(a, b)


def test_gated_table_overflow_redoes_the_count(partitioned, monkeypatch):
    """The counting pass from the kept partitions into a table too small for the gated k-mers
    (KC_BF_TABLE=tiny: an eighth of new_in_second; KC_BF_TABLE=fit sizes it new_in_second + 30 %):
    a region overflows, and the ordinary counting pass redoes the batch into the reference-sized
    table (2 x new_in_second) with the counters as they were."""
    torch = pytest.importorskip("torch")
    k = 51
    img = _image(torch, 300_000, 150, 3_000_000, 14)
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    want = _exact_solid(img, chunks, k)
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=0.01)
    monkeypatch.setenv("KC_FUSE", "0")
    with ka.KmerCounter(cfg) as kc:
        st_ok, got_ok = _bloom_job(kc, img, chunks)
    monkeypatch.setenv("KC_BF_TABLE", "tiny")
    with ka.KmerCounter(cfg) as kc:
        st, got = _bloom_job(kc, img, chunks)
    assert st_ok["reused_passes"] == 1 and st["reused_passes"] == 0
    assert st["windows"] == st_ok["windows"] == 300_000 * (150 - k + 1)
    assert np.array_equal(got, want) and np.array_equal(got_ok, want)
