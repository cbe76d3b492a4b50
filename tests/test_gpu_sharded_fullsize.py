"""The whole C4 job through the sharded merge at 8 ranks (the exchange and the
owner insert at full size), on one GPU with the ranks emulated in turn: every rank counts its 1/8
of the 100 M reads into its local table (sized from the distinct estimate, one size for every rank
as bench.py's ranks agree on it), routes the table as owner-grouped {key, count} records
(kc_route_table_device, ShardedCounter's route), and every owner adds the groups addressed to it, in
rank order, into its owner table (kc_insert_counts_runs_device: the region-sorted runs merge).  The
owners' output digests combined (kc_output_digest, bench.py's N > 1 parity record) must equal the
whole job's digest in tests/golden/fullsize.json (C4: the pinned CPU restatement's), and the owners'
distinct k-mers must add up to the job's.  The all-to-all itself is data movement checked by
per-peer sums (kaarme_amd.sharded.exchange; tests/test_sharded.py, tests/test_gpu_sharded_mp.py).
"""
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_c4_whole_job_through_the_merge_at_8_ranks():
    import torch
    import kaarme_amd as ka
    from kaarme_amd.sharded import DeviceEngine

    doc = json.load(open(os.path.join(GOLDEN, "fullsize.json")))
    fx = doc["cases"].get("C4")
    if not fx or not fx.get("digest"):
        pytest.skip("no C4 whole-job digest")
    G, N, L, genome, k, slots = 8, 100_000_000, 150, 500_000_000, 51, 2_600_000_000
    lib = ka.load_library()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    W = ka.words_for_k(k)

    def image(r):
        first = N * r // G
        n = N * (r + 1) // G - first
        nbytes = lib.kc_synth_bytes(first, n, L, 0)
        img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        assert lib.kc_synth_device(img.data_ptr(), first, n, 42, genome, L, 0, 0.001, 0.0, stream) == 0
        torch.cuda.synchronize()
        return img, ka.plan_chunks_device(img.data_ptr(), nbytes, k, ka.FMT_FASTA), n * (L - k + 1)

    # the ranks' distinct estimates, one local-table size for all (the max, as bench.py's ranks agree)
    est = []
    for r in range(G):
        img, chunks, _ = image(r)
        with ka.KmerCounter(ka.Config(k=k, mode=2, table_slots=1 << 16, batch_bytes=2 << 30)) as probe:
            est.append(probe.estimate_distinct_device(img.data_ptr(), chunks, ka.FMT_FASTA, stream))
        del img
    local_slots = int(1.1 * max(est)) + (1 << 20)
    cfg = ka.Config(k=k, mode=2, table_slots=-(-slots // G), min_abundance=1, batch_bytes=2 << 30)
    recs, groups, windows, local_distinct = [], [], 0, 0
    for r in range(G):
        img, chunks, win = image(r)
        eng = DeviceEngine(cfg, local_slots=local_slots, world=G)
        eng.count(img.data_ptr(), chunks, ka.FMT_FASTA, stream)
        rec, counts = eng.route_table(G, stream)
        torch.cuda.synchronize()
        st = eng.kc.finish()
        assert st["windows"] == win
        windows += st["windows"]
        local_distinct += st["distinct"]
        assert sum(counts) == st["distinct"]
        recs.append(rec[: sum(counts) * (W + 1)].clone())
        groups.append(counts)
        eng.close()
        del img, rec
        torch.cuda.empty_cache()
    assert windows == fx["count_sum"]
    digests, distinct = [], 0
    owner_cfg = ka.Config(k=k, mode=2, table_slots=local_slots, min_abundance=1)  # the local tables' geometry
    for o in range(G):
        parts, gc = [], []
        for r in range(G):
            lo = sum(groups[r][:o]) * (W + 1)
            parts.append(recs[r][lo: lo + groups[r][o] * (W + 1)])
            gc.append(groups[r][o])
        recv = torch.cat(parts)
        with ka.KmerCounter(owner_cfg) as own:
            own.insert_counts_runs_device(recv.data_ptr(), gc, stream)
            st = own.finish()
            distinct += st["distinct"]
            digests.append(own.output_digest())
        del recv
    assert distinct == fx["distinct"]
    got = ka.combine_digests(digests)
    assert ka.same_digest(got, fx["digest"]), (got, fx["digest"])
    assert local_distinct > distinct  # (k-mers seen by several ranks merged at their owner)
