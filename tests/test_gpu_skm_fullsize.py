"""The whole C4 job through the super-k-mer exchange at G ranks, on one GPU with
the ranks emulated in turn: every rank tokenizes its 1/G of the 100 M reads and routes its windows
as super-k-mers to their canonical-minimizer owners (kc_route_superkmers_device); every owner counts
the streams addressed to it by all ranks, concatenated in rank order as the all-to-all delivers them
(kc_count_packed_device), into its own table at its 1/G share of -s.  The owners' output digests
combined (bench.py's N > 1 parity record) must equal the whole job's digest in
tests/golden/fullsize.json (C4: the pinned CPU restatement's), the owners' windows must add up to the
job's, and the bytes a rank sends must be the few the design promises.  The times of the
route and of each owner's count are printed (`-s`): the per-rank work of a G-GPU step.
"""
import json
import os
import time

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def emulate(G, out=None):
    import torch
    import kaarme_amd as ka
    from kaarme_amd.sharded import owner_share

    doc = json.load(open(os.path.join(GOLDEN, "fullsize.json")))
    fx = doc["cases"]["C4"]
    N, L, genome, k, slots = 100_000_000, 150, 500_000_000, 51, 2_600_000_000
    lib = ka.load_library()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    route = ka.KmerCounter(ka.Config(k=k, mode=2, table_slots=1 << 16, batch_bytes=2 << 30))
    rec = {"G": G, "route_ms": [], "count_ms": [], "sent_bytes": [], "windows": 0}
    streams = [[] for _ in range(G)]  # per owner: (pk, bk, words, windows) from every rank
    for r in range(G):
        first = N * r // G
        n = N * (r + 1) // G - first
        nbytes = lib.kc_synth_bytes(first, n, L, 0)
        img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        assert lib.kc_synth_device(img.data_ptr(), first, n, 42, genome, L, 0, 0.001, 0.0, stream) == 0
        torch.cuda.synchronize()
        chunks = ka.plan_chunks_device(img.data_ptr(), nbytes, k, ka.FMT_FASTA)
        need, _ = route.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, G, stream=stream)
        cap = int(max(need) * 1.05) + 64
        pk = torch.empty(G * cap + 2, dtype=torch.int64, device="cuda")
        bk = torch.empty(G * cap + 2, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        words, wins = route.route_superkmers_device(img.data_ptr(), chunks, ka.FMT_FASTA, G, pk.data_ptr(),
                                                    bk.data_ptr(), cap, stream=stream)
        torch.cuda.synchronize()
        rec["route_ms"].append(round((time.perf_counter() - t0) * 1e3, 2))
        assert words == need and sum(wins) == n * (L - k + 1)
        rec["windows"] += sum(wins)
        rec["sent_bytes"].append(sum(w for o, w in enumerate(words) if o != r) * 12)
        for o in range(G):
            streams[o].append((pk[o * cap: o * cap + words[o]].clone(), bk[o * cap: o * cap + words[o]].clone(),
                               words[o], wins[o]))
        del img, pk, bk
        torch.cuda.empty_cache()
    route.close()
    assert rec["windows"] == fx["count_sum"]
    digests, distinct = [], 0
    # one owner context for every owner in turn (kc_reset between them), as a rank keeps its owner
    # table and partition buffers from step to step; a first owner job warms it up
    cfg = ka.Config(k=k, mode=2, table_slots=owner_share(slots, G), min_abundance=1)
    kc = ka.KmerCounter(cfg)
    for o in [0] + list(range(G)):
        pk = torch.cat([s[0] for s in streams[o]] + [streams[o][0][0].new_zeros(2)])
        bk = torch.cat([s[1] for s in streams[o]] + [streams[o][0][1].new_zeros(2)])
        n_words, windows = sum(s[2] for s in streams[o]), sum(s[3] for s in streams[o])
        kc.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kc.count_packed_device(pk.data_ptr(), bk.data_ptr(), n_words, windows, stream)
        st = kc.finish()
        ms = round((time.perf_counter() - t0) * 1e3, 2)
        del pk, bk
        if "warm" not in rec:
            rec["warm"] = ms
            continue
        streams[o] = None
        rec["count_ms"].append(ms)
        rec.setdefault("owner_stats", []).append({x: st[x] for x in ("deferred_level3", "part_fallbacks",
                                                                      "spilled", "heavy_records", "distinct")})
        assert st["windows"] == windows
        distinct += st["distinct"]
        digests.append(kc.output_digest())
        torch.cuda.empty_cache()
    kc.close()
    rec["distinct"] = distinct
    rec["digest"] = ka.combine_digests(digests)
    rec["match"] = distinct == fx["distinct"] and ka.same_digest(rec["digest"], fx["digest"])
    rec["bytes_per_window_sent"] = round(sum(rec["sent_bytes"]) / rec["windows"] * G / (G - 1), 4)
    if out:
        with open(out, "w") as f:
            json.dump(rec, f)
    return rec


@pytest.mark.timeout(900)
@pytest.mark.parametrize("G", [8])
def test_c4_whole_job_through_superkmers(G):
    rec = emulate(G)
    print(json.dumps(rec))
    assert rec["match"], rec
    # about 1.6 bytes per window at 8 ranks (10.8 GB of records per rank in round 5)
    assert max(rec["sent_bytes"]) < 2.5e9, rec["sent_bytes"]


if __name__ == "__main__":
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "canonical-k-mer-hash-table_amd"))
    for g in map(int, sys.argv[2:] or ["8"]):
        print(json.dumps(emulate(g, sys.argv[1].replace("G", str(g)) if len(sys.argv) > 1 else None)), flush=True)
