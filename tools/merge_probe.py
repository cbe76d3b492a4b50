"""GPU probe: time the shard-merge inserts on one C2-sized local table's records.
general = kc_insert_counts_device; runs = kc_insert_counts_runs_device on the routed
(table-order) records; runs_shuf = runs on records sorted by region but shuffled within."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "canonical-k-mer-hash-table_amd"))
import kaarme_amd as ka  # noqa: E402
from kaarme_amd.sharded import DeviceEngine  # noqa: E402

N, L, G, k = int(os.environ.get("N", "10000000")), 150, 50_000_000, 31
lib = ka.load_library()
nbytes = lib.kc_synth_bytes(0, N, L, 0)
img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 42, G, L, 0, 0.001, 0.0, 0) == 0
torch.cuda.synchronize()
chunks = ka.plan_chunks(img.cpu().numpy().tobytes(), k, ka.FMT_FASTA)
cfg = ka.Config(k=k, table_slots=200_000_000, min_abundance=2)
e = DeviceEngine(cfg)
e.kc.reset()
e.count(img.data_ptr(), chunks, ka.FMT_FASTA)
recs, counts = e.route_table(1)
torch.cuda.synchronize()
n = counts[0]
rec = recs[: n * 2].view(n, 2).clone()
R = None
owner = e.owner_table()


def run(name, fn):
    for rep in range(3):
        owner.reset()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) * 1e3
    st = owner.finish()
    print(f"{name:10s} {dt:8.3f} ms  distinct {st['distinct']} inserted {st['inserted']}", flush=True)


run("general", lambda: owner.insert_counts_device(rec.data_ptr(), n))
run("runs", lambda: owner.insert_counts_runs_device(rec.data_ptr(), [n]))
# sorted by region, shuffled inside
print("shuffling", flush=True)
R = owner.finish()["table_slots"] // (512 * 8)
hi = (rec[:, 0] >> 32) & 0xFFFFFFFF
region = (hi * R) >> 32
key = region * (1 << 31) + torch.randint(0, 1 << 31, (n,), device="cuda")
order = torch.sort(key).indices
rec2 = rec[order].contiguous()
torch.cuda.synchronize()
print("shuffled", flush=True)
run("runs_shuf", lambda: owner.insert_counts_runs_device(rec2.data_ptr(), [n]))
