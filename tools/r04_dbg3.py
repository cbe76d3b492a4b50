"""Debug: owner-sharded Bloom filter fill and counters vs one filter (emulated ranks)."""
import os, sys, subprocess, tempfile
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "canonical-k-mer-hash-table_amd"))
import numpy as np
import torch
import kaarme_amd as ka
from kaarme_amd.sharded import DeviceEngine
GEN = os.path.join(REPO, "canonical-k-mer-hash-table_amd", "bin", "kc_gen")
td = tempfile.mkdtemp()
fa = os.path.join(td, "w.fasta")
subprocess.run([GEN, fa, "16000", "150", "40000"], check=True)
data = open(fa, "rb").read()
img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
k = 31
ch = ka.plan_chunks(data, k, ka.FMT_FASTA)
with ka.KmerCounter(ka.Config(k=k, mode=2, table_slots=4_000_000, min_abundance=1)) as kc:
    kc.count_device(img.data_ptr(), ch, ka.FMT_FASTA)
    st = kc.finish()
    recs = kc.dump()
distinct = st["distinct"]
solid = int((recs[:, -1] >= 2).sum())
print("distinct", distinct, "solid", solid, flush=True)

def fill(kc):
    w = kc.bloom_read().reshape(-1, 16)
    f1 = np.unpackbits(w[:, :8].view(np.uint8)).mean()
    f2 = np.unpackbits(w[:, 8:].view(np.uint8)).mean()
    return round(float(f1), 4), round(float(f2), 4)

cfg = ka.Config(k=k, mode=2, bf_enable=True, est_unique=distinct, fpr=0.01, min_abundance=1)
with ka.KmerCounter(cfg) as kc:
    kc.bloom_device(img.data_ptr(), ch, ka.FMT_FASTA)
    kc.bloom_finalize()
    print("single fill", fill(kc), kc.bloom_info(), flush=True)
    kc.count_device(img.data_ptr(), ch, ka.FMT_FASTA)
    st1 = kc.finish()
    print("single", {x: st1[x] for x in ("distinct", "new_in_first", "new_in_second", "failed_in_first", "inserted")}, flush=True)
for G in (1, 2):
    e = DeviceEngine(cfg, local_slots=4_000_000, world=G)
    e.bloom(img.data_ptr(), ch, ka.FMT_FASTA)
    r, counts = e.route_table(G)
    torch.cuda.synchronize()
    W = e.W
    tot = 0
    engines = [DeviceEngine(cfg, local_slots=1 << 16, world=G) for _ in range(G)]
    for d in range(G):
        lo = sum(counts[:d]) * (W + 1)
        rec = r[lo: lo + counts[d] * (W + 1)].clone()
        n = counts[d]
        rr = rec.view(-1, W + 1).cpu().numpy()
        print("G", G, "owner", d, "records", n, "count>=2", int((rr[:, -1] >= 2).sum()), "max", int(rr[:, -1].max()), flush=True)
        engines[d].bloom_records(rec, n)
        print("  unique", engines[d]._nuniq, flush=True)
        nis = engines[d].owner_bloom_finalize()
        o = engines[d].owner_table()
        print("  fill", fill(o), o.bloom_info(), "nis", nis, flush=True)
        engines[d].count_records(rec, n)
        st = o.finish()
        print("  ", {x: st[x] for x in ("distinct", "new_in_first", "new_in_second", "failed_in_first", "inserted")}, flush=True)
