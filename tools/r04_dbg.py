"""Debug: the fused pass's decisions for the Bloom test shapes (KC_REUSE_DEBUG output)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "canonical-k-mer-hash-table_amd"))
os.environ["KC_REUSE_DEBUG"] = "1"
os.environ["KC_INSERT_PATH"] = "partitioned"
import torch
import kaarme_amd as ka
lib = ka.load_library()
N, L, G = 300_000, 150, 3_000_000
nbytes = lib.kc_synth_bytes(0, N, L, 0)
img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 11, G, L, 0, 0.002, 0.0, 0) == 0
torch.cuda.synchronize()
for k, fpr in [(95, 0.05), (127, 0.01), (51, 0.01)]:
    chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
    cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=8_000_000, fpr=fpr)
    with ka.KmerCounter(cfg) as kc:
        kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        kc.bloom_finalize()
        kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
        st = kc.finish()
        print(k, fpr, st, flush=True)
