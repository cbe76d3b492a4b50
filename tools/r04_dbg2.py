"""Debug: the fused pass's overflow fallback vs KC_FUSE=0 at -u 2e5 (k=51)."""
import os, sys, subprocess
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "canonical-k-mer-hash-table_amd"))
os.environ["KC_REUSE_DEBUG"] = "1"
os.environ["KC_INSERT_PATH"] = "partitioned"
mode = sys.argv[1]
if mode == "nofuse":
    os.environ["KC_FUSE"] = "0"
elif mode == "force16":
    os.environ["KC_FUSE_R"] = "16"
import torch
import kaarme_amd as ka
lib = ka.load_library()
N, L, G = 300_000, 150, 3_000_000
nbytes = lib.kc_synth_bytes(0, N, L, 0)
img = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 12, G, L, 0, 0.002, 0.0, 0) == 0
torch.cuda.synchronize()
k = 51
chunks = ka.plan_chunks(bytes(img.cpu().numpy()), k, ka.FMT_FASTA)
cfg = ka.Config(k=k, min_abundance=2, bf_enable=True, est_unique=200_000, fpr=0.01)
with ka.KmerCounter(cfg) as kc:
    kc.bloom_device(img.data_ptr(), chunks, ka.FMT_FASTA)
    print("nis", kc.bloom_finalize(), flush=True)
    kc.count_device(img.data_ptr(), chunks, ka.FMT_FASTA)
    try:
        st = kc.finish()
        print(mode, st, flush=True)
    except Exception as e:
        print(mode, "ERR", e, flush=True)
