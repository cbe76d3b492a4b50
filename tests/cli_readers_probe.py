"""The drop-in CLI on a whole strong workload's file (C4: 16 GB, k = 51, -s 2.6e9; C5: 10 GB,
k = 127, -s 3.6e9) with several upload reader counts (--readers), its timer lines and its phase
lines (--phases, stderr).  Not a test; run on a GPU box:
    python3 -u tests/cli_readers_probe.py [C4|C5] [readers ...]"""
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "canonical-k-mer-hash-table_amd"))
import torch  # noqa: E402

import kaarme_amd as ka  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].startswith("C") else "C4"
readers = [int(x) for x in sys.argv[2 if len(sys.argv) > 1 and sys.argv[1].startswith("C") else 1:]] or [1, 2, 4, 8]
N, L, k, s = (100_000_000, 150, 51, "2600000000") if cfg == "C4" else (1_000_000, 10_000, 127, "3600000000")
s = os.environ.get("PROBE_S", s)  # (diagnosis: a smaller -s, i.e. a smaller table allocated at kc_create)
lib = ka.load_library()
nb = lib.kc_synth_bytes(0, N, L, 0)
img = torch.empty(nb, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 42, 500_000_000, L, 0, 0.001, 0.0, 0) == 0
torch.cuda.synchronize()
cli = os.path.join(ROOT, "canonical-k-mer-hash-table_amd", "bin", "kaarme")
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    fa = os.path.join(td, "input.fasta")
    with open(fa, "wb") as f:
        f.write(memoryview(img.cpu().numpy()))
    del img
    torch.cuda.empty_cache()
    with open(fa, "rb") as f:
        while f.read(1 << 24):
            pass
    for rd in readers:
        t0 = time.perf_counter()
        p = subprocess.run([cli, fa, str(k), "-m", "2", "-s", s, "-a", "1", "-t", "18", "-o", os.path.join(td, "o.txt"),
                            "--digest-only", "--phases", "--readers", str(rd)], capture_output=True, text=True)
        wall = time.perf_counter() - t0
        keep = [l for l in (p.stdout + p.stderr).splitlines() if l.strip()]
        print(f"== {cfg} readers {rd} rc {p.returncode} wall {wall:.2f}", flush=True)
        print("\n".join(keep[-40:]), flush=True)
