"""The drop-in CLI on the whole 16 GB C4 file with 1 / 2 / 4 / 8 upload readers (--readers): its
timer line (file read + chunking + estimate + count) and its stdout's phase lines, to pick the
reader count for big inputs.  Not a test; run on a GPU box: python3 -u tests/cli_readers_probe.py"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "canonical-k-mer-hash-table_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import kaarme_amd as ka  # noqa: E402

lib = ka.load_library()
N, L = 100_000_000, 150
nb = lib.kc_synth_bytes(0, N, L, 0)
img = torch.empty(nb, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 42, 500_000_000, L, 0, 0.001, 0.0, 0) == 0
torch.cuda.synchronize()
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    fa = os.path.join(td, "input.fasta")
    with open(fa, "wb") as f:
        f.write(memoryview(img.cpu().numpy()))
    del img
    torch.cuda.empty_cache()
    with open(fa, "rb") as f:
        while f.read(1 << 24):
            pass
    for rd in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        r = bench.run_cli(fa, ["51", "-m", "2", "-s", "2600000000", "-a", "1", "-t", "18"], os.path.join(td, "o.txt"),
                          ["--digest-only", "--readers", str(rd)])
        if r is None:
            print("readers", rd, "failed", flush=True)
            continue
        secs, write_s, wall, out = r
        lines = [l for l in out.splitlines() if "Time used" in l or "Input" in l or "digest" in l.lower()]
        print("readers", rd, "build_s", round(secs, 3), "wall", round(wall, 2), "|", " | ".join(lines)[:600], flush=True)
