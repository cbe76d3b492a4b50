"""The route of one C4/8 share (12.5 M reads, k = 51, G = 8), twice after a dry run: the workload
profiled for k_skm_route (rocprofv3 --kernel-trace / --pmc -- python3 -u tests/skm_route_probe.py).
Not a test (no assertions on results); the parity of the route is tests/test_gpu_skm*.py."""
import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "canonical-k-mer-hash-table_amd"))
import torch, kaarme_amd as ka
lib = ka.load_library(); torch.cuda.set_device(0); st = torch.cuda.current_stream().cuda_stream
N, L, G = 12_500_000, 150, 8
nb = lib.kc_synth_bytes(0, N, L, 0); img = torch.empty(nb, dtype=torch.uint8, device="cuda")
assert lib.kc_synth_device(img.data_ptr(), 0, N, 42, 500_000_000, L, 0, 0.001, 0.0, st) == 0
torch.cuda.synchronize()
ch = ka.plan_chunks_device(img.data_ptr(), nb, 51, ka.FMT_FASTA)
r = ka.KmerCounter(ka.Config(k=51, mode=2, table_slots=1 << 16, batch_bytes=2 << 30))
need, _ = r.route_superkmers_device(img.data_ptr(), ch, ka.FMT_FASTA, G, stream=st)
cap = int(max(need) * 1.05) + 64
pk = torch.empty(G * cap + 2, dtype=torch.int64, device="cuda"); bk = torch.empty(G * cap + 2, dtype=torch.int32, device="cuda")
for _ in range(2):
    r.route_superkmers_device(img.data_ptr(), ch, ka.FMT_FASTA, G, pk.data_ptr(), bk.data_ptr(), cap, stream=st)
torch.cuda.synchronize(); print("ok", sum(need))
