"""Achievable HBM streaming rates on this box (reference points for the roofline):
device-to-device copy (read + write) and a pure read (sum) of a C2-sized key stream."""
import time

import torch

n = 1_200_000_000  # 9.6 GB of u64 keys: one C2 key stream
a = torch.empty(n, dtype=torch.int64, device="cuda")
a.fill_(1)
b = torch.empty_like(a)
for what, fn, bytes_ in (("copy (r+w)", lambda: b.copy_(a), 2 * 8 * n),
                         ("read (sum)", lambda: a.sum(), 8 * n),
                         ("write (fill)", lambda: b.fill_(3), 8 * n)):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"{what:14s} {bytes_ / dt / 1e12:6.2f} TB/s  ({dt * 1e3:.2f} ms for {bytes_ / 1e9:.1f} GB)")
