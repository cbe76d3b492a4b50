"""The sharded engine across processes: two ranks, both on cuda:0, over
gloo (the device tensors of the exchange cross through host memory; on a node the same code
runs over RCCL).  Every rank runs ShardedCounter with the HIP DeviceEngine on its share of the
reference chunks (every other chunk): the Bloom pass and the filter combine (-b), the local
count, the pre-aggregated merge (kc_route_table_device -> all-to-all -> kc_insert_counts_*) -- or the
super-k-mer exchange (kc_route_superkmers_device -> two all-to-alls -> kc_count_packed_device, and
the owners' own Bloom passes over what they receive).
The union of the owners' outputs must equal the reference's output on the whole input
(tests/golden/cases.json); the reference's single shared table is kmer_hash_table.cpp:2207.
"""
import json
import os
import socket

import numpy as np
import pytest

from conftest import lines_digest, load_cases, sorted_digest_lines

pytestmark = pytest.mark.gpu

CASES = {(c["input"], c["k"], " ".join(c["args"])): c for c in load_cases()["cases"]}
PICK = [("reads_w60.fasta", 31, "-m 2 -a 1 -s 1000000"),
        ("reads_w60.fasta", 51, "-b -u 100000 -f 0.05 -a 2"),
        ("big_skew.fasta", 63, "-b -u 12000000 -a 2")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _options(args):
    a = args.split()
    o = {"mode": 2, "a": 2, "slots": 0, "bf": False, "u": 0, "fpr": 0.01}
    i = 0
    while i < len(a):
        if a[i] == "-b":
            o["bf"] = True
            i += 1
            continue
        key = {"-m": "mode", "-a": "a", "-s": "slots", "-u": "u", "-f": "fpr"}[a[i]]
        o[key] = float(a[i + 1]) if key == "fpr" else int(a[i + 1])
        i += 2
    return o


def _rank(rank, world, port, path, k, args, out_dir, exchange="records"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import kaarme_amd as ka
    from kaarme_amd.sharded import ShardedCounter

    o = _options(args)
    data = open(path, "rb").read()
    chunks = ka.plan_chunks(data, k, ka.FMT_FASTA, 256 << 10)  # many chunks: every rank gets a share
    mine = chunks[rank::world]
    img = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cfg = ka.Config(k=k, mode=o["mode"], table_slots=o["slots"] or (1 << 20), bf_enable=o["bf"],
                    est_unique=o["u"], fpr=o["fpr"], min_abundance=o["a"])
    sc = ShardedCounter(cfg, dist, exchange=exchange)
    stream = torch.cuda.current_stream().cuda_stream
    if o["bf"]:
        sc.bloom_device(img.data_ptr(), mine, ka.FMT_FASTA, stream)
        sc.bloom_finalize()
    sc.count_device(img.data_ptr(), mine, ka.FMT_FASTA, stream)
    st = sc.finish()
    d = sc.output_digest()  # collective: the owners' digests combined (bench.py's N > 1 parity)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), sc.dump())
    with open(os.path.join(out_dir, f"dg{rank}.json"), "w") as f:
        json.dump(d, f)
    with open(os.path.join(out_dir, f"st{rank}.txt"), "w") as f:
        f.write(f"{st['windows']} {st['chunks']}\n")
    sc.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("exchange", ["records", "superkmers"])
@pytest.mark.parametrize("name,k,args", PICK, ids=[f"{n}-k{k}" for n, k, _ in PICK])
def test_two_processes_equal_the_reference(name, k, args, exchange, golden_input, tmp_path):
    import torch.multiprocessing as mp

    import kaarme_amd as ka

    case = CASES[(name, k, args)]
    path = golden_input(name)
    mp.start_processes(_rank, args=(2, _free_port(), path, k, args, str(tmp_path), exchange), nprocs=2, join=True,
                       start_method="spawn")
    recs = [np.load(tmp_path / f"r{r}.npy") for r in range(2)]
    keys = [set(map(tuple, r[:, :-1].tolist())) for r in recs]
    assert not (keys[0] & keys[1]), "owners must be disjoint"
    lines = []
    for r in recs:
        lines += [f"{s} {c}" for s, c in ka.decode_records(r.reshape(-1), k)]
    assert sorted_digest_lines(lines) == (case["sorted_sha256"], case["lines"])
    want = lines_digest(lines)
    for r in range(2):
        assert json.load(open(tmp_path / f"dg{r}.json")) == want, r
    windows = sum(int(open(tmp_path / f"st{r}.txt").read().split()[0]) for r in range(2))
    assert windows > 0
