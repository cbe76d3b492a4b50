#!/usr/bin/env python3
"""Summarise profiles/collect_pmc.sh output: per-kernel mean counters per dispatch and
the HBM traffic of one counting pass (bench.py's roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are
the L2 memory-side request counters; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so reads are doubled.  The unit of both (KiB in rocprofv3) was
calibrated on k_gather's stores, 16-byte streaming writes of exactly `stage_bytes`
bytes per step (a known byte count), and is applied to every kernel.

usage: pmc_summary.py OUTDIR [--write profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# the roofline window: the tokenizer + the counting pass (+ the reuse checksum beside them; the
# distinct estimate of the strong presets, whose tokenized batches the counting pass reads)
COUNT_PASS = ("k_p1<", "k_p2<", "k_p2f<", "k_p3<", "k_b3<", "k_bf3<", "k_bprobe<", "k_scanA", "k_scanB", "k_scanC",
              "k_count<", "k_tile_map", "k_tile_summary", "k_tscan_block", "k_tscan_top", "k_zero_edges", "k_emit",
              "k_checksum", "k_hll<", "k_skm_route")
# FETCH_SIZE / WRITE_SIZE unit: 1023.99998 bytes per unit measured in r01_v5 against
# k_gather's WRITE_SIZE for a known byte count (k_gather no longer exists: the tokenizer
# reads device images in place), i.e. the counters are in KiB.
KIB_CALIBRATED = 1024.0

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_digest  # noqa: E402


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("kc::", "")
    return n


def load(outdir):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    for f in glob.glob(os.path.join(outdir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            vals[short(names[d])][c].append(v)
    return vals


def main():
    outdir = sys.argv[1]
    dest = sys.argv[sys.argv.index("--write") + 1] if "--write" in sys.argv else None
    vals = load(outdir)
    bench = None
    for j in sorted(glob.glob(os.path.join(outdir, "pmc*.json"))):
        try:
            bench = json.loads(open(j).read().strip().splitlines()[-1])
            break
        except (ValueError, IndexError):
            continue
    steps = bench["steps"] + bench["warmup"]
    mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    gather = [k for k in mean if k.startswith("k_gather")]
    unit = KIB_CALIBRATED
    if gather and "WRITE_SIZE" in mean[gather[0]] and bench.get("stage_bytes"):
        unit = bench["stage_bytes"] / mean[gather[0]]["WRITE_SIZE"]
        print(f"unit (bytes per counter unit, from k_gather writes): {unit}")
    else:
        print(f"unit (bytes per counter unit): {unit} (calibrated in r01_v5 on k_gather's 16-B stores)")
    print(f"{'kernel':60s} {'calls':>5s} {'read GB':>9s} {'write GB':>9s}")
    total = 0.0
    per_kernel = {}
    for k in sorted(mean, key=lambda x: -mean[x].get("FETCH_SIZE", 0)):
        m = mean[k]
        calls = max(len(v) for v in vals[k].values())
        rd = 2 * m.get("FETCH_SIZE", 0) * (unit or 1)
        wr = m.get("WRITE_SIZE", 0) * (unit or 1)
        per_kernel[k] = {"calls": calls, "read_bytes": rd, "write_bytes": wr,
                         **{c: m[c] for c in m if c not in ("FETCH_SIZE", "WRITE_SIZE")}}
        print(f"{k[:60]:60s} {calls:5d} {rd / 1e9:9.3f} {wr / 1e9:9.3f}")
        if k.startswith(COUNT_PASS):
            total += (rd + wr) * calls / steps
    # bench.py's roofline unit: one counting pass per staged batch, or with the Bloom
    # filter (-b) one Bloom pass + one counting pass over the same batch
    per_step = bench["config"].get("batches_per_step", 1.0)
    units = per_step / 2 if " -b " in bench["config"]["workload"] else per_step
    total /= max(units, 1e-9)
    print(f"count pass HBM bytes per launch: {total / 1e9:.3f} GB")
    if dest:
        # one entry per workload (bench.py looks its own up); earlier entries are kept
        try:
            with open(dest) as f:
                old = json.load(f)
        except (OSError, ValueError):
            old = {}
        book = old.get("workloads", {})
        if "workload" in old:  # the single-workload layout of earlier versions
            book.setdefault(old["workload"], {c: v for c, v in old.items() if c != "workload"})
        book[bench["config"]["workload"]] = {
            "bytes_per_launch": int(total), "unit_bytes": unit,
            # the kernel sources this was measured with (bench.py marks the entry stale when
            # the sources differ) and the commit, when the caller passes it (KC_COMMIT)
            "source_sha": kernel_source_digest(), "commit": os.environ.get("KC_COMMIT"),
            "method": "2*FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM), unit calibrated on k_gather 16-B "
                      "stores; count-pass kernels (with -b: Bloom pass + counting pass) summed per launch",
            "per_kernel": per_kernel}
        with open(dest, "w") as f:
            json.dump({"workloads": book}, f, indent=1)
        print("wrote", dest)

if __name__ == "__main__":
    main()
