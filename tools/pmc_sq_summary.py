"""Per-kernel SQ counter summary of tools/gpu_pmc_sq.sh output: python tools/pmc_sq_summary.py DIR [kernel-prefix ...]"""
import collections
import csv
import sys

d0 = sys.argv[1]
pref = tuple(sys.argv[2:]) or ("k_",)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for g in ("pmc1", "pmc2"):
    for r in csv.DictReader(open(f"{d0}/{g}/run_counter_collection.csv")):
        n = r["Kernel_Name"].split("(")[0].replace("void kc::", "").replace("kc::", "")
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(g, n)].add(r["Dispatch_Id"])
for n, d in agg.items():
    if not n.startswith(pref) or not d["SQ_WAVES"]:
        continue
    c = len(disp[("pmc1", n)])
    w = d["SQ_WAVES"]
    print(f"{n[:60]:60s} calls {c}  per wave: VALU {d['SQ_INSTS_VALU']/w:9.0f} SALU {d['SQ_INSTS_SALU']/w:8.0f} "
          f"LDS {d['SQ_INSTS_LDS']/w:7.0f} VMEM_RD {d['SQ_INSTS_VMEM_RD']/w:7.1f} WR {d['SQ_INSTS_VMEM_WR']/w:6.1f} "
          f"cyc {d['SQ_WAVE_CYCLES']/w:8.0f} waitAny {d['SQ_WAIT_ANY']/w:8.0f} actLDS {d['SQ_ACTIVE_INST_LDS']/w:7.0f} "
          f"waves/call {w/c:8.0f} bankconf/call {d['SQ_LDS_BANK_CONFLICT']/c:.3g}")
