"""Per-kernel mean per dispatch of every counter under a pmc.sh output directory (k_p1/k_p2f/k_p3),
with per-wave figures for the SQ counters and GB for FETCH_SIZE (x2, gfx950 wide reads) / WRITE_SIZE."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kc::", "")
        if not any(n.startswith(p) for p in ("k_p1<", "k_p2f<", "k_p3<1, true")):
            continue
        vals[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(n, r["Counter_Name"])].add(r["Dispatch_Id"])
for n, c in vals.items():
    m = {k: v / max(1, len(disp[(n, k)])) for k, v in c.items()}
    w = m.get("SQ_WAVES", 1) or 1
    out = [n[:48].ljust(48)]
    for k, lab in (("SQ_INSTS_VALU", "VALU"), ("SQ_INSTS_SALU", "SALU"), ("SQ_INSTS_LDS", "LDS"),
                   ("SQ_INSTS_VMEM_RD", "VMRD"), ("SQ_INSTS_VMEM_WR", "VMWR"), ("SQ_WAVE_CYCLES", "cyc"),
                   ("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "waitI"), ("SQ_ACTIVE_INST_VALU", "aVALU"),
                   ("SQ_ACTIVE_INST_LDS", "aLDS")):
        if k in m:
            out.append(f"{lab} {m[k] / w:.0f}")
    if "SQ_LDS_BANK_CONFLICT" in m:
        out.append(f"bankconf {m['SQ_LDS_BANK_CONFLICT']:.3g}")
    if "SQ_WAVES" in m:
        out.append(f"waves {w:.0f}")
    if "FETCH_SIZE" in m:
        out.append(f"rdGB {2 * m['FETCH_SIZE'] * 1024 / 1e9:.2f}")
    if "WRITE_SIZE" in m:
        out.append(f"wrGB {m['WRITE_SIZE'] * 1024 / 1e9:.2f}")
    print(" ".join(out))
