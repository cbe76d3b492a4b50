"""Counter / known bytes per calibration kernel (tools/pmc_calib/run.sh)."""
import csv
import glob
import os
import sys

out = sys.argv[1]
known = {}
for line in open(os.path.join(out, "known.txt")):
    name, recs, byts = line.split()
    known[name] = int(byts.split("=")[1])
vals = {}
for f in glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        name = next((n for n in known if k.startswith(n + "(") or k == n or k.startswith(n)), None)
        if name:
            vals.setdefault(name, {})[row["Counter_Name"]] = vals.setdefault(name, {}).get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
print(f"{'kernel':14s} {'known GB':>9s} {'FETCH GB':>9s} {'ratio':>7s} {'WRITE GB':>9s} {'ratio':>7s}")
for name, b in known.items():
    v = vals.get(name, {})
    fe, wr = v.get("FETCH_SIZE"), v.get("WRITE_SIZE")
    # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB (1024 bytes)
    fgb = fe * 1024 / 1e9 if fe is not None else float("nan")
    wgb = wr * 1024 / 1e9 if wr is not None else float("nan")
    print(f"{name:14s} {b / 1e9:9.3f} {fgb:9.3f} {fgb / (b / 1e9):7.3f} {wgb:9.3f} {wgb / (b / 1e9):7.3f}")
