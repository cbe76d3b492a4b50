"""Per-kernel LDS stall summary of tools/gpu_pmc_lds.sh output: python tools/pmc_lds_summary.py DIR [kernel-prefix ...]

Per wave: cycles, cycles parked (SQ_WAIT_ANY: s_waitcnt / barrier), LDS instructions, cycles
a ready LDS instruction could not issue (SQ_WAIT_INST_LDS: the LDS queue is full -- atomics
and conflicted accesses hold it), cycles an LDS instruction was in flight (SQ_ACTIVE_INST_LDS);
per call: LDS-array cycles (SQ_LDS_IDX_ACTIVE) and the extra ones from bank conflicts."""
import collections
import csv
import glob
import sys

d0 = sys.argv[1]
pref = tuple(sys.argv[2:]) or ("k_",)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{d0}/p/**/run_counter_collection.csv", recursive=True) or [f"{d0}/p/run_counter_collection.csv"]:
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void kc::", "").replace("kc::", "")
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
print(f"{'kernel':58s} {'calls':>5s} {'cyc/w':>8s} {'park%':>6s} {'LDS/w':>7s} {'ldsStall%':>9s} "
      f"{'ldsAct%':>7s} {'arrayCyc/call':>13s} {'conflict%':>9s}")
for n, d in sorted(agg.items(), key=lambda x: -x[1]["SQ_WAVE_CYCLES"]):
    if not n.startswith(pref) or not d["SQ_WAVES"]:
        continue
    c = len(disp[n])
    w = d["SQ_WAVES"]
    cyc = d["SQ_WAVE_CYCLES"] or 1
    arr = d["SQ_LDS_IDX_ACTIVE"] or 1
    print(f"{n[:58]:58s} {c:5d} {cyc / w:8.0f} {100 * d['SQ_WAIT_ANY'] / cyc:6.1f} {d['SQ_INSTS_LDS'] / w:7.0f} "
          f"{100 * d['SQ_WAIT_INST_LDS'] / cyc:9.2f} {100 * d['SQ_ACTIVE_INST_LDS'] / cyc:7.1f} {arr / c:13.3g} "
          f"{100 * d['SQ_LDS_BANK_CONFLICT'] / arr:9.1f}")
