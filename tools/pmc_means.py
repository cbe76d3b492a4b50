"""Per-kernel mean of every PMC counter over its dispatches (the committed form of a
rocprofv3 --pmc run): python tools/pmc_means.py run_counter_collection.csv > out.csv"""
import collections
import csv
import sys

acc = collections.defaultdict(float)
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    key = (r["Kernel_Name"], r["Counter_Name"])
    acc[key] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
w = csv.writer(sys.stdout)
w.writerow(["Kernel_Name", "Counter_Name", "Dispatches", "Mean_Per_Dispatch"])
for (k, c), v in acc.items():
    w.writerow([k, c, len(disp[(k, c)]), v / len(disp[(k, c)])])
