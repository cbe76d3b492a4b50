"""Print a rocprofv3 kernel_stats.csv as name / calls / avg ms / total ms."""
import csv
import sys

for x in csv.DictReader(open(sys.argv[1])):
    print(x["Name"][:100].ljust(100), x["Calls"].rjust(4), f"{float(x['AverageNs']) / 1e6:9.3f}",
          f"{float(x['TotalDurationNs']) / 1e6:9.2f}")
