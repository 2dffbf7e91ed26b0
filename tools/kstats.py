"""Print a rocprofv3 kernel_stats.csv as name / calls / average us (tools only)."""
import csv
import sys

for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        print(f"   {r['Name'][:44]:44s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1000:9.1f} us {float(r['Percentage']):6.2f}%")
