"""Print the pw:: rows of a rocprofv3 kernel_stats.csv: name and average µs.  Usage: kstat.py <csv>"""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    name = r["Name"][5:] if r["Name"].startswith("void ") else r["Name"]  # (templates: "void pw::k<..>(...)")
    if name.startswith("pw::"):
        print(f"   {name.split('(')[0]:28s} {float(r['AverageNs']) / 1000:9.1f} us")
