"""Print a rocprofv3 run_kernel_stats.csv compactly.  Usage: python tools/kstats.py <csv>"""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(anonymous namespace\)::|spt::|void ", "", r["Name"]).split("(")[0]
    print(f"{name[:44]:44s} calls {r['Calls']:>5s} total {float(r['TotalDurationNs']) / 1e6:8.3f} ms "
          f"avg {float(r['AverageNs']) / 1e3:8.1f} us")
