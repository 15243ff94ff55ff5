"""Summarise a rocprofv3 --stats kernel_stats.csv: name (shortened), calls, average and total ms."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("void ", "").split("(")[0][:60]
    print(f"{name:62s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us {float(r['TotalDurationNs'])/1e6:9.3f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}%")
