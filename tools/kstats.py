"""Summarise a rocprofv3 *_kernel_stats.csv (development tool)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    n = r["Name"]
    n = n[:n.find("(")] if "(" in n else n
    print(f"{n[:62]:62s} calls={r['Calls']:>7s} avg_us={float(r['AverageNs'])/1e3:8.1f} "
          f"pct={100*float(r['TotalDurationNs'])/tot:5.1f}")
