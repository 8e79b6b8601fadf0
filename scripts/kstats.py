"""Summarise a rocprofv3 kernel_stats.csv per step: python scripts/kstats.py <csv> [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.3f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) // steps:5d}/step "
          f"{float(r['AverageNs']) / 1e3:8.1f} us {float(r['Percentage']):5.1f}%  {r['Name'][:70]}")
