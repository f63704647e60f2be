"""Summarise a rocprofv3 kernel_stats.csv: per-step time by kernel."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else None
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':80s} {'calls':>6s} {'avg_us':>8s} {'%':>6s}")
for r in rows:
    print(f"{r['Name'][:80]:80s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:8.2f} {float(r['Percentage']):6.2f}")
if steps:
    print(f"total kernel time per step: {tot/1e3/steps:.1f} us")
