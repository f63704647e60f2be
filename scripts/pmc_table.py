"""Per-kernel mean of each PMC counter from a rocprofv3 counter_collection.csv."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(lambda: defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
ctrs = sorted({c for k in agg.values() for c in k})
print("kernel".ljust(60), *[c[-22:].rjust(22) for c in ctrs])
for k, v in sorted(agg.items()):
    print(k.ljust(60), *[f"{(sum(v[c]) / len(v[c])) if v[c] else float('nan'):22.0f}" for c in ctrs])
