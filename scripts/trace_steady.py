"""Steady-state per-step kernel table from a rocprofv3 kernel_trace.csv.

Steps are delimited by a marker kernel that runs once per training step (the
optimizer); the last N steps are summarised, so one-time work (MIOpen Find,
warm-up, graph capture) is excluded.

    python scripts/trace_steady.py run_kernel_trace.csv [marker-substring] [N]
"""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "amp_sgd"
n_last = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(marks) < n_last + 1:
    raise SystemExit(f"only {len(marks)} marker kernels")
lo, hi = marks[-n_last - 1] + 1, marks[-1] + 1
sel = rows[lo:hi]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
print(f"steady state over the last {n_last} steps: wall {wall / n_last:.1f} us/step, kernel busy {busy / n_last:.1f} us/step, "
      f"{len(sel) / n_last:.0f} launches/step")
print(f"{'kernel':90s} {'/step':>6s} {'us/step':>9s} {'%':>6s}")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[:90]:90s} {c / n_last:6.1f} {t / n_last:9.1f} {100 * t / busy:6.2f}")
