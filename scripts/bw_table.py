"""Per-kernel HBM traffic and achieved bandwidth from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE, KB per dispatch, one pass each: they need 5 TCC counters together, the limit is 4)
and a kernel-trace CSV of a run of the same program (durations).

    python scripts/bw_table.py FETCH.csv WRITE.csv KERNEL_TRACE.csv [top]

Kernels are matched by their name's first 80 characters; every number is a mean per dispatch.
"""
import csv
import sys
from collections import defaultdict


def counters(path, name):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            acc[r["Kernel_Name"][:80]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def durations(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"][:80]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)  # us
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch, write = counters(sys.argv[1], "FETCH_SIZE"), counters(sys.argv[2], "WRITE_SIZE")
    dur = durations(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows = []
    for k, (us, n) in dur.items():
        if k not in fetch and k not in write:
            continue
        f, w = fetch.get(k, 0.0) / 1024.0, write.get(k, 0.0) / 1024.0  # MB per dispatch
        rows.append((us * n, k, n, us, f, w, (f + w) * 1.048576 / us if us > 0 else 0.0))  # MiB/us -> TB/s
    rows.sort(reverse=True)
    print(f"{'kernel':80s} {'calls':>6s} {'us/call':>8s} {'read MB':>8s} {'write MB':>8s} {'TB/s':>6s}")
    for _, k, n, us, f, w, bw in rows[:top]:
        print(f"{k:80s} {n:6d} {us:8.1f} {f:8.1f} {w:8.1f} {bw:6.2f}")


if __name__ == "__main__":
    main()
