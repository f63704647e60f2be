"""One steady-state step of a rocprofv3 kernel_trace.csv as a launch sequence: every
dispatch of the last complete step (between the last two marker kernels) with its grid,
workgroup size, registers, LDS and duration, so each launch can be matched to the layer
that issued it (ResNet-50: per-shape attribution of the steady table).

    python scripts/trace_seq.py run_kernel_trace.csv [marker-substring]
"""
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "amp_sgd"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(marks) < 2:
    raise SystemExit(f"only {len(marks)} marker kernels")
sel = rows[marks[-2] + 1:marks[-1] + 1]


def col(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    return "?"


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("dpa::", "").replace("__hip_bfloat16", "bf16")
    return name[:70]


tot = 0.0
print(f"{'#':>4s} {'kernel':70s} {'grid':>10s} {'wg':>5s} {'vgpr':>5s} {'lds':>6s} {'us':>8s}")
for i, r in enumerate(sel):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    grid = col(r, "Grid_Size", "Grid_Size_X")
    wg = col(r, "Workgroup_Size", "Workgroup_Size_X")
    try:
        grid = str(int(grid) // max(1, int(wg)))  # workgroups
    except ValueError:
        pass
    print(f"{i:4d} {short(r['Kernel_Name']):70s} {grid:>10s} {wg:>5s} {col(r, 'VGPR_Count', 'Arch_VGPR_Count'):>5s} "
          f"{col(r, 'LDS_Block_Size', 'Group_Segment_Size', 'LDS_Size'):>6s} {us:8.1f}")
print(f"total {tot:.1f} us over {len(sel)} launches")
