"""Per-kernel VGPR / scratch / LDS / occupancy of one HIP source (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

sys.path.insert(0, __file__.rsplit("/scripts", 1)[0])
from ddp_practice_amd import build as b  # noqa: E402

src = sys.argv[1]
r = subprocess.run(["hipcc", "-x", "hip", *b._flags(), "--offload-device-only",
                    "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/_ru.o"],
                   capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for row in rows:
    n = subprocess.run(["c++filt", row["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{n[:95]:95s} v={row.get('VGPRs')} a={row.get('AGPRs')} scr={row.get('ScratchSize')} "
          f"lds={row.get('LDS Size')} occ={row.get('Occupancy')}")
