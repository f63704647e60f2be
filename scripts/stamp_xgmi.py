"""Phase timing of the one-shot xGMI all-reduce at world size 1 (experiment build):
    DPA_BUILD_TAG=timing DPA_EXTRA_CFLAGS=-DDPA_TIMING python -m ddp_practice_amd.build
    DPA_EXT_SO=ddp_practice_amd/_C_timing.so python scripts/stamp_xgmi.py
Stamps: s1 = granules pushed, s2 = every granule polled, s3 = end (us from block start)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_practice_amd import _ext  # noqa: E402

X = _ext.load().xgmi
x = X.XgmiComm(0, 1, 0, 1 << 20, 10.0)
x.open([x.handle()])
for n in (33, 4224, 29034):
    t = torch.randn(n, device="cuda")
    out = torch.empty_like(t)
    for it in range(5):
        X.clear_stamps()
        x.all_reduce(t, "sum", out)
        st = X.read_stamps().double()
    rows = st[st[:, 0] > 0]
    t0 = rows[:, 0].min()
    line = f"n={n:6d} blocks={len(rows):3d} span={(rows.max(dim=1).values.max() - t0).item() / 100:6.2f}us " \
           f"skew={(rows[:, 0].max() - t0).item() / 100:5.2f}us"
    for i in range(1, 4):
        line += f" s{i}={((rows[:, i] - rows[:, 0]).mean() / 100).item():5.2f}"
    print(line, flush=True)
    assert torch.allclose(out, t)
