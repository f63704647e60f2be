"""Phase timing of the fused ConvNet kernels (experiment build with -DDPA_TIMING):
    DPA_BUILD_TAG=timing DPA_EXTRA_CFLAGS=-DDPA_TIMING python -m ddp_practice_amd.build
    DPA_EXT_SO=ddp_practice_amd/_C_timing.so python scripts/stamp_conv.py
Per kernel: blocks, span (first start -> last end), start skew, and the mean
time of each stamped phase relative to the block's start (us)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
cn = C.convnet
names = ["conv1_fwd_pack", "conv2_fwd", "head_fwd", "head_bwd", "conv2_dgrad", "conv_wgrad_bn"]
report = []


def wrap(name):
    f = getattr(cn, name)

    def g(*a):
        cn.clear_stamps()
        torch.cuda.synchronize()
        f(*a)
        st = cn.read_stamps().double()
        rows = st[st[:, 0] > 0]
        if len(rows) == 0:
            report.append((name, 0, "no stamps"))
            return
        t0 = rows[:, 0].min()
        end = rows.max(dim=1).values
        line = f"{name:16s} blocks={len(rows):4d} span={(end.max() - t0).item() / 100:6.2f}us " \
               f"skew={(rows[:, 0].max() - t0).item() / 100:5.2f}us phases:"
        for i in range(1, 16):
            col = rows[:, i]
            ok = col > 0
            if ok.any():
                line += f" s{i}={((col[ok] - rows[ok, 0]).mean() / 100).item():5.2f}"
        report.append((name, len(rows), line))
    setattr(cn, name, g)


for n in names:
    wrap(n)

from ddp_practice_amd.models import ConvNet  # noqa: E402
from ddp_practice_amd.ops import convnet_fused  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = ConvNet().to(dev)
for it in range(3):
    x = torch.rand(32, 1, 28, 28, device=dev).to(torch.bfloat16)
    out = convnet_fused.convnet_forward(m, x, cdtype=torch.bfloat16)
    out.float().sum().backward()
    torch.cuda.synchronize()
    if it == 2:
        for r in report[-7:]:
            print(r[2])
    else:
        report.clear()
