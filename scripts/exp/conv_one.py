"""Run one ResNet-50 conv shape on conv_glds_kernel N times (a PMC / trace target).

  python scripts/exp/conv_one.py Cin H Cout R stride [N] [WIDE]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

K_ = _ext.load().conv_igemm
Cin, H, K, R, st = (int(a) for a in sys.argv[1:6])
n = int(sys.argv[6]) if len(sys.argv) > 6 else 50
if len(sys.argv) > 7:
    K_.wide_config(int(sys.argv[7]))
B, pad, CL = 128, R // 2, torch.channels_last
g = torch.Generator().manual_seed(1)
x = torch.randn(B, Cin, H, H, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
w = (torch.randn(K, Cin, R, R, generator=g) / (Cin * R * R) ** 0.5).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
OH = (H + 2 * pad - R) // st + 1
y = torch.empty(B, K, OH, OH, dtype=torch.bfloat16, device="cuda", memory_format=CL)
for _ in range(n):
    K_.conv_fwd(x, w, y, st, pad)
torch.cuda.synchronize()
print("ok")
