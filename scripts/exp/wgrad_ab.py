"""Per-shape A/B of the implicit-GEMM weight-gradient kernels on every ResNet-50 (bs 128)
conv shape, interleaved rounds in one process (median of 5):
  a: default (1x1 on the LDS-DMA kernel, KxK register-staged), 4 waves
  b: the same with 8-wave LDS-DMA workgroups (conv_igemm.wgrad_waves_config(8))
  c: every conv on the LDS-DMA kernel, 8 waves (wgrad_config(2))
with each arm's error against an fp32 torch reference.

  python scripts/exp/wgrad_ab.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402
from ddp_practice_amd.ops.conv_igemm import conv_wgrad  # noqa: E402

C = _ext.load()
K_ = C.conv_igemm
CL = torch.channels_last
B = int(os.environ.get("BS", "128"))
SHAPES = [(64, 56, 64, 3, 1, 3), (128, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 3), (256, 28, 256, 3, 2, 1),
          (256, 14, 256, 3, 1, 5), (512, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 2),
          (64, 56, 64, 1, 1, 1), (64, 56, 256, 1, 1, 4), (256, 56, 64, 1, 1, 2), (256, 56, 128, 1, 1, 1),
          (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (256, 56, 512, 1, 2, 1), (512, 28, 256, 1, 1, 1),
          (256, 14, 1024, 1, 1, 6), (1024, 14, 256, 1, 1, 5), (512, 28, 1024, 1, 2, 1), (1024, 14, 512, 1, 1, 1),
          (512, 7, 2048, 1, 1, 3), (2048, 7, 512, 1, 1, 2), (1024, 14, 2048, 1, 2, 1)]
ARMS = {"a": (1, 4), "b": (1, 8), "c": (2, 8)}


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


tot = {a: 0.0 for a in ARMS}
print(f"{'shape (Cin,H,Cout,R,s)':26s} {'GFLOP':>6s} " + " ".join(f"{a:>8s}" for a in ARMS) + "  rel-err a/b/c")
for Cin, H, K, R, st, cnt in SHAPES:
    pad = R // 2
    g = torch.Generator().manual_seed(Cin + K + H)
    x = torch.randn(B, Cin, H, H, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // st + 1
    dy = torch.randn(B, K, OH, OH, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
    wshape = (K, Cin, R, R)
    fl = 2.0 * B * OH * OH * K * Cin * R * R / 1e9
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), torch.empty(wshape, device="cuda"), None,
                                              [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    ts = {a: [] for a in ARMS}
    err = {}
    for _ in range(5):
        for a, (gl, wv) in ARMS.items():
            p0, p1 = K_.wgrad_config(gl), K_.wgrad_waves_config(wv)
            ts[a].append(timeit(lambda: conv_wgrad(dy, x, wshape, st, pad)))
            gw = conv_wgrad(dy, x, wshape, st, pad)
            err[a] = ((gw - ref).abs().max() / ref.abs().max()).item()
            K_.wgrad_config(p0)
            K_.wgrad_waves_config(p1)
    med = {a: statistics.median(v) for a, v in ts.items()}
    for a in ARMS:
        tot[a] += med[a] * cnt
    print(f"{str((Cin, H, K, R, st)):26s} {fl:6.2f} " + " ".join(f"{med[a]:8.1f}" for a in ARMS)
          + f"  {err['a']:.1e}/{err['b']:.1e}/{err['c']:.1e} x{cnt}", flush=True)
print("network wgrad (x count, incl. the split reduction): " + ", ".join(f"{a} {tot[a]:.0f} us" for a in ARMS))
