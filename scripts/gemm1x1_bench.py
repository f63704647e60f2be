"""Microbench: ResNet-50 (bs 128) 1x1-conv GEMMs on hipBLASLt vs MIOpen.

For every distinct 1x1 conv shape: forward rows[P,Cin] x W^T, dgrad dY[P,Cout] x W,
wgrad dY^T[Cout,P] x rows[P,Cin] as (a) one mm, (b) split-K bmm over S chunks with
fp32 output + sum, (c) MIOpen convolution_backward (weight) on channels_last.
"""
import sys
import time

import torch

dev = torch.device("cuda")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
shapes = []  # (H, Cin, Cout, stride)
for H, planes, blocks, stride in ((56, 64, 3, 1), (28, 128, 4, 2), (14, 256, 6, 2), (7, 512, 3, 2)):
    inpl = 64 if planes == 64 else planes * 2
    Hin = H * stride
    shapes.append((H, inpl, planes, 1, Hin))           # conv1 of first block (input res Hin, stride 1 conv)
    shapes.append((H, planes, planes * 4, 1, H))       # conv3
    shapes.append((H, inpl, planes * 4, stride, Hin))  # downsample
    if blocks > 1:
        shapes.append((H, planes * 4, planes, 1, H))   # conv1 of later blocks
shapes = sorted(set(shapes))


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


bf = torch.bfloat16
tot = {}
for (H, Cin, Cout, stride, Hin) in shapes:
    P = N * H * H
    x = torch.randn(P, Cin, device=dev, dtype=bf)
    dy = torch.randn(P, Cout, device=dev, dtype=bf)
    w = torch.randn(Cout, Cin, device=dev, dtype=bf)
    fl = 2.0 * P * Cin * Cout
    r = {}
    r["fwd_mm"] = timeit(lambda: torch.mm(x, w.t()))
    r["dgrad_mm"] = timeit(lambda: torch.mm(dy, w))
    r["wgrad_mm"] = timeit(lambda: torch.mm(dy.t(), x))
    r["wgrad_mm_f32"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    for S in (4, 8, 16, 32, 64):
        if P % S:
            continue
        xb, db = x.view(S, P // S, Cin), dy.view(S, P // S, Cout)
        r[f"wgrad_bmm{S}"] = timeit(lambda: torch.bmm(db.transpose(1, 2), xb, out_dtype=torch.float32).sum(0))
    xc = x.view(N, H, H, Cin).permute(0, 3, 1, 2)
    dyc = dy.view(N, H, H, Cout).permute(0, 3, 1, 2)
    w4 = w.view(Cout, Cin, 1, 1).contiguous(memory_format=torch.channels_last)
    r["miopen_fwd"] = timeit(lambda: torch.nn.functional.conv2d(xc, w4))
    r["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dyc, xc, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, False, True]))
    r["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dyc, xc, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]))
    best_w = min((v, k) for k, v in r.items() if k.startswith("wgrad"))
    print(f"H={H:3d} Cin={Cin:4d} Cout={Cout:4d} P={P:7d} GF={fl/1e9:6.1f} | " +
          " ".join(f"{k}={v:7.1f}" for k, v in r.items()) + f" | best wgrad {best_w[1]} {fl/best_w[0]/1e6:.0f} TF/s",
          flush=True)
