"""NHWC BatchNorm statistics kernels: write-through vs fenced ticket hand-off
(bn_nhwc.set_handoff) x workgroup-count target, on ResNet-50 (bs 128) shapes,
plus the elementwise targets.  Per-call microseconds and implied HBM TB/s."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts", 1)[0])
from ddp_practice_amd import _ext  # noqa: E402
from ddp_practice_amd.ops.bn_nhwc import _Workspace  # noqa: E402

K = _ext.load().bn_nhwc
dev = torch.device("cuda")
shapes = [(128 * 56 * 56, 64), (128 * 56 * 56, 256), (128 * 28 * 28, 128), (128 * 28 * 28, 512),
          (128 * 14 * 14, 1024), (128 * 7 * 7, 2048)]


def tm(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


f32 = dict(dtype=torch.float32, device=dev)
for M, C in shapes:
    x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    yb = torch.randn_like(x)
    res = torch.randn_like(x)
    shift = torch.zeros(C, **f32)
    gamma = torch.ones(C, **f32)
    beta = torch.zeros(C, **f32)
    rm, rv = torch.zeros(C, **f32), torch.ones(C, **f32)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    part, tick = _Workspace.get(dev, C)
    stats = torch.empty(3 * C + 4, **f32)
    save = torch.empty(2 * C, **f32)
    out = torch.empty(2 * C, **f32)
    dg, db = torch.empty(C, **f32), torch.empty(C, **f32)
    dx = torch.empty_like(x)
    dres = torch.empty_like(x)
    gb = M * C * 2 / 1e9
    K.fwd_stats(x, C, shift, part, tick, stats, nbt)
    K.apply(x, None, yb, C, stats, gamma, beta, rm, rv, nbt, 0.1, 1e-5, True, True, save)
    ref = {}
    for wt in (0, 1):
        K.set_handoff(wt)
        for st in (128, 256, 512, 1024, 2048):
            K.set_grid_targets(st, 512, 1024)
            a = tm(lambda: K.bwd_stats(dy, yb, x, C, 1, save, gamma, beta, part, tick, out, dg, db))
            b = tm(lambda: K.bwd_stats(dy, None, x, C, 2, save, gamma, beta, part, tick, out, dg, db))
            same = bool(torch.equal(out, ref[st])) if wt else True  # fixed-order sums: bitwise equal
            ref[st] = out.clone()
            print(f"M={M:7d} C={C:4d} wt={wt} st={st:5d} bstats_y={a:7.1f}us({3 * gb / a * 1e3:4.1f}TB/s) "
                  f"bstats_rc={b:7.1f}us({2 * gb / b * 1e3:4.1f}TB/s) same={same}", flush=True)
    K.set_handoff(1)
    K.set_grid_targets(0, 512, 1024)
    for el in (512, 1024, 2048, 4096):
        K.set_grid_targets(0, el, el)
        a = tm(lambda: K.apply(x, res, yb, C, stats, gamma, beta, rm, rv, nbt, 0.1, 1e-5, True, True, save))
        b = tm(lambda: K.bwd_elemt(dy, yb, x, C, 1, save, out, stats, gamma, beta, dx, dres))
        c = tm(lambda: K.bwd_elemt(dy, None, x, C, 2, save, out, stats, gamma, beta, dx, None))
        print(f"M={M:7d} C={C:4d} el={el:5d} apply_res={a:7.1f}us({3 * gb / a * 1e3:4.1f}TB/s) "
              f"belemt_y={b:7.1f}us({5 * gb / b * 1e3:4.1f}TB/s) belemt_rc={c:7.1f}us({3 * gb / c * 1e3:4.1f}TB/s)",
              flush=True)
    K.set_grid_targets(0, 512, 1024)
