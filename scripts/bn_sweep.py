"""Sweep the NHWC BatchNorm kernels' workgroup-count targets on ResNet-50 (bs 128)
activation shapes: per-call time of forward stats / apply / backward stats /
backward elemt, and the implied HBM bandwidth."""
import itertools
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts", 1)[0])
from ddp_practice_amd import _ext  # noqa: E402
from ddp_practice_amd.ops.bn_nhwc import _Workspace  # noqa: E402

K = _ext.load().bn_nhwc
dev = torch.device("cuda")
shapes = [(128 * 56 * 56, 64), (128 * 56 * 56, 256), (128 * 28 * 28, 512), (128 * 14 * 14, 1024),
          (128 * 7 * 7, 2048), (128 * 28 * 28, 128)]


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
    best = {}
    for st, el in itertools.product((64, 128, 256, 512), (256, 512, 1024, 2048)):
        K.set_grid_targets(st, el, el)
        r = {
            "fstats": (tm(lambda: K.fwd_stats(x, C, shift, part, tick, stats, None)), 1),
            "apply_res": (tm(lambda: K.apply(x, res, yb, C, stats, gamma, beta, rm, rv, nbt, 0.1, 1e-5, True, True,
                                             save)), 3),
            "bstats_y": (tm(lambda: K.bwd_stats(dy, yb, x, C, 1, save, gamma, beta, part, tick, out, dg, db)), 3),
            "bstats_rc": (tm(lambda: K.bwd_stats(dy, None, x, C, 2, save, gamma, beta, part, tick, out, dg, db)), 2),
            "belemt_y": (tm(lambda: K.bwd_elemt(dy, yb, x, C, 1, save, out, stats, gamma, beta, dx, dres)), 5),
            "belemt_rc": (tm(lambda: K.bwd_elemt(dy, None, x, C, 2, save, out, stats, gamma, beta, dx, None)), 3),
        }
        for k, (us, nt) in r.items():
            key = k
            tgt = st if "stats" in k else el
            if key not in best or us < best[key][0]:
                best[key] = (us, tgt, nt * gb / us * 1e3)
        print(f"M={M:7d} C={C:4d} st={st:5d} el={el:5d} " +
              " ".join(f"{k}={us:7.1f}us({nt * gb / us * 1e3:4.1f}TB/s)" for k, (us, nt) in r.items()), flush=True)
    print(f"BEST M={M} C={C}: " + " ".join(f"{k}:{v[0]:.1f}us@{v[1]}({v[2]:.1f}TB/s)" for k, v in best.items()),
          flush=True)
