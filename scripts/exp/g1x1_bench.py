"""ResNet-50 (bs 128) 1x1 conv shapes: conv_glds_kernel (256- and 128-pixel tiles, +BN
statistics) vs the general implicit-GEMM kernel vs hipBLASLt (torch.mm), with the error
of each against an fp32 reference.  Forward shapes and the data-gradient GEMMs
(dX[P, Cin] = dY[P, Cout] @ W: the 1x1 conv Cout -> Cin on dy, stride 1).

  python scripts/exp/g1x1_bench.py  [BS=128]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
K_ = C.conv_igemm
DEFER_DEFAULT = K_.stat_defer_config()
CL = torch.channels_last
B = int(os.environ.get("BS", "128"))
# (Cin, H, Cout, stride, count in the network) -- forward 1x1 convs
FWD = [(64, 56, 64, 1, 1), (64, 56, 256, 1, 4), (256, 56, 64, 1, 2), (256, 56, 128, 1, 1),
       (128, 28, 512, 1, 4), (512, 28, 128, 1, 3), (256, 56, 512, 2, 1), (512, 28, 256, 1, 1),
       (256, 14, 1024, 1, 6), (1024, 14, 256, 1, 5), (512, 28, 1024, 2, 1), (1024, 14, 512, 1, 1),
       (512, 7, 2048, 1, 3), (2048, 7, 512, 1, 2), (1024, 14, 2048, 2, 1)]
# data gradients: conv Cin -> Cout at output size OH becomes Cout -> Cin on dy (stride 1)
DGRAD = sorted({(k, (h + s - 1) // s, c, 1, n) for c, h, k, s, n in FWD})


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


def run(table, title, stats):
    print(f"## {title} ({'with' if stats else 'no'} BN statistics)")
    # bp256 / bp128: that tile, in-launch statistics tree; auto / old: default tile and tree
    # placement (deferred past DPA_STAT_DEFER_MIN workgroups) on the 1x1 / general kernel
    print(f"{'shape (Cin,H,Cout,s)':26s} {'GFLOP':>6s} {'bp256':>7s} {'bp128':>7s} {'auto':>7s} {'old':>7s} "
          f"{'hipBLASLt':>9s} {'TF/s':>5s} {'vsLib':>5s} err")
    tot = {"auto": 0.0, "old": 0.0, "lib": 0.0}
    for Cin, H, K, st, cnt in table:
        g = torch.Generator().manual_seed(Cin + K + H)
        x = torch.randn(B, Cin, H, H, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(K, Cin, 1, 1, generator=g) / Cin ** 0.5).to("cuda", torch.bfloat16).contiguous(
            memory_format=CL)
        OH = (H - 1) // st + 1
        M = B * OH * OH
        y = torch.empty(B, K, OH, OH, dtype=torch.bfloat16, device="cuda", memory_format=CL)
        part = torch.empty(K_.stat_part_len(M, K), device="cuda")
        tk = torch.zeros(K_.stat_tickets_len(M, K), dtype=torch.int32, device="cuda")
        sts = torch.empty(3 * K + 4, device="cuda")
        shift = torch.zeros(K, device="cuda")
        args = (part, tk, sts, shift, None) if stats else ()
        fn = lambda: K_.conv_fwd(x, w, y, st, 0, *args)  # noqa: E731
        ref = torch.nn.functional.conv2d(x.float(), w.float(), None, st)
        res, errs = {}, []
        for name, cfg in (("bp256", (1, 256, -1)), ("bp128", (1, 128, -1)), ("auto", (1, 0, DEFER_DEFAULT)),
                          ("old", (0, 0, DEFER_DEFAULT))):
            K_.g1x1_config(cfg[0], cfg[1])
            K_.stat_defer_config(cfg[2])  # -1: never defer
            res[name] = timeit(fn)
            fn()
            torch.cuda.synchronize()
            errs.append(((y.float() - ref).abs().max() / ref.abs().max()).item())
            if stats and name != "old":
                yr = y.float().permute(0, 2, 3, 1).reshape(-1, K)
                assert torch.allclose(sts[:K], yr.sum(0), rtol=1e-3, atol=1e-1 * (M / 1e4)), name
        K_.g1x1_config(1, 0)
        K_.stat_defer_config(DEFER_DEFAULT)
        xs = x[:, :, ::st, ::st] if st > 1 else x
        rows = xs.permute(0, 2, 3, 1).contiguous().reshape(-1, Cin)
        wm = w.reshape(K, Cin)
        res["lib"] = timeit(lambda: torch.mm(rows, wm.t()))
        fl = 2.0 * M * K * Cin / 1e9
        for k in tot:
            tot[k] += res[k] * cnt
        print(f"{str((Cin, H, K, st)):26s} {fl:6.2f} {res['bp256']:7.1f} {res['bp128']:7.1f} {res['auto']:7.1f} "
              f"{res['old']:7.1f} {res['lib']:9.1f} {fl / res['auto'] * 1e3:5.0f} {res['lib'] / res['auto']:5.2f} "
              f"{max(errs):.1e} x{cnt}")
    print(f"network total (x count): auto {tot['auto']:.0f} us, old kernel {tot['old']:.0f} us, "
          f"hipBLASLt {tot['lib']:.0f} us\n")


if __name__ == "__main__":
    run(FWD, "forward 1x1 convs", True)
    run(DGRAD, "data-gradient GEMMs", False)
