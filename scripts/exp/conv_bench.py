"""ResNet-50 (bs 128) conv shapes: conv_igemm.conv_fwd (+stats) vs MIOpen / hipBLASLt."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
CL = torch.channels_last
B = int(os.environ.get("BS", "128"))
# (Cin, H, Cout, R, stride, count in the network)
SHAPES = [(64, 56, 64, 3, 1, 3), (128, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 3), (256, 28, 256, 3, 2, 1),
          (256, 14, 256, 3, 1, 5), (512, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 2),
          (64, 56, 64, 1, 1, 1), (64, 56, 256, 1, 1, 4), (256, 56, 64, 1, 1, 2), (256, 56, 128, 1, 1, 1),
          (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (256, 56, 512, 1, 2, 1), (512, 28, 256, 1, 1, 1),
          (256, 14, 1024, 1, 1, 6), (1024, 14, 256, 1, 1, 5), (512, 28, 1024, 1, 2, 1), (1024, 14, 512, 1, 1, 1),
          (512, 7, 2048, 1, 1, 3), (2048, 7, 512, 1, 1, 2), (1024, 14, 2048, 1, 2, 1)]


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


tot_me = tot_ref = tot_wme = tot_wref = tot_wold = 0.0
from ddp_practice_amd.ops.conv_igemm import conv_wgrad  # noqa: E402
print(f"{'shape':34s} {'GFLOP':>7s} {'mine us':>8s} {'TF/s':>6s} {'nostat':>7s} {'ref us':>8s} {'TF/s':>6s} "
      "(gen: the register-staged kernel for KxK)")
for Cin, H, K, R, st, cnt in SHAPES:
    pad = R // 2
    x = torch.randn(B, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    w = torch.randn(K, Cin, R, R, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // st + 1
    y = torch.empty(B, K, OH, OH, dtype=torch.bfloat16, device="cuda", memory_format=CL)
    M = B * OH * OH
    part = torch.empty(C.conv_igemm.stat_part_len(M, K), device="cuda")
    tk = torch.zeros(C.conv_igemm.stat_tickets_len(M, K), dtype=torch.int32, device="cuda")
    sts = torch.empty(3 * K + 4, device="cuda")
    shift = torch.zeros(K, device="cuda")
    fl = 2.0 * M * K * Cin * R * R / 1e9
    prev3 = C.conv_igemm.g3x3_config(0)
    t_gen = timeit(lambda: C.conv_igemm.conv_fwd(x, w, y, st, pad, part, tk, sts, shift, None))
    C.conv_igemm.g3x3_config(prev3)
    t_me = timeit(lambda: C.conv_igemm.conv_fwd(x, w, y, st, pad, part, tk, sts, shift, None))
    t_ns = timeit(lambda: C.conv_igemm.conv_fwd(x, w, y, st, pad))
    if R == 1:
        xs = x[:, :, ::st, ::st] if st > 1 else x
        rows = xs.permute(0, 2, 3, 1).reshape(-1, Cin) if st == 1 else xs.permute(0, 2, 3, 1).contiguous().reshape(-1, Cin)
        wm = w.reshape(K, Cin)
        t_ref = timeit(lambda: torch.mm(rows, wm.t()))
    else:
        t_ref = timeit(lambda: torch.ops.aten.convolution(x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1))
    ref = torch.ops.aten.convolution(x.float(), w.float(), None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1)
    C.conv_igemm.conv_fwd(x, w, y, st, pad, part, tk, sts, shift, None)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    dy = torch.randn_like(y)
    wshape = tuple(w.shape)
    C.conv_igemm.wgrad_config(0)
    t_wold = timeit(lambda: conv_wgrad(dy, x, wshape, st, pad))
    C.conv_igemm.wgrad_config(2)
    t_wme = timeit(lambda: conv_wgrad(dy, x, wshape, st, pad))
    t_wref = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                [0, 0], 1, [False, True, False]))
    C.conv_igemm.wgrad_config(1)
    gw = conv_wgrad(dy, x, wshape, st, pad)
    rw = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [st, st], [pad, pad], [1, 1],
                                             False, [0, 0], 1, [False, True, False])[1]
    werr = ((gw - rw).abs().max() / rw.abs().max()).item()
    tot_wme += t_wme * cnt
    tot_wold += t_wold * cnt
    tot_wref += t_wref * cnt
    tot_me += t_me * cnt
    tot_ref += t_ref * cnt
    print(f"{str((Cin, H, K, R, st)):34s} {fl:7.2f} {t_me:8.1f} {fl / t_me * 1e3:6.0f} {t_ns:7.1f} {t_ref:8.1f} "
          f"{fl / t_ref * 1e3:6.0f}  gen {t_gen:6.1f} err={err:.1e} | wgrad glds {t_wme:7.1f} reg {t_wold:7.1f} MIOpen {t_wref:7.1f} "
          f"err={werr:.1e} x{cnt}")
print(f"network forward convs (x count): mine {tot_me:.0f} us, reference {tot_ref:.0f} us "
      "(mine includes the BN statistics; reference does not)")
print(f"network wgrad (x count): glds {tot_wme:.0f} us, register-staged {tot_wold:.0f} us, MIOpen {tot_wref:.0f} us")
