"""Per-shape A/B of conv_glds_kernel variants on every ResNet-50 (bs 128) forward conv
shape, with the BN statistics, interleaved rounds in one process (median of 5).

  STAGES=2,3,4 python scripts/exp/stage_ab.py   LDS stages (2: one tile in flight, two
                                                workgroups per CU; 3-4: one workgroup per CU)
  WIDE=0,2,3,4 python scripts/exp/stage_ab.py   tiles (conv_igemm.wide_config: 0 the 4-wave
                                                128 x 128, 2: 256 x 128, 3: 256 x 256, 4: 128 x
                                                128 on 8 waves)
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
K_ = C.conv_igemm
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


WIDE = "WIDE" in os.environ
STAGES = [int(s) for s in os.environ.get("WIDE" if WIDE else "STAGES", "2,3").split(",")]
cfg = K_.wide_config if WIDE else K_.glds_config
tot = {s: 0.0 for s in STAGES}
best = 0.0
print(f"{'shape (Cin,H,Cout,R,s)':26s} {'GFLOP':>6s} {'WGs':>6s} " + " ".join(f"{('w' if WIDE else 'ns') + str(s):>8s}" for s in STAGES))
for Cin, H, K, R, st, cnt in SHAPES:
    pad = R // 2
    g = torch.Generator().manual_seed(Cin + K + H)
    x = torch.randn(B, Cin, H, H, generator=g).to("cuda", torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(K, Cin, R, R, generator=g) / (Cin * R * R) ** 0.5).to("cuda", torch.bfloat16).contiguous(
        memory_format=CL)
    OH = (H + 2 * pad - R) // st + 1
    y = torch.empty(B, K, OH, OH, dtype=torch.bfloat16, device="cuda", memory_format=CL)
    M = B * OH * OH
    part = torch.empty(K_.stat_part_len(M, K), device="cuda")
    tk = torch.zeros(K_.stat_tickets_len(M, K), dtype=torch.int32, device="cuda")
    sts = torch.empty(3 * K + 4, device="cuda")
    shift = torch.zeros(K, device="cuda")
    fl = 2.0 * M * K * Cin * R * R / 1e9
    ts = {s: [] for s in STAGES}
    outs = {}
    for _ in range(5):
        for s in STAGES:
            prev = cfg(s)
            ts[s].append(timeit(lambda: K_.conv_fwd(x, w, y, st, pad, part, tk, sts, shift, None)))
            outs[s] = (y.clone(), sts.clone())
            cfg(prev)
    med = {s: statistics.median(v) for s, v in ts.items()}
    for s in STAGES:
        tot[s] += med[s] * cnt
    best += min(med.values()) * cnt
    same = all(torch.equal(outs[s][0], outs[STAGES[0]][0]) for s in STAGES)
    # statistics: the same sums in another association when the tiles differ
    serr = max(((outs[s][1][:2 * K] - outs[STAGES[0]][1][:2 * K]).abs().max()
                / outs[STAGES[0]][1][:2 * K].abs().max().clamp_min(1e-30)).item() for s in STAGES)
    wgs = (M + 127) // 128 * (K // (128 if K % 128 == 0 else 64))
    print(f"{str((Cin, H, K, R, st)):26s} {fl:6.2f} {wgs:6d} " + " ".join(f"{med[s]:8.1f}" for s in STAGES)
          + f"  x{cnt} {'bitwise-same' if same else 'DIFFERENT'} stats-rel {serr:.1e}", flush=True)
print("network forward convs (x count): " + ", ".join(f"{'w' if WIDE else 'ns'}{s} {tot[s]:.0f} us" for s in STAGES)
      + f", best per shape {best:.0f} us")
