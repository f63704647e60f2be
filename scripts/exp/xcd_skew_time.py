"""Is the per-XCC start offset real or a clock offset?  Time 50 back-to-back launches
of the probe in one graph (spin = 0 / 2 / 5 us per workgroup) for several grids: a real
dispatch stagger adds ~the offset to every launch; a clock offset adds nothing."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
for blocks in (1, 8, 32, 256):
    for spin in (0, 200, 500):
        out = torch.zeros(3 * blocks, dtype=torch.int64, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            C.xcd_probe(out, blocks, spin)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(50):
                C.xcd_probe(out, blocks, spin)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        per = e0.elapsed_time(e1) / 200 * 1e3
        r = out.view(-1, 3).cpu()
        sk = (r[:, 0].max() - r[:, 0].min()).item() / 100
        print(f"blocks={blocks:4d} spin={spin / 100:4.1f}us: {per:6.2f} us per launch (measured start skew {sk:.2f} us)",
              flush=True)
