"""Dispatch skew per XCD: start time (s_memrealtime, 10 ns) and XCC id of every
workgroup of one launch, for a few grid sizes, eager and graph-replayed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
dev = "cuda"
for blocks in (8, 32, 64, 256, 1024):
    for spin in (0, 200):
        out = torch.zeros(3 * blocks, dtype=torch.int64, device=dev)
        for _ in range(3):
            C.xcd_probe(out, blocks, spin)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            C.xcd_probe(out, blocks, spin)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            C.xcd_probe(out, blocks, spin)
        for mode in ("eager", "graph"):
            (C.xcd_probe(out, blocks, spin) if mode == "eager" else g.replay())
            torch.cuda.synchronize()
            r = out.view(-1, 3).cpu()
            t0 = r[:, 0].min()
            st = (r[:, 0] - t0).float() / 100  # us
            xcc = r[:, 1]
            per = []
            for x in range(8):
                m = xcc == x
                per.append(f"{st[m].min().item():5.2f}/{st[m].max().item():5.2f}" if m.any() else "  -  ")
            mapping = "id%8==xcc" if bool((xcc == torch.arange(blocks) % 8).all()) else "other"
            print(f"blocks={blocks:5d} spin={spin:4d} {mode:5s} skew={st.max().item():5.2f}us "
                  f"map={mapping} per-xcc first/last start: {' '.join(per)}", flush=True)
