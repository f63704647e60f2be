"""Measure the per-kernel launch floor on this box (eager vs hipGraph, C++ and torch)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
buf = torch.zeros(16, device="cuda")
res = {}
for blocks in (1, 64):
    res[f"cpp_eager_b{blocks}"] = C.launch_floor(buf, 200, 20, False, blocks)
    res[f"cpp_graph_b{blocks}"] = C.launch_floor(buf, 200, 20, True, blocks)
# torch graph of tiny torch ops
x = torch.zeros(1, device="cuda")
def f():
    for _ in range(100):
        x.add_(1)
for _ in range(3):
    f()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    f()
torch.cuda.synchronize()
res["torch_eager_add"] = (time.perf_counter() - t0) / 1000 * 1e6
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    f()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    f()
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
res["torch_graph_add"] = (time.perf_counter() - t0) / 2000 * 1e6
res["env"] = {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "HSA_", "GPU_", "AMD_"))}
print(json.dumps(res, indent=1))
