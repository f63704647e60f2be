"""Eager vs 1-step-graph training of the same ConvNet (amp, head step): parameter and
loss differences after every step, to find the first step that diverges."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd.amp import GradScaler  # noqa: E402
from ddp_practice_amd.data import DeviceLoader, ImageDataset, synthetic  # noqa: E402
from ddp_practice_amd.engine import TrainLoop  # noqa: E402
from ddp_practice_amd.models import ConvNet  # noqa: E402
from ddp_practice_amd.nn import CrossEntropyLoss  # noqa: E402
from ddp_practice_amd.optim import SGD  # noqa: E402


def mk(model, ds, graph):
    loader = DeviceLoader(ImageDataset(ds.images, ds.labels), batch_size=32, shuffle=False, device="cuda",
                          dtype=torch.bfloat16)
    loop = TrainLoop(model, CrossEntropyLoss(), SGD(model.parameters(), lr=0.05), loader, GradScaler(),
                     use_graph=graph, steps_per_graph=1)
    return loop


ds = synthetic(32 * 8, seed=11)
torch.manual_seed(0)
base = ConvNet(amp_dtype=torch.bfloat16).cuda()
a, b = copy.deepcopy(base), copy.deepcopy(base)
la, lb = mk(a, ds, False), mk(b, ds, True)
la.loader.start_epoch()
lb.loader.start_epoch()
g = lb._graph(1)
print("graph captured:", g is not None, lb.graph_error, flush=True)
for i in range(8):
    la._eager_step()
    g.run()
    torch.cuda.synchronize()
    worst = max(((p.float() - q.float()).abs().max().item(), n)
                for (n, p), (_, q) in zip(a.state_dict().items(), b.state_dict().items()))
    ga = {n: p.grad for n, p in a.named_parameters()}
    gd = max(((ga[n].float() - p.grad.float()).abs().max().item(), n) for n, p in b.named_parameters()
             if p.grad is not None and ga[n] is not None)
    print(f"step {i}: worst param diff {worst}, worst grad diff {gd}, scale {la.scaler._scale.item()} "
          f"{lb.scaler._scale.item()}", flush=True)
