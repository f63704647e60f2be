"""Experiment: eager training steps on the default stream, then hipGraph capture of the
same step (torch.cuda.graph).  MODE=torch: plain torch modules/optimizer; MODE=native:
this package's ConvNet + SGD + GradScaler."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
mode = os.environ.get("MODE", "torch")
dev = torch.device("cuda", 0)
torch.manual_seed(0)
x = torch.rand(32, 1, 28, 28, device=dev)
y = torch.randint(0, 10, (32,), device=dev)
if mode == "torch":
    m = torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(784, 10)).to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)

    def step():
        loss = torch.nn.functional.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
else:
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD

    m = ConvNet(amp_dtype=torch.bfloat16 if mode == "native" else None).to(dev)
    x = x.to(torch.bfloat16) if mode == "native" else x
    opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(enabled=mode == "native"), CrossEntropyLoss()

    def step():
        loss = crit(m(x), y)
        opt.zero_grad(set_to_none=True)
        if mode == "native":
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward()
            opt.step()
for _ in range(int(os.environ.get("EAGER", "3"))):
    step()
torch.cuda.synchronize()
if os.environ.get("GC") == "1":
    import collections
    import gc

    gc.set_debug(gc.DEBUG_SAVEALL)
    print("gc found", gc.collect(), "unreachable objects", flush=True)
    cnt = collections.Counter(type(o).__name__ for o in gc.garbage)
    print(cnt.most_common(30), flush=True)
    for o in gc.garbage:
        if type(o).__name__ in ("function", "cell", "dict", "tuple"):
            try:
                print(type(o).__name__, repr(o)[:300], flush=True)
            except Exception:
                pass
    gc.set_debug(0)
    gc.garbage.clear()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print("capturing", flush=True)
with torch.cuda.graph(g):
    step()
g.replay()
torch.cuda.synchronize()
print(f"{mode}: capture after eager ok", flush=True)
