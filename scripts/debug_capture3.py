"""Isolate which piece of the reducer breaks hipGraph capture."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._dist import free_port
import ddp_practice_amd.distributed as dist
from ddp_practice_amd import _ext

stage = sys.argv[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
torch.cuda.set_device(0)
c = dist.init_process_group("nccl")
C = _ext.load()
rc = c.native
flat = torch.zeros(1000, device="cuda")
ts = [torch.ones(10, device="cuda"), torch.ones(20, device="cuda")]
w = torch.nn.Parameter(torch.ones(10, device="cuda"))

def body():
    if stage == "flatcopy":
        C.optim.flat_copy(ts, [0, 10], flat, 0.5, 0)
    elif stage == "async_main":
        flat.add_(1)
        rc.all_reduce_async(flat, "sum", 0)
        rc.wait(0)
    elif stage in ("hook_async", "hook_fenced", "hook_flatcopy"):
        w.grad = None
        (w * 2).sum().backward()
    elif stage == "reducer":
        w.grad = None
        red.prepare_for_backward(True)
        (w * 2).sum().backward()

if stage.startswith("hook"):
    def hook(p):
        if stage == "hook_async":
            rc.all_reduce_async(p.grad, "sum", 0)
            rc.wait(0)
        elif stage == "hook_fenced":
            rc.all_reduce(p.grad, "sum")
        else:
            C.optim.flat_copy([p.grad], [0], flat, 1.0, 0)
    w.register_post_accumulate_grad_hook(hook)
if stage == "reducer":
    red = C.ddp.Reducer([w], [[0]], rc, False)

s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("warmup ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
print("capture ok", flush=True)
g.replay()
torch.cuda.synchronize()
print("replay ok", stage, flush=True)
