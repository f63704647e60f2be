"""Bisect hipGraph capture of the DDP step: python scripts/debug_capture.py STAGE"""
import copy, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._dist import free_port
import ddp_practice_amd.distributed as dist
from ddp_practice_amd.parallel import comm as comm_mod
from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
from ddp_practice_amd.models import ConvNet
from ddp_practice_amd.ops.head import cross_entropy

stage = sys.argv[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
torch.cuda.set_device(0)
dist.init_process_group("nccl")
comm_mod.Communicator.force_active = True
torch.manual_seed(0)
m = ConvNet().cuda()
if "sync" in stage:
    m = convert_sync_batchnorm(m)
if "ddp" in stage:
    m = DistributedDataParallel(m, device_ids=[0])
x = torch.rand(32, 1, 28, 28, device="cuda")
y = torch.randint(0, 10, (32,), device="cuda")

def step():
    out = m(x)
    if "fwd" in stage:
        return
    loss = cross_entropy(out, y)
    for p in m.parameters():
        p.grad = None
    loss.backward()

s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("warmup ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
print("capture ok", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("replay ok", stage, flush=True)
dist.destroy_process_group()
