import copy, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._dist import free_port
import ddp_practice_amd.distributed as dist
from ddp_practice_amd.parallel import comm as comm_mod
from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
from ddp_practice_amd.models import ConvNet
from ddp_practice_amd.data import synthetic
from tests.test_dist_gpu import _train

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
torch.cuda.set_device(0)
dist.init_process_group("nccl")
comm_mod.Communicator.force_active = True
ds = synthetic(32 * 9 + 5, seed=11)

def cmp(a, b, tag):
    worst = max(((p.float() - q.float()).abs().max().item(), n) for (n, p), (_, q) in zip(a.state_dict().items(), b.state_dict().items()))
    print(tag, worst, flush=True)

for variant in ["syncbn_only", "ddp_plainbn", "ddp_syncbn"]:
    torch.manual_seed(0)
    plain = ConvNet().cuda()
    m = copy.deepcopy(plain)
    if variant in ("syncbn_only", "ddp_syncbn"):
        m = convert_sync_batchnorm(m)
    if variant.startswith("ddp"):
        m = DistributedDataParallel(m, device_ids=[0])
    _train(plain, 1, ds.images, ds.labels, False, use_graph=False)
    _train(m, 1, ds.images, ds.labels, False, use_graph=False)
    mm = m.module if hasattr(m, "module") else m
    cmp(mm, plain, variant)
dist.destroy_process_group()
