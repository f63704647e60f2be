"""Which conv1-wgrad path do the plain / DDP(forced) runs take, eager vs graph? (debug)"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
calls = {}


def spy(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        calls[name] = calls.get(name, 0) + 1
        return f(*a, **k)
    setattr(mod, name, g)


for mod, name in ((C.convnet, "convnet_amp_step"), (C.convnet, "conv1_wgrad_slab2"), (C.convblock, "slab_reduce"),
                  (C.convnet, "conv_wgrad_bn"), (C.optim, "amp_sgd_fused")):
    spy(mod, name)

import ddp_practice_amd.distributed as dist  # noqa: E402
from tests.test_dist_gpu import _train  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
from bench import _force_collectives  # noqa: E402

_force_collectives()
dist.init_process_group("nccl")
from ddp_practice_amd.data import synthetic  # noqa: E402
from ddp_practice_amd.models import ConvNet  # noqa: E402
from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm  # noqa: E402

ds = synthetic(32 * 9 + 5, seed=11)
from ddp_practice_amd.ops import convnet_fused as cf  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "all"
for tag, defer, wrap, graph in (("plain graph (merged)", True, False, True), ("ddp graph, no wgrad1 defer", False, True, True),
                                ("ddp graph (merged)", True, True, True)):
    cf._DEFER_WGRAD1 = defer
    torch.manual_seed(0)
    plain = ConvNet(amp_dtype=torch.bfloat16).cuda()
    ref = copy.deepcopy(plain)
    model = DistributedDataParallel(convert_sync_batchnorm(copy.deepcopy(plain)), device_ids=[0]) if wrap else plain
    _train(ref, 2, ds.images, ds.labels, True, use_graph=False)
    calls.clear()
    _train(model, 2, ds.images, ds.labels, True, use_graph=graph)
    mm = model.module if wrap else model
    worst = max(((p.float() - q.float()).abs().max().item(), n)
                for (n, p), (_, q) in zip(mm.state_dict().items(), ref.state_dict().items()))
    print(tag, dict(calls), "worst", worst, flush=True)
