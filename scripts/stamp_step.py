"""Phase timing of the fused ConvNet step kernels (experiment build with -DDPA_TIMING):
    DPA_BUILD_TAG=timing DPA_EXTRA_CFLAGS=-DDPA_TIMING python -m ddp_practice_amd.build
    DPA_EXT_SO=ddp_practice_amd/_C_timing.so python scripts/stamp_step.py [--forced]
--forced: the W>1 step shape on one GPU (DDP + SyncBN with every collective forced at W=1,
the xGMI engine's in-kernel exchanges), as bench.py --force-collectives.
For the head step (convnet_head.head_step) and the merged layer-2 backward
(convnet.conv2_bwd, roles split by block range): blocks, span (first start ->
last stamp), start skew, and the mean time of each stamped phase relative to
the block's own start (us)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddp_practice_amd import _ext  # noqa: E402

C = _ext.load()
report = []


DUMP_STARTS = "--starts" in sys.argv


def starts_line(name, rows):
    """Workgroup start offsets (us after the first) by block index: dispatch order / rate."""
    st = (rows[:, 0] - rows[:, 0].min()) / 100
    n = len(st)
    q = [st[int(i * (n - 1) / 8)].item() for i in range(9)]
    srt = st.sort().values
    qs = [srt[int(i * (n - 1) / 8)].item() for i in range(9)]
    # the hardware deals workgroup i to XCD i % 8: mean start per XCD (a consistent late XCD
    # would be worth giving the least work)
    bx = torch.arange(n) % 8
    xcd = [st[bx == x].mean().item() if (bx == x).any() else float("nan") for x in range(8)]
    return (f"{name:18s} start by block index (every n/8-th): " + " ".join(f"{v:4.2f}" for v in q) +
            " | sorted quantiles: " + " ".join(f"{v:4.2f}" for v in qs) +
            " | mean by XCD: " + " ".join(f"{v:4.2f}" for v in xcd))


def summarize(name, rows):
    if len(rows) == 0:
        return f"{name:18s} no stamps"
    if DUMP_STARTS:
        report.append(starts_line(name, rows))
    t0 = rows[:, 0].min()
    end = rows.max(dim=1).values
    line = (f"{name:18s} blocks={len(rows):4d} span={(end.max() - t0).item() / 100:6.2f}us "
            f"skew={(rows[:, 0].max() - t0).item() / 100:5.2f}us phases:")
    for i in range(1, 16):
        col = rows[:, i]
        ok = col > 0
        if ok.any():
            rel = (col[ok] - rows[ok, 0]) / 100
            line += f" s{i}={rel.mean().item():5.2f}/{rel.max().item():5.2f}"
    return line


def wrap(mod, name, roles):
    f = getattr(mod, name)

    def g(*a):
        mod.clear_stamps()
        torch.cuda.synchronize()
        f(*a)
        st = mod.read_stamps().double()
        for rname, sel in roles(a):
            rows = st[sel]
            rows = rows[rows[:, 0] > 0]
            report.append(summarize(rname, rows))
    setattr(mod, name, g)


B = 32
wrap(C.convnet_head, "head_step", lambda a: [("head_step", slice(0, 32))])
wrap(C.convnet, "conv2_bwd", lambda a: [("conv2_bwd/dgrad", slice(0, 2 * B)),
                                         ("conv2_bwd/wgrad", slice(2 * B, 2 * B + 4 * B))])
wrap(C.convnet, "conv2_fwd", lambda a: [("conv2_fwd", slice(0, 2 * B))])
wrap(C.convnet, "wgrad1_reduce", lambda a: [("wgrad1_reduce/wgrad", slice(0, 7 * B))])
wrap(C.convnet, "conv1_wgrad_slab2", lambda a: [("wgrad1_slab2/wgrad", slice(0, 7 * B)),
                                                 ("wgrad1_slab2/sums", slice(7 * B, 512))])
wrap(C.convnet, "convnet_amp_step", lambda a: [("amp_step/producers", slice(0, 7 * B)),
                                                ("amp_step/amp", slice(7 * B, 512))])
wrap(C.optim, "amp_sgd_fused", lambda a: [("amp_sgd_fused", slice(0, 512))])
FORCED = "--forced" in sys.argv
if FORCED:
    from ddp_practice_amd.parallel import comm as comm_mod  # noqa: E402
    import ddp_practice_amd.distributed as ddist  # noqa: E402

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29517"), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    comm_mod.Communicator.force_active = True
    torch.cuda.set_device(0)
    ddist.init_process_group("nccl")

from ddp_practice_amd.amp import GradScaler  # noqa: E402
from ddp_practice_amd.data import DeviceLoader  # noqa: E402
from ddp_practice_amd.models import ConvNet  # noqa: E402
from ddp_practice_amd.nn import CrossEntropyLoss  # noqa: E402
from ddp_practice_amd.optim import SGD  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = ConvNet(amp_dtype=torch.bfloat16).to(dev)
if FORCED:
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm  # noqa: E402

    m = DistributedDataParallel(convert_sync_batchnorm(m), device_ids=[0])
opt = SGD(m.parameters(), lr=1e-4)
scaler = GradScaler()
if not FORCED or m.defer_grad_sync_to(opt):  # as engine.TrainLoop
    m.set_slab_sink(opt)  # conv1's weight-gradient sums inside the optimizer launch
crit = CrossEntropyLoss()
for it in range(4):
    x = torch.rand(B, 1, 28, 28, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev)
    DeviceLoader.pair(x, y)
    report.clear()
    loss = crit(m(x), y)
    opt.zero_grad(set_to_none=True)
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    torch.cuda.synchronize()
for r in report:
    print(r)
