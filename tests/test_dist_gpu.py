"""Single-GPU checks of the distributed stack: native RCCL communicator, DDP
reducer, SyncBN-in-fused-block, all under hipGraph capture.

World size is 1 on the test box; ``Communicator.force_active`` makes every
collective code path run anyway (RCCL all-reduce of a world of one is the
identity, so results must equal the non-distributed run).
"""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl(C):
    import ddp_practice_amd.distributed as dist
    from ddp_practice_amd.parallel import comm as comm_mod

    from ._dist import free_port

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    old = comm_mod.Communicator.force_active
    comm_mod.Communicator.force_active = True  # W=1 without it gets the LocalCommunicator
    c = dist.init_process_group("nccl")
    assert isinstance(c, comm_mod.RcclCommunicator)
    yield c
    comm_mod.Communicator.force_active = old
    dist.destroy_process_group()


def test_rccl_collectives_world1(rccl):
    t = torch.arange(8, dtype=torch.float32, device="cuda")
    rccl.all_reduce_(t)
    assert t.tolist() == list(range(8))
    o = rccl.all_reduce(t, "max")
    assert torch.equal(o, t) and o.data_ptr() != t.data_ptr()
    rccl.broadcast_(t, 0)
    rccl.reduce_(t, 0)
    out = torch.empty(8, device="cuda")
    rccl.all_gather_into_tensor(out, t)
    assert torch.equal(out, t)
    rccl.reduce_scatter_tensor(out, t)
    rccl.all_to_all_single(out, t)
    assert torch.equal(out, t)
    for dt in (torch.bfloat16, torch.float16, torch.int64):
        x = torch.ones(5, dtype=dt, device="cuda")
        rccl.all_reduce_(x)
        assert x.float().sum().item() == 5
    rccl.barrier()
    assert rccl.async_error() == ""


def test_rccl_under_graph_capture(rccl):
    x = torch.ones(1024, device="cuda")
    y = torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        rccl.all_reduce_(x)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        x.mul_(2)
        rccl.all_reduce_(x)
        y.copy_(x)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert y[0].item() == 8.0


def _train(model, steps, images, labels, scaler_on, use_graph, batch=32):
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, ImageDataset
    from ddp_practice_amd.engine import TrainLoop
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD

    ds = ImageDataset(images, labels)
    loader = DeviceLoader(ds, batch_size=batch, shuffle=False, device="cuda",
                          dtype=torch.bfloat16 if scaler_on else torch.float32)
    opt = SGD(model.parameters(), lr=0.05)
    scaler = GradScaler() if scaler_on else None
    loop = TrainLoop(model, CrossEntropyLoss(), opt, loader, scaler, use_graph=use_graph, steps_per_graph=4)
    for _ in range(steps):
        loop.run_epoch()
    assert loop.graph_error is None, loop.graph_error
    return model


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("amp", [False, True])
def test_ddp_syncbn_fused_graph_matches_plain(rccl, amp, graph):
    """DDP(SyncBN ConvNet) with forced collectives, graph-captured, == plain ConvNet eager."""
    from ddp_practice_amd.data import synthetic
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    ds = synthetic(32 * 9 + 5, seed=11)  # 9 full batches (2 graph replays + 1-step graph) + a tail of 5
    torch.manual_seed(0)
    dt = torch.bfloat16 if amp else None
    plain = ConvNet(amp_dtype=dt).cuda()
    ddp = DistributedDataParallel(convert_sync_batchnorm(copy.deepcopy(plain)), device_ids=[0], gradient_as_bucket_view=True)
    assert ddp.reducer is not None
    _train(plain, 2, ds.images, ds.labels, amp, use_graph=False)
    _train(ddp, 2, ds.images, ds.labels, amp, use_graph=graph)
    tol = 1e-5 if not amp else 2e-3
    for (n, p), (_, q) in zip(ddp.module.state_dict().items(), plain.state_dict().items()):
        torch.testing.assert_close(p.float(), q.float(), rtol=tol, atol=tol, msg=n)
    assert int(ddp.module.layer1[1].num_batches_tracked) == 2 * 10


def test_ddp_syncbn_batch80_takes_launch_path(rccl):
    """Batch 80: the conv1 weight-gradient site would need 7 * 80 = 560 workgroups, more than
    a site's 512 epoch words (comm/xsite.h kEpochWords), so the ConvNet must take the
    all-reduce launch path (ops/convnet_fused._fused_site_engine) -- and still train exactly
    like the plain model (advisor round 4: the words were not checked on the host)."""
    from ddp_practice_amd._ext import load
    from ddp_practice_amd.data import synthetic
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    C = load()
    assert C.convnet.sites_resident(32, torch.bfloat16)
    assert not C.convnet.sites_resident(80, torch.bfloat16)
    ds = synthetic(80 * 3 + 7, seed=5)
    torch.manual_seed(0)
    plain = ConvNet(amp_dtype=torch.bfloat16).cuda()
    ddp = DistributedDataParallel(convert_sync_batchnorm(copy.deepcopy(plain)), device_ids=[0], gradient_as_bucket_view=True)
    _train(plain, 2, ds.images, ds.labels, True, use_graph=False, batch=80)
    _train(ddp, 2, ds.images, ds.labels, True, use_graph=True, batch=80)
    for (n, p), (_, q) in zip(ddp.module.state_dict().items(), plain.state_dict().items()):
        torch.testing.assert_close(p.float(), q.float(), rtol=2e-3, atol=2e-3, msg=n)
    assert rccl.xgmi is not None and rccl.xgmi.error() == 0


def test_xgmi_debug_state_names_sites_and_words(rccl):
    """The watchdog's exchange-state report (csrc/comm/xgmi_allreduce.hip debug_state): error /
    abort words, the used sites' epochs and the peers' newest granule epochs, read from a
    side stream with a bounded wait."""
    from ddp_practice_amd.data import synthetic
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    x = rccl.xgmi
    assert x is not None
    ds = synthetic(32 * 3, seed=3)
    torch.manual_seed(0)
    ddp = DistributedDataParallel(convert_sync_batchnorm(ConvNet(amp_dtype=torch.bfloat16).cuda()), device_ids=[0], gradient_as_bucket_view=True)
    _train(ddp, 1, ds.images, ds.labels, True, use_graph=False)
    torch.cuda.synchronize()
    st = x.debug_state(2.0)
    assert st.startswith("xgmi rank 0/1: err=0 abort=0"), st
    assert "fwd1 ep=" in st and "peers[par0|par1]=" in st and "oneshot blk ep=" in st, st
    # the host-side issue counts (readable when the device is wedged): the training above
    # attached launches to the SyncBN sites
    import re

    m = re.search(r"host issued: oneshot (\d+) twoshot (\d+) \(last (\d+) B\), site handles ([\d,]+)", st)
    assert m is not None, st
    assert sum(int(v) for v in m.group(4).split(",")) > 0, st


def test_xgmi_engine_passes_its_selftest_at_forced_world1(rccl):
    """The RCCL communicator's start-up self-test (parallel/comm.setup_xgmi) must pass on a
    healthy device, or every multi-GPU run silently loses the xGMI engine (round 2's self-test
    probed a SyncBN site with 1568 floats > its 128-float row and failed on every box)."""
    assert rccl.xgmi_status.startswith("on"), rccl.xgmi_status
    assert rccl.xgmi is not None and rccl.xgmi_max_bytes > 0


@pytest.mark.parametrize("amp", [None, torch.bfloat16])
def test_resnet_syncbn_sites_match_launch_path(rccl, monkeypatch, amp):
    """ResNet-50 SyncBN with the statistics exchanged inside the finisher workgroups (the
    xGMI engine's wide site, ops/bn_nhwc.sync_site) == the all-reduce-launch path
    (DPA_FUSED_SYNC=0).  At W=1 both reduce to the local sums, so the output, every
    gradient and every buffer must be bitwise equal -- and the site path must launch no
    all-reduce kernel for the statistics."""
    import torch.nn.functional as F

    from ddp_practice_amd.models import resnet50
    from ddp_practice_amd.ops.bn_nhwc import sync_site
    from ddp_practice_amd.parallel import convert_sync_batchnorm

    assert sync_site(rccl) is not None
    torch.manual_seed(0)
    base = convert_sync_batchnorm(resnet50(num_classes=10, amp_dtype=amp)).cuda()
    x = torch.rand(8, 3, 64, 64, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    res = {}
    calls = {}
    # a warm-up pass first: library convolutions (the fp32 model's) pick their algorithms on
    # the first call of a shape, which must not land on one of the two compared runs
    for flag in ("w", "0", "1"):
        monkeypatch.setenv("DPA_FUSED_SYNC", "0" if flag == "w" else flag)
        m = copy.deepcopy(base)
        n = [0]
        orig = type(rccl).all_reduce_, type(rccl).all_reduce

        def count_(self, t, op="sum", _f=orig[0]):
            n[0] += 1
            return _f(self, t, op)

        def count(self, t, op="sum", _f=orig[1]):
            n[0] += 1
            return _f(self, t, op)

        monkeypatch.setattr(type(rccl), "all_reduce_", count_)
        monkeypatch.setattr(type(rccl), "all_reduce", count)
        out = m(x)
        F.cross_entropy(out.float(), y).backward()
        torch.cuda.synchronize()
        monkeypatch.setattr(type(rccl), "all_reduce_", orig[0])
        monkeypatch.setattr(type(rccl), "all_reduce", orig[1])
        calls[flag] = n[0]
        res[flag] = (out.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()},
                     {k: b.clone() for k, b in m.named_buffers()})
    assert rccl.xgmi.error() == 0, rccl.xgmi.error_string()
    assert calls["0"] >= 2 * 53 and calls["1"] == 0, calls  # 53 BatchNorms, fwd + bwd each
    (o0, g0, b0), (o1, g1, b1), (ow, gw, _) = res["0"], res["1"], res["w"]

    def rel(a, b):
        return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()

    # bf16: every kernel of the step is the framework's own (deterministic): bitwise.  fp32:
    # the library convolutions vary run to run (~1e-5): within a few times that spread
    bitwise = amp is not None
    if bitwise:
        assert torch.equal(ow, o0), ("launch path run to run", rel(ow, o0))
    floor = 0.0 if bitwise else 10 * max(rel(ow, o0), max(rel(gw[k], g0[k]) for k in g0), 1e-6)

    def same(a, b, what):
        if bitwise:
            assert torch.equal(a, b), (what, rel(a, b))
        else:
            assert rel(a, b) <= floor, (what, rel(a, b), floor)

    same(o1, o0, "output")
    for k in g0:
        same(g1[k], g0[k], k)
    for k in b0:
        if b0[k].dtype.is_floating_point:
            same(b1[k], b0[k], k)
        else:
            assert torch.equal(b0[k], b1[k]), k


def test_ddp_bucket_replan_never_inside_capture(rccl):
    """DDP re-plans its buckets at iteration 1's forward; when that forward is being captured
    (CapturedStep warm-up of one step) the plan is kept instead: a re-plan would allocate and
    zero the new bucket buffers as graph nodes re-run on every replay (round 4's forced
    steady table showed that FillFunctor<float>).  No fill / zero op is issued under capture."""
    from torch.utils._python_dispatch import TorchDispatchMode

    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel
    from ddp_practice_amd.runtime import CapturedStep

    torch.manual_seed(0)
    ddp = DistributedDataParallel(ConvNet().cuda(), device_ids=[0], bucket_cap_mb=0.01, gradient_as_bucket_view=True)
    opt, crit = SGD(ddp.parameters(), lr=0.01), CrossEntropyLoss()
    x = torch.randn(32, 1, 28, 28, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")
    fills = []

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.__name__.split(".")[0].strip("_")
            if name in ("fill", "zero", "zeros", "full") and torch.cuda.is_current_stream_capturing():
                fills.append(str(func))
            return func(*args, **(kwargs or {}))

    def step():
        loss = crit(ddp(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    before = [list(b) for b in ddp.reducer.bucket_indices()]
    runner = CapturedStep(step, warmup=1, steps_per_graph=2)
    with Spy():
        assert runner.capture()
    assert fills == [], fills
    assert ddp._rebuilt and [list(b) for b in ddp.reducer.bucket_indices()] == before
    for _ in range(3):
        runner.run()
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in ddp.parameters())
