"""GradScaler state machine and SGD parity with torch (CPU paths)."""
import pytest
import torch

from ddp_practice_amd.amp import GradScaler, autocast, compute_dtype
from ddp_practice_amd.optim import SGD


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(n, generator=g)) for n in (3, 17, 64)]


@pytest.mark.parametrize("momentum,wd,nesterov,damp", [(0.0, 0.0, False, 0.0), (0.9, 1e-4, False, 0.1),
                                                       (0.9, 0.0, True, 0.0)])
def test_sgd_matches_torch(momentum, wd, nesterov, damp):
    a, b = _params(), _params()
    oa = SGD(a, lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov, dampening=damp)
    ob = torch.optim.SGD(b, lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov, dampening=damp)
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        grads = [torch.randn(p.shape, generator=g) for p in a]
        for p, q, gr in zip(a, b, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        oa.step()
        ob.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p, q)


def test_grad_scaler_state_machine_matches_torch():
    """Scripted found_inf sequence: scale / growth tracker must track torch.amp.GradScaler."""
    ours = GradScaler(device="cpu", init_scale=8.0, growth_interval=3)
    ref = torch.amp.GradScaler("cpu", init_scale=8.0, growth_interval=3)
    pa, pb = _params(), _params()
    oa, ob = SGD(pa, lr=0.01), torch.optim.SGD(pb, lr=0.01)
    pattern = [False, False, False, True, False, False, False, False, True, True, False]
    for bad in pattern:
        ours.scale(torch.tensor(1.0))
        ref.scale(torch.tensor(1.0))
        for p, q in zip(pa, pb):
            gr = torch.ones_like(p) * 8.0
            if bad:
                gr[0] = float("inf")
            p.grad = gr.clone()
            q.grad = gr.clone()
        ours.step(oa)
        ref.step(ob)
        ours.update()
        ref.update()
        assert ours.get_scale() == ref.get_scale()
        assert ours.state_dict()["_growth_tracker"] == ref.state_dict()["_growth_tracker"]
        for p, q in zip(pa, pb):
            torch.testing.assert_close(p, q)
    sd_o, sd_r = ours.state_dict(), ref.state_dict()
    assert set(sd_o) == set(sd_r)
    for k in sd_r:
        assert sd_o[k] == sd_r[k], k
        assert type(sd_o[k]) is type(sd_r[k]), k


def test_grad_scaler_scale_and_load_state():
    s = GradScaler(device="cpu")
    loss = torch.tensor(2.0, requires_grad=True)
    out = s.scale(loss)
    assert out.dim() == 0 and out.item() == 2.0 * 65536
    s2 = GradScaler(device="cpu")
    s2.load_state_dict({"scale": 4.0, "growth_factor": 3.0, "backoff_factor": 0.25, "growth_interval": 7,
                        "_growth_tracker": 2})
    assert s2.get_scale() == 4.0 and s2.get_growth_factor() == 3.0
    loss2 = torch.tensor(1.0, requires_grad=True)
    assert s2.scale(loss2).item() == 4.0
    assert s2.state_dict()["_growth_tracker"] == 2


def test_grad_scaler_disabled_passthrough():
    s = GradScaler(device="cpu", enabled=False)
    x = torch.tensor(3.0)
    assert s.scale(x) is x and s.state_dict() == {}


def test_autocast_policy():
    x = torch.zeros(2)
    assert compute_dtype(x) == torch.float32
    with autocast(dtype=torch.bfloat16, device_type="cpu"):
        assert compute_dtype(x) == torch.bfloat16
        with autocast(enabled=False, device_type="cpu"):
            assert compute_dtype(x) == torch.float32
    assert compute_dtype(x.half()) == torch.float16
    with pytest.raises(ValueError):
        with autocast(dtype=torch.float32):
            pass


def test_seeded_backward_matches_autograd_backward():
    """GradScaler's engine-direct seeded backward == torch.autograd.backward(t, seed):
    same grads, `inputs=` restricts accumulation, retain_graph allows a second pass,
    a seed of another floating dtype is cast like torch does."""
    from ddp_practice_amd.amp.grad_scaler import _seeded_backward

    torch.manual_seed(0)
    w = torch.randn(5, 3, requires_grad=True)
    b = torch.randn(3, requires_grad=True)
    x = torch.randn(4, 5)

    def loss():
        return ((x @ w + b).relu() ** 2).mean()

    seed = torch.tensor(512.0)
    torch.autograd.backward(loss(), grad_tensors=seed)
    gw, gb = w.grad.clone(), b.grad.clone()
    w.grad = b.grad = None
    _seeded_backward(loss(), seed, None, None)
    assert torch.equal(w.grad, gw) and torch.equal(b.grad, gb)
    w.grad = b.grad = None
    _seeded_backward(loss(), seed, None, [b])
    assert w.grad is None and torch.equal(b.grad, gb)
    b.grad = None
    lv = loss()
    _seeded_backward(lv, seed, True, None)
    _seeded_backward(lv, seed, None, None)
    assert torch.allclose(w.grad, 2 * gw)
    w.grad = b.grad = None
    lh = loss().to(torch.float64)
    _seeded_backward(lh, seed, None, None)  # fp32 seed into an fp64 output
    assert torch.allclose(w.grad, gw)
    with pytest.raises(RuntimeError):
        _seeded_backward(loss(), seed, None, [])


def test_optimizer_and_scaler_do_not_import_dynamo_or_sympy():
    """SGD construction/zero_grad/state_dict and a scaled backward stay clear of the lazy
    torch._dynamo / sympy imports (~2.5 s on a fresh box), checked in a fresh interpreter."""
    import subprocess
    import sys

    code = (
        "import sys, torch\n"
        "from ddp_practice_amd.optim import SGD\n"
        "from ddp_practice_amd.amp.grad_scaler import _seeded_backward\n"
        "p = torch.nn.Parameter(torch.randn(4))\n"
        "o = SGD([p], lr=0.1)\n"
        "_seeded_backward((p * p).sum(), torch.tensor(2.0), None, None)\n"
        "o.step(); o.zero_grad(); o.load_state_dict(o.state_dict())\n"
        "bad = [m for m in ('torch._dynamo', 'sympy') if m in sys.modules]\n"
        "assert not bad, bad\n"
    )
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


def test_prechecked_bookkeeping():
    """The producer-check registration (ops/convnet_fused.py -> SGD.set_prechecked) lasts until
    the next fused step or any gradient reader: flush_slab (GradScaler.unscale_, DDP flush,
    grad hooks) and a new backward drop it, and the check words are never created inside a
    graph capture (here: none on CPU either way)."""
    p = torch.nn.Parameter(torch.zeros(8))
    opt = SGD([p], lr=0.1)
    out = torch.zeros(8)
    chk = torch.zeros(2, dtype=torch.int32)
    scale = torch.ones(1)
    opt.set_prechecked(chk, scale, out)
    pc = opt.__dict__["_prechecked"]
    assert pc[0] is chk and pc[1] is scale and pc[3] - pc[2] == out.numel() * out.element_size()
    opt.flush_slab()
    assert "_prechecked" not in opt.__dict__
    opt.set_prechecked(chk, scale, out)
    opt.clear_prechecked()
    assert "_prechecked" not in opt.__dict__
    t = opt.grad_chk(2, torch.device("cpu"))
    assert t.dtype == torch.int32 and t.numel() == 2 and opt.grad_chk(2, torch.device("cpu")) is t
