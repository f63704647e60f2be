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
