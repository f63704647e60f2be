"""Generic SyncBatchNorm (parallel/sync_bn.py) on 4-D device inputs runs the native
channels_last kernels (ops/bn_nhwc.py): forward / backward / running statistics vs
torch's BatchNorm2d, including momentum=None (cumulative average, no host sync) and
a non-affine module."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("affine", [True, False])
@pytest.mark.parametrize("cl", [False, True])
def test_syncbn_native_matches_torch(C, momentum, affine, cl):
    from ddp_practice_amd.parallel import SyncBatchNorm

    torch.manual_seed(0)
    ref = torch.nn.BatchNorm2d(24, momentum=momentum, affine=affine).cuda()
    mine = SyncBatchNorm(24, momentum=momentum, affine=affine).cuda()
    if affine:
        with torch.no_grad():
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.uniform_(-0.5, 0.5)
            mine.weight.copy_(ref.weight)
            mine.bias.copy_(ref.bias)
    calls = {"n": 0}
    orig = C.bn_nhwc.apply

    def spy(*a):
        calls["n"] += 1
        return orig(*a)

    C.bn_nhwc.apply = spy
    try:
        for it in range(3):
            x = (torch.randn(6, 24, 9, 11, device="cuda") * 2 + 1)
            if cl:
                x = x.contiguous(memory_format=torch.channels_last)
            xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
            ya, yb = ref(xa), mine(xb)
            g = torch.randn_like(ya)
            ya.backward(g)
            yb.backward(g)
            torch.testing.assert_close(yb, ya, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-4, atol=1e-4)
    finally:
        C.bn_nhwc.apply = orig
    assert calls["n"] == 3, "the native kernels did not run"
    torch.testing.assert_close(mine.running_mean, ref.running_mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mine.running_var, ref.running_var, rtol=1e-5, atol=1e-5)
    assert int(mine.num_batches_tracked) == 3
    if affine:
        torch.testing.assert_close(mine.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(mine.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape,ref_cls", [((40, 24), torch.nn.BatchNorm1d), ((6, 24, 37), torch.nn.BatchNorm1d),
                                           ((3, 24, 4, 5, 6), torch.nn.BatchNorm3d)])
def test_syncbn_native_non_4d(C, shape, ref_cls):
    """BatchNorm1d / BatchNorm3d inputs (2-D, 3-D, 5-D) run the same native kernels as the
    4-D view [N, C, prod(rest), 1] (they ran eager torch ops)."""
    from ddp_practice_amd.parallel import SyncBatchNorm

    torch.manual_seed(1)
    ref = ref_cls(24).cuda()
    mine = SyncBatchNorm(24).cuda()
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
        mine.weight.copy_(ref.weight)
        mine.bias.copy_(ref.bias)
    calls = {"n": 0}
    orig = C.bn_nhwc.apply

    def spy(*a):
        calls["n"] += 1
        return orig(*a)

    C.bn_nhwc.apply = spy
    try:
        for _ in range(2):
            x = torch.randn(*shape, device="cuda") * 3 - 1
            xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
            ya, yb = ref(xa), mine(xb)
            assert yb.shape == ya.shape and yb.is_contiguous()
            g = torch.randn_like(ya)
            ya.backward(g)
            yb.backward(g)
            torch.testing.assert_close(yb, ya, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(xb.grad, xa.grad, rtol=1e-4, atol=1e-4)
    finally:
        C.bn_nhwc.apply = orig
    assert calls["n"] == 2, "the native kernels did not run"
    torch.testing.assert_close(mine.running_var, ref.running_var, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(mine.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
