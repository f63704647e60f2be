"""ops/bn_nhwc.BNTap host-side contract: the consumer conv's BN backward sums
are reused only for the exact, unmodified gradient tensor, and a tap holds no strong
reference to the BN's activations (no output -> grad_fn -> tap -> output cycle)."""
import gc
import weakref

import torch

from ddp_practice_amd.ops.bn_nhwc import BNTap


class _Id(torch.autograd.Function):
    """Stands in for BNActFn: saves (x, y) and binds the tap to its own node."""

    @staticmethod
    def forward(ctx, x, tap):
        y = x * 2
        ctx.save_for_backward(x, y)
        tap.bind(ctx, 0, 1, 1, None, None, None)
        ctx.tap = tap
        return y

    @staticmethod
    def backward(ctx, g):
        return g * 2, None


def test_matches_requires_same_unmodified_tensor():
    bt = BNTap()
    dx = torch.zeros(8)
    bt.sums = (torch.zeros(2), torch.zeros(1), torch.zeros(1))
    bt.grad_ptr, bt.grad_ver = dx.data_ptr(), dx._version
    assert bt.matches(dx)
    assert not bt.matches(torch.zeros(8))  # another tensor
    dx.add_(1.0)  # autograd accumulating a second consumer's gradient in place
    assert not bt.matches(dx)
    bt.sums = None
    assert not bt.matches(dx)


def test_tap_reads_saved_tensors_through_node():
    x = torch.randn(4, requires_grad=True)
    bt = BNTap()
    y = _Id.apply(x, bt)
    assert torch.equal(bt.x, x.detach()) and torch.equal(bt.y, y.detach())
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((4,), 2.0))


def test_tap_forms_no_reference_cycle():
    """A training forward not followed by backward frees its activations by reference
    counting alone (the cycle collector is disabled here)."""
    gc.disable()
    try:
        x = torch.randn(1024, requires_grad=True)
        bt = BNTap()
        y = _Id.apply(x, bt)
        alive = weakref.ref(y)
        node = weakref.ref(y.grad_fn)
        del y
        assert alive() is None and node() is None
        assert bt.x is None and bt.y is None  # the node is gone: the consumer falls back
    finally:
        gc.enable()


def test_bind_tensors_holds_direct_inputs():
    bt = BNTap()
    x = torch.ones(3)
    bt.bind_tensors(x, None, 2, None, None, None)
    assert bt.x is x and bt.y is None and bt.act == 2
    bt.clear()
    assert bt.x is None
