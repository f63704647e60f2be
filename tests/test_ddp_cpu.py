"""DDP / SyncBN / communicator semantics on 2 CPU ranks (gloo)."""
import pytest
import torch

from ddp_practice_amd.parallel import compute_bucket_assignment

from . import _ddp_workers as W
from ._dist import run

pytestmark = pytest.mark.slow


def test_ddp_syncbn_matches_single_process_full_batch():
    outs = run(W.ddp_syncbn_equivalence, world=2, args=(8,))
    keys = outs[0]["keys"]
    assert keys[0] == "module.layer1.0.weight" and len(keys) == 16
    assert "module.layer2.1.running_var" in keys and "module.fc.bias" in keys
    # one bucket like torch's (29,034 floats); every param view starts 16-B aligned,
    # which pads fc.bias (10 -> 12) and the 5x5 bias of 16/32 floats not at all
    sizes = [10, 15680, 32, 32, 32, 12800, 16, 16, 16, 400]
    assert outs[0]["buckets"] == [sum((n + 3) // 4 * 4 for n in sizes) * 4]


def test_ddp_no_sync_and_find_unused():
    assert run(W.ddp_no_sync_and_unused, world=2) == [True, True]


def test_comm_collectives_gloo():
    assert run(W.comm_collectives, world=3) == [True] * 3


def _torch_buckets(params, first, cap):
    import torch.distributed as dist

    idx, _ = dist._compute_bucket_assignment_by_size(
        params[::-1], [first, cap], [False] * len(params))
    n = len(params)
    return [[n - 1 - i for i in b] for b in idx]


@pytest.mark.parametrize("shapes", [
    [(16, 1, 5, 5), (16,), (16,), (16,), (32, 16, 5, 5), (32,), (32,), (32,), (10, 1568), (10,)],
    [(2048, 2048), (2048,), (512, 512), (1000, 2048), (1000,), (64, 3, 7, 7)],
])
def test_bucket_assignment_matches_torch(shapes):
    params = [torch.empty(s) for s in shapes]
    first, cap = 1 << 20, 25 << 20
    ours = compute_bucket_assignment(params, cap, first)
    ref = _torch_buckets(params, first, cap)
    assert sorted(map(sorted, ours)) == sorted(map(sorted, ref))


def test_ddp_deferred_grad_sync_flush():
    assert run(W.ddp_deferred_flush, world=2) == [True, True]


def test_distributed_facade_async_op_returns_work():
    assert run(W.facade_async_work, world=2) == [True, True]


@pytest.mark.parametrize("kind,needle", [("ok", ""), ("shape", "parameter 0 has shape (3, 8)"),
                                         ("dtype", "dtype torch.float64"), ("count", "parameters")])
def test_ddp_exact_shape_and_dtype_check(kind, needle):
    outs = run(W.ddp_shape_mismatch, world=2, args=(kind,))
    if kind == "ok":
        assert outs == ["", ""]
    else:
        assert all(needle in o for o in outs), outs


def test_ddp_slab_sink_requires_deferred_zero_copy():
    assert run(W.ddp_slab_sink_guard, world=2) == [True, True]


def test_ddp_gradient_as_bucket_view_false_copies_back():
    """gradient_as_bucket_view=False keeps autograd's gradient tensors (values averaged
    into them), VERDICT r3 minor API item."""
    from ._ddp_workers import ddp_grad_not_bucket_view

    assert all(run(ddp_grad_not_bucket_view, world=2))


def test_ddp_syncbn_world8_epoch_tail():
    """World 8 (BASELINE configs 3-5) on gloo: the per-rank tail of an epoch (12 train /
    2 test samples per rank, as MNIST's at W=8), padding wrapped from the front, SyncBN
    statistics over 8 ranks, DDP average of 8 and test() reduced to rank 0 -- the
    result equals one process on each step's concatenated global batch."""
    world, batch = 8, 32
    n_train, n_test = world * (batch + 12) - 3, world * (batch + 2)
    outs = run(W.ddp_syncbn_epoch_tail, world=world, args=(n_train, n_test, batch), timeout=600)
    for o in outs:
        assert o["sizes"] == [32, 12] and o["test_sizes"] == [32, 2]
    assert outs[0]["size"] == world * (batch + 2)  # the padded test set: 272 samples counted
    assert 0 <= outs[0]["correct"] <= outs[0]["size"]
