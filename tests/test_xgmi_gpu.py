"""One-shot xGMI all-reduce (csrc/comm/xgmi_allreduce.hip) with W processes
sharing the single GPU of the test box: values vs a CPU fp32 reference,
bit-identical results on every rank, graph replay, bounded waits.  World 8 is the
driver's node size: every ``kMaxRanks = 8`` path (8-row site polls, 7-peer pushes,
two-shot shards of 1/8) runs here before it runs on eight GPUs."""
import pytest

from ._dist import launch
from .conftest import W8

pytestmark = pytest.mark.gpu


def _run(world, mode, timeout=None):
    timeout = timeout or (150 if world <= 4 else 300)
    from ._xgmi_worker import worker

    return launch(worker, world, (mode,), timeout)


@pytest.mark.parametrize("world", [2, 4, pytest.param(8, marks=W8)])
def test_xgmi_allreduce_multiprocess(C, world):
    outs = _run(world, "full")
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"


def test_xgmi_wait_is_bounded(C):
    _run(2, "timeout")


@pytest.mark.parametrize("world", [2, 3, pytest.param(8, marks=W8)])
def test_xsite_exchange_multiprocess(C, world):
    """The in-kernel SyncBN exchange (csrc/comm/xsite.h) every fused consumer runs."""
    outs = _run(world, "site")
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"


@pytest.mark.parametrize("world", [1, 2, 4, pytest.param(8, marks=W8)])
def test_wide_site_exchange_multiprocess(C, world):
    """The positioned exchange of the ResNet statistics finishers (SyncBN rows up to
    2*2048+1 floats over several finisher workgroups, csrc/comm/xsite.h kSiteWide)."""
    outs = _run(world, "wide")
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"


@pytest.mark.parametrize("mode", ["site_timeout", "sgd_timeout"])
def test_in_kernel_exchange_wait_is_bounded(C, mode):
    """A fused SyncBN site and the fused AMP-SGD gradient exchange whose peer never
    arrives end with the error word set; the optimizer applies nothing."""
    _run(2, mode)


@pytest.mark.parametrize("world", [2, 3, 4, pytest.param(8, marks=W8)])
def test_xgmi_twoshot_multiprocess(C, world):
    """Two-shot (reduce-scatter + all-gather) engine for large messages: 1-32 MiB,
    ragged sizes, every dtype/op, interleaved sizes, graph replay; bit-identical ranks."""
    outs = _run(world, "twoshot", timeout=240 if world <= 4 else 360)
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"
