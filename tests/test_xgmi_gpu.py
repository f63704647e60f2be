"""One-shot xGMI all-reduce (csrc/comm/xgmi_allreduce.hip) with W processes
sharing the single GPU of the test box: values vs a CPU fp32 reference,
bit-identical results on every rank, graph replay, bounded waits."""
import pytest

from ._dist import launch

pytestmark = pytest.mark.gpu


def _run(world, mode, timeout=150):
    from ._xgmi_worker import worker

    return launch(worker, world, (mode,), timeout)


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_multiprocess(C, world):
    outs = _run(world, "full")
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"


def test_xgmi_wait_is_bounded(C):
    _run(2, "timeout")
