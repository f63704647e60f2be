"""DDP + SyncBN ConvNet with 2 processes on the test box's single GPU, all
all-reduces on the one-shot xGMI engine: the result must equal one process
training on the global batch, and every rank must end bit-identical."""
import pytest

from ._dist import launch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("amp,graph", [(False, False), (False, True), (True, True)])
def test_ddp_syncbn_xgmi_two_processes(C, amp, graph):
    from ._xgmi_ddp_worker import worker

    world = 2
    outs = launch(worker, world, (amp, graph), timeout=240)
    res = dict(enumerate(outs))
    print("grad errs", res[0]["grad_errs"])
    print("param errs", res[0]["errs"])
    assert res[0]["digest"] == res[1]["digest"], "ranks diverged"


def test_prechecked_step_agrees_across_ranks(C):
    """DDP + SyncBN ConvNet over the xGMI engine with the pre-checked AMP step: one rank's
    overflow makes every rank skip (the flagged rank pushes NaN in its gradient exchange)."""
    from ._xgmi_ddp_worker import worker_poison

    outs = launch(worker_poison, 2, (), timeout=240)
    assert len(outs) == 2 and outs[0]["scale"] < outs[1]["scale"]  # rank 0 backed off; rank 1 stays inf
