"""DDP + SyncBN ConvNet with 2 processes on the test box's single GPU, all
all-reduces on the one-shot xGMI engine: the result must equal one process
training on the global batch, and every rank must end bit-identical."""
import pytest
import torch.multiprocessing as mp

from ._dist import free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("amp,graph", [(False, False), (False, True), (True, True)])
def test_ddp_syncbn_xgmi_two_processes(C, amp, graph):
    from ._xgmi_ddp_worker import worker

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, amp, graph, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, st, out = q.get(timeout=240)
            assert st == "ok", f"rank {rank} failed:\n{out}"
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    print("grad errs", res[0]["grad_errs"])
    print("param errs", res[0]["errs"])
    assert res[0]["digest"] == res[1]["digest"], "ranks diverged"
