"""One-shot xGMI all-reduce (csrc/comm/xgmi_allreduce.hip) with W processes
sharing the single GPU of the test box: values vs a CPU fp32 reference,
bit-identical results on every rank, graph replay, bounded waits."""
import pytest
import torch
import torch.multiprocessing as mp

from ._dist import free_port

pytestmark = pytest.mark.gpu


def _run(world, mode, timeout=150):
    from ._xgmi_worker import worker

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, st, out = q.get(timeout=timeout)
            assert st == "ok", f"rank {rank} failed:\n{out}"
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_multiprocess(C, world):
    outs = _run(world, "full")
    for k, v in outs[0].items():
        for r in range(1, world):
            assert v == outs[r][k], f"rank {r} differs from rank 0 on {k}"


def test_xgmi_wait_is_bounded(C):
    _run(2, "timeout")
