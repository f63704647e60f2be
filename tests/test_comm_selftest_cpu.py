"""The xGMI engine's start-up self-test (parallel/comm._xgmi_selftest) on gloo with a
stand-in engine: every rank issues the same collectives whatever fails locally, and a
failure on any one rank -- a wrong all-reduce or a failing in-kernel exchange site --
keeps every rank off the engine (no rank may leave the test early)."""
import pytest

from tests import _selftest_worker
from tests._dist import launch


@pytest.mark.parametrize("bad,kind", [(-1, "none"), (1, "oneshot"), (0, "site"), (2, "site")])
def test_selftest_votes_symmetrically(bad, kind):
    outs = launch(_selftest_worker.run, 3, (bad, kind), timeout=120)
    goods = {o[0] for o in outs}
    assert goods == {bad < 0}, outs
    if bad >= 0:
        assert any(o[1] for o in outs)  # the failing rank names why
    counts = outs[0][2]
    assert len(set(counts)) == 1, f"ranks issued different numbers of collectives: {counts}"
