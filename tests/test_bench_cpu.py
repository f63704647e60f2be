"""bench.py contract on CPU: the self-launcher (``--gpus N`` with no WORLD_SIZE spawns N
ranks before any GPU call; gloo here), exact step counts, one JSON line from rank 0."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _bench(args, timeout=300, extra_env=None):
    env = dict(os.environ)
    env.update(extra_env or {})
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_self_launches_two_ranks():
    r = _bench(["--gpus", "2", "--steps", "7", "--warmup", "3", "--epochs", "1", "--train-samples", "640",
                "--test-samples", "128"])
    assert r.returncode == 0, r.stdout + r.stderr
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2
    assert rec["steps"] == 7 and rec["warmup"] == 3
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 64
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["epochs"] == 1 and rec["steps_per_rank_per_epoch"] == 10  # 320 samples per rank / 32
    assert rec["wall_3epoch_s"] > 0 and 0.0 <= rec["accuracy"] <= 1.0
    for k in ("metric", "unit", "vs_baseline", "dtype", "data", "config"):
        assert k in rec


def test_bench_rejects_bad_gpu_count():
    r = _bench(["--gpus", "0"])
    assert r.returncode == 2 and "--gpus must be >= 1" in r.stderr


_SMALL = ["--gpus", "2", "--steps", "7", "--warmup", "3", "--epochs", "1", "--train-samples", "640",
          "--test-samples", "128"]


def test_bench_hung_rank_falls_back_with_comm_error():
    """rank 1 hangs at step 3 -> both ranks' watchdogs report and exit 124 (no
    30-min gloo stall), the supervisor re-runs fresh ranks (--comm rccl) and prints ONE line
    carrying the value, ``fallback`` and the first attempt's ``comm_error``; rc 0."""
    # the healthy fallback must not trip the watchdog: scripts/asan_check.sh runs every step
    # several times slower and stretches the budget through DPA_TEST_TIME_SCALE
    wd = 4 * float(os.environ.get("DPA_TEST_TIME_SCALE", "1"))
    r = _bench(_SMALL, extra_env={"DPA_FAULT": "1:3:hang", "DPA_BENCH_WATCHDOG": f"{wd:g}"})
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1
    rec = recs[0]
    assert rec["value"] > 0 and rec["fallback"] == "rccl"
    assert "rank 1" in rec["comm_error"] and "watchdog" in rec["comm_error"]
    assert [a["ok"] for a in rec["attempts"]] == [False, True]


def test_bench_every_attempt_failing_reports_rc3():
    """A fault that recurs in the fallback: one line, value null, comm_error set, rc 3."""
    r = _bench(_SMALL, extra_env={"DPA_FAULT": "1:2:exit:9", "DPA_FAULT_RETRY": "1"})
    assert r.returncode == 3, r.stdout + r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1 and recs[0]["value"] is None
    assert "rank 1: exit 9" in recs[0]["comm_error"]


def test_bench_under_torchrun_one_line():
    """The driver's N > 1 launch: every torchrun worker supervises one fresh rank; rank 0
    prints the only line."""
    from tests._dist import free_port

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(ROOT, "bench.py"), *_SMALL], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    assert recs[0]["n_gpus"] == 2 and recs[0]["ranks_seen"] == 2 and recs[0]["comm_error"] == ""


def test_bench_under_torchrun_eight_ranks():
    """The driver's N = 8 launch shape on gloo: 8 torchrun workers, each supervising one
    fresh rank; an epoch of one full batch and a 12-sample tail per rank; rank 0 prints
    the only line and saw all 8 ranks."""
    from tests._dist import free_port

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    args = ["--gpus", "8", "--steps", "3", "--warmup", "2", "--epochs", "1", "--train-samples", str(8 * 44),
            "--test-samples", str(8 * 34)]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 8 and rec["ranks_seen"] == 8 and rec["comm_error"] == ""
    assert rec["config"]["parallelism"] == "dp8" and rec["config"]["global_batch"] == 256
    assert rec["steps"] == 3 and rec["steps_per_rank_per_epoch"] == 2  # 32 + the 12-sample tail


def test_bench_under_torchrun_rank_failure_falls_back():
    """torchrun shape with rank 0's child dying at step 2: every worker's supervisor sees the
    shared failure flag, kills its child, and all of them re-run fresh children; rank 0's
    supervisor prints one line with the fallback and the error."""
    from tests._dist import free_port

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(CUDA_VISIBLE_DEVICES="", DPA_FAULT="0:2:exit:7", DPA_BENCH_GRACE="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(ROOT, "bench.py"), *_SMALL], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["fallback"] == "rccl" and rec["value"] > 0
    assert "rank 0: exit 7" in rec["comm_error"]


def test_supervisor_rejects_multi_node_torchrun(monkeypatch):
    """The per-attempt child store is on the leader's localhost: a multi-node torchrun run
    is refused up front instead of timing out as a comm failure."""
    from ddp_practice_amd.runtime.supervisor import Supervisor

    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("MASTER_PORT", "1")
    with pytest.raises(ValueError, match="single-node"):
        Supervisor(16)


def test_timed_chunk_plan_covers_exactly_the_steps(monkeypatch):
    """bench.py's timed regions replay graphs in a plan of a one-step lead, the remainder and
    full graphs: it runs exactly the requested number of steps, with a lead step unless
    DPA_BENCH_LEAD=0 or one step per graph."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class Plan(bench._Chunks):
        def __init__(self, spg):  # no graphs, no loader: the plan only
            self.spg = spg

    for spg, n in [(16, 20), (16, 2000), (16, 1875), (16, 5), (16, 1), (16, 17), (1, 7), (16, 0)]:
        plan = Plan(spg)._plan(n)
        assert sum(plan) == n and all(1 <= k <= spg for k in plan), (spg, n, plan)
        if n and spg > 1:
            assert plan[0] == 1
    assert Plan(16)._plan(20) == [1, 3, 16]
    monkeypatch.setenv("DPA_BENCH_LEAD", "0")
    assert Plan(16)._plan(20) == [4, 16]
