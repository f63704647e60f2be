"""bench.py contract on CPU: the self-launcher (``--gpus N`` with no WORLD_SIZE spawns N
ranks before any GPU call; gloo here), exact step counts, one JSON line from rank 0."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _bench(args, timeout=300):
    env = dict(os.environ)
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
