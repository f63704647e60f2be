"""bench.py contract on the MI355X: exact --steps/--warmup, the measured 3-epoch run,
the same-node torch baseline, the self-launcher with ranks sharing the one GPU, and a
clear refusal of more ranks than GPUs."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, timeout=110):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, recs


def test_bench_one_gpu_contract(C):
    r, recs = _bench(["--steps", "20", "--warmup", "5", "--baseline-steps", "30"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(recs) == 1
    rec = recs[0]
    assert rec["n_gpus"] == 1 and rec["steps"] == 20 and rec["warmup"] == 5 and rec["ranks_seen"] == 1
    assert rec["dtype"] == "bf16" and rec["config"]["hipgraph"] is True
    assert rec["epochs"] == 3 and rec["steps_per_rank_per_epoch"] == 1875
    assert rec["wall_3epoch_s"] > 0 and rec["accuracy"] > 0.5  # trains on the synthetic set
    assert rec["baseline_same_node_img_s"] > 0, rec.get("baseline_error")
    assert rec["vs_baseline"] == pytest.approx(rec["value"] / rec["baseline_same_node_img_s"], rel=1e-2)
    # the other precisions and the steady state, same run
    for dt in ("fp16", "fp32"):
        assert rec[f"value_{dt}"] > 0 and rec[f"ms_per_step_{dt}"] > 0, rec.get(f"error_{dt}")
    assert rec["steady_steps"] >= 1875 and rec["steady_img_s"] > 0
    assert rec["comm_error"] == ""


def test_bench_shared_gpu_two_ranks(C):
    r, recs = _bench(["--gpus", "2", "--share-gpu", "--steps", "20", "--warmup", "5", "--epochs", "1"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(recs) == 1
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["ranks_seen"] == 2 and rec["steps"] == 20 and rec["warmup"] == 5
    assert rec["config"]["shared_gpu"] is True and rec["config"]["sync_bn"] is True
    assert rec["steps_per_rank_per_epoch"] == 938
    assert rec["comm_error"] == "" and rec["fallback"] is None
    assert "xgmi" in rec["config"]["comm"].lower()


def test_bench_shared_gpu_site_timeout_falls_back(C):
    """Rank 1 stops entering collectives for longer than the exchange timeout at step 3:
    rank 0's in-kernel exchange times out (error word), its watchdog reports and exits, the
    supervisor kills rank 1 and re-runs both as fresh processes on the host-staged
    communicator -> one line with the measured value, ``fallback`` and the original error."""
    env = {"DPA_FAULT": "1:3:slow:6", "DPA_XGMI_TIMEOUT": "1", "DPA_BENCH_WATCHDOG": "20", "DPA_BENCH_GRACE": "3"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        r, recs = _bench(["--gpus", "2", "--share-gpu", "--steps", "5", "--warmup", "2", "--epochs", "1",
                          "--train-samples", "2048", "--test-samples", "256", "--extra-dtypes", ""], timeout=110)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert len(recs) == 1
    rec = recs[0]
    assert rec["fallback"] == "host" and rec["value"] > 0
    assert "timeout" in rec["comm_error"] or "watchdog" in rec["comm_error"], rec["comm_error"]
    assert [a["ok"] for a in rec["attempts"]] == [False, True]


def test_bench_refuses_more_ranks_than_gpus(C):
    n = torch.cuda.device_count() + 1
    r, recs = _bench(["--gpus", str(n), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2 and not recs
    assert "GPU(s) are visible" in r.stderr
