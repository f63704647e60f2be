"""End-to-end CLI runs on CPU (BASELINE config 1 plumbing + gloo DDP), small synthetic sets."""
import os
import subprocess
import sys

import pytest
import torch

from ._dist import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow

REF_KEYS = ["layer1.0.weight", "layer1.0.bias", "layer1.1.weight", "layer1.1.bias", "layer1.1.running_mean",
            "layer1.1.running_var", "layer1.1.num_batches_tracked", "layer2.0.weight", "layer2.0.bias",
            "layer2.1.weight", "layer2.1.bias", "layer2.1.running_mean", "layer2.1.running_var",
            "layer2.1.num_batches_tracked", "fc.weight", "fc.bias"]


def _run(args, cwd, env_extra=None, timeout=600, stderr=False):
    env = dict(os.environ)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, *args], cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return (r.stdout, r.stderr) if stderr else r.stdout


def _check_stdout(out, epochs):
    lines = [ln for ln in out.splitlines() if ln.strip()]
    for e in range(epochs):
        assert f"begin training of epoch {e + 1}/{epochs}" in lines
    assert "begin testing" in lines
    acc = [ln for ln in lines if ln.startswith("Accuracy is ")]
    assert len(acc) == 1 and acc[0].endswith("%")
    assert any(ln.startswith("time elapsed: ") and ln.endswith(" seconds") for ln in lines)
    return float(acc[0][len("Accuracy is "):-1])


def test_origin_main_cpu(tmp_path):
    out = _run([os.path.join(ROOT, "origin_main.py"), "-e", "2", "--synthetic", "--train-samples", "2048",
                "--test-samples", "512", "--seed", "0"], tmp_path)
    acc = _check_stdout(out, 2)
    assert acc > 15.0  # learns something in 128 tiny steps at lr 1e-4 (chance: 10 %)
    ck = torch.load(tmp_path / "origin_checkpoint.pt", weights_only=True)
    assert list(ck) == ["model"] and list(ck["model"]) == REF_KEYS
    from ddp_practice_amd.models import ConvNet

    m = ConvNet()
    m.load_state_dict(ck["model"])


def test_ddp_main_spawn_cpu(tmp_path):
    out = _run([os.path.join(ROOT, "ddp_main.py"), "-e", "1", "--synthetic", "--train-samples", "1024",
                "--test-samples", "256", "--cpu-procs", "2", "--amp-dtype", "fp32"], tmp_path,
               {"MASTER_PORT": str(free_port()), "DPA_MASTER_ADDR": "127.0.0.1"})
    _check_stdout(out, 1)
    ck = torch.load(tmp_path / "ddp_checkpoint.pt", weights_only=True)
    assert list(ck["model"]) == ["module." + k for k in REF_KEYS]


def test_ddp_main_torchrun_cpu(tmp_path):
    port = free_port()
    out = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
                f"--master-port={port}", os.path.join(ROOT, "ddp_main_torchrun.py"), "--gpu", "", "-e", "1",
                "--synthetic", "--train-samples", "1024", "--test-samples", "256", "--amp-dtype", "bf16"], tmp_path)
    _check_stdout(out, 1)
    ck = torch.load(tmp_path / "ddp_checkpoint.pt", weights_only=True)
    assert list(ck["model"]) == ["module." + k for k in REF_KEYS]
    assert set(ck["scaler"]) == {"scale", "growth_factor", "backoff_factor", "growth_interval", "_growth_tracker"}


def test_origin_main_resnet50_cpu(tmp_path):
    """``--model resnet50`` (BASELINE.json config 5) through the reference CLI: the
    synthetic ImageNet-shaped set at a small image size, torchvision state_dict keys."""
    out = _run([os.path.join(ROOT, "origin_main.py"), "-e", "1", "-b", "8", "--model", "resnet50",
                "--image-size", "32", "--num-classes", "10", "--train-samples", "32", "--test-samples", "16",
                "--seed", "0"], tmp_path)
    _check_stdout(out, 1)
    ck = torch.load(tmp_path / "origin_checkpoint.pt", weights_only=True)
    from ddp_practice_amd.models import resnet50

    m = resnet50(num_classes=10)
    assert list(ck["model"]) == list(m.state_dict())
    m.load_state_dict(ck["model"])


def test_ddp_main_resnet50_cpu(tmp_path):
    out = _run([os.path.join(ROOT, "ddp_main.py"), "-e", "1", "-b", "4", "--model", "resnet50", "--image-size", "32",
                "--num-classes", "10", "--train-samples", "16", "--test-samples", "8", "--cpu-procs", "2",
                "--amp-dtype", "fp32"], tmp_path, {"MASTER_PORT": str(free_port()), "DPA_MASTER_ADDR": "127.0.0.1"})
    _check_stdout(out, 1)
    ck = torch.load(tmp_path / "ddp_checkpoint.pt", weights_only=True)
    from ddp_practice_amd.models import resnet50

    assert list(ck["model"]) == ["module." + k for k in resnet50(num_classes=10).state_dict()]


@pytest.mark.parametrize("spawn", ["forkserver", "spawn"])
def test_ddp_main_timer_includes_child_interpreter(tmp_path, spawn):
    """``time elapsed`` has the reference's scope (/root/reference/ddp_main.py:175-177: the
    parent times mp.spawn): the interpreter that imports torch for the ranks starts after
    ``time_start`` -- with the fork server as with plain spawn (Missing 2)."""
    out, err = _run([os.path.join(ROOT, "ddp_main.py"), "-e", "1", "--synthetic", "--train-samples", "256",
                     "--test-samples", "64", "--cpu-procs", "2", "--amp-dtype", "fp32"], tmp_path,
                    {"MASTER_PORT": str(free_port()), "DPA_MASTER_ADDR": "127.0.0.1", "DPA_PHASES": "1",
                     "DPA_SPAWN": spawn}, stderr=True)
    _check_stdout(out, 1)
    t0 = [float(ln.split("wall=")[1]) for ln in err.splitlines() if "time_start wall=" in ln]
    starts = [float(ln.split("wall=")[1]) for ln in err.splitlines() if "interpreter_start wall=" in ln]
    assert len(t0) == 1 and len(starts) == 2, err
    assert all(s >= t0[0] for s in starts), (t0, starts)
    elapsed = float([ln for ln in out.splitlines() if ln.startswith("time elapsed: ")][0].split()[2])
    assert elapsed >= max(starts) - t0[0]


def test_shared_cu_mask_gives_each_rank_its_own_cus(monkeypatch):
    """--share-gpu from 3 ranks: disjoint CU ranges (HSA_CU_MASK) covering the device, and the
    residency checks told the per-rank count (DPA_RESIDENT_CUS)."""
    from ddp_practice_amd.runtime.device import shared_cu_mask

    for k in ("HSA_CU_MASK", "DPA_RESIDENT_CUS", "DPA_SHARED_CUS", "DPA_SHARED_CU_MASK"):
        monkeypatch.delenv(k, raising=False)
    assert shared_cu_mask(2, 1) is None and "HSA_CU_MASK" not in os.environ
    masks = [shared_cu_mask(8, r) for r in range(8)]
    assert masks[0] == "0:0-31" and masks[7] == "0:224-255" and os.environ["DPA_RESIDENT_CUS"] == "32"
    cus = [set(range(int(m[2:].split("-")[0]), int(m.split("-")[1]) + 1)) for m in masks]
    assert set().union(*cus) == set(range(256)) and sum(len(c) for c in cus) == 256
    monkeypatch.setenv("DPA_SHARED_CU_MASK", "0")
    assert shared_cu_mask(8, 3) is None


def test_spin_sync_is_opt_in_and_uses_the_loaded_runtime(monkeypatch):
    """runtime/device.spin_sync: nothing without DPA_SPIN_SYNC=1; opted in, it talks only to
    the HIP runtime this process already loaded (torch's), never a second copy by name --
    with torch's runtime loaded on a GPU-less host it calls it and reports the hipError."""
    import torch  # noqa: F401  (loads torch's libamdhip64, as bench.py has by then)

    from ddp_practice_amd.runtime import device

    monkeypatch.delenv("DPA_SPIN_SYNC", raising=False)
    assert device.spin_sync(0) is None
    monkeypatch.setenv("DPA_SPIN_SYNC", "1")
    lib = device._loaded_hip()
    rc = device.spin_sync(0)
    if lib is None:  # a CPU-only torch build: no HIP runtime in the process
        assert rc is None
    else:
        assert isinstance(rc, int)  # hipSuccess on a GPU box, an error code (no device) here
    monkeypatch.setattr(device, "_loaded_hip", lambda: None)
    assert device.spin_sync(0) is None


def test_shared_gpu_env_one_hw_queue_from_three_ranks(monkeypatch):
    """--share-gpu: ranks get the fused-path gates, and from 3 ranks one HIP hardware queue
    per process (4 processes with 4 queues each stalled on one MI355X; profiles/r5v_*)."""
    from ddp_practice_amd.runtime.device import shared_gpu_env

    for k in ("DPA_SHARED_GPU", "GPU_MAX_HW_QUEUES", "DPA_SHARED_HW_QUEUES"):
        monkeypatch.delenv(k, raising=False)
    shared_gpu_env(2)
    assert os.environ["DPA_SHARED_GPU"] == "1" and "GPU_MAX_HW_QUEUES" not in os.environ
    shared_gpu_env(4)
    assert os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.setenv("DPA_SHARED_HW_QUEUES", "2")
    shared_gpu_env(4)
    assert os.environ["GPU_MAX_HW_QUEUES"] == "2"
