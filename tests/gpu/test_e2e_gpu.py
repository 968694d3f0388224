"""End-to-end on one MI355X: vae-hpo.py with the fused HIP path (single trial,
world of 1), output formats, images, metrics; plus the native reducer on a
size-1 RCCL group (no-op path) and graph capture through the trainer."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_vae_hpo_single_gpu(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "vae-hpo.py"), "--ngroups", "1", "--epochs", "2",
                        "--metrics-dir", "m", "--ckpt-dir", "ck"],
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path), env=env)
    text = r.stdout + r.stderr
    assert r.returncode == 0, text[-4000:]
    assert "Distributed data parallel: nccl master at 127.0.0.1:29611" in text
    assert re.search(r"^\[0:0\] Train Epoch: 1 \[0/60000 \(0%\)\]\tLoss: \d+\.\d{6}$", text, re.M)
    assert re.search(r"^\[0:0\] ====> Epoch: 2 Average loss: \d+\.\d{4}$", text, re.M)
    assert re.search(r"^\[0:0\] ====> Test set loss: \d+\.\d{4}$", text, re.M)
    assert re.search(r"^0 Done\. time: \d+\.\d{6}$", text, re.M)
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["samples"] == 120000 and agg["value"] > 1e5
    # the loss actually decreases over training
    losses = [float(x) for x in re.findall(r"Average loss: (\d+\.\d+)", text)]
    assert losses[-1] < losses[0]
    assert (tmp_path / "results-0" / "reconstruction_2.png").exists()
    assert (tmp_path / "ck" / "trial-0" / "epoch-2.pt").exists()


def test_bench_gpu_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "10"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29612"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["backend"] == "hip" and out["config"]["valid"] and out["value"] > 1e5


def test_vae_hpo_packed_trials_gpu(tmp_path):
    """Two trials packed on one MI355X (one HIP stream each), conv model."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29613")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "vae-hpo.py"), "--ngroups", "1", "--epochs", "1",
                        "--trials-per-group", "2", "--model", "conv", "--train-samples", "4096",
                        "--test-samples", "512", "--metrics-dir", "m"],
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path), env=env)
    text = r.stdout + r.stderr
    assert r.returncode == 0, text[-4000:]
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["trials"] == 2 and agg["samples"] == 2048 * 1 + 2048 * 2 and agg["failed_trials"] == []
    assert re.search(r"^\[0:0\] \(trial 1\) ====> Epoch: 2 Average loss: \d+\.\d{4}$", text, re.M)
    assert (tmp_path / "results-t1-0" / "sample_2.png").exists()


def _hpo(tmp_path, port, *args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "vae-hpo.py"), "--ngroups", "1"] + list(args),
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path), env=env)
    text = r.stdout + r.stderr
    assert r.returncode == 0, text[-4000:]
    assert "FAILED" not in text, text[-4000:]
    return text


def _epoch_losses(text):
    return {int(e): float(v) for e, v in re.findall(r"====> Epoch: (\d+) Average loss: (\d+\.\d+)", text)}


def test_vae_hpo_conv28_ckpt_resume_gpu(tmp_path):
    """The 28x28 conv VAE through vae-hpo on the fused HIP step: 2 epochs
    straight vs 1 epoch + checkpoint + --resume for epoch 2. The resumed run
    restores weights, Adam moments, step counter and data cursor, so its
    epoch-2 loss matches the straight run's (same kernels, same order)."""
    common = ["--model", "conv", "--train-samples", "8192", "--test-samples", "1024", "--no-results"]
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    straight = _hpo(tmp_path / "a", 29615, "--epochs", "2", *common)
    _hpo(tmp_path / "b", 29616, "--epochs", "1", "--ckpt-dir", "ck", *common)
    assert (tmp_path / "b" / "ck" / "trial-0" / "epoch-1.pt").exists()
    resumed = _hpo(tmp_path / "b", 29617, "--epochs", "2", "--ckpt-dir", "ck", "--resume", *common)
    assert "resumed trial 0" in resumed and 1 not in _epoch_losses(resumed)
    la, lb = _epoch_losses(straight), _epoch_losses(resumed)
    assert la[2] < la[1]
    assert abs(la[2] - lb[2]) <= 1e-3 * la[2], (la, lb)
    import torch

    ck = torch.load(str(tmp_path / "b" / "ck" / "trial-0" / "epoch-2.pt"), weights_only=True)
    assert ck["progress"]["epoch"] == 2 and ck["arch"]["kind"] == "conv"


def test_vae_hpo_conv128_gpu(tmp_path):
    """The 128x128 conv VAE (direct-conv + im2col kernels, graphs) through
    vae-hpo for one short epoch: finite decreasing-per-log loss, PNGs, aggregate."""
    text = _hpo(tmp_path, 29618, "--model", "conv", "--image-size", "128", "--epochs", "1",
                "--batch-size", "64", "--train-samples", "2048", "--test-samples", "256", "--metrics-dir", "m")
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["samples"] == 2048 and agg["failed_trials"] == [] and agg["value"] > 1e3
    logs = [float(x) for x in re.findall(r"Train Epoch: 1 .*Loss: (\d+\.\d+)", text)]
    assert len(logs) >= 2 and logs[-1] < logs[0], logs
    assert (tmp_path / "results-0" / "reconstruction_1.png").exists()


def test_bench_trial_packing():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "10",
                        "--trials-per-gpu", "2"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29614"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["trials"] == 2 and out["config"]["valid"]
