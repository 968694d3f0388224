#!/usr/bin/env python3
"""Throughput harness for the five BASELINE.json configurations + scaling curve.

Each configuration is one ``bench.py`` run launched with
``torch.distributed.run`` (one process per GPU, 127.0.0.1 rendezvous). Its
single JSON line is collected, and everything is written to one JSON file.
Configurations that need more GPUs than this node has are reported as
skipped. They are never oversubscribed, because RCCL rejects two ranks on
one GPU.

  #1  world 2 on CPU/gloo, 2 subgroups x 1 rank, MLP-VAE (plumbing)
  #2  1 subgroup x 1 MI355X, conv-VAE 28x28 bf16
  #3  8 subgroups x 1 MI355X, 8 concurrent trials, MLP-VAE (headline shape)
  #4  4 subgroups x 2 MI355X, conv-VAE 28x28 with intra-group all-reduce
  #5  2 subgroups x 4 MI355X, conv-VAE 128x128 with per-layer buckets

``--scaling`` adds the headline weak-scaling curve at N = 1, 2, 4, 8 GPUs (one
trial per GPU) with efficiency = value(N) / (N * value(1)).

usage: python bench/run_configs.py [--out bench_configs.json] [--steps 100] [--scaling] [--only 2,3]
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    1: dict(desc="world 2 CPU/gloo, 2 subgroups x 1 rank, MLP-VAE plumbing", nproc=2, gpus=0,
            args=["--model", "mlp", "--ngroups", "2", "--backend", "torch", "--no-graphs"], env={"DDP_BACKEND": "gloo"}),
    2: dict(desc="1 subgroup x 1 MI355X, conv-VAE 28x28 bf16", nproc=1, gpus=1,
            args=["--model", "conv28", "--ngroups", "1"]),
    3: dict(desc="8 subgroups x 1 MI355X, conv-VAE 28x28 (lr, beta) sweep (headline)", nproc=8, gpus=8,
            args=["--model", "conv28", "--ngroups", "8"]),
    4: dict(desc="4 subgroups x 2 MI355X, conv-VAE 28x28 + intra-group all-reduce", nproc=8, gpus=8,
            args=["--model", "conv28", "--ngroups", "4"]),
    5: dict(desc="2 subgroups x 4 MI355X, conv-VAE 128x128 + per-layer buckets", nproc=8, gpus=8,
            args=["--model", "conv128", "--ngroups", "2", "--batch-size", "64", "--bucket-mb", "4"]),
}


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def run_bench(nproc: int, args, steps: int, warmup: int, env_extra=None, timeout: int = 900):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", str(steps),
           "--warmup", str(warmup)] + list(args)
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + cmd[1:]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    line = next((l for l in reversed(r.stdout.splitlines()) if l.startswith("{")), None)
    if r.returncode != 0 or line is None:
        return {"error": f"rc={r.returncode}", "tail": (r.stdout + r.stderr)[-2000:]}
    return json.loads(line)


def ddp_structure(model: str, timeout: int = 600):
    """Per-step time of the reducer-free step and of the DDP step with forced
    one-rank collectives (RCCL, fused xGMI jobs), and their ratios."""
    out = os.path.join("/tmp", f"mdt_ddp_structure_{model}_{os.getpid()}.json")
    cmd = [sys.executable, os.path.join(ROOT, "bench", "ddp_structure.py"), "--model", model, "--steps", "10",
           "--json", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    if r.returncode != 0 or not os.path.exists(out):
        return {"error": f"rc={r.returncode}", "tail": (r.stdout + r.stderr)[-1000:]}
    with open(out) as f:
        d = json.load(f)
    os.unlink(out)
    d.pop("xgmi_overlap_job_spans", None)
    return d


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="bench_configs.json")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--only", default=None, help="comma list of config numbers")
    ap.add_argument("--scaling", action="store_true")
    ap.add_argument("--model", default="conv28", help="model of the 1/2/4/8-GPU scaling curve")
    a = ap.parse_args(argv)
    ngpu = gpu_count()
    only = {int(x) for x in a.only.split(",")} if a.only else set(CONFIGS)
    results = {"gpus_available": ngpu, "configs": {}, "scaling": None}
    for k in sorted(only):
        c = CONFIGS[k]
        if c["gpus"] > ngpu:
            rec = {"desc": c["desc"], "skipped": f"needs {c['gpus']} GPUs, have {ngpu}"}
            if k in (4, 5) and ngpu >= 1:
                # what one GPU CAN measure: the intra-group DDP step's structure cost
                # with every collective forced on a one-rank group (bench/ddp_structure.py)
                rec["one_gpu_ddp_structure"] = ddp_structure("conv28" if k == 4 else "conv128")
            results["configs"][k] = rec
            print(f"config #{k}: skipped ({c['gpus']} GPUs needed); one-GPU DDP structure: "
                  f"{json.dumps(rec.get('one_gpu_ddp_structure'))[:300]}", flush=True)
            continue
        res = run_bench(c["nproc"], c["args"], a.steps, a.warmup, c.get("env"))
        res["desc"] = c["desc"]
        results["configs"][k] = res
        print(f"config #{k}: {json.dumps(res)[:300]}", flush=True)
    if a.scaling:
        curve = []
        for n in (1, 2, 4, 8):
            if n > ngpu:
                curve.append({"n_gpus": n, "skipped": True})
                continue
            r = run_bench(n, ["--model", a.model], a.steps, a.warmup)
            curve.append({"n_gpus": n, "value": r.get("value"), "ms_per_step": r.get("ms_per_step")})
        base = next((c["value"] for c in curve if c.get("n_gpus") == 1 and c.get("value")), None)
        for c in curve:
            if base and c.get("value"):
                c["efficiency"] = round(c["value"] / (c["n_gpus"] * base), 4)
        results["scaling"] = curve
    if os.path.dirname(a.out):
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
