#!/usr/bin/env python3
"""Reference-equivalent baseline on MI355X (for BASELINE.md's "reference on MI355X" rows).

The reference publishes no numbers and cannot run unmodified on the GPU box
(no torchvision, no network). This harness re-creates its per-trial behaviour
with stock PyTorch-ROCm, mirroring /root/reference/vae-hpo.py:
  * MLP VAE 784-400-20, fp32, torch eager (vae-hpo.py:19-45)
  * DistributedDataParallel(model, process_group=group) (vae-hpo.py:130)
  * Adam(lr=1e-3) (vae-hpo.py:131)
  * DataLoader(batch 128, DistributedSampler(rank=g, num_replicas=K), CPU
    tensors -> .to(device) every step) over a synthetic [N,1,28,28] dataset in
    [0,1] (stand-in for torchvision MNIST + ToTensor; no PIL decode, so this
    is generous to the reference) (vae-hpo.py:146-150)
  * BCE(sum) + KLD loss and loss.item() each step (vae-hpo.py:49-58, :73)
With ``--model conv28|conv128`` the same loop trains the conv-VAE of
``multidisttorch_amd/models/conv_vae.py`` in stock torch ops (MIOpen convs,
bf16 autocast, channels-last left to torch's defaults): the reference's
training loop with the north-star model swapped in, so bench.py's conv numbers
have a same-GPU torch-eager anchor.
Reports the hot training-loop throughput (samples/s over full epochs of the
shard), and optionally the full reference epoch (train + test pass + 64-sample
decode) as one JSON line. Single process or torchrun (one trial per rank).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn, optim

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class RefVAE(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(784, 400)
        self.fc21 = nn.Linear(400, 20)
        self.fc22 = nn.Linear(400, 20)
        self.fc3 = nn.Linear(20, 400)
        self.fc4 = nn.Linear(400, 784)

    def forward(self, x):
        h1 = F.relu(self.fc1(x.view(-1, 784)))
        mu, logvar = self.fc21(h1), self.fc22(h1)
        z = mu + torch.randn_like(mu) * torch.exp(0.5 * logvar)
        return torch.sigmoid(self.fc4(F.relu(self.fc3(z)))), mu, logvar


def ref_loss(recon_x, x, mu, logvar):
    bce = F.binary_cross_entropy(recon_x, x.view(-1, 784), reduction="sum")
    kld = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
    return bce + kld


class ConvRef(nn.Module):
    """Conv-VAE whose forward returns the ELBO (randn_like eps like the
    reference's reparameterize), so DDP sees one module call per step."""

    def __init__(self, net):
        super().__init__()
        self.net = net

    def forward(self, x):
        n = self.net
        mu, lv = n.encode(x)
        zz = mu + torch.randn_like(mu) * torch.exp(0.5 * lv)
        t = n.decode_logits(zz).float()
        bce = F.binary_cross_entropy_with_logits(t, x.view_as(t), reduction="sum")
        mu, lv = mu.float(), lv.float()
        return bce - 0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp())


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--ngroups", type=int, default=None)
    ap.add_argument("--full-epoch", action="store_true", help="also time test pass + sampling like the reference")
    ap.add_argument("--model", default="mlp", choices=["mlp", "conv28", "conv128"])
    ap.add_argument("--max-steps", type=int, default=None, help="cap the timed steps per epoch")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"], help="conv models: autocast bf16 or fp32")
    ap.add_argument("--no-miopen", action="store_true",
                    help="torch.backends.cudnn.enabled = False: torch's own conv kernels instead of MIOpen "
                         "(the 28x28 bf16 autocast run aborts inside a MIOpen backward kernel on this stack)")
    a = ap.parse_args(argv)
    if a.no_miopen:
        torch.backends.cudnn.enabled = False

    from multidisttorch_amd.runtime import setup_ddp
    from multidisttorch_amd.parallel.groups import setup_ddp_groups
    from multidisttorch_amd.data.datasets import synthetic_images

    world, rank = setup_ddp(verbose=False)
    K = a.ngroups or world
    groups = setup_ddp_groups(K, verbose=False)
    n_per = world // K
    gid = rank // n_per
    group = groups[gid]
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    img = 128 if a.model == "conv128" else 28
    ntr, nte = (60000, 10000) if img == 28 else (8192, 1024)
    train = synthetic_images(ntr, seed=0, size=img).view(ntr, 1, img, img)
    test = synthetic_images(nte, seed=1, size=img).view(nte, 1, img, img)
    trainset = torch.utils.data.TensorDataset(train, torch.zeros(ntr))
    testset = torch.utils.data.TensorDataset(test, torch.zeros(nte))
    sampler = torch.utils.data.distributed.DistributedSampler(trainset, rank=gid, num_replicas=world // n_per)
    loader = torch.utils.data.DataLoader(trainset, batch_size=a.batch_size, shuffle=False, sampler=sampler)
    test_loader = torch.utils.data.DataLoader(testset, batch_size=a.batch_size, shuffle=False)

    if a.model == "mlp":
        model = RefVAE().to(dev)
        amp = None
    else:
        from multidisttorch_amd.models.conv_vae import TorchConvVAE, conv_vae_spec

        z = 32 if img == 28 else 64
        model = ConvRef(TorchConvVAE(conv_vae_spec(img, 1, z), img, 1, z)).to(dev)
        amp = torch.bfloat16 if (dev.type == "cuda" and a.dtype == "bf16") else None
    model = torch.nn.parallel.DistributedDataParallel(model, process_group=group)
    opt = optim.Adam(model.parameters(), lr=1e-3)

    def step_loss(data):
        if a.model == "mlp":
            recon, mu, lv = model(data)
            return ref_loss(recon, data, mu, lv)
        if amp is None:
            return model(data)
        with torch.autocast(device_type="cuda", dtype=amp):
            return model(data)

    def train_epoch():
        model.train()
        n = 0
        for bi, (data, _) in enumerate(loader):
            if a.max_steps is not None and bi >= a.max_steps:
                break
            data = data.to(dev)
            opt.zero_grad()
            loss = step_loss(data)
            loss.backward()
            loss.item()
            opt.step()
            n += data.shape[0]
        return n

    # warm-up: a few steps (allocator, kernels), then timed epochs
    it = iter(loader)
    for _ in range(5):
        data, _ = next(it)
        data = data.to(dev)
        opt.zero_grad()
        step_loss(data).backward()
        opt.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    samples = 0
    for _ in range(a.epochs):
        samples += train_epoch()
        if a.full_epoch and a.model == "mlp":
            model.eval()
            with torch.no_grad():
                for data, _ in test_loader:
                    data = data.to(dev)
                    r, mu, lv = model(data)
                    ref_loss(r, data, mu, lv).item()
                model.module.fc3  # decode 64 latents like vae-hpo.py:163-170
                z = torch.randn(64, 20).to(dev)
                torch.sigmoid(model.module.fc4(F.relu(model.module.fc3(z)))).cpu()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    total = samples * K  # samples counted once per trial
    if rank == 0:
        print(json.dumps({"what": "reference-equivalent torch eager (DDP + DataLoader + .item())",
                          "model": a.model, "amp": str(amp), "miopen": not a.no_miopen,
                          "device": str(dev), "trials": K, "world": world, "epochs": a.epochs,
                          "full_epoch": a.full_epoch, "samples_per_trial": samples, "wall_s": round(dt, 4),
                          "aggregate_samples_per_s": round(total / dt, 1),
                          "ms_per_step": round(dt / (samples / a.batch_size) * 1e3, 4)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
