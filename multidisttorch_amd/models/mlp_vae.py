"""MLP-VAE: reference topology, flat-arena parameter layout, reference math.

Parity: ``VAE`` <- /root/reference/vae-hpo.py:19-45 (fc1 784->400, fc21/fc22
400->20, fc3 20->400, fc4 400->784), ``loss_function`` <- vae-hpo.py:49-58.
``VAE`` here is a plain ``nn.Module`` with the same parameter names, so a
``state_dict`` moves between the reference, this module and the fused engine.

``arena_layout`` mirrors ``MlpVaeEngine``'s C++ layout (csrc/runtime/vae_engine.cpp):
fc4 last so that the first-ready gradient bucket is the arena tail.
``reference_step`` is the explicit forward/backward the HIP kernels implement,
written in torch ops; it is the CPU backend and the fp32 oracle in the tests.
"""

from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F
from torch import nn

__all__ = ["VAE", "loss_function", "arena_layout", "ARENA_ALIGN", "init_params_",
           "reference_forward", "reference_step", "views"]

ARENA_ALIGN = 64


class VAE(nn.Module):
    def __init__(self, D: int = 784, H: int = 400, Z: int = 20):
        super().__init__()
        self.D, self.H, self.Z = D, H, Z
        self.fc1 = nn.Linear(D, H)
        self.fc21 = nn.Linear(H, Z)
        self.fc22 = nn.Linear(H, Z)
        self.fc3 = nn.Linear(Z, H)
        self.fc4 = nn.Linear(H, D)

    def encode(self, x):
        h1 = F.relu(self.fc1(x))
        return self.fc21(h1), self.fc22(h1)

    def reparameterize(self, mu, logvar, eps=None):
        std = torch.exp(0.5 * logvar)
        if eps is None:
            eps = torch.randn_like(std)
        return mu + eps * std

    def decode(self, z):
        h3 = F.relu(self.fc3(z))
        return torch.sigmoid(self.fc4(h3))

    def forward(self, x, eps=None):
        mu, logvar = self.encode(x.view(-1, self.D))
        z = self.reparameterize(mu, logvar, eps)
        return self.decode(z), mu, logvar


def loss_function(recon_x, x, mu, logvar, beta: float = 1.0):
    """BCE(sum) + beta * KLD (beta = 1 is the reference's ELBO)."""
    D = recon_x.shape[-1]
    bce = F.binary_cross_entropy(recon_x, x.view(-1, D), reduction="sum")
    kld = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
    return bce + beta * kld


def _a(v: int) -> int:
    return (v + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN


def arena_layout(D: int = 784, H: int = 400, Z: int = 20) -> Tuple[List[Tuple[str, int, Tuple[int, ...]]], int, int]:
    """[(name, offset, shape)], total numel, bucket split offset (start of fc4)."""
    out = []
    off = 0
    out.append(("fc1.weight", off, (H, D))); off = _a(off + H * D)
    out.append(("fc1.bias", off, (H,))); off = _a(off + H)
    w2 = off; off = _a(off + 2 * Z * H)
    b2 = off; off = _a(off + 2 * Z)
    out += [("fc21.weight", w2, (Z, H)), ("fc22.weight", w2 + Z * H, (Z, H)),
            ("fc21.bias", b2, (Z,)), ("fc22.bias", b2 + Z, (Z,))]
    out.append(("fc3.weight", off, (H, Z))); off = _a(off + H * Z)
    out.append(("fc3.bias", off, (H,))); off = _a(off + H)
    split = off
    out.append(("fc4.weight", off, (D, H))); off = _a(off + D * H)
    out.append(("fc4.bias", off, (D,))); off = _a(off + D)
    return out, off, split


def views(flat: torch.Tensor, layout) -> Dict[str, torch.Tensor]:
    return {n: flat.narrow(0, o, math.prod(s)).view(s) for n, o, s in layout}


@torch.no_grad()
def init_params_(flat: torch.Tensor, layout, generator: torch.Generator = None):
    """nn.Linear default init: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for W and b."""
    v = views(flat, layout)
    for n, t in v.items():
        layer = n.split(".")[0]
        fan_in = v[layer + ".weight"].shape[1]
        bound = 1.0 / math.sqrt(fan_in)
        r = torch.rand(t.shape, generator=generator, dtype=torch.float32)
        t.copy_((r * 2 - 1) * bound)


def _w(v):
    W2 = torch.cat([v["fc21.weight"], v["fc22.weight"]], 0)
    b2 = torch.cat([v["fc21.bias"], v["fc22.bias"]], 0)
    return v["fc1.weight"], v["fc1.bias"], W2, b2, v["fc3.weight"], v["fc3.bias"], v["fc4.weight"], v["fc4.bias"]


def _bce_terms(t, x):
    sp_pos = torch.clamp(t, min=0) + torch.log1p(torch.exp(-t.abs()))  # -log(1-p)
    sp_neg = sp_pos - t                                                 # -log p
    return x * torch.clamp(sp_neg, max=100.0) + (1 - x) * torch.clamp(sp_pos, max=100.0)


def _relu(pre, mask):
    return torch.relu(pre) if mask is None else pre * mask.to(pre.dtype)


def reference_forward(v, x, eps, beta: float = 1.0, masks=None):
    """Forward + loss pieces exactly as kernels F1-F3 compute them.

    ``masks=(m1, m3)`` optionally pins the ReLU masks (tests: a pre-activation
    within rounding of 0 may legitimately flip between summation orders).
    """
    W1, b1, W2, b2, W3, b3, W4, b4 = _w(v)
    Z = W3.shape[1]
    m1, m3 = masks if masks is not None else (None, None)
    h1 = _relu(x @ W1.t() + b1, m1)
    mulv = h1 @ W2.t() + b2
    mu, lv = mulv[:, :Z], mulv[:, Z:]
    sd = torch.exp(0.5 * lv)
    z = mu + eps * sd
    h3 = _relu(z @ W3.t() + b3, m3)
    t = h3 @ W4.t() + b4
    p = torch.sigmoid(t)
    bce = _bce_terms(t, x).sum()
    kld = -0.5 * (1 + lv - mu * mu - sd * sd).sum()
    return dict(h1=h1, mulv=mulv, mu=mu, lv=lv, sd=sd, z=z, h3=h3, t=t, p=p,
                bce=bce, kld=kld, loss=bce + beta * kld)


def reference_step(v, g, x, eps, beta: float = 1.0, masks=None):
    """Explicit backward (kernels B1-B3) writing into grad views ``g``. Returns fwd dict."""
    f = reference_forward(v, x, eps, beta, masks)
    W1, b1, W2, b2, W3, b3, W4, b4 = _w(v)
    Z = W3.shape[1]
    dlog = f["p"] - x
    g["fc4.weight"].copy_(dlog.t() @ f["h3"])
    g["fc4.bias"].copy_(dlog.sum(0))
    dh3 = (dlog @ W4) * (f["h3"] > 0)
    g["fc3.weight"].copy_(dh3.t() @ f["z"])
    g["fc3.bias"].copy_(dh3.sum(0))
    dz = dh3 @ W3
    dmu = dz + beta * f["mu"]
    dlv = 0.5 * dz * eps * f["sd"] + 0.5 * beta * (f["sd"] * f["sd"] - 1)
    dmulv = torch.cat([dmu, dlv], 1)
    gW2 = dmulv.t() @ f["h1"]
    gb2 = dmulv.sum(0)
    g["fc21.weight"].copy_(gW2[:Z]); g["fc22.weight"].copy_(gW2[Z:])
    g["fc21.bias"].copy_(gb2[:Z]); g["fc22.bias"].copy_(gb2[Z:])
    dh1 = (dmulv @ W2) * (f["h1"] > 0)
    g["fc1.weight"].copy_(dh1.t() @ x)
    g["fc1.bias"].copy_(dh1.sum(0))
    f["dlog"], f["dh3"], f["dmulv"], f["dh1"] = dlog, dh3, dmulv, dh1
    return f


@torch.no_grad()
def reference_adam_(p, g, m, v, step: int, lr, beta1, beta2, eps, weight_decay=0.0,
                    grad_scale=1.0, decoupled=False):
    """torch.optim.Adam arithmetic on flat tensors (step = 1-based t)."""
    gr = g * grad_scale
    if weight_decay != 0:
        if decoupled:
            p.mul_(1 - lr * weight_decay)
        else:
            gr = gr + weight_decay * p
    m.lerp_(gr, 1 - beta1)
    v.mul_(beta2).addcmul_(gr, gr, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
