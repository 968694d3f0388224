"""Convolutional VAE (28x28 and 128x128) on hand-written bf16 MFMA kernels.

North-star extension (BASELINE.json configs #2 and #5; absent from the
reference, whose model is the MLP of /root/reference/vae-hpo.py:19-45):
a conv/deconv encoder-decoder with the same ELBO (BCE(sum) + beta*KLD) and
reparameterisation as the reference.

Layout and precision: NHWC activations in bf16, fp32 master weights + fp32
gradients + fp32 Adam moments in flat arenas (one ``adam_cast`` launch per step
updates the masters and re-emits the bf16 weights AND their [Cin][KH][KW][Cout]
transposes), f32 accumulation everywhere, f32 mu/logvar/logits and loss.

Every layer maps onto the LDS-tiled implicit-GEMM kernels of
csrc/kernels/conv_igemm.hip (conv view: a convT is the conv whose backward-data
is its forward):
  conv    fwd = igemm(conv mode),   d_in = igemm(parity mode, Wt),  dW = wgrad(G=d_out, X=in)
  linear  = conv 1x1 on a 1x1 "image" (split-K when deep and narrow)
  convT   fwd = igemm(parity mode, Wt), d_in = igemm(conv mode),    dW = wgrad(G=in, X=d_out)
ReLU backward and the bias-gradient column sums are fused into the epilogue
that produces each gradient; weight gradients are m-split partial slabs that
one finalize launch reduces (deterministically) and feeds to a fused Adam.
``TorchConvVAE`` is the same network in stock torch ops (fp32, NCHW): the CPU
backend and the numerical oracle of the GPU tests.
"""

from __future__ import annotations

import math
import os
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from ..ops import native
from ..ops.philox import reparam_eps
from .eval_graphs import GraphedEval
from .mlp_vae import reference_adam_

__all__ = ["Layer", "conv_vae_spec", "TorchConvVAE", "ConvVaeTrainer", "conv_layout"]

EVAL_STREAM = 1 << 30


@dataclass(frozen=True)
class Layer:
    name: str
    kind: str          # conv | convT | linear
    cin: int
    cout: int
    k: int
    s: int
    p: int
    relu: bool
    in_hw: int         # input spatial size (1 for linear)
    out_hw: int


def conv_vae_spec(image: int = 28, channels: int = 1, z: int = 32) -> List[Layer]:
    if image == 28:
        enc = [(channels, 32), (32, 64)]
    elif image == 128:
        enc = [(channels, 32), (32, 64), (64, 128), (128, 256)]
    else:
        raise ValueError("image must be 28 or 128")
    L, hw = [], image
    for i, (ci, co) in enumerate(enc):
        L.append(Layer(f"enc{i + 1}", "conv", ci, co, 4, 2, 1, True, hw, hw // 2))
        hw //= 2
    flat = enc[-1][1] * hw * hw
    L.append(Layer("enc_head", "linear", flat, 2 * z, 1, 1, 0, False, 1, 1))
    L.append(Layer("dec_fc", "linear", z, flat, 1, 1, 0, True, 1, 1))
    dec = [(co, ci) for (ci, co) in reversed(enc)]
    for i, (ci, co) in enumerate(dec):
        last = i == len(dec) - 1
        L.append(Layer(f"dec{i + 1}", "convT", ci, co, 4, 2, 1, not last, hw, hw * 2))
        hw *= 2
    return L


def _w_shape(l: Layer):
    """Our weight layout: conv/linear [Cout][K][K][Cin]; convT [Cin_t][K][K][Cout_t]."""
    if l.kind == "convT":
        return (l.cin, l.k, l.k, l.cout)
    return (l.cout, l.k, l.k, l.cin)


def conv_layout(spec: List[Layer]):
    """[(name, offset, shape)], total; weights then bias per layer, 64-aligned."""
    a = lambda v: (v + 63) // 64 * 64
    out, off = [], 0
    for l in spec:
        ws = _w_shape(l)
        out.append((l.name + ".weight", off, ws))
        off = a(off + math.prod(ws))
        out.append((l.name + ".bias", off, (l.cout,)))
        off = a(off + l.cout)
    return out, off


# --------------------------------------------------------------------------
class TorchConvVAE(nn.Module):
    """Reference network in stock torch ops (fp32, NCHW; Linear inputs flattened
    in NHWC order so weights map 1:1 onto the kernel layout)."""

    def __init__(self, spec: List[Layer], image: int, channels: int, z: int):
        super().__init__()
        self.spec, self.image, self.channels, self.z = spec, image, channels, z
        mods = {}
        for l in spec:
            if l.kind == "conv":
                mods[l.name] = nn.Conv2d(l.cin, l.cout, l.k, l.s, l.p)
            elif l.kind == "convT":
                mods[l.name] = nn.ConvTranspose2d(l.cin, l.cout, l.k, l.s, l.p)
            else:
                mods[l.name] = nn.Linear(l.cin, l.cout)
        self.layers = nn.ModuleDict(mods)

    def _run(self, layers, h):
        for l in layers:
            m = self.layers[l.name]
            if l.kind == "linear":
                if h.dim() == 4:  # NCHW -> NHWC flatten
                    h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)
                h = m(h)
            else:
                if h.dim() == 2:  # NHWC flat -> NCHW
                    c = l.cin
                    hw = int(round(math.sqrt(h.shape[1] // c)))
                    h = h.view(h.shape[0], hw, hw, c).permute(0, 3, 1, 2)
                h = m(h)
            if l.relu:
                h = F.relu(h)
        return h

    def encode(self, x):
        enc = [l for l in self.spec if l.name.startswith("enc")]
        h = self._run(enc, x.view(-1, self.channels, self.image, self.image))
        return h[:, : self.z], h[:, self.z:]

    def decode_logits(self, zz):
        dec = [l for l in self.spec if l.name.startswith("dec")]
        return self._run(dec, zz)

    def forward(self, x, eps):
        mu, lv = self.encode(x)
        zz = mu + eps * torch.exp(0.5 * lv)
        t = self.decode_logits(zz)
        return t, mu, lv

    def loss(self, x, eps, beta: float = 1.0):
        t, mu, lv = self.forward(x, eps)
        xt = x.view(x.shape[0], self.image, self.image, self.channels).permute(0, 3, 1, 2)
        sp_pos = torch.clamp(t, min=0) + torch.log1p(torch.exp(-t.abs()))
        bce = (xt * torch.clamp(sp_pos - t, max=100.0) + (1 - xt) * torch.clamp(sp_pos, max=100.0)).sum()
        kld = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp())
        return bce + beta * kld, t, mu, lv

    # weight mapping between torch modules and the kernel arena layout
    def to_arena(self) -> Dict[str, torch.Tensor]:
        out = {}
        for l in self.spec:
            m = self.layers[l.name]
            w = m.weight.detach()
            if l.kind in ("conv", "convT"):
                w = w.permute(0, 2, 3, 1).contiguous()
            else:
                w = w.reshape(l.cout, 1, 1, l.cin)
            out[l.name + ".weight"] = w
            out[l.name + ".bias"] = m.bias.detach()
        return out

    @torch.no_grad()
    def from_arena(self, d: Dict[str, torch.Tensor]):
        for l in self.spec:
            m = self.layers[l.name]
            w = d[l.name + ".weight"].to(m.weight.device, m.weight.dtype)
            if l.kind in ("conv", "convT"):
                m.weight.copy_(w.permute(0, 3, 1, 2))
            else:
                m.weight.copy_(w.reshape(l.cout, l.cin))
            m.bias.copy_(d[l.name + ".bias"])

    def grads_to_arena(self) -> Dict[str, torch.Tensor]:
        out = {}
        for l in self.spec:
            m = self.layers[l.name]
            g = m.weight.grad
            if l.kind in ("conv", "convT"):
                g = g.permute(0, 2, 3, 1).contiguous()
            else:
                g = g.reshape(l.cout, 1, 1, l.cin)
            out[l.name + ".weight"] = g
            out[l.name + ".bias"] = m.bias.grad
        return out


# --------------------------------------------------------------------------
class ConvVaeTrainer(GraphedEval):
    """One trial of the conv VAE. Same driver-facing API as MlpVaeTrainer."""

    def __init__(self, batch_size: int = 128, image: int = 28, channels: int = 1, z: int = 32, device=None,
                 backend: Optional[str] = None, seed: int = 0, lr: float = 1e-3, kl_beta: float = 1.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, decoupled_wd: bool = False,
                 rng_stream: int = 0, use_graphs: bool = True, graph_steps: int = 10, init_seed: Optional[int] = None):
        self.B, self.image, self.channels, self.Z = batch_size, image, channels, z
        self.D = image * image * channels
        self.H = None
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        backend = backend or ("hip" if self.device.type == "cuda" else "torch")
        self.backend = backend
        self.seed, self.rng_stream = int(seed), int(rng_stream)
        self.hp = dict(lr=lr, beta1=betas[0], beta2=betas[1], eps=eps, weight_decay=weight_decay,
                       kl_beta=kl_beta, grad_scale=1.0)
        self.decoupled_wd = decoupled_wd
        self.spec = conv_vae_spec(image, channels, z)
        self.layout, self.numel = conv_layout(self.spec)
        # first decoder parameter: the default bucket boundary (decoder grads are ready first)
        self.split = next(o for n, o, _ in self.layout if n.startswith("dec"))
        self.use_graphs = use_graphs and backend == "hip"
        self.graph_steps = max(1, graph_steps)
        self._graphs = {}
        self.reducer = None
        # horizontal fusion of independent backward launches (conv_jobs.hip);
        # MDT_CONV_JOBS=0 issues every op as its own kernel (A/B, bitwise equal)
        self.fuse_jobs = os.getenv("MDT_CONV_JOBS", "1") != "0"
        # finalize+Adam of each layer spread over the backward launches (third
        # job of the launch after its gradients completed) instead of all in
        # the optimizer tail (MDT_CONV_SPREAD_FIN, bitwise equal). Measured
        # neutral at 28x28 with the transposes in the tail (the tail shrinks,
        # the hosting launches grow by as much) and 0.7 % slower at 128x128
        # (profiles/r1_tail); with the transposes deferred (below) 1 % faster
        # at 28x28 (0.1208 -> 0.1196 ms, profiles/r1_defer). Round 4 (16-B
        # transposes, 64x32 shallow-Linear tiles) re-measured 128x128 B=64:
        # 0.3572-0.3585 spread vs 0.3595-0.3608 ms tail (profiles/r4_tiles):
        # on at every size now
        self.spread_fin = os.getenv("MDT_CONV_SPREAD_FIN", "1") == "1"
        # two-launch tail without the transposes (MDT_CONV_DEFER_WT=1|2, no
        # ticket, no fences): the tail's second launch is the first layer's
        # finalize alone, and the transposed weight copies ride in the next
        # step's first launch (=1) or in the decoder Linear's launch (=2: a
        # 50-block GEMM at 28x28 that leaves most CUs free for the copies).
        # Measured (profiles/r1_defer): 28x28 0.1249 -> 0.1232 (=1) -> 0.1209
        # ms/step (=2); 128x128 B=64 0.4517 -> 0.460 (=1) / 0.4545 (=2), so
        # the default is 2 up to 64x64 images and 0 above
        mode = os.getenv("MDT_CONV_DEFER_WT", "2" if image <= 64 else "0")
        self.defer_wt = mode in ("1", "2")
        self.wt_in_dec = mode == "2"
        # per-sample fused 28x28 step (csrc/kernels/conv28_fused.hip): forward,
        # backward-data, weight gradients and optimizer in 4 launches instead of
        # the layer-by-layer path's 15. MDT_CONV_F28=0 keeps the layer path.
        self.f28 = (backend == "hip" and image == 28 and channels == 1 and z == 32
                    and os.getenv("MDT_CONV_F28", "1") != "0")
        self._plans28 = {}
        self.f28_skip_adam = False  # tests: leave the reduced gradients in `grads`, no update
        # forward and backward of the fused step in one launch (MDT_F28_MERGE=0: two)
        self.f28_merge = os.getenv("MDT_F28_MERGE", "1") != "0"
        # the merged step with two workgroups per sample (conv28_pair.h): a
        # B = 128 trial fills all 256 CUs instead of 128. MDT_F28_PAIR=0 (A/B): one per sample
        self.f28_pair = os.getenv("MDT_F28_PAIR", "1") != "0"
        # eval passes through the same paired form, forward only (MDT_F28_EVAL_PAIR=0: solo f28_fwd_k)
        self._eval_pair = os.getenv("MDT_F28_EVAL_PAIR", "1") != "0"
        # DDP on the fused 28x28 step: the decoder bucket goes out before the
        # encoder weight gradients (True), or every bucket after the whole
        # backward on one stream (False); "auto" (default): overlap only when
        # the decoder bucket's transfer over one xGMI link outweighs the
        # measured cost of splitting the weight-gradient launch
        # (parallel/ddp.py::overlap_pays, profiles/r4_ddp_fused)
        ov = os.getenv("MDT_DDP_OVERLAP", "auto")
        self.ddp_overlap = None if ov == "auto" else ov != "0"
        # tests: > 0 delays every partner workgroup (forces the solo fallback); < 0 stalls sample 0's
        # role-1 half after pairing (forces an exchange timeout: f28_err, health_error());
        # MDT_F28_TEST_STALL_US=N sets -N (fault drills through the HPO runner / bench)
        self.f28_pair_delay_us = -int(os.getenv("MDT_F28_TEST_STALL_US", "0"))
        # profiling: int64 [B*16] tensors (fwd, bwd) receiving per-workgroup
        # phase-end s_memrealtime stamps (obs/f28_phases.py); None = off
        self.f28_stamps = (None, None)
        self._fused_launches = 0
        self._comm_packs = {}
        self._comm_tables = {}
        # profiling: int64 tensors ([grid][2] each) receiving per-workgroup start/end
        # stamps of the fused-reducer step's job launches (bench/ddp_structure.py); None = off
        self.comm_stamps = None
        # one-GPU multi-process rehearsals (eager only): push and reduce in separate
        # launches with ``comm_phase_hook()`` (e.g. device sync + host barrier)
        # between them, so no rank's reduce ever spins on a peer that shares
        # the GPU (tests/gpu/conv_ddp_worker.py)
        self.comm_split_tail = False
        self.comm_phase_hook = None
        self._data = None
        torch.manual_seed(self.seed if init_seed is None else init_seed)
        ref = TorchConvVAE(self.spec, image, channels, z)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.params = torch.zeros(self.numel, **f32)
        self.grads = torch.zeros(self.numel, **f32)
        self.exp_avg = torch.zeros(self.numel, **f32)
        self.exp_avg_sq = torch.zeros(self.numel, **f32)
        for name, t in ref.to_arena().items():
            self.named_parameters()[name].copy_(t)
        if backend == "torch":
            self.model = ref.to(self.device)
            self._st = dict(step=0, cursor=0, nbatches=0, epoch_loss=0.0, epoch_count=0.0)
            self._st_eval = dict(step=0, cursor=0, nbatches=0, epoch_loss=0.0, epoch_count=0.0)
            self._hist = np.zeros(4096, np.float32)
            self._hist_eval = np.zeros(4096, np.float32)
        else:
            self.C = native.require()
            self.state = self.C.TrialState(self.device.index or 0)
            self._alloc_hip()
        self._push_hparams()

    # ----------------------------------------------------------- arenas
    def model_meta(self) -> dict:
        """Architecture record stored in checkpoints and validated on load."""
        return {"kind": "conv", "image": int(self.image), "channels": int(self.channels), "Z": int(self.Z),
                "layers": [[l.name, l.kind, l.cin, l.cout, l.k, l.s, l.p] for l in self.spec]}

    def named_parameters(self):
        return {n: self.params.narrow(0, o, math.prod(s)).view(s) for n, o, s in self.layout}

    def named_grads(self):
        return {n: self.grads.narrow(0, o, math.prod(s)).view(s) for n, o, s in self.layout}

    def state_dict(self):
        return {k: v.detach().cpu().clone() for k, v in self.named_parameters().items()}

    @torch.no_grad()
    def load_state_dict(self, sd):
        for k, t in self.named_parameters().items():
            t.copy_(sd[k].to(t.device, torch.float32))
        if self.backend == "hip":
            self._cast_weights()
        else:
            self.model.from_arena(self.named_parameters())

    def optimizer_state(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg.cpu().clone(), "exp_avg_sq": self.exp_avg_sq.cpu().clone()}

    @torch.no_grad()
    def load_optimizer_state(self, st):
        self.exp_avg.copy_(st["exp_avg"])
        self.exp_avg_sq.copy_(st["exp_avg_sq"])
        self.set_step(int(st["step"]))

    def set_hparams(self, **kw):
        for k, v in kw.items():
            self.hp[k] = float(v)
        self._push_hparams()

    def _push_hparams(self):
        if self.backend == "hip":
            h = self.hp
            self.state.set_hparams(h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"], h["kl_beta"],
                                   h["grad_scale"], self.seed, self.decoupled_wd)

    # ----------------------------------------------------------- state
    @property
    def step_count(self):
        return int(self.read_state()["step"])

    @property
    def comm_jobs(self) -> bool:
        """The step can host the fused all-reduce jobs (comm_jobs.h): the
        default intra-node reducer for this trainer is then kind "xgmi"."""
        return self.backend == "hip" and self.fuse_jobs

    def _invalidate_prefetch(self):
        """The host moved the cursor, the step or the data: rows the last
        finalize gathered are not the next step's (f28 P0 falls back to the
        index chain until the next finalize gathers again)."""
        xt = getattr(self, "f28_xtag", None)
        if xt is not None:
            xt.fill_(-1)

    def set_step(self, step):
        self._invalidate_prefetch()
        if self.backend == "hip":
            red = self.reducer
            if red is not None and hasattr(red, "rebase_epochs"):
                # the fused jobs' epoch is step + base: keep it increasing
                red.rebase_epochs(self.step_count, int(step))
            self.state.set_step(False, int(step))
        else:
            self._st["step"] = int(step)

    def set_cursor(self, cursor, nbatches, eval=False):
        if not eval:
            self._invalidate_prefetch()
        if self.backend == "hip":
            self.state.set_cursor(eval, int(cursor), int(nbatches))
        else:
            st = self._st_eval if eval else self._st
            st["cursor"], st["nbatches"] = int(cursor), int(nbatches)

    def reset_loss(self, eval=False):
        if self.backend == "hip":
            self.state.reset_loss(eval)
        else:
            st = self._st_eval if eval else self._st
            st["epoch_loss"], st["epoch_count"] = 0.0, 0.0

    def read_state(self, eval=False):
        if self.backend == "hip":
            s = self.state.read_state(eval)
            return dict(step=int(s[0]), cursor=int(s[1]), nbatches=int(s[2]), epoch_loss=s[3], epoch_count=s[4])
        return dict(self._st_eval if eval else self._st)

    def loss_history(self, eval=False):
        if self.backend == "hip":
            return self.state.loss_history(eval).numpy()
        return (self._hist_eval if eval else self._hist).copy()

    def bind_train_data(self, X, idx):
        assert X.dim() == 2 and X.shape[1] == self.D and X.dtype == torch.float32
        n = idx.numel()
        nb = -(-n // self.B)
        idx = idx.to(device=self.device, dtype=torch.int32)
        pad = nb * self.B - n
        if pad:
            idx = torch.cat([idx, idx[:1].expand(pad)])
        self._data = (X.contiguous(), idx.contiguous(), n, nb)
        self._invalidate_prefetch()
        self._graphs.clear()
        self._plans28.clear()

    def attach_reducer(self, reducer):
        """Reducer over ``self.grads`` whose bucket bounds fall on layer starts
        (see ``bucket_bounds``); buckets launch as their layers' backward ends.
        A fused xGMI reducer (``XgmiP2PReducer(fused=True)``, kind "xgmi")
        instead contributes all-reduce JOBS to the step's own launches
        (csrc/kernels/comm_jobs.h): no second stream, no events."""
        self.reducer = reducer
        self._graphs.clear()
        from ..parallel.ddp import graph_capturable

        # a host-blocking (c10d/gloo) reducer cannot live inside a step graph: eager steps
        if not hasattr(self, "_graphs_wanted"):
            self._graphs_wanted = self.use_graphs
        self.use_graphs = self._graphs_wanted and graph_capturable(reducer)
        self._plans28.clear()
        self._comm_packs = {}
        self._comm_tables = {}

    def health_error(self) -> Optional[str]:
        """Silent-corruption check after an epoch (host sync): a paired-workgroup
        exchange of the fused 28x28 step that timed out (the step then trained on
        zero-filled partial sums, and an all-reduce would make the replicas agree
        on the corrupted gradient) or a reducer wait that gave up on a peer.
        None when healthy."""
        if self.backend != "hip":
            return None
        msgs = []
        if self.f28:
            err = int(self.f28_err.item())
            if err:
                msgs.append(f"fused 28x28 step: a paired-workgroup exchange timed out (f28_err={err}); "
                            f"the trial trained on incomplete partial sums")
            derr = int(self.f28_dep[self._dep_err_idx].item())
            if derr:
                msgs.append(f"fused 28x28 step: a finalize job gave up waiting for job {derr - 1} of its launch; "
                            f"the trial's update used incomplete weight gradients")
        red = self.reducer
        if red is not None and hasattr(red, "status"):
            st = int(red.status())
            if st:
                msgs.append(f"xGMI all-reduce gave up waiting for a peer (status {st})")
        return "; ".join(msgs) or None

    def _comm_ctx(self):
        """Device address of the fused reducer's CommCtx, or 0 (no reducer, or
        one that runs its collectives on its own stream)."""
        red = self.reducer
        if red is None or not hasattr(red, "comm_ctx") or not red.fused():
            return 0
        return int(red.comm_ctx())

    def _comm_job(self, segs, units, u0, u1, mode, adam, job=None):
        """A recorded all-reduce job over finalize units [u0, u1) of a plan
        (into ``job`` when given)."""
        st = self.state
        j = self.C.Job() if job is None else job
        self.C.comm_job(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, segs,
                        units.narrow(0, u0 * 12, (u1 - u0) * 12), u1 - u0, st.train_state, st.hparams, adam,
                        self._comm_ctx(), mode, j)
        return j

    def layer_ranges(self):
        """[(layer, begin, end)] arena range of each layer's (weight, bias)."""
        lay = {n: (o, s) for n, o, s in self.layout}
        out = []
        for l in self.spec:
            b = lay[l.name + ".weight"][0]
            ob, sb = lay[l.name + ".bias"]
            out.append((l, b, ob + sb[0]))
        return out

    def bucket_bounds(self, bucket_mb=None):
        """Bucket bounds in gradient-ready (reverse-layer) order, closed at layer
        boundaries once a bucket holds >= bucket_mb MiB of f32 gradients.
        None -> two buckets (decoder | encoder); 0 -> one bucket."""
        ranges = self.layer_ranges()
        if bucket_mb == 0:
            return [0, self.numel]
        if bucket_mb is None:
            dec0 = next(b for l, b, e in ranges if l.name.startswith("dec"))
            return [0, dec0, self.numel]
        cap = float(bucket_mb) * (1 << 20)
        bounds, acc = [self.numel], 0.0
        for l, b, e in reversed(ranges):
            acc += 4.0 * (e - b)
            if acc >= cap and b > 0:
                bounds.append(b)
                acc = 0.0
        bounds.append(0)
        return sorted(set(bounds))

    def default_bucket_bounds(self):
        return self.bucket_bounds(None)

    @torch.no_grad()
    def refresh_weights(self):
        """Re-derive the bf16 compute copies after ``params`` changed outside a
        step (replica broadcast, checkpoint load)."""
        if self.backend == "hip":
            self._cast_weights()
        else:
            self.model.from_arena(self.named_parameters())

    # ----------------------------------------------------------- HIP path
    def _alloc_hip(self):
        dev = self.device
        B = self.B
        bf = dict(dtype=torch.bfloat16, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.w16 = torch.zeros(self.numel, **bf)
        toff, self._toff = 0, {}
        for l in self.spec:
            self._toff[l.name] = toff
            toff = (toff + math.prod(_w_shape(l)) + 63) // 64 * 64
        self.w16t = torch.zeros(max(toff, 64), **bf)
        rows = self._seg_rows({})
        self.segs = self.C.make_grad_segs(rows, dev.index or 0)
        self.nseg = 2 * len(self.spec)
        tr = []
        self._tr_layer = []  # layer li owns transpose units [_tr_layer[li], _tr_layer[li + 1])
        for si, r in enumerate(rows):
            if si % 2 == 0:
                self._tr_layer.append(len(tr))
            if r[8] < 0:
                continue
            co, k, ci = r[4], r[5], r[7]
            for tap in range(k * k):
                for co0 in range(0, co, 64):
                    for ci0 in range(0, ci, 64):
                        tr.append([si, tap, co0, ci0])
        self._tr_layer.append(len(tr))
        self.tr_units = self.C.make_tr_units(tr, dev.index or 0)
        self.n_tr = len(tr)
        self.xb = torch.zeros(B, self.D, **f32)
        self.acts, self.gacts = {}, {}
        for l in self.spec:
            n_out = B * l.out_hw * l.out_hw * l.cout
            self.acts[l.name] = torch.zeros(n_out, **bf)
            self.gacts[l.name] = torch.zeros(n_out, **bf)
        zf = self.Z
        self.mulv = torch.zeros(B, 2 * zf, **f32)
        self.eps = torch.zeros(B, zf, **f32)
        self.z16 = torch.zeros(B, zf, **bf)
        self.dz = torch.zeros(B, zf, **f32)
        self.dmulv = torch.zeros(B, 2 * zf, **f32)
        self.dmulv16 = torch.zeros(B, 2 * zf, **bf)
        self.logits = torch.zeros(B * self.D, **f32)
        self.recon = torch.zeros(B * self.D, **f32)
        self.dlog16 = torch.zeros(B * self.D, **bf)
        first, last = self.spec[0], self.spec[-1]
        # single-channel edge layers run on the direct kernels of conv_thin.hip
        self._thin_first = first.kind == "conv" and first.cin == 1 and first.cout in (16, 32, 64) and first.k <= 4
        self._thin_last = (last.kind == "convT" and last.cout == 1 and last.cin in (16, 32, 64) and last.k % last.s == 0
                           and last.out_hw % last.s == 0)
        self.bce_part = torch.zeros(max(self._n_bce(B), 1), **f32)
        self.kld_part = torch.zeros(B * zf, **f32)  # >= KLD partials of reparam / combine_reparam
        self._plans = {}
        if self.f28:
            self.dlog32 = torch.zeros(B * self.D, **f32)
            self.f28_part = torch.zeros(3 * B, **f32)                  # bce | kld | dec2-bias partials
            # bias partials: dec_fc [B][3136] | dec1 [B][32] | enc2 [2][B][64] (a row per pair half) | enc1 [B][32]
            self.f28_bias = torch.zeros(B * (3136 + 32 + 128 + 32), **f32)
            # paired step state: exchange granules, pairing words, error word (all zero between launches)
            self.f28_xg = torch.zeros(B * 2 * self.C.f28_pair_words(), dtype=torch.int64, device=dev)
            self.f28_pairw = torch.zeros(B, dtype=torch.int32, device=dev)
            self.f28_err = torch.zeros(1, dtype=torch.int32, device=dev)
            # next-batch prefetch: the finalize of step k gathers step k+1's rows
            # into f28_xn and tags them with the step they are for (f28_xtag);
            # -1 = nothing gathered (the host invalidates on cursor/data/step moves)
            self.f28_xn = torch.zeros(B * self.D, **f32)
            self.f28_xtag = torch.full((B,), -1, dtype=torch.int32, device=dev)
            self.f28_prefetch = os.getenv("MDT_F28_PREFETCH", "1") != "0"
            # MDT_F28_FIN_MERGE=1: finalize + Adam (and the prefetch gather)
            # inside the weight-gradient launch, each layer's units released by
            # in-launch counters as that layer's weight gradient completes
            # (conv_jobs.hip JobPackN deps). Bitwise the two-launch tail but
            # slower (0.079 vs 0.061 ms/step: the waiting workgroups and the
            # producers' store drains slow the weight gradients 30-80 %,
            # profiles/r6_fin_merge), so off by default
            self.f28_fin_merge = os.getenv("MDT_F28_FIN_MERGE", "0") == "1"
            words, self._dep_err_idx = self.C.jobs_dep_layout()
            self.f28_dep = torch.zeros(words, dtype=torch.int32, device=dev)  # counters, zero between launches
        self._cast_weights()

    def _n_bce(self, M):
        """Number of BCE loss partials the forward writes for a batch of M."""
        if self._thin_last:
            return self.C.thin_blocks(True, self._desc(self.spec[-1], M))
        return -(-M * self.D // 256)

    def _n_kld(self, M):
        """Number of KLD partials the forward writes for a batch of M (one per
        block of the reparameterisation kernel that ends the encoder)."""
        head = [l for l in self.spec if l.name.startswith("enc")][-1]
        ks = self.C.igemm_plan(0, self._desc(head, M), True, fwd=True)[10]
        if ks > 1:
            return self.C.combine_reparam_blocks(ks, M, self.Z)
        return -(-M * self.Z // 256)

    def _wf32(self, l):
        """f32 master weight of a layer (read directly by the thin kernels)."""
        o, s = next((o, s) for n, o, s in self.layout if n == l.name + ".weight")
        return self.params.narrow(0, o, math.prod(s))

    def _seg_rows(self, slabs):
        """GradSeg rows (off, numel, slab_ptr, nsplit, co, k, s, ci, toff) for every
        weight and bias; ``slabs`` maps a parameter name to (tensor, nsplit)."""
        rows = []
        lay = {n: (o, s) for n, o, s in self.layout}
        for l in self.spec:
            for suffix in (".weight", ".bias"):
                name = l.name + suffix
                o, shp = lay[name]
                t, ns = slabs.get(name, (None, 1))
                ptr = t.data_ptr() if t is not None else 0
                if suffix == ".weight":
                    rows.append([o, math.prod(shp), ptr, ns, shp[0], shp[1], l.s, shp[3], self._toff[l.name]])
                else:
                    rows.append([o, shp[0], ptr, ns, 0, 0, 0, 0, -1])
        return rows

    def _plan(self, M):
        """Per-batch-size backward plan: partial-slab buffers sized from the
        native planners, the GradSeg/GradUnit tables of the finalize kernel and
        the split-K workspace (built once per M, reused by every step/graph)."""
        p = self._plans.get(M)
        if p is not None:
            return p
        C, dev = self.C, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        slabs, ws_need = {}, 0
        spec = self.spec
        names = [l.name for l in spec]
        colsum = {}
        for i, l in enumerate(spec):
            d = self._desc(l, M)
            info = C.wgrad_plan(d)
            ns = info[6]
            wn = math.prod(_w_shape(l))
            if ns > 1:
                slabs[l.name + ".weight"] = (torch.empty(ns * wn, **f32), ns)
            # backward-data producing the previous layer's gradient
            if i == 0:
                continue
            prev = spec[i - 1]
            if i == len(spec) - 1 and self._thin_last:
                rows, ncols = C.thin_blocks(False, d), prev.cout
                t = torch.empty(rows * ncols, **f32)
                colsum[prev.name] = t
                slabs[prev.name + ".bias"] = (t, rows)
                continue
            mode = 0 if l.kind == "convT" else 1
            split_ok = l.name == "dec_fc"
            q = C.igemm_plan(mode, d, split_ok)
            if split_ok and q[10] > 1:
                ws_need = max(ws_need, q[10] * q[4] * q[5])
            if prev.name in ("dec_fc",) or l.name == "dec_fc":
                continue  # per-feature / reparam biases: colsum kernel below
            rows, ncols = q[11], q[5]
            t = torch.empty(rows * ncols, **f32)
            colsum[prev.name] = t
            slabs[prev.name + ".bias"] = (t, rows * (ncols // prev.cout))
        for l in spec:  # forward split-K (deep, narrow conv-mode layers such as enc_head)
            if l.kind != "convT":
                q = C.igemm_plan(0, self._desc(l, M), True, fwd=True)
                if q[10] > 1:
                    ws_need = max(ws_need, q[10] * q[4] * q[5])
        # the layer feeding the encoder head, when it runs split-K: its combine
        # is folded into the head GEMM's A staging (APro, conv_igemm_dev.h)
        ws_a, ks_a = None, 0
        enc = [l for l in spec if l.name.startswith("enc")]
        if len(enc) >= 3 and os.getenv("MDT_CONV_APRO", "1") != "0":
            src = enc[-2]
            if not (src is spec[0] and self._thin_first) and src.kind == "conv" and src.cout % 8 == 0:
                q = C.igemm_plan(0, self._desc(src, M), True, fwd=True)
                if q[10] > 1:
                    ks_a = q[10]
                    ws_a = torch.empty(ks_a * q[4] * q[5], **f32)
        rows_per = 8  # colsum kernel partial rows for the per-feature biases
        ncs = -(-M // rows_per)
        for l in spec:
            if l.name in ("dec_fc", "enc_head"):
                t = torch.empty(ncs * l.cout, **f32)
                colsum[l.name] = t
                slabs[l.name + ".bias"] = (t, ncs)
        last = spec[-1]
        nb = self._n_bce(M)
        gpart = torch.empty(nb, **f32)
        if self.channels == 1:
            slabs[last.name + ".bias"] = (gpart, nb)
        else:
            raise NotImplementedError("conv-VAE HIP path: multi-channel images need the per-channel dlogits sum")
        segs = self._seg_rows(slabs)
        units, layer_units = self._finalize_units(segs)
        p = dict(slabs=slabs, colsum=colsum, gpart=gpart, ws=torch.empty(max(ws_need, 1), **f32), rows_per=rows_per,
                 ws_a=ws_a, ks_a=ks_a,
                 segs=C.make_grad_segs(segs, dev.index or 0), units=C.make_grad_units(units, dev.index or 0),
                 nunits=len(units), layer_units=layer_units)
        self._plans[M] = p
        return p

    @staticmethod
    def _finalize_units(segs):
        """GradUnit rows (seg, start, count) of the finalize kernel for GradSeg
        rows ``segs``; layer i owns units [layer_units[i], layer_units[i+1])."""
        units, layer_units = [], []
        for si, (off, numel, ptr, ns, *_rest) in enumerate(segs):
            if si % 2 == 0:
                layer_units.append(len(units))
            rp = 1  # partial rows per unit column; 256-thread finalize blocks (kFinalizeThreads)
            if ptr:
                while rp < 256 and rp * 16 < ns:
                    rp *= 2
            cnt = 256 // rp
            if rp == 1 and numel % 4 == 0 and off % 4 == 0 and ptr % 16 == 0:
                cnt = 4 * 256  # grad_finalize_vec4: 4 elements per thread, 16-B accesses
            for st in range(0, numel, cnt):
                units.append([si, st, min(cnt, numel - st)])
        layer_units.append(len(units))
        return units, layer_units

    def _cast_weights(self):
        h = self.state
        self.C.adam_cast(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, self.segs, self.nseg,
                         h.train_state, h.hparams, False)
        self._transpose_weights()

    def _transpose_weights(self):
        """bf16 weights -> parity-ordered transposed copies (one coalesced launch)."""
        self.C.wtrans(self.w16, self.w16t, self.segs, self.tr_units, self.n_tr)

    def _w(self, l):
        o, s = next((o, s) for n, o, s in self.layout if n == l.name + ".weight")
        return self.w16.narrow(0, o, math.prod(s))

    def _wt(self, l):
        s = _w_shape(l)
        return self.w16t.narrow(0, self._toff[l.name], math.prod(s))

    def _b(self, l):
        return self.named_parameters()[l.name + ".bias"]

    def _gw(self, l):
        o, s = next((o, s) for n, o, s in self.layout if n == l.name + ".weight")
        return self.grads.narrow(0, o, math.prod(s))

    def _gb(self, l):
        return self.named_grads()[l.name + ".bias"]

    @staticmethod
    def _desc(l: Layer, M: int):
        if l.kind == "convT":  # conv geometry: conv input = convT output
            return [M, l.out_hw, l.out_hw, l.cout, l.in_hw, l.in_hw, l.cin, l.k, l.k, l.s, l.p]
        return [M, l.in_hw, l.in_hw, l.cin, l.out_hw, l.out_hw, l.cout, l.k, l.k, l.s, l.p]

    def _layer_fwd(self, l, h, M, o16, o32, ws, **pro):
        """conv / linear: conv-mode GEMM; convT: parity-class GEMM on the
        transposed weights (no zero-insertion taps); single-channel edge
        layers: direct kernels."""
        d = self._desc(l, M)
        if l is self.spec[0] and self._thin_first:
            self.C.thin_conv(h, self._wf32(l), d, self._b(l), l.relu, o16)
        elif l is self.spec[-1] and self._thin_last:
            self.C.thin_tconv(h, self._wf32(l), d, self._b(l), y32=o32)
        elif l.kind == "convT":
            self.C.igemm(1, h, self._wt(l), d, self._b(l), l.relu, o16, o32, fwd=True)
        else:
            self.C.igemm(0, h, self._w(l), d, self._b(l), l.relu, o16, o32, ws=ws, fwd=True, **pro)

    def _forward_hip(self, M, state, stream, want_recon=False, train=True, src=None):
        """Forward of one batch. ``src = (X, idx)``: the batch is gathered from
        the dataset by the step's first kernel (and the step begun there) when
        the first layer runs on the direct kernel; otherwise by gather_rows."""
        C = self.C
        p = self._plan(M)
        hp = self.state.hparams
        enc = [l for l in self.spec if l.name.startswith("enc")]
        dec = [l for l in self.spec if l.name.startswith("dec")]
        h = self.xb
        first = 0
        # w16t of the previous step's update still to be written (an eval
        # forward finds them current: evaluate() ran _ensure_wt first)
        wt = self._wt_deferred() and train
        if src is not None:
            X, idx = src
            l = enc[0]
            if self.fuse_jobs and self._thin_first and len(enc) > 1:
                first_conv = (lambda job, l=l: C.thin_conv(X, self._wf32(l), self._desc(l, M), self._b(l), l.relu,
                                                           self.acts[l.name], job=job, idx=idx, state=state,
                                                           hparams=hp, B=self.B, xb=self.xb))
                if wt and not self.wt_in_dec:
                    # the transposed copies share the step's first launch (nothing in it reads them)
                    self._run_group([first_conv, lambda job: self._wtrans_layers(1, len(self.spec), job)])
                    wt = False
                else:
                    first_conv(None)
                h, first = self.acts[l.name], 1
            else:
                C.step_begin(state, hp)
                C.gather_rows(X, idx, state, self.B, M, self.xb)
        if wt and not (self.wt_in_dec and self.fuse_jobs):
            self._wtrans_layers(1, len(self.spec))
            wt = False
        pro = {}
        for l in enc[first:]:
            last = l is enc[-1]
            if not last and p["ws_a"] is not None and l is enc[-2]:
                # split-K partials only; the head's A staging combines them (+bias, ReLU)
                # and writes this layer's activations for the backward
                C.igemm(0, h, self._w(l), self._desc(l, M), None, False, None, None, ws=p["ws_a"], combine=False,
                        fwd=True)
                pro = dict(a_slab=p["ws_a"], a_ks=p["ks_a"], a_bias=self._b(l), a_relu=l.relu,
                           a_out16=self.acts[l.name])
                h = self.acts[l.name]
                continue
            if last:
                q = C.igemm_plan(0, self._desc(l, M), True, fwd=True)
                if q[10] > 1:  # split-K head: combine fused with the reparameterisation
                    C.igemm(0, h, self._w(l), self._desc(l, M), self._b(l), False, None, self.mulv, ws=p["ws"],
                            combine=False, fwd=True, **pro)
                    C.combine_reparam(p["ws"], q[10], self._b(l), self.mulv, self.eps, self.z16, None, M, self.Z,
                                      state, hp, stream, self.kld_part)
                    break
            self._layer_fwd(l, h, M, None if last else self.acts[l.name], self.mulv if last else None, p["ws"],
                            **(pro if last else {}))
            h = self.acts[l.name]
        else:
            C.reparam(self.mulv, self.eps, self.z16, None, M, self.Z, state, hp, stream, self.kld_part)
        h = self.z16
        for l in dec:
            last = l is dec[-1]
            if wt:
                # the transposed copies share the first decoder launch: nothing
                # before it reads them, the parity-mode layers after it do
                wt = False
                d = self._desc(l, M)
                if (l.kind != "convT" and not last and C.igemm_plan(0, d, p["ws"] is not None)[10] == 1):
                    self._run_group([lambda job, l=l, d=d, h=h: C.igemm(0, h, self._w(l), d, self._b(l), l.relu,
                                                                        self.acts[l.name], None, job=job),
                                     lambda job: self._wtrans_layers(1, len(self.spec), job)])
                    h = self.acts[l.name]
                    continue
                self._wtrans_layers(1, len(self.spec))
            if last and self._thin_last:  # last layer + BCE + dlogits + bias-grad partials, one launch
                C.thin_tconv(h, self._wf32(l), self._desc(l, M), self._b(l), X=self.xb,
                             dlog16=self.dlog16 if train else None, recon=self.recon if want_recon else None,
                             part=self.bce_part, gpart=p["gpart"] if train else None)
                return
            self._layer_fwd(l, h, M, None if last else self.acts[l.name], self.logits if last else None, p["ws"])
            h = self.acts[l.name]
        C.bce_logits(self.logits, self.xb, None, M, self.D, self.dlog16 if train else None,
                     self.recon if want_recon else None, self.bce_part, p["gpart"] if train else None)

    def _run_group(self, fns):
        """Run independent launches ``fns`` (each ``f(job)``): recorded as jobs
        and issued as ONE fused kernel when conv_jobs.hip has an instantiation
        for their kinds, else each op's own kernel (same bodies, same results)."""
        if self.fuse_jobs and 1 < len(fns) <= 3:
            jobs = [self.C.Job() for _ in fns]
            for f, j in zip(fns, jobs):
                f(j)
            if all(j.kind > 0 for j in jobs) and self.C.launch_jobs(jobs):
                self._fused_launches += 1
                return
            if os.getenv("MDT_JOBS_DEBUG"):
                print(f"[jobs] not fused: kinds={sorted(j.kind for j in jobs)} post={[j.has_post for j in jobs]}",
                      file=sys.stderr, flush=True)
        for f in fns:
            f(None)

    def _backward_hip(self, M, with_loss=False, optimizer=False):
        """Reverse sweep: per layer one weight-gradient GEMM (partial slabs) and
        one backward-data GEMM whose epilogue applies the previous layer's ReLU
        mask and emits its bias-gradient column sums. The two (plus any bias
        column sum or loss reduction that became ready) are independent and
        share one launch (``_run_group``). ``with_loss`` adds the loss reduction
        of the forward to the first launch; ``optimizer`` (no reducer) appends
        the optimizer tail: first-layer weight gradient || finalize+Adam of the
        other layers, then first-layer finalize || transposed weight copies."""
        C = self.C
        p = self._plan(M)
        spec = self.spec
        st = self.state
        g = self.dlog16
        red = self.reducer
        # fused xGMI all-reduce (comm_jobs.h): a backward launch with a free job
        # slot also pushes the layers the previous launches completed
        # (``pending``); the tail pushes the rest, reduces and applies Adam
        fused = red is not None and self.fuse_jobs and bool(self._comm_ctx())
        pend_lo = pend_hi = len(spec)  # layers [pend_lo, pend_hi) complete, not yet pushed
        if fused:
            red = None
        if red is not None:
            bounds = list(red.bounds())
            starts = {b: i for i, (l, b, e) in enumerate(self.layer_ranges())}
            assert all(b in starts or b == self.numel for b in bounds), "bucket bounds must fall on layer starts"
        carry = []  # launches that depend on the previous group's outputs
        # spread mode: layers [fin_hi, L) already finalized (+Adam) as the third
        # job of a backward launch -- layer j's gradients are complete once the
        # launch of layer j ran, and nothing later in the step reads its weights
        spread = (optimizer and self.spread_fin and self.fuse_jobs and self.reducer is None)
        fin_hi = len(spec)
        if with_loss:
            carry.append(lambda job: C.loss_finalize2(self.bce_part, self._n_bce(M), self.kld_part,
                                                      self._n_kld(M), st.train_state, st.hparams, True,
                                                      job=job))
        for i in range(len(spec) - 1, -1, -1):
            if red is not None and i + 1 < len(spec):
                self._maybe_launch_bucket(red, bounds, starts, i + 1, M)
            l = spec[i]
            prev = spec[i - 1] if i > 0 else None
            d = self._desc(l, M)
            if i == 0:
                a_in = self.xb
            elif l.name == "dec_fc":
                a_in = self.z16
            else:
                a_in = self.acts[prev.name]
            wslab = p["slabs"].get(l.name + ".weight")
            wout = wslab[0] if wslab is not None else self._gw(l)
            fns, carry, after = carry, [], []
            if l.kind == "convT":  # conv view: output = convT input, input = convT output
                fns.append(lambda job, a_in=a_in, g=g, d=d, wout=wout: C.wgrad(a_in, g, d, wout, job=job))
            else:
                fns.append(lambda job, a_in=a_in, g=g, d=d, wout=wout: C.wgrad(g, a_in, d, wout, job=job))
            gin = None
            if prev is not None:
                omask = a_in if prev.relu else None
                if l.name == "dec_fc":
                    ks = C.igemm_plan(1, d, True)[10]
                    fns.append(lambda job, g=g, l=l, d=d, ks=ks: C.igemm(1, g, self._wt(l), d, None, False, None,
                                                                         self.dz, ws=p["ws"], job=job,
                                                                         combine=ks == 1))
                    if ks > 1:  # split-K combine fused with the reparameterisation backward
                        after.append(lambda ks=ks: C.combine_reparam_bwd(p["ws"], ks, self.mulv, self.eps, self.dmulv,
                                                                         self.dmulv16, self.dz, M, self.Z,
                                                                         st.hparams))
                    else:
                        after.append(lambda: C.reparam_bwd(self.dz, self.mulv, self.eps, self.dmulv, self.dmulv16,
                                                           M, self.Z, st.hparams))
                    cso = p["colsum"][prev.name]
                    carry.append(lambda job, cso=cso: C.colsum(self.dmulv16, M, 2 * self.Z, p["rows_per"], cso,
                                                               job=job))
                    gin = self.dmulv16
                elif i == len(spec) - 1 and self._thin_last:
                    gin = self.gacts[prev.name]
                    cso = p["colsum"][prev.name]
                    fns.append(lambda job, g=g, l=l, d=d, gin=gin, omask=omask, cso=cso:
                               C.thin_conv(g, self._wf32(l), d, None, False, gin, omask, cso, job=job))
                else:
                    gin = self.gacts[prev.name]
                    cs = None if prev.name == "dec_fc" else p["colsum"].get(prev.name)
                    mode = 0 if l.kind == "convT" else 1
                    w = self._w(l) if l.kind == "convT" else self._wt(l)
                    fns.append(lambda job, g=g, w=w, d=d, gin=gin, omask=omask, cs=cs, mode=mode:
                               C.igemm(mode, g, w, d, None, False, gin, None, omask, cs, job=job))
                    if prev.name == "dec_fc":
                        cso = p["colsum"][prev.name]
                        carry.append(lambda job, gin=gin, n=prev.cout, cso=cso:
                                     C.colsum(gin, M, n, p["rows_per"], cso, job=job))
            if prev is None and optimizer:
                L = len(spec)
                if fin_hi > 1:
                    fns.append(lambda job, hi=fin_hi: self._finalize_layers(M, 1, hi, job))
                self._run_group(fns)
                if self._wt_deferred():
                    self._finalize_layers(M, 0, 1)
                else:
                    self._run_group([lambda job: self._finalize_layers(M, 0, 1, job),
                                     lambda job: self._wtrans_layers(1, L, job)])
                break
            if spread and len(fns) == 2 and i + 1 < fin_hi and self._run_with_finalize(fns, M, i + 1, fin_hi):
                fin_hi = i + 1
            elif fused and len(fns) in (1, 2) and pend_lo < pend_hi and \
                    self._run_with_comm(fns, M, pend_lo, pend_hi):
                pend_hi = pend_lo
            else:
                self._run_group(fns)
            for f in after:
                f()
            if fused:
                pend_lo = i  # layer i's gradients are complete now
            if prev is None:
                assert not carry
                if red is not None:
                    self._maybe_launch_bucket(red, bounds, starts, 0, M)
                if fused:
                    self._comm_tail(M, pend_lo, pend_hi)
                break
            g = gin

    def _run_with_finalize(self, fns, M, lo, hi):
        """Launch the two jobs ``fns`` plus finalize+Adam of layers [lo, hi) as
        ONE kernel; False (nothing launched) when that combination has no
        instantiation."""
        if not self.fuse_jobs:
            return False
        jobs = [self.C.Job() for _ in range(3)]
        for f, j in zip(fns, jobs):
            f(j)
        self._finalize_layers(M, lo, hi, jobs[2])
        if all(j.kind > 0 for j in jobs) and self.C.launch_jobs(jobs):
            self._fused_launches += 1
            return True
        if os.getenv("MDT_JOBS_DEBUG"):
            print(f"[jobs] no finalize fusion: kinds={sorted(j.kind for j in jobs)}", file=sys.stderr, flush=True)
        return False

    def _run_with_comm(self, fns, M, lo, hi):
        """Launch the jobs ``fns`` plus the push (comm_jobs.h, mode 1) of layers
        [lo, hi) as ONE kernel; False (nothing launched) when that combination
        has no instantiation."""
        jobs = [self.C.Job() for _ in range(len(fns) + 1)]
        for f, j in zip(fns, jobs):
            f(j)
        p = self._plan(M)
        lu = p["layer_units"]
        self._comm_job(p["segs"], p["units"], lu[lo], lu[hi], 1, True, job=jobs[-1])
        if all(j.kind > 0 for j in jobs) and self.C.launch_jobs(jobs):
            self._fused_launches += 1
            return True
        if os.getenv("MDT_JOBS_DEBUG"):
            print(f"[jobs] no comm fusion: kinds={sorted(j.kind for j in jobs)}", file=sys.stderr, flush=True)
        return False

    def _comm_tail(self, M, lo, hi):
        """After the first layer's backward launch: push+reduce+Adam of the
        layers not pushed yet ([lo, hi), the first layer included) || reduce+Adam
        of the ones pushed by the backward launches ([hi, L)), one launch."""
        p, L = self._plan(M), len(self.spec)
        lu = p["layer_units"]
        jobs = [self._comm_job(p["segs"], p["units"], lu[lo], lu[hi], 3, True)]
        if hi < L:
            jobs.append(self._comm_job(p["segs"], p["units"], lu[hi], lu[L], 2, True))
        if len(jobs) == 2:
            ok = self.C.launch_jobs(jobs)
            assert ok, "jobs_k<JComm, JComm> missing from conv_jobs.hip"
        else:
            pack, grid = self._comm_single_pack(("tail", M, lo, hi), jobs[0])
            self.C.launch_jobs_multi(pack, grid)

    def _comm_single_pack(self, key, job):
        """Device job table of a single comm job (cached by ``key``: replayed
        graphs keep reading it)."""
        if key not in self._comm_packs:
            pack, grid = self.C.pack_jobs_multi([job])
            self._comm_packs[key] = (pack.to(self.device), grid)
        return self._comm_packs[key]

    def _wt_deferred(self):
        """The transposed weight copies (w16t) of a step's update are written by
        the next step's first launch or the first decoder launch (MDT_CONV_DEFER_WT)."""
        return self.defer_wt and self.fuse_jobs and self._thin_first and self.reducer is None and len(self.spec) > 1

    def _finalize_layers(self, M, lo, hi, job=None):
        """Finalize + Adam + bf16 cast of layers [lo, hi) (their units of the plan)."""
        p, st = self._plan(M), self.state
        u0, u1 = p["layer_units"][lo], p["layer_units"][hi]
        self.C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"],
                             p["units"].narrow(0, u0 * 12, (u1 - u0) * 12), u1 - u0, st.train_state, st.hparams,
                             True, job=job)

    def _wtrans_layers(self, lo, hi, job=None):
        """Parity-ordered transposed copies of layers [lo, hi) (the first layer's
        copy is never read: it has no backward-data GEMM)."""
        t0, t1 = self._tr_layer[lo], self._tr_layer[hi]
        self.C.wtrans(self.w16, self.w16t, self.segs, self.tr_units.narrow(0, t0 * 16, (t1 - t0) * 16), t1 - t0,
                      job=job)

    def _maybe_launch_bucket(self, red, bounds, starts, i, M):
        """Layer i's gradients just became final (all layers >= i are done): if
        i starts a bucket, reduce that bucket's partial slabs into the arena and
        launch its all-reduce (it overlaps the rest of the backward)."""
        _, b, _ = self.layer_ranges()[i]
        if b not in bounds[:-1]:
            return
        k = bounds.index(b)
        end = bounds[k + 1]
        last = next((j for j, (l, bb, e) in enumerate(self.layer_ranges()) if bb >= end), len(self.spec))
        p, st = self._plan(M), self.state
        u0, u1 = p["layer_units"][i], p["layer_units"][last]
        units = p["units"].narrow(0, u0 * 12, (u1 - u0) * 12)
        self.C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"], units,
                             u1 - u0, st.train_state, st.hparams, False)
        red.launch(k)

    def _step_hip(self, M):
        if self.f28:
            self._step28(M)
            return
        C = self.C
        X, idx = self._data[0], self._data[1]
        st = self.state
        self._forward_hip(M, st.train_state, self.rng_stream, src=(X, idx))
        if self.reducer is None:
            # backward + optimizer tail (finalize/Adam/bf16 cast/transposes) in fused launches
            self._backward_hip(M, with_loss=True, optimizer=True)
            return
        # intra-group DDP: the backward finalizes + launches each gradient bucket
        # as it completes (loss reduction in its first launch); Adam after the
        # all-reduces. Fused xGMI reducer: pushes ride in the backward launches,
        # the tail reduces + applies Adam (no stream-side collectives to wait for)
        self._backward_hip(M, with_loss=True)
        if self.fuse_jobs and self._comm_ctx():
            self._wtrans_layers(1, len(self.spec))  # the first layer's copy is never read
            return
        self.reducer.wait_all()
        C.adam_cast(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, self.segs, self.nseg,
                    st.train_state, st.hparams, True)
        self._transpose_weights()

    # ----------------------------------------------------------- fused 28x28
    def _plan28(self, M):
        """Pointer tables, weight-gradient jobs and finalize units of the fused
        28x28 step for a batch of M (built once per M and data binding; the
        tensors never move, so captured graphs stay valid)."""
        p = self._plans28.get(M)
        if p is not None:
            return p
        C, dev, B = self.C, self.device, self.B
        f32 = dict(dtype=torch.float32, device=dev)
        L = {l.name: l for l in self.spec}
        X, idx = self._data[0], self._data[1]
        st = self.state
        w = self._f28_weights()
        part = self.f28_part
        bce, kld, db4 = part.narrow(0, 0, B), part.narrow(0, B, B), part.narrow(0, 2 * B, B)
        bias = self.f28_bias
        dbd = bias.narrow(0, 0, B * 3136)
        db3 = bias.narrow(0, B * 3136, B * 32)
        db2 = bias.narrow(0, B * 3168, 2 * B * 64)  # [2][M][64] for a batch of M
        db1 = bias.narrow(0, B * 3296, B * 32)
        a1, a2, d0, d1 = self.acts["enc1"], self.acts["enc2"], self.acts["dec_fc"], self.acts["dec1"]
        gd1, gd0, ga2, ga1 = self.gacts["dec1"], self.gacts["dec_fc"], self.gacts["enc2"], self.gacts["enc1"]
        fwd = w + [X, idx, st.train_state, st.hparams, self.xb, a1, a2, self.mulv, self.eps, self.z16, d0, d1,
                   self.dlog32, None, bce, kld, db4, self.f28_stamps[0], self.f28_xn, self.f28_xtag]
        bwd = w + [st.hparams, self.mulv, self.eps, a1, a2, d0, d1, self.dlog32, gd1, gd0, dbd, self.dmulv,
                   self.dmulv16, ga2, ga1, db3, db2, db1, self.f28_stamps[1]]
        # weight gradients: (G, X) per layer in the conv view (see _backward_hip)
        srcs = {"enc1": (ga1, self.xb), "enc2": (ga2, a1), "enc_head": (self.dmulv16, a2),
                "dec_fc": (gd0, self.z16), "dec1": (d0, gd1), "dec2": (d1, self.dlog32)}
        slabs, jobs = {}, []
        for name, (G, Xw) in srcs.items():
            l = L[name]
            d = self._desc(l, M)
            ns = C.wgrad_plan(d)[6]
            t = torch.empty(ns * math.prod(_w_shape(l)), **f32)
            slabs[name + ".weight"] = (t, ns)
            j = C.Job()
            C.wgrad(G, Xw, d, t, job=j)
            jobs.append(j)
        j = C.Job()
        C.loss_finalize2(bce, M, kld, M, st.train_state, st.hparams, True, job=j, advance_step=True)
        jobs.append(j)
        # bias gradients: per-sample partial rows written by the fused kernels
        for name, t, rows in (("enc1", db1, M), ("enc2", db2, 2 * M), ("enc_head", self.dmulv, M),
                              ("dec_fc", dbd, M), ("dec1", db3, M), ("dec2", db4, M)):
            slabs[name + ".bias"] = (t, rows)
        segs = self._seg_rows(slabs)
        units, layer_units = self._finalize_units(segs)
        pack, grid = C.pack_jobs_multi(jobs)
        # intra-group DDP: the decoder's weight gradients (ready first in the
        # reference's backward order) get a launch of their own, so their
        # bucket's all-reduce runs while the encoder's are still computed
        names = list(srcs)
        dec_pack, dec_grid = C.pack_jobs_multi([jobs[i] for i, n in enumerate(names) if n.startswith("dec")] +
                                               [jobs[len(names)]])
        enc_pack, enc_grid = C.pack_jobs_multi([jobs[i] for i, n in enumerate(names) if not n.startswith("dec")])
        first_dec = next(i for i, l in enumerate(self.spec) if l.name.startswith("dec"))
        p = dict(fwd=fwd, bwd=bwd, jobs=jobs, jobs_pack=pack.to(dev), jobs_grid=grid, slabs=slabs,
                 segs=C.make_grad_segs(segs, dev.index or 0), units=C.make_grad_units(units, dev.index or 0),
                 nunits=len(units), layer_units=layer_units, first_dec=first_dec,
                 dec_pack=dec_pack.to(dev), dec_grid=dec_grid, enc_pack=enc_pack.to(dev), enc_grid=enc_grid)
        p["names"] = names
        self._plans28[M] = p
        return p

    # finalize jobs of the merged launch, ordered by when their layer's weight
    # gradient completes (profiles/r6_jobs28: dec_fc 5.4, enc_head 5.8, enc1
    # 7.2, enc2 8.5, dec2 8.8, dec1 9.1 us into the launch)
    _FIN_ORDER28 = ("dec_fc", "enc_head", "enc1", "enc2", "dec2", "dec1")

    def _merged_pack28(self, p):
        """One jobs_multi_k table for the whole optimizer tail of the fused
        28x28 step: the six weight gradients and the loss/step job, then the
        next-batch gather (waits for the loss job: it needs the advanced
        cursor), then one finalize+Adam job per layer (waits for that layer's
        weight gradient and for the loss job's advanced step). Each waiting
        workgroup is released by in-launch counters (conv_jobs.hip JobPackN),
        so a layer's update runs while later layers' gradients are still being
        computed and the step loses a launch boundary. Bitwise the two-launch
        form: the same bodies, the same per-element summation order."""
        adam = not self.f28_skip_adam
        key = ("merged", adam, bool(self.f28_prefetch))
        hit = p.get(key)
        if hit is not None:
            return hit
        C, st, names = self.C, self.state, p["names"]
        jobs = list(p["jobs"])  # names order + loss/step
        loss_i = len(names)
        wait = [0] * len(jobs)
        if self.f28_prefetch:
            j = C.Job()
            C.gather_job(self._data[0], self._data[1], st.train_state, self.f28_xn, self.f28_xtag, self.B, j)
            jobs.append(j)
            wait.append(1 << loss_i)
        lu = p["layer_units"]
        for name in self._FIN_ORDER28:
            i = next(k for k, l in enumerate(self.spec) if l.name == name)
            u0, u1 = lu[i], lu[i + 1]
            j = C.Job()
            C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"],
                            p["units"].narrow(0, u0 * 12, (u1 - u0) * 12), u1 - u0, st.train_state, st.hparams,
                            adam, job=j, dep=True)
            jobs.append(j)
            wait.append((1 << names.index(name)) | (1 << loss_i))
        pack, grid = C.pack_jobs_multi(jobs, wait=wait, dep_ctr=self.f28_dep)
        hit = p[key] = (pack.to(self.device), grid, jobs, wait)
        return hit

    def _step28(self, M):
        """Fused 28x28 step: forward + backward-data (one launch: f28_step_k,
        or two with MDT_F28_MERGE=0) || weight gradients + loss/step ||
        finalize + Adam (DDP: finalize without Adam, bucket all-reduce, then
        Adam + bf16 cast)."""
        C, p, st = self.C, self._plan28(M), self.state
        if self.f28_merge:
            C.f28_step(p["fwd"], p["bwd"], self.B, M, self.rng_stream,
                       pair=[self.f28_xg, self.f28_pairw, self.f28_err] if self.f28_pair else [],
                       pair_delay_us=self.f28_pair_delay_us)
        else:
            C.f28_forward(p["fwd"], self.B, M, self.rng_stream, True)
            C.f28_backward(p["bwd"], M)
        red = self.reducer
        if red is None:
            if self.f28_fin_merge:
                pack, grid, _, _ = self._merged_pack28(p)
                C.launch_jobs_multi(pack, grid, dep=True)
                return
            C.launch_jobs_multi(p["jobs_pack"], p["jobs_grid"])
            C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"], p["units"],
                            p["nunits"], st.train_state, st.hparams, not self.f28_skip_adam,
                            gather=([self._data[0], self._data[1], self.f28_xn, self.f28_xtag]
                                    if self.f28_prefetch else []), gather_B=self.B)
            return
        if self._comm_ctx():
            # fused xGMI all-reduce (comm_jobs.h), one stream: decoder weight
            # gradients | encoder weight gradients || decoder push (its bytes
            # cross the links while the encoder's are computed) | encoder
            # push+reduce || decoder reduce, both with Adam + bf16 cast.
            # MDT_DDP_OVERLAP=0: all weight gradients | push+reduce+Adam.
            packs = self._comm_packs28(M, p)
            for i, (pack, grid) in enumerate(packs):
                C.launch_jobs_multi(pack, grid)
                if self.comm_phase_hook is not None and i == len(packs) - 2:
                    self.comm_phase_hook()
            return
        # DDP (reference: the Reducer's bucket all-reduces launched from the
        # autograd hooks while backward continues, /root/reference/vae-hpo.py:72,
        # :130): decoder weight gradients -> their finalize -> every bucket
        # that holds only decoder parameters goes out on the comm stream ->
        # encoder weight gradients (overlapping those all-reduces) -> their
        # finalize -> the remaining buckets -> wait -> Adam + bf16 cast.
        lu, fd, L = p["layer_units"], p["first_dec"], len(self.spec)
        dec0 = self.layer_ranges()[fd][1]
        bounds = list(red.bounds())
        nbk = len(bounds) - 1
        early = self._overlap28(fused=False)
        if hasattr(red, "set_inline"):
            red.set_inline(not early)
        if not early:
            # one stream: all weight gradients | finalize | the bucket
            # collectives in issue order on the compute stream (no events) | Adam
            C.launch_jobs_multi(p["jobs_pack"], p["jobs_grid"])
            self._finalize_unit_range(p, lu[0], lu[L])
            for k in reversed(range(nbk)):
                red.launch(k)
            red.wait_all()
            if not self.f28_skip_adam:
                C.adam_cast(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, self.segs, self.nseg,
                            st.train_state, st.hparams, True)
            return
        C.launch_jobs_multi(p["dec_pack"], p["dec_grid"])
        self._finalize_unit_range(p, lu[fd], lu[L])
        for k in reversed(range(nbk)):
            if bounds[k] >= dec0:
                red.launch(k)
        C.launch_jobs_multi(p["enc_pack"], p["enc_grid"])
        self._finalize_unit_range(p, lu[0], lu[fd])
        for k in reversed(range(nbk)):
            if bounds[k] < dec0:
                red.launch(k)
        red.wait_all()
        if not self.f28_skip_adam:
            C.adam_cast(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, self.segs, self.nseg,
                        st.train_state, st.hparams, True)

    def _comm_packs28(self, M, p):
        """Job tables of the fused-reducer 28x28 step after the f28_step_k
        launch: [(device pack, grid)], built once per (M, Adam, overlap)."""
        adam = not self.f28_skip_adam
        overlap = self._overlap28(fused=True) and not self.comm_split_tail
        key = (M, adam, overlap, self.comm_split_tail)
        packs = self._comm_packs.get(key)
        if packs is not None:
            return packs
        C, dev = self.C, self.device
        lu, fd, L = p["layer_units"], p["first_dec"], len(self.spec)
        segs, units = p["segs"], p["units"]
        jobs = p["jobs"]  # six weight-gradient jobs (enc1, enc2, enc_head, dec_fc, dec1, dec2) + loss/step
        names = ["enc1", "enc2", "enc_head", "dec_fc", "dec1", "dec2"]
        enc = [jobs[i] for i, n in enumerate(names) if not n.startswith("dec")]
        dec = [jobs[i] for i, n in enumerate(names) if n.startswith("dec")] + [jobs[len(names)]]
        if self.comm_split_tail:
            tables = [jobs, [self._comm_job(segs, units, lu[0], lu[L], 1, adam)],
                      [self._comm_job(segs, units, lu[0], lu[L], 2, adam)]]
        elif overlap:
            tables = [dec,
                      enc + [self._comm_job(segs, units, lu[fd], lu[L], 1, adam)],
                      [self._comm_job(segs, units, lu[0], lu[fd], 3, adam),
                       self._comm_job(segs, units, lu[fd], lu[L], 2, adam)]]
        else:
            tables = [jobs, [self._comm_job(segs, units, lu[0], lu[L], 3, adam)]]
        self._comm_tables[key] = tables
        packs = []
        for i, t in enumerate(tables):
            st = self.comm_stamps[i] if self.comm_stamps is not None and i < len(self.comm_stamps) else None
            pack, grid = C.pack_jobs_multi(t, stamps=st)
            packs.append((pack.to(dev), grid))
        self._comm_packs[key] = packs
        return packs

    def _overlap28(self, fused: bool) -> bool:
        """Resolve MDT_DDP_OVERLAP (``ddp_overlap``; None = auto) for the fused
        28x28 DDP step: the split costs ~6 us with the fused xGMI jobs and
        ~31 us with RCCL on its own stream (profiles/r4_ddp_fused)."""
        if self.ddp_overlap is not None:
            return bool(self.ddp_overlap)
        from ..parallel.ddp import overlap_pays

        dec0 = next(b for l, b, e in self.layer_ranges() if l.name.startswith("dec"))
        return overlap_pays(4 * (self.numel - dec0), 6.0 if fused else 31.0)

    def _finalize_unit_range(self, p, u0, u1):
        """Slab reduction into the gradient arena (no Adam) of finalize units [u0, u1)."""
        if u1 > u0:
            st = self.state
            self.C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"],
                                 p["units"].narrow(0, u0 * 12, (u1 - u0) * 12), u1 - u0, st.train_state,
                                 st.hparams, False)

    def _finalize_grads(self, M, do_adam):
        """Reduce the partial slabs into the gradient arena (deterministic order);
        with ``do_adam`` also apply Adam and re-emit the bf16 weight copies."""
        p, st = self._plan(M), self.state
        self.C.grad_finalize(self.params, self.grads, self.exp_avg, self.exp_avg_sq, self.w16, p["segs"], p["units"],
                             p["nunits"], st.train_state, st.hparams, do_adam)

    # ----------------------------------------------------------- torch path
    def _step_torch(self, M):
        X, idx = self._data[0], self._data[1]
        st = self._st
        rows = idx[st["cursor"] * self.B: st["cursor"] * self.B + M].long()
        x = X[rows]
        eps = torch.from_numpy(reparam_eps(M, self.Z, self.seed, self.rng_stream, st["step"])).to(self.device)
        self.model.zero_grad(set_to_none=True)
        loss, *_ = self.model.loss(x, eps, self.hp["kl_beta"])
        loss.backward()
        with torch.no_grad():
            gv = self.named_grads()
            for k, v in self.model.grads_to_arena().items():
                gv[k].copy_(v)
            if self.reducer is not None:
                self.reducer.launch_all()
                self.reducer.wait_all()
            h = self.hp
            reference_adam_(self.params, self.grads, self.exp_avg, self.exp_avg_sq, st["step"] + 1, h["lr"],
                            h["beta1"], h["beta2"], h["eps"], h["weight_decay"], h["grad_scale"], self.decoupled_wd)
            self.model.from_arena(self.named_parameters())
        lv = float(loss.detach())
        self._hist[st["step"] % 4096] = lv
        st["epoch_loss"] += lv
        st["epoch_count"] += 1
        st["step"] += 1
        st["cursor"] += 1
        if st["nbatches"] and st["cursor"] >= st["nbatches"]:
            st["cursor"] = 0

    # ----------------------------------------------------------- driver API
    def train_steps(self, n, M=None):
        M = self.B if M is None else M
        if n <= 0:
            return
        if self.backend == "torch":
            for _ in range(n):
                self._step_torch(M)
            return
        if not self.use_graphs:
            for _ in range(n):
                self._step_hip(M)
        else:
            S = self.graph_steps
            while n >= S:
                self._replay(S, M)
                n -= S
            for _ in range(n):
                self._replay(1, M)
        if self._wt_deferred() or self.f28:
            # the last step's transposed weight copies (deferred to the next
            # step's first launch, or never needed by the fused 28x28 step) are
            # stale now: eval / decode write them first (_ensure_wt)
            self._wt_stale = True

    _wt_stale = False

    def _ensure_wt(self):
        """Write the transposed weight copies (w16t) if training left them
        stale. Only eval / decode read them outside a training step: a step of
        the layer path writes its own in its first launch, and the fused 28x28
        step never reads them."""
        if self._wt_stale:
            self._wtrans_layers(1, len(self.spec))
            self._wt_stale = False

    def prepare(self, batch_sizes, eval_rows=None):
        """Set-up work done once before timing starts: capture the step graphs
        for the batch sizes an epoch uses and run the eval / decode kernels
        once (code-object load). Training state is left unchanged."""
        if self.backend != "hip":
            return
        if self.use_graphs and self._data is not None:
            for M in sorted({int(m) for m in batch_sizes if m and m > 0}):
                for S in {self.graph_steps, 1}:
                    if (S, M) not in self._graphs:
                        self._graphs[(S, M)] = self._capture(S, M)
        if eval_rows is not None and eval_rows.numel():
            st = self.read_state(eval=True)
            n = eval_rows.shape[0]
            self.evaluate(eval_rows, torch.arange(n, device=eval_rows.device, dtype=torch.int32))
            self.decode(torch.zeros(1, self.Z, device=self.device))
            self.set_cursor(st["cursor"], st["nbatches"], eval=True)
            self.reset_loss(eval=True)
        torch.cuda.synchronize(self.device)

    # strict_graphs: a replay that finds no captured graph raises instead of
    # capturing lazily (bench.py / autotune set it after ``prepare`` so no
    # capture ever lands inside a timed region)
    strict_graphs = False

    def _replay(self, S, M):
        g = self._graphs.get((S, M))
        if g is None:
            if self.strict_graphs:
                raise RuntimeError(f"no captured step graph for (steps={S}, M={M}); call prepare() first")
            g = self._capture(S, M)
            self._graphs[(S, M)] = g
        g.replay()

    def _capture(self, S, M):
        red = self.reducer
        k0 = self.step_count if red is not None and hasattr(red, "rebase_epochs") else None
        snap = [t.clone() for t in (self.params, self.exp_avg, self.exp_avg_sq, self.state.train_state)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._step_hip(M)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(S):
                self._step_hip(M)
        for t, v in zip((self.params, self.exp_avg, self.exp_avg_sq, self.state.train_state), snap):
            t.copy_(v)
        if k0 is not None:
            # the warm-up step ran the fused all-reduce jobs at epoch k0 + 1 and
            # published flags for it; the step counter now goes back to k0, so
            # the next real step must not reuse that epoch (every member
            # captures at the same points: the rebase is the same everywhere)
            red.rebase_epochs(k0 + 1, k0)
        self._cast_weights()
        native.upload_graph(g)
        return g

    @torch.no_grad()
    # graph-replayed eval passes (models/eval_graphs.py)
    def _eval_batch(self, M, X, idx, want_recon):
        st = self.state
        if self.f28:
            # the fused 28x28 forward in eval mode (f28_fwd_k, one workgroup
            # per sample, no activation stores): one launch instead of the
            # layer path's dozen; its loss job advances the eval step exactly
            # like the layer path's step_begin (same Philox keys, same ring slot)
            bce, kld = self.f28_part.narrow(0, 0, self.B), self.f28_part.narrow(0, self.B, self.B)
            # paired (two workgroups per sample, 2M CUs) unless MDT_F28_EVAL_PAIR=0
            pair = [self.f28_xg, self.f28_pairw, self.f28_err] if self.f28_pair and self._eval_pair else []
            self.C.f28_forward(self._eval_fwd28(X, idx, want_recon), self.B, M, EVAL_STREAM + self.rng_stream,
                               False, pair=pair)
            self.C.loss_finalize2(bce, M, kld, M, st.eval_state, st.hparams, True, advance_step=True)
            return
        self._forward_hip(M, st.eval_state, EVAL_STREAM + self.rng_stream, want_recon=want_recon, train=False,
                          src=(X, idx))
        self.C.loss_finalize2(self.bce_part, self._n_bce(M), self.kld_part, self._n_kld(M), st.eval_state,
                              st.hparams, True)

    def _f28_weights(self):
        L = {l.name: l for l in self.spec}
        return [self._wf32(L["enc1"]), self._b(L["enc1"]), self._w(L["enc2"]), self._b(L["enc2"]),
                self._w(L["enc_head"]), self._b(L["enc_head"]), self._w(L["dec_fc"]), self._b(L["dec_fc"]),
                self._w(L["dec1"]), self._b(L["dec1"]), self._wf32(L["dec2"]), self._b(L["dec2"])]

    def _eval_fwd28(self, X, idx, want_recon):
        """Pointer table of the fused forward over an eval set: the eval state,
        no activation outputs (train = 0), the reconstruction when wanted."""
        st = self.state
        part = self.f28_part
        bce, kld, db4 = part.narrow(0, 0, self.B), part.narrow(0, self.B, self.B), part.narrow(0, 2 * self.B, self.B)
        return self._f28_weights() + [X, idx, st.eval_state, st.hparams, self.xb, None, None, self.mulv, self.eps,
                                      self.z16, None, None, None, self.recon if want_recon else None, bce, kld, db4,
                                      None]

    def _eval_state(self):
        return self.state.eval_state

    def _eval_recon(self, M):
        return self.recon[: M * self.D].view(M, self.D).clone()

    def evaluate(self, X, idx, want_first_recon=True):
        self._ensure_wt()
        idx = idx.to(device=self.device, dtype=torch.int32).contiguous()
        n = idx.numel()
        nb = -(-n // self.B)
        pad = nb * self.B - n
        if pad:
            idx = torch.cat([idx, idx[:1].expand(pad)])
        if self.backend == "hip" and self.use_graphs:
            first = self._eval_graphed(X.contiguous(), idx, n, want_first_recon)
            return self.read_state(eval=True)["epoch_loss"], first
        self.set_cursor(0, nb, eval=True)
        self.reset_loss(eval=True)
        first = None
        for b in range(nb):
            M = min(self.B, n - b * self.B)
            if self.backend == "hip":
                want = want_first_recon and b == 0
                self._eval_batch(M, X.contiguous(), idx, want)
                if want:
                    first = self._eval_recon(M)
            else:
                st = self._st_eval
                rows = idx[b * self.B: b * self.B + M].long()
                x = X[rows]
                eps = torch.from_numpy(reparam_eps(M, self.Z, self.seed, EVAL_STREAM + self.rng_stream,
                                                   st["step"])).to(self.device)
                loss, t, _, _ = self.model.loss(x, eps, self.hp["kl_beta"])
                if want_first_recon and b == 0:
                    first = torch.sigmoid(t).permute(0, 2, 3, 1).reshape(M, self.D).clone()
                lv = float(loss.detach())
                self._hist_eval[st["step"] % 4096] = lv
                st["epoch_loss"] += lv
                st["epoch_count"] += 1
                st["step"] += 1
        return self.read_state(eval=True)["epoch_loss"], first

    @torch.no_grad()
    def decode(self, zz):
        zz = zz.to(self.device, torch.float32)
        if self.backend == "torch":
            t = self.model.decode_logits(zz)
            return torch.sigmoid(t).permute(0, 2, 3, 1).reshape(zz.shape[0], self.D)
        self._ensure_wt()
        outs = []
        dec = [l for l in self.spec if l.name.startswith("dec")]
        for i in range(0, zz.shape[0], self.B):
            zc = zz[i:i + self.B]
            M = zc.shape[0]
            self.z16[:M].copy_(zc.to(torch.bfloat16))
            h = self.z16
            for l in dec:
                last = l is dec[-1]
                self._layer_fwd(l, h, M, None if last else self.acts[l.name], self.logits if last else None,
                                self._plan(M)["ws"])
                h = self.acts[l.name]
            outs.append(torch.sigmoid(self.logits[: M * self.D].view(M, self.D)).clone())
        return torch.cat(outs)

    def flops_per_sample(self):
        f = 0
        for l in self.spec:
            f += 2 * l.out_hw * l.out_hw * l.cout * l.k * l.k * l.cin if l.kind != "convT" else \
                2 * l.in_hw * l.in_hw * l.cin * l.k * l.k * l.cout
        return 3 * f
