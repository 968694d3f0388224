"""One HPO trial's MLP-VAE training state and step, on the fused HIP path or
the torch reference path.

Replaces the reference's per-step chain (DataLoader collate -> H2D copy ->
DDP forward -> loss -> autograd backward -> DDP bucket all-reduce ->
``loss.item()`` sync -> foreach Adam; /root/reference/vae-hpo.py:67-74) with:

* ``backend="hip"``: ``_C.MlpVaeEngine`` — seven fused CDNA4 launches per step
  (csrc/kernels/vae_mlp.hip, adam.hip) reading the batch rows straight out of
  a device-resident dataset through the epoch's sampler index list, gradient
  buckets all-reduced by the native ``BucketReducer`` while later backward
  kernels run, and the whole step (optionally S steps) captured in one
  hipGraph and replayed; the loss stays on the device (ring buffer) and is
  read at log points only.
* ``backend="torch"``: the same math in torch ops (``reference_step``), used on
  CPU hosts and as the fp32 oracle for the kernel tests.

Both backends share the flat-arena layout, the Philox noise stream and Adam
arithmetic, so a run is reproducible across them up to fp32 rounding.
"""

from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import native
from ..ops.philox import reparam_eps
from .eval_graphs import GraphedEval
from .mlp_vae import arena_layout, init_params_, reference_adam_, reference_forward, reference_step, views

__all__ = ["MlpVaeTrainer"]

EVAL_STREAM = 1 << 30
LOSS_HIST = 4096


class MlpVaeTrainer(GraphedEval):
    def __init__(self, batch_size: int = 128, D: int = 784, H: int = 400, Z: int = 20,
                 device=None, backend: Optional[str] = None, seed: int = 0, init_seed: Optional[int] = None,
                 lr: float = 1e-3, kl_beta: float = 1.0, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, decoupled_wd: bool = False, rng_stream: int = 0,
                 use_graphs: bool = True, graph_steps: int = 10):
        self.B, self.D, self.H, self.Z = batch_size, D, H, Z
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        if backend is None:
            backend = "hip" if self.device.type == "cuda" else "torch"
        if backend == "hip" and self.device.type != "cuda":
            raise ValueError("hip backend needs a GPU device")
        self.backend = backend
        self.seed = int(seed)
        self.rng_stream = int(rng_stream)
        self.hp = dict(lr=lr, beta1=betas[0], beta2=betas[1], eps=eps, weight_decay=weight_decay,
                       kl_beta=kl_beta, grad_scale=1.0)
        self.decoupled_wd = decoupled_wd
        self.layout, self.numel, self.split = arena_layout(D, H, Z)
        self.use_graphs = use_graphs and backend == "hip"
        self.graph_steps = max(1, int(graph_steps))
        self._graphs: Dict[tuple, "torch.cuda.CUDAGraph"] = {}
        self.reducer = None
        # DDP structure (MDT_DDP_OVERLAP, as ConvVaeTrainer): True = the fc4
        # bucket goes out on the reducer's stream between backward parts;
        # False = one stream, the whole backward then every bucket inline;
        # None (auto) = overlap only when the fc4 bucket's transfer over one
        # xGMI link outweighs the measured cost of the split (overlap_pays)
        ov = os.getenv("MDT_DDP_OVERLAP", "auto")
        self.ddp_overlap = None if ov == "auto" else ov != "0"
        self._data = None
        if backend == "hip":
            C = native.require()
            self.engine = C.MlpVaeEngine(batch_size, D, H, Z, self.device.index or 0)
            lay = [(n, o, tuple(s)) for n, o, s in self.engine.layout()]
            assert sorted(lay) == sorted(self.layout) and self.engine.numel() == self.numel, \
                "C++/Python arena layouts disagree"
            self.params, self.grads = self.engine.params, self.engine.grads
            self.exp_avg, self.exp_avg_sq = self.engine.exp_avg, self.engine.exp_avg_sq
        else:
            self.engine = None
            z = lambda: torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            self.params, self.grads, self.exp_avg, self.exp_avg_sq = z(), z(), z(), z()
            self._st = dict(step=0, cursor=0, nbatches=0, epoch_loss=0.0, epoch_count=0.0)
            self._st_eval = dict(step=0, cursor=0, nbatches=0, epoch_loss=0.0, epoch_count=0.0)
            self._hist = np.zeros(LOSS_HIST, np.float32)
            self._hist_eval = np.zeros(LOSS_HIST, np.float32)
        g = torch.Generator().manual_seed(self.seed if init_seed is None else int(init_seed))
        host = torch.zeros(self.numel, dtype=torch.float32)
        init_params_(host, self.layout, g)
        self.params.copy_(host)
        self._push_hparams()

    # ------------------------------------------------------------------ params
    def named_parameters(self) -> Dict[str, torch.Tensor]:
        return views(self.params, self.layout)

    def named_grads(self) -> Dict[str, torch.Tensor]:
        return views(self.grads, self.layout)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Model weights under the reference's parameter names (cpu copies)."""
        return {k: v.detach().cpu().clone() for k, v in self.named_parameters().items()}

    @torch.no_grad()
    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        v = self.named_parameters()
        for k, t in v.items():
            t.copy_(sd[k].to(t.device, torch.float32))

    def optimizer_state(self) -> dict:
        return {"step": self.step_count, "exp_avg": self.exp_avg.detach().cpu().clone(),
                "exp_avg_sq": self.exp_avg_sq.detach().cpu().clone()}

    @torch.no_grad()
    def load_optimizer_state(self, st: dict):
        self.exp_avg.copy_(st["exp_avg"])
        self.exp_avg_sq.copy_(st["exp_avg_sq"])
        self.set_step(int(st["step"]))

    # ------------------------------------------------------------------ hparams
    def set_hparams(self, **kw):
        for k, v in kw.items():
            if k not in self.hp:
                raise KeyError(k)
            self.hp[k] = float(v)
        self._push_hparams()

    def _push_hparams(self):
        if self.engine is not None:
            h = self.hp
            self.engine.set_hparams(h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"],
                                    h["kl_beta"], h["grad_scale"], self.seed, self.decoupled_wd)

    # ------------------------------------------------------------------ state
    @property
    def step_count(self) -> int:
        if self.engine is not None:
            return int(self.engine.read_state(False)[0])
        return self._st["step"]

    def set_step(self, step: int):
        if self.engine is not None:
            self.engine.set_step(int(step))
        else:
            self._st["step"] = int(step)

    def set_cursor(self, cursor: int, nbatches: int, eval: bool = False):
        if self.engine is not None:
            self.engine.set_cursor(eval, int(cursor), int(nbatches))
        else:
            st = self._st_eval if eval else self._st
            st["cursor"], st["nbatches"] = int(cursor), int(nbatches)

    def reset_loss(self, eval: bool = False):
        if self.engine is not None:
            self.engine.reset_loss(eval)
        else:
            st = self._st_eval if eval else self._st
            st["epoch_loss"], st["epoch_count"] = 0.0, 0.0

    def read_state(self, eval: bool = False) -> dict:
        if self.engine is not None:
            s = self.engine.read_state(eval)
            return dict(step=int(s[0]), cursor=int(s[1]), nbatches=int(s[2]), epoch_loss=s[3],
                        epoch_count=s[4])
        return dict(self._st_eval if eval else self._st)

    def loss_history(self, eval: bool = False) -> np.ndarray:
        if self.engine is not None:
            return self.engine.loss_history(eval).numpy()
        return (self._hist_eval if eval else self._hist).copy()

    # ------------------------------------------------------------------ data
    def bind_train_data(self, X: torch.Tensor, idx: torch.Tensor):
        """X: [N, D] float32 on device; idx: int32 index list for the epoch."""
        assert X.dtype == torch.float32 and X.dim() == 2 and X.shape[1] == self.D
        n = idx.numel()
        nb = -(-n // self.B)
        pad = nb * self.B - n
        idx = idx.to(device=self.device, dtype=torch.int32)
        if pad:
            idx = torch.cat([idx, idx[:1].expand(pad)])  # never read (rows >= M)
        self._data = (X.contiguous(), idx.contiguous(), n, nb)
        self._graphs.clear()

    # ------------------------------------------------------------------ step
    def attach_reducer(self, reducer):
        """BucketReducer over ``self.grads`` with bounds [0, split, numel] (fc4
        first, overlapping the rest of the backward) or [0, numel]."""
        self.reducer = reducer
        self._graphs.clear()
        from ..parallel.ddp import graph_capturable

        # a host-blocking (c10d/gloo) reducer cannot live inside a step graph: eager steps
        if not hasattr(self, "_graphs_wanted"):
            self._graphs_wanted = self.use_graphs
        self.use_graphs = self._graphs_wanted and graph_capturable(reducer)

    def bucket_bounds(self, bucket_mb=None):
        """The fused step finishes gradients in two groups (fc4 after B2,
        the rest after B3): two buckets, or one when bucket_mb == 0."""
        return [0, self.numel] if bucket_mb == 0 else [0, self.split, self.numel]

    def default_bucket_bounds(self):
        return self.bucket_bounds(None)

    def refresh_weights(self):
        """Params are the compute weights here (fp32 views): nothing to re-derive."""

    # measured cost (us per step) of splitting the MLP backward around a
    # side-stream bucket launch, per reducer family: overlap minus inline with
    # forced one-rank collectives, 77.5 - 56.9 (RCCL) and 81.9 - 68.0 (p2p
    # kernel) on a 49.0 us step (profiles/r4_ddp_fused/ddp_structure_mlp.json)
    SPLIT_COST_US = {"rccl": 20.5, "p2p": 14.0}

    def _overlap(self) -> bool:
        red = self.reducer
        if red is None or red.num_buckets() != 2:
            return False
        if self.ddp_overlap is not None:
            return bool(self.ddp_overlap)
        from ..parallel.ddp import overlap_pays

        fam = "rccl" if type(red).__name__.startswith("Rccl") else "p2p"
        return overlap_pays(4 * (self.numel - self.split), self.SPLIT_COST_US[fam])

    def _step_hip(self, M: int):
        X, idx = self._data[0], self._data[1]
        e = self.engine
        e.forward(X, idx, M, True, False, self.rng_stream, False)
        early = self._overlap()
        if self.reducer is not None and hasattr(self.reducer, "set_inline"):
            self.reducer.set_inline(not early)
        if early:
            e.backward(X, idx, M, 1, False)
            e.backward(X, idx, M, 2, False)
            self.reducer.launch(1)          # fc4 bucket (final after B2): overlaps B3
            e.backward(X, idx, M, 3, False)
            self.reducer.launch(0)
            self.reducer.wait_all()
            e.adam()
        elif self.reducer is not None:      # every bucket after the whole backward
            e.backward(X, idx, M, 0, False)
            for k in reversed(range(self.reducer.num_buckets())):
                self.reducer.launch(k)
            self.reducer.wait_all()
            e.adam()
        else:
            # Adam fused into the weight-gradient epilogues of B3
            e.backward(X, idx, M, 0, True)

    _CPU_ORDER = ("fc1.weight", "fc1.bias", "fc21.weight", "fc21.bias", "fc22.weight", "fc22.bias",
                  "fc3.weight", "fc3.bias", "fc4.weight", "fc4.bias")

    def _cpu_native(self):
        """The fused native CPU step (csrc/runtime/cpu_mlp.cpp) when the torch
        backend runs on the host and the extension is built; None otherwise
        (stock torch ops, ``reference_step``)."""
        if self.device.type != "cpu" or not native.available():
            return None
        if getattr(self, "_cpu", None) is None:
            self._cpu = native.require().MlpCpuStep(self.B, self.D, self.H, self.Z)
            v, g = self.named_parameters(), self.named_grads()
            self._cpu_w = [v[n] for n in self._CPU_ORDER]
            self._cpu_g = [g[n] for n in self._CPU_ORDER]
        return self._cpu

    @torch.no_grad()
    def _step_torch(self, M: int):
        X, idx = self._data[0], self._data[1]
        st = self._st
        h = self.hp
        cpu = self._cpu_native()
        if cpu is not None:
            loss = cpu.forward_backward(self._cpu_w, self._cpu_g, X, idx, st["cursor"] * self.B, M, self.seed,
                                        self.rng_stream, st["step"], h["kl_beta"])
        else:
            rows = idx[st["cursor"] * self.B: st["cursor"] * self.B + M].long()
            x = X[rows]
            eps = torch.from_numpy(reparam_eps(M, self.Z, self.seed, self.rng_stream, st["step"])).to(self.device)
            f = reference_step(self.named_parameters(), self.named_grads(), x, eps, h["kl_beta"])
            loss = None
        if self.reducer is not None:
            self.reducer.launch(1)
            self.reducer.launch(0)
            self.reducer.wait_all()
        if cpu is not None:
            cpu.adam(self.params, self.grads, self.exp_avg, self.exp_avg_sq, st["step"] + 1, h["lr"], h["beta1"],
                     h["beta2"], h["eps"], h["weight_decay"], h["grad_scale"], self.decoupled_wd)
        else:
            reference_adam_(self.params, self.grads, self.exp_avg, self.exp_avg_sq, st["step"] + 1,
                            h["lr"], h["beta1"], h["beta2"], h["eps"], h["weight_decay"], h["grad_scale"],
                            self.decoupled_wd)
            loss = float(f["loss"])
        self._hist[st["step"] % LOSS_HIST] = loss
        st["epoch_loss"] += loss
        st["epoch_count"] += 1
        st["step"] += 1
        st["cursor"] += 1
        if st["nbatches"] and st["cursor"] >= st["nbatches"]:
            st["cursor"] = 0

    def train_steps(self, n: int, M: Optional[int] = None):
        """Run ``n`` training steps of ``M`` rows from the current cursor."""
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
            return
        S = self.graph_steps
        while n >= S:
            self._replay(S, M)
            n -= S
        for _ in range(n):
            self._replay(1, M)

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

    def model_meta(self) -> dict:
        """Architecture record stored in checkpoints and validated on load."""
        return {"kind": "mlp", "D": int(self.D), "H": int(self.H), "Z": int(self.Z)}

    # see ConvVaeTrainer.strict_graphs: no lazy capture once set
    strict_graphs = False

    def _replay(self, S: int, M: int):
        key = (S, M)
        g = self._graphs.get(key)
        if g is None:
            if self.strict_graphs:
                raise RuntimeError(f"no captured step graph for (steps={S}, M={M}); call prepare() first")
            g = self._capture(S, M)
            self._graphs[key] = g
        g.replay()

    def _capture(self, S: int, M: int):
        # Capture with the device state preserved: warm-up launches advance the
        # step counter / cursor / Adam moments, so snapshot and restore them.
        snap = [t.clone() for t in (self.params, self.exp_avg, self.exp_avg_sq,
                                     self.engine.train_state)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._step_hip(M)  # warm-up (communicator init, code-object load)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(S):
                self._step_hip(M)
        for t, v in zip((self.params, self.exp_avg, self.exp_avg_sq, self.engine.train_state), snap):
            t.copy_(v)
        native.upload_graph(g)
        return g

    # ------------------------------------------------------------------ eval / sample
    @torch.no_grad()
    # graph-replayed eval passes (models/eval_graphs.py)
    def _eval_batch(self, M, X, idx, want_recon):
        self.engine.forward(X, idx, M, False, True, EVAL_STREAM + self.rng_stream, want_recon)
        self.engine.loss_finalize(True)

    def _eval_state(self):
        return self.engine.eval_state

    def _eval_recon(self, M):
        return self.engine.act("recon", M).clone()

    def evaluate(self, X: torch.Tensor, idx: torch.Tensor, want_first_recon: bool = True):
        """Forward + loss over (X[idx]); returns (sum_loss, recon of the first batch or None)."""
        idx = idx.to(device=self.device, dtype=torch.int32).contiguous()
        n = idx.numel()
        nb = -(-n // self.B)
        pad = nb * self.B - n
        if pad:
            idx = torch.cat([idx, idx[:1].expand(pad)])
        X = X.contiguous()
        if self.backend == "hip" and self.use_graphs:
            first = self._eval_graphed(X, idx, n, want_first_recon)
            return self.read_state(eval=True)["epoch_loss"], first
        self.set_cursor(0, nb, eval=True)
        self.reset_loss(eval=True)
        first = None
        for b in range(nb):
            M = min(self.B, n - b * self.B)
            if self.backend == "hip":
                want = want_first_recon and b == 0
                self._eval_batch(M, X, idx, want)
                if want:
                    first = self._eval_recon(M)
            else:
                st = self._st_eval
                cpu = self._cpu_native()
                if cpu is not None:  # fused native forward + loss (csrc/runtime/cpu_mlp.cpp)
                    loss = cpu.forward_backward(self._cpu_w, self._cpu_g, X, idx, b * self.B, M, self.seed,
                                                EVAL_STREAM + self.rng_stream, st["step"], self.hp["kl_beta"],
                                                backward=False)
                    if want_first_recon and b == 0:
                        first = cpu.recon()
                else:
                    rows = idx[b * self.B: b * self.B + M].long()
                    x = X[rows]
                    eps = torch.from_numpy(reparam_eps(M, self.Z, self.seed, EVAL_STREAM + self.rng_stream,
                                                       st["step"])).to(self.device)
                    f = reference_forward(self.named_parameters(), x, eps, self.hp["kl_beta"])
                    if want_first_recon and b == 0:
                        first = f["p"].clone()
                    loss = float(f["loss"])
                self._hist_eval[st["step"] % LOSS_HIST] = loss
                st["epoch_loss"] += loss
                st["epoch_count"] += 1
                st["step"] += 1
                st["cursor"] = (st["cursor"] + 1) % nb
        return self.read_state(eval=True)["epoch_loss"], first

    @torch.no_grad()
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        z = z.to(self.device, torch.float32).contiguous()
        if self.backend == "hip":
            out = []
            for i in range(0, z.shape[0], self.B):
                out.append(self.engine.decode(z[i:i + self.B].contiguous()))
            return torch.cat(out)
        v = self.named_parameters()
        h3 = torch.relu(z @ v["fc3.weight"].t() + v["fc3.bias"])
        return torch.sigmoid(h3 @ v["fc4.weight"].t() + v["fc4.bias"])

    # ------------------------------------------------------------------ info
    def flops_per_sample(self) -> float:
        D, H, Z = self.D, self.H, self.Z
        fwd = D * H + H * 2 * Z + Z * H + H * D
        bwd = 2 * fwd - D * H  # no dX for the input layer
        return 2.0 * (fwd + bwd)
