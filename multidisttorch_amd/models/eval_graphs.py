"""Graph-replayed evaluation passes for the HIP trainers.

Reference: ``test()`` runs the model over the whole 10 000-image test set
after every epoch (/root/reference/vae-hpo.py:95-119), and its time is part of
the per-trial wall time the aggregate samples/s metric divides by
(:159, :172-174). Issued eagerly from Python, each test
batch costs a dozen kernel launches plus their host overhead: ~230 us per
batch, 17-19 ms per epoch for the 28x28 conv-VAE -- 37 % of an epoch whose
training takes 29 ms (`profiles/r5_e2e`).

The trainers' eval kernels take the batch rows from a device-resident cursor
(the eval ``TrainState``) and write the loss into its ring, exactly like the
training step, so a whole pass is capturable: batch 0 runs eagerly (it may
also produce the reconstruction images), the remaining full batches replay one
captured graph of S batches, the tail batch a graph of its own. The index list
lives in a persistent buffer (its address is baked into the graphs; each pass
copies the caller's indices into it), graphs are keyed by (S, M, dataset
address and length, buffer address; only the latest dataset's are kept), and
capturing restores the eval state
the warm-up batch advanced. Numerics are those of the eager pass (same kernels
in the same order).
"""

from __future__ import annotations

import torch

from ..ops import native

__all__ = ["GraphedEval"]


class GraphedEval:
    """Mixin: requires ``self.B``, ``self.device``, ``self.use_graphs``,
    ``self.set_cursor``, ``self.reset_loss``, ``self._eval_batch(M, X, idx,
    want_recon)``, ``self._eval_state()`` (the eval TrainState tensor) and
    ``self._eval_recon(M)`` (the first batch's reconstruction)."""

    _eval_idx = None
    _eval_graphs = None

    def _eval_bind(self, idx_padded: torch.Tensor) -> torch.Tensor:
        n = idx_padded.numel()
        buf = self._eval_idx
        if buf is None or buf.numel() != n:
            self._eval_idx = buf = torch.empty(n, dtype=torch.int32, device=self.device)
            self._eval_graphs = {}
        buf.copy_(idx_padded)
        return buf

    def _eval_graph(self, S: int, M: int, X: torch.Tensor, idx: torch.Tensor):
        key = (S, M, X.data_ptr(), X.shape[0], idx.data_ptr())
        # graphs of the latest eval set only: a caller that passes
        # a new (e.g. temporary) X drops the graphs -- and their private memory
        # pools -- captured for the previous one instead of accumulating them
        xkey = (X.data_ptr(), X.shape[0], idx.data_ptr())
        if getattr(self, "_eval_xkey", None) != xkey:
            self._eval_graphs = {}
            self._eval_xkey = xkey
        g = self._eval_graphs.get(key)
        if g is None:
            st = self._eval_state()
            snap = st.clone()
            cur = torch.cuda.current_stream()
            s = torch.cuda.Stream()
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                self._eval_batch(M, X, idx, False)  # warm-up: plans / workspaces exist before capture
            cur.wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(S):
                    self._eval_batch(M, X, idx, False)
            st.copy_(snap)
            native.upload_graph(g)
            self._eval_graphs[key] = g
        return g

    def _eval_graphed(self, X: torch.Tensor, idx_padded: torch.Tensor, n: int, want_first_recon: bool):
        """One eval pass over rows idx[:n] of X (graphs after batch 0)."""
        B = self.B
        nb = -(-n // B)
        idx = self._eval_bind(idx_padded)
        self.set_cursor(0, nb, eval=True)
        self.reset_loss(eval=True)
        M0 = min(B, n)
        self._eval_batch(M0, X, idx, want_first_recon)
        first = self._eval_recon(M0) if want_first_recon else None
        full, tail = n // B, n % B
        if n > B:
            if full > 1:
                self._eval_graph(full - 1, B, X, idx).replay()
            if tail:
                self._eval_graph(1, tail, X, idx).replay()
        return first
