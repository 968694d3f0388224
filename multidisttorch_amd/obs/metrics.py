"""Per-trial JSONL metrics and the aggregate samples/s metric.

The reference only prints ``"{rank} Done. time: {t1-t0}"`` (/root/reference/
vae-hpo.py:159, 172-174). Here every trial's group rank 0 appends JSON lines
(epoch, loss, samples/s, step_ms, eval time, ...) to
``<metrics_dir>/trial-{g}.jsonl``, and world rank 0 computes the headline
metric: Σ_g (epochs_g · |shard_g|) / max_rank(t1 - t0), samples
counted once per trial (replicas of a group share the shard).
"""

from __future__ import annotations

import json
import os
import time
from typing import Optional

__all__ = ["TrialMetrics", "aggregate_samples_per_s", "StepTimer"]


class TrialMetrics:
    def __init__(self, metrics_dir: Optional[str], group_id: int, enabled: bool = True):
        self.path = None
        if metrics_dir and enabled:
            os.makedirs(metrics_dir, exist_ok=True)
            self.path = os.path.join(metrics_dir, f"trial-{group_id}.jsonl")
        self.group_id = group_id

    def log(self, **kw):
        if self.path is None:
            return
        rec = {"ts": time.time(), "trial": self.group_id}
        rec.update(kw)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def aggregate_samples_per_s(trial_samples, wall_s: float) -> float:
    """Σ samples over trials / slowest rank's wall time (BASELINE.md definition)."""
    return float(sum(trial_samples)) / max(wall_s, 1e-12)


class StepTimer:
    """Device-event timer (HIP events) with host fallback."""

    def __init__(self, device):
        import torch

        self.cuda = getattr(device, "type", str(device)) == "cuda"
        self.torch = torch
        self.t0 = None
        self.e0 = self.e1 = None

    def start(self):
        if self.cuda:
            self.e0 = self.torch.cuda.Event(enable_timing=True)
            self.e1 = self.torch.cuda.Event(enable_timing=True)
            self.e0.record()
        self.t0 = time.perf_counter()

    def stop(self) -> float:
        """Elapsed seconds (device time when on GPU)."""
        if self.cuda:
            self.e1.record()
            self.e1.synchronize()
            return self.e0.elapsed_time(self.e1) / 1e3
        return time.perf_counter() - self.t0
