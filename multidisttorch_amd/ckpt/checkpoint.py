"""Per-trial checkpoint / resume (absent from the reference).

Layout (beside the reference's ``results-{group_rank}/`` images):

    <ckpt_dir>/trial-{g}/epoch-{e}.pt      one file per completed epoch
    <ckpt_dir>/trial-{g}/latest            text file: name of the newest epoch file

Each file holds only tensors and plain Python scalars/strings, so it loads
with ``torch.load(weights_only=True)`` (never unpickles code):
  model        state_dict under the reference's parameter names (fc1.weight, ...)
  optimizer    {"step", "exp_avg", "exp_avg_sq"} flat arenas (layout recorded)
  trial        TrialSpec fields (group_id, epochs, lr, beta, seed)
  progress     {"epoch": completed epochs, "step": optimizer steps}
  rng          {"seed", "rng_stream"} (Philox is counter-based: the step
               counter + seed fully determine the noise stream)
  layout       [[name, offset, shape...]] of the arena, for validation
  arch         model kind + dims (mlp: D/H/Z; conv: image/channels/Z + the
               layer table), validated on load before any tensor is copied
Only group rank 0 writes (replicas are identical after the all-reduce);
writes go to a temp file + atomic rename so a crash never leaves a torn file.
"""

from __future__ import annotations

import os
from typing import Optional

import torch

__all__ = ["trial_dir", "save_trial", "load_latest", "latest_path"]


def trial_dir(ckpt_dir: str, group_id: int) -> str:
    return os.path.join(ckpt_dir, f"trial-{group_id}")


def save_trial(ckpt_dir: str, trainer, spec, epoch: int, extra: Optional[dict] = None) -> str:
    d = trial_dir(ckpt_dir, spec.group_id)
    os.makedirs(d, exist_ok=True)
    opt = trainer.optimizer_state()
    payload = {
        "format": "multidisttorch_amd.trial.v1",
        "model": trainer.state_dict(),
        "optimizer": {"step": int(opt["step"]), "exp_avg": opt["exp_avg"], "exp_avg_sq": opt["exp_avg_sq"]},
        "trial": {k: (float(v) if isinstance(v, float) else int(v)) for k, v in spec.to_dict().items()},
        "progress": {"epoch": int(epoch), "step": int(opt["step"])},
        "rng": {"seed": int(trainer.seed), "rng_stream": int(trainer.rng_stream)},
        "layout": [[n, int(o)] + [int(x) for x in s] for n, o, s in trainer.layout],
        "arch": trainer.model_meta(),
    }
    if extra:
        payload["extra"] = extra
    name = f"epoch-{epoch}.pt"
    path = os.path.join(d, name)
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)
    with open(os.path.join(d, "latest.tmp"), "w") as f:
        f.write(name + "\n")
    os.replace(os.path.join(d, "latest.tmp"), os.path.join(d, "latest"))
    return path


def latest_path(ckpt_dir: str, group_id: int) -> Optional[str]:
    d = trial_dir(ckpt_dir, group_id)
    p = os.path.join(d, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    path = os.path.join(d, name)
    return path if os.path.exists(path) else None


def load_latest(ckpt_dir: str, group_id: int, trainer) -> Optional[dict]:
    """Restore model + optimizer into ``trainer``; returns the progress dict or None."""
    path = latest_path(ckpt_dir, group_id)
    if path is None:
        return None
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if ck.get("format") != "multidisttorch_amd.trial.v1":
        raise ValueError(f"{path}: unknown checkpoint format {ck.get('format')!r}")
    arch = ck.get("arch")
    if arch is not None and arch != trainer.model_meta():
        raise ValueError(f"{path}: checkpoint is for {arch.get('kind')} model {arch}, "
                         f"trainer is {trainer.model_meta()}")
    lay = [[n, int(o)] + [int(x) for x in s] for n, o, s in trainer.layout]
    if ck["layout"] != lay:
        raise ValueError(f"{path}: parameter arena layout mismatch")
    trainer.load_state_dict(ck["model"])
    trainer.load_optimizer_state(ck["optimizer"])
    return dict(ck["progress"], path=path, trial=ck["trial"])
