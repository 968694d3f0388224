"""Failure detection, isolation and fault injection for concurrent trials.

The reference has none: a failing trial, or leftover idle
ranks, crash or hang everyone at the global barriers, and RCCL waits for the
10-minute watchdog. Here:

* **Isolation** — ``run_trial`` executes inside ``guarded`` : an exception in
  one trial is caught, logged (stdout + metrics JSONL), and the rank still
  joins the gloo control-plane barriers, so the other K-1 trials finish and
  report. A trial whose group has >1 rank also aborts its own communicator so
  peers blocked in a collective fail fast instead of hanging.
* **Detection** — sub-group collectives are created with a bounded timeout
  (``MDT_GROUP_TIMEOUT_S``, default 600 s) and the control plane with a long
  one; ``ProcessGroupNCCL``'s async error handling turns a stuck collective
  into an exception on every member.
* **Agreement** — a trial group of more than one rank agrees on its health
  over its own small gloo group (``create_health_groups``): every member
  checks in before each epoch and once after the last one. A member that
  failed checks in exactly once with "not ok", so however the failure
  happened (Python error between epochs, a replica stuck in a collective that
  timed out and aborted its communicator) all members leave the trial at the
  same check and mark it failed; nobody blocks forever in graph replay.
* **Injection** — ``MDT_FAULT`` triggers a deterministic failure for tests and
  drills: ``MDT_FAULT="trial=1,epoch=1"`` (before the epoch starts) or
  ``"rank=3,step=5"`` (mid-epoch: the rank stops issuing steps at optimizer
  step 5 while its peers are already enqueued for the whole epoch)
  (comma-separated key=value; all given keys must match).
"""

from __future__ import annotations

import datetime as _dt
import os
import traceback
from contextlib import contextmanager
from typing import Dict, Optional

__all__ = ["InjectedFault", "TrialTimeout", "maybe_inject", "fault_step", "guarded", "group_timeout_s",
           "parse_fault", "create_health_groups", "health_group", "agree_healthy"]


class InjectedFault(RuntimeError):
    pass


class TrialTimeout(RuntimeError):
    """A replica's epoch did not complete within the group timeout (a peer is gone)."""


_HEALTH: Dict[int, object] = {}


def create_health_groups(num_groups: int, world_size: Optional[int] = None):
    """World collective: one gloo group per trial group for health agreement.

    Call on every rank, in the same order relative to other ``new_group``
    calls (right after ``setup_ddp_groups`` / ``control_group``). Members keep
    their own group's handle; ``health_group(g)`` returns it.
    """
    import torch.distributed as dist

    from ..parallel.groups import GroupPlan
    from .bootstrap import _stdout_to_stderr

    if not dist.is_initialized():
        return
    W = world_size or dist.get_world_size()
    plan = GroupPlan(W, num_groups)
    me = dist.get_rank()
    _HEALTH.clear()
    with _stdout_to_stderr():  # gloo connect banners stay off stdout
        for g in range(num_groups):
            pg = dist.new_group(ranks=plan.ranks(g), backend="gloo", timeout=_dt.timedelta(hours=6))
            if me in plan.ranks(g):
                _HEALTH[g] = pg


def health_group(group_id: int):
    return _HEALTH.get(group_id)


def agree_healthy(group_id: int, ok: bool) -> bool:
    """All-reduce(MIN) of this member's ``ok`` over the trial's health group.
    Without a health group (single-rank trial, or groups not created) -> ``ok``."""
    pg = _HEALTH.get(group_id)
    if pg is None:
        return ok
    import torch
    import torch.distributed as dist

    if dist.get_world_size(pg) == 1:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pg)
    return bool(t.item())


def fault_step(**where) -> Optional[int]:
    """Optimizer step at which MDT_FAULT's ``step=`` key fires for this
    (rank, trial, ...), or None. Keys other than ``step`` must all match."""
    f = parse_fault()
    if not f or "step" not in f:
        return None
    for k, v in f.items():
        if k != "step" and where.get(k) != v:
            return None
    return int(f["step"])


def parse_fault(spec: Optional[str] = None) -> Optional[dict]:
    spec = os.getenv("MDT_FAULT", "") if spec is None else spec
    if not spec:
        return None
    out = {}
    for part in spec.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip()] = int(v)
    return out or None


def maybe_inject(**where):
    """Raise InjectedFault if MDT_FAULT matches every key it names (a spec
    with a ``step`` key fires through ``fault_step`` instead)."""
    f = parse_fault()
    if not f or "step" in f:
        return
    for k, v in f.items():
        if where.get(k) != v:
            return
    raise InjectedFault(f"injected fault at {where}")


def group_timeout_s() -> float:
    return float(os.getenv("MDT_GROUP_TIMEOUT_S", "600"))


@contextmanager
def guarded(label: str, group=None, on_error=None):
    """Run a trial; on exception report and (for groups > 1) abort the group's
    communicator, then swallow so the rank can still join global barriers."""
    try:
        yield
    except Exception as e:  # noqa: BLE001 - isolation boundary
        msg = f"[mdt] {label} FAILED: {type(e).__name__}: {e}"
        print(msg, flush=True)
        if os.getenv("MDT_FAULT_TRACEBACK", "0") == "1":
            traceback.print_exc()
        if group is not None:
            try:
                import torch.distributed as dist

                if dist.get_world_size(group) > 1:
                    backend = group._get_backend(__import__("torch").device("cuda")) if hasattr(group, "_get_backend") else None
                    if backend is not None and hasattr(backend, "abort"):
                        backend.abort()
            except Exception:
                pass
        if on_error is not None:
            on_error(e)
