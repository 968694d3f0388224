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
* **Injection** — ``MDT_FAULT`` triggers a deterministic failure for tests and
  drills: ``MDT_FAULT="trial=1,epoch=1"`` or ``"rank=3,step=5"``
  (comma-separated key=value; all given keys must match).
"""

from __future__ import annotations

import os
import traceback
from contextlib import contextmanager
from typing import Optional

__all__ = ["InjectedFault", "maybe_inject", "guarded", "group_timeout_s", "parse_fault"]


class InjectedFault(RuntimeError):
    pass


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
    """Raise InjectedFault if MDT_FAULT matches every key it names."""
    f = parse_fault()
    if not f:
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
