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
* **Heartbeat** — while a replica waits for its enqueued epoch it beats on
  the c10d store and watches its peers (``TrialWatch``): a peer that raised
  publishes a "failed" key (seen within ~0.5 s), a peer whose process died
  stops beating (``MDT_HEARTBEAT_S``, default 30 s); either aborts the trial's
  communicator at once instead of after the group timeout. The stall bound
  (``MDT_GROUP_TIMEOUT_S``) counts from the last completed chunk of steps,
  not from the start of the epoch, so a long healthy epoch never trips it.
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

__all__ = ["InjectedFault", "TrialTimeout", "TrialCorrupted", "maybe_inject", "fault_step", "guarded", "group_timeout_s",
           "heartbeat_s", "parse_fault", "create_health_groups", "health_group", "trial_watch", "agree_healthy",
           "TrialWatch", "injected_rank"]


class InjectedFault(RuntimeError):
    pass


class TrialTimeout(RuntimeError):
    """A replica's epoch did not complete within the group timeout (a peer is gone)."""


class TrialCorrupted(RuntimeError):
    """A kernel reported that the epoch's results are not trustworthy (an
    in-kernel exchange or all-reduce wait timed out); the trial fails instead
    of reporting healthy numbers."""


_HEALTH: Dict[int, object] = {}
_WATCH: Dict[int, "TrialWatch"] = {}
_GEN = [0]


class TrialWatch:
    """Host-side liveness of the replicas of one trial over the c10d store:
    ``beat()`` advances this member's counter, ``fail(msg)`` publishes a
    failure, ``check()`` reports a published failure or a peer whose counter
    has not moved for ``silent_s`` seconds (``reset()`` restarts those clocks,
    e.g. when a new epoch starts)."""

    def __init__(self, store, rank: int, size: int):
        self.store, self.rank, self.size = store, rank, size
        self.beats = 0
        self.seen: Dict[int, tuple] = {}

    def beat(self):
        self.beats += 1
        self.store.set(f"hb/{self.rank}", str(self.beats))

    def fail(self, msg: str):
        try:
            self.store.set("failed", f"rank {self.rank}: {msg}")
        except Exception:  # noqa: BLE001 - the store may be gone with rank 0
            pass

    def reset(self):
        self.seen.clear()

    def check(self, silent_s: Optional[float] = None) -> Optional[str]:
        import time

        silent_s = heartbeat_s() if silent_s is None else silent_s
        if self.store.check(["failed"]):
            return "a replica failed (" + self.store.get("failed").decode(errors="replace") + ")"
        now = time.monotonic()
        for p in range(self.size):
            if p == self.rank:
                continue
            key = f"hb/{p}"
            v = self.store.get(key) if self.store.check([key]) else b""
            old = self.seen.get(p)
            if old is None or old[0] != v:
                self.seen[p] = (v, now)
            elif now - old[1] > silent_s:
                return f"replica {p} of the trial sent no heartbeat for {now - old[1]:.0f} s (process lost?)"
        return None


def create_health_groups(num_groups: int, world_size: Optional[int] = None):
    """One gloo group per multi-rank trial for health agreement, plus its
    ``TrialWatch``. Call on every rank (it is NOT a world collective).

    Built without ``dist.new_group``: on a device-bound RCCL world torch makes
    every NON-member of a new group take part in a ``ncclCommSplit(NOCOLOR)``
    of the world communicator -- for gloo groups too -- while the gloo group's
    members make no split call, so an idle leftover rank (W % K != 0) would
    issue one split more than the trial members and hang in it.
    Here each member connects a ``ProcessGroupGloo`` of its own trial straight
    through the default store (keys under a per-call prefix, the same
    constructor ``new_group`` uses); non-members and idle ranks do nothing.
    ``health_group(g)`` / ``trial_watch(g)`` return this member's handles.
    """
    import torch.distributed as dist

    from ..parallel.groups import GroupPlan
    from .bootstrap import _stdout_to_stderr

    _HEALTH.clear()
    _WATCH.clear()
    if not dist.is_initialized():
        return
    _GEN[0] += 1
    W = world_size or dist.get_world_size()
    plan = GroupPlan(W, num_groups)
    me = dist.get_rank()
    g = plan.group_of(me)
    if g is None or plan.ranks_per_group == 1:
        return
    ranks = plan.ranks(g)
    store = dist.PrefixStore(f"mdt_health/{_GEN[0]}/{g}/", dist.distributed_c10d._get_default_store())
    with _stdout_to_stderr():  # gloo connect banners stay off stdout
        _HEALTH[g] = dist.ProcessGroupGloo(dist.PrefixStore("pg/", store), me - ranks[0], len(ranks),
                                           _dt.timedelta(hours=6))
    _WATCH[g] = TrialWatch(dist.PrefixStore("watch/", store), me - ranks[0], len(ranks))


def health_group(group_id: int):
    return _HEALTH.get(group_id)


def trial_watch(group_id: int) -> Optional[TrialWatch]:
    return _WATCH.get(group_id)


def agree_healthy(group_id: int, ok: bool) -> bool:
    """All-reduce(MIN) of this member's ``ok`` over the trial's health group.
    Without a health group (single-rank trial, or groups not created) -> ``ok``."""
    pg = _HEALTH.get(group_id)
    if pg is None:
        return ok
    import torch
    import torch.distributed as dist

    if pg.size() == 1:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    opts = dist.AllreduceOptions()
    opts.reduceOp = dist.ReduceOp.MIN
    pg.allreduce([t], opts).wait()
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


def injected_rank(name: str) -> Optional[int]:
    """Test-only seam of the data-plane fallbacks: the group rank named by
    ``MDT_TEST_<name>_RANK`` (e.g. ``IPC_FAIL``: that member's peer mapping
    fails; ``XGMI_SELFTEST_FAIL``: its data-plane self-test reports a
    mismatch), or None. Production never sets these; every consumer is a
    collective decision, so an injected failure exercises exactly the path a
    real one takes."""
    v = os.getenv(f"MDT_TEST_{name}_RANK", "")
    return int(v) if v.strip().lstrip("-").isdigit() else None


def group_timeout_s() -> float:
    return float(os.getenv("MDT_GROUP_TIMEOUT_S", "600"))


def heartbeat_s() -> float:
    return float(os.getenv("MDT_HEARTBEAT_S", "30"))


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
