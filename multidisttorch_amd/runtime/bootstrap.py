"""Process-group bootstrap: backend choice, device binding, world + control plane.

Parity: ``setup_ddp`` <- /root/reference/utils.py:93-144 (backend choice
``:96-103``, env export ``:122-131``, banner ``:133-136``, idempotent init
``:138-139``). ``get_comm_size_and_rank`` <- /root/reference/utils.py:28-38.

MI355X-first differences:
  * one process per GPU: the local rank is bound with ``torch.cuda.set_device``
    *before* the RCCL world is created (the reference binds nothing and relies
    on the launcher hiding GPUs);
  * a separate **gloo control plane** (``control_group()``) carries the global
    barriers of the HPO driver, so trials of different length never trip the
    RCCL watchdog (10 min) at the final barrier and idle leftover ranks can
    still join it;
  * eager, device-bound RCCL world by default when every local rank has its
    own GPU (``eager_comm_requested``), so trial groups are produced by
    ``ncclCommSplit`` instead of a fresh bootstrap each.
"""

from __future__ import annotations

import datetime as _dt
import contextlib
import os
import sys
from typing import Optional

import torch
import torch.distributed as dist

from . import env as _envmod

__all__ = [
    "choose_backend",
    "setup_ddp",
    "get_comm_size_and_rank",
    "control_group",
    "global_barrier",
    "bound_device",
    "shutdown",
]

_STATE = {"control": None, "device": None, "launch": None}


def choose_backend() -> str:
    """``$DDP_BACKEND`` > ``nccl`` (=RCCL on ROCm) if a GPU exists > ``gloo``."""
    if os.getenv("DDP_BACKEND") is not None:
        return os.environ["DDP_BACKEND"]
    if dist.is_nccl_available() and torch.cuda.is_available():
        return "nccl"
    if dist.is_gloo_available():
        return "gloo"
    raise RuntimeError("No parallel backends available")


def get_comm_size_and_rank():
    """(world_size, world_rank) after init; (1, 0) when not initialised."""
    if dist.is_available() and dist.is_initialized():
        return int(dist.get_world_size()), int(dist.get_rank())
    return 1, 0


def eager_comm_requested(info: Optional[_envmod.LaunchInfo] = None, ndev: Optional[int] = None) -> bool:
    """Bind the RCCL world to the local device at init (eager communicator),
    so trial groups are split from it (``ncclCommSplit``) instead of each
    bootstrapping a fresh communicator at its first collective.

    ``MDT_EAGER_COMM=1`` forces it, ``=0`` forbids it; by default it is on
    whenever every rank of this node has its own GPU (the launcher reports a
    local size no larger than the visible device count) -- the one-process-
    per-MI355X layout. Ranks sharing a GPU (RCCL rejects duplicate devices in
    one communicator) or an unknown local size keep the lazy path."""
    v = os.getenv("MDT_EAGER_COMM", "auto")
    if v in ("0", "1"):
        return v == "1"
    info = info or _STATE.get("launch")
    if info is None or info.local_size is None or not ndev:
        return False
    return info.local_size <= ndev


def world_is_device_bound() -> bool:
    """True when the default group is an eagerly initialised, device-bound RCCL world."""
    if not dist.is_initialized() or dist.get_backend() != "nccl":
        return False
    return getattr(dist.distributed_c10d._get_default_group(), "bound_device_id", None) is not None


def bound_device() -> torch.device:
    """Device this process computes on (``cuda:<local_rank>`` or ``cpu``)."""
    if _STATE["device"] is not None:
        return _STATE["device"]
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _bind_local_device(info: _envmod.LaunchInfo, backend: Optional[str] = None) -> torch.device:
    if not torch.cuda.is_available():
        return torch.device("cpu")
    ndev = torch.cuda.device_count()
    # If the launcher already isolated one GPU per process (jsrun resource
    # sets, --gpus-per-task, HIP_VISIBLE_DEVICES) ndev == 1 and this is cuda:0.
    # ndev == 1 is the launcher-isolated layout (each rank sees its own GPU as
    # cuda:0); with several visible GPUs, more local ranks than GPUs means sharing
    shared = ndev > 1 and ((info.local_size is not None and info.local_size > ndev) or info.local_rank >= ndev)
    if shared and backend == "nccl":
        # more ranks than GPUs on this node: RCCL would later abort with
        # "Duplicate GPU detected" inside the first collective; say so now
        raise RuntimeError(
            f"{info.local_size if info.local_size is not None else '>' + str(info.local_rank)} ranks on this node "
            f"but {ndev} visible GPUs: RCCL needs one process per GPU (launch at most {ndev} ranks per node, or "
            f"use DDP_BACKEND=gloo to share GPUs)")
    if shared:
        print(f"[mdt] warning: local rank {info.local_rank} shares a GPU ({ndev} visible); "
              f"cuda:{info.local_rank % max(ndev, 1)}", file=sys.stderr, flush=True)
    idx = info.local_rank % max(ndev, 1)
    torch.cuda.set_device(idx)
    return torch.device("cuda", idx)


def setup_ddp(backend: Optional[str] = None, verbose: bool = True,
              timeout_s: Optional[float] = None, bind_device: bool = True):
    """Initialise the global world. Returns ``(world_size, world_rank)``.

    Same observable contract as the reference: exports ``MASTER_ADDR``,
    ``MASTER_PORT``, ``WORLD_SIZE``, ``RANK`` (and ``GLOO_SOCKET_IFNAME`` for
    gloo), prints ``"Distributed data parallel: <backend> master at A:P"`` and
    initialises the default process group once.
    """
    backend = backend or choose_backend()
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else None
    info = _envmod.discover(ndev=ndev)
    _STATE["launch"] = info
    world_size, world_rank = info.world_size, info.world_rank
    master_addr, master_port = info.master_addr, info.master_port

    if backend in ("nccl", "gloo", "cpu:gloo,cuda:nccl"):
        os.environ["MASTER_ADDR"] = master_addr
        os.environ["MASTER_PORT"] = master_port
        os.environ["WORLD_SIZE"] = str(world_size)
        os.environ["RANK"] = str(world_rank)
    if backend == "gloo" and "GLOO_SOCKET_IFNAME" not in os.environ:
        ifname = _envmod.find_ifname(master_addr)
        if ifname is not None:
            os.environ["GLOO_SOCKET_IFNAME"] = ifname

    _STATE["device"] = _bind_local_device(info, backend) if bind_device else bound_device()

    if verbose:
        print("Distributed data parallel: %s master at %s:%s" % (backend, master_addr, master_port))

    if not dist.is_initialized():
        kwargs = {}
        if timeout_s is not None:
            kwargs["timeout"] = _dt.timedelta(seconds=timeout_s)
        if backend == "nccl" and _STATE["device"].type == "cuda" and eager_comm_requested(info, ndev):
            kwargs["device_id"] = _STATE["device"]
        dist.init_process_group(backend=backend, init_method="env://",
                                world_size=world_size, rank=world_rank, **kwargs)
    return world_size, world_rank


@contextlib.contextmanager
def _stdout_to_stderr():
    """Point fd 1 at fd 2 for the duration (native libraries write to fd 1 directly)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def control_group():
    """World-spanning gloo process group for control-plane barriers.

    Created lazily; every rank must call it in the same order as any other
    ``new_group`` (it is itself a world collective). On a gloo world the
    default group is returned.
    """
    if not dist.is_initialized():
        return None
    if _STATE["control"] is None:
        if dist.get_backend() == "gloo":
            _STATE["control"] = dist.group.WORLD
        else:
            # gloo's C++ connect banner goes to fd 1; keep stdout for the
            # caller's own output (bench.py's single JSON line)
            with _stdout_to_stderr():
                _STATE["control"] = dist.new_group(backend="gloo",
                                                   timeout=_dt.timedelta(hours=6))
    return _STATE["control"]


def global_barrier():
    """Barrier over the whole world on the gloo control plane."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    dist.barrier(group=control_group())


def shutdown():
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        finally:
            _STATE["control"] = None
