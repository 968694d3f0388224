"""Launcher environment discovery (pure Python, no torch.distributed needed).

Parity with the reference bootstrap layer:
  * ``init_comm_size_and_rank``  <- /root/reference/utils.py:9-26
  * ``parse_slurm_nodelist``     <- /root/reference/utils.py:59-90
  * ``find_ifname``              <- /root/reference/utils.py:40-56
  * master discovery             <- /root/reference/utils.py:108-119

Extensions:
  * torchrun's ``RANK``/``WORLD_SIZE`` are honoured *after* OMPI and SLURM
    (the reference ignores them, so two torchrun processes became two
    isolated worlds of size 1).
  * a *local rank* is discovered as well, so every process can bind exactly
    one MI355X (``OMPI_COMM_WORLD_LOCAL_RANK`` / ``SLURM_LOCALID`` /
    ``LOCAL_RANK``), which the reference never does.
"""

from __future__ import annotations

import os
import re
import socket
from dataclasses import dataclass
from typing import Mapping, Optional

__all__ = [
    "LaunchInfo",
    "discover",
    "init_comm_size_and_rank",
    "local_rank_from_env",
    "parse_slurm_nodelist",
    "parse_slurm_tasks_per_node",
    "find_ifname",
    "discover_master",
]


def _env(env: Optional[Mapping[str, str]]) -> Mapping[str, str]:
    return os.environ if env is None else env


def init_comm_size_and_rank(env: Optional[Mapping[str, str]] = None):
    """World (size, rank) from launcher variables, *before* process-group init.

    Precedence (OMPI -> SLURM identical to /root/reference/utils.py:13-20):
      1. ``OMPI_COMM_WORLD_SIZE`` + ``OMPI_COMM_WORLD_RANK``  (jsrun / mpirun)
      2. ``SLURM_NPROCS`` + ``SLURM_PROCID``                  (srun)
      3. ``WORLD_SIZE`` + ``RANK``                             (torchrun, mdtrun) [extension]
      4. ``(1, 0)``
    """
    e = _env(env)
    if e.get("OMPI_COMM_WORLD_SIZE") and e.get("OMPI_COMM_WORLD_RANK"):
        return int(e["OMPI_COMM_WORLD_SIZE"]), int(e["OMPI_COMM_WORLD_RANK"])
    if e.get("SLURM_NPROCS") and e.get("SLURM_PROCID"):
        return int(e["SLURM_NPROCS"]), int(e["SLURM_PROCID"])
    if e.get("WORLD_SIZE") and e.get("RANK"):
        return int(e["WORLD_SIZE"]), int(e["RANK"])
    return 1, 0


def local_rank_from_env(env: Optional[Mapping[str, str]] = None,
                        world_rank: int = 0,
                        ndev: Optional[int] = None) -> int:
    """Node-local rank used for ``hipSetDevice`` binding (one process per GPU)."""
    e = _env(env)
    for key in ("OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID", "LOCAL_RANK", "MPI_LOCALRANKID"):
        v = e.get(key)
        if v not in (None, ""):
            return int(v)
    if ndev:
        return world_rank % ndev
    return 0


def parse_slurm_tasks_per_node(spec: str) -> list:
    """Expand SLURM's compressed per-node task counts (``SLURM_TASKS_PER_NODE``
    / ``SLURM_STEP_TASKS_PER_NODE``): ``"8(x2)"`` -> [8, 8], ``"4,2"`` -> [4, 2],
    ``"2(x3),1"`` -> [2, 2, 2, 1]. Raises ValueError on anything else."""
    out = []
    for part in spec.strip().split(","):
        part = part.strip()
        if not part:
            raise ValueError(f"bad task count list {spec!r}")
        if part.endswith(")") and "(x" in part:
            n, rep = part[:-1].split("(x", 1)
            out += [int(n)] * int(rep)
        else:
            out.append(int(part))
    if not out or min(out) < 1:
        raise ValueError(f"bad task count list {spec!r}")
    return out


def local_size_from_env(env: Optional[Mapping[str, str]] = None) -> Optional[int]:
    """Number of ranks on this node, when the launcher says (torchrun
    ``LOCAL_WORLD_SIZE``, Open MPI ``OMPI_COMM_WORLD_LOCAL_SIZE``, MPICH
    ``MPI_LOCALNRANKS``, SLURM ``SLURM_NTASKS_PER_NODE`` or the per-node lists
    ``SLURM_STEP_TASKS_PER_NODE`` / ``SLURM_TASKS_PER_NODE`` indexed by
    ``SLURM_NODEID``, e.g. ``8(x2)``); None if unknown.

    A plain ``srun`` exports only the lists (the reference's primary launcher
    path, /root/reference/utils.py:17-20), so without them the device-bound
    RCCL world (ncclCommSplit trial groups) would never turn on under SLURM."""
    e = _env(env)
    for key in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE"):
        v = e.get(key)
        if v not in (None, ""):
            try:
                return int(v)
            except ValueError:  # e.g. SLURM's "8(x2)"
                continue
    for key in ("SLURM_STEP_TASKS_PER_NODE", "SLURM_TASKS_PER_NODE"):
        v = e.get(key)
        if v in (None, ""):
            continue
        try:
            counts = parse_slurm_tasks_per_node(v)
        except ValueError:
            continue
        try:
            node = int(e.get("SLURM_NODEID", ""))
        except ValueError:  # unset or malformed: fall through to the same-count rule
            node = -1
        if 0 <= node < len(counts):
            return counts[node]
        if len(set(counts)) == 1:  # same count on every node: the node id does not matter
            return counts[0]
    return None


def parse_slurm_nodelist(nodelist: str):
    """Expand a SLURM compressed host list.

    ``"or-condo-g[05,07-08,13],or-condo-h[01,12]"`` -> 6 hosts, zero padding of
    range starts preserved (parity: /root/reference/utils.py:59-90).
    Written as a small bracket-aware tokenizer rather than a regex pass.
    """
    hosts = []
    i, n = 0, len(nodelist)
    while i < n:
        # read a prefix up to '[' or ','
        j = i
        while j < n and nodelist[j] not in "[,":
            j += 1
        prefix = nodelist[i:j]
        if j < n and nodelist[j] == "[":
            k = nodelist.index("]", j)
            body = nodelist[j + 1:k]
            for part in body.split(","):
                part = part.strip()
                if not part:
                    continue
                if "-" in part:
                    lo, hi = part.split("-", 1)
                    width = len(lo)
                    for v in range(int(lo), int(hi) + 1):
                        hosts.append(f"{prefix}{v:0{width}d}")
                else:
                    hosts.append(prefix + part)
            j = k + 1
            # tolerate a suffix after the bracket: "node[1-2]-ib" (rare); the
            # reference drops it too, so we do the same.
            while j < n and nodelist[j] != ",":
                j += 1
        elif prefix:
            hosts.append(prefix)
        i = j + 1 if j < n and nodelist[j] == "," else j
        if j >= n:
            break
    return hosts


def find_ifname(myaddr: str):
    """NIC owning ``myaddr`` (hostname or IP), for ``GLOO_SOCKET_IFNAME``.

    Parity: /root/reference/utils.py:40-56. Returns ``None`` if not found.
    """
    import psutil

    try:
        ipaddr = socket.gethostbyname(myaddr)
    except OSError:
        return None
    for nic, addrs in psutil.net_if_addrs().items():
        for addr in addrs:
            if addr.address == ipaddr:
                return nic
    return None


def discover_master(env: Optional[Mapping[str, str]] = None):
    """(master_addr, master_port) with LSF/SLURM overrides.

    Defaults ``127.0.0.1:8889``; ``LSB_HOSTS`` second token (Summit, first is
    the batch node), else ``LSB_MCPU_HOSTS`` third token, else first host of
    ``SLURM_NODELIST`` (parity: /root/reference/utils.py:108-119).
    """
    e = _env(env)
    addr = e.get("MASTER_ADDR", "127.0.0.1")
    port = e.get("MASTER_PORT", "8889")
    if e.get("LSB_HOSTS") is not None:
        addr = e["LSB_HOSTS"].split()[1]
    elif e.get("LSB_MCPU_HOSTS") is not None:
        addr = e["LSB_MCPU_HOSTS"].split()[2]
    elif e.get("SLURM_NODELIST") is not None:
        addr = parse_slurm_nodelist(e["SLURM_NODELIST"])[0]
    return addr, port


@dataclass(frozen=True)
class LaunchInfo:
    world_size: int
    world_rank: int
    local_rank: int
    master_addr: str
    master_port: str
    launcher: str
    local_size: Optional[int] = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


def _launcher_name(e: Mapping[str, str]) -> str:
    if e.get("OMPI_COMM_WORLD_SIZE") and e.get("OMPI_COMM_WORLD_RANK"):
        return "ompi"
    if e.get("SLURM_NPROCS") and e.get("SLURM_PROCID"):
        return "slurm"
    if e.get("WORLD_SIZE") and e.get("RANK"):
        return "torchrun"
    return "single"


def discover(env: Optional[Mapping[str, str]] = None, ndev: Optional[int] = None) -> LaunchInfo:
    e = _env(env)
    ws, wr = init_comm_size_and_rank(e)
    addr, port = discover_master(e)
    lr = local_rank_from_env(e, wr, ndev)
    return LaunchInfo(ws, wr, lr, addr, port, _launcher_name(e), local_size_from_env(e))


def cu_split_mask(local_rank: int, local_size: int, device: int = 0, ncu: int = 256) -> str:
    """``HSA_CU_MASK`` value giving local rank r of s ranks that share ONE GPU
    the disjoint CU range [r*ncu/s, (r+1)*ncu/s) of device ``device``."""
    if local_size < 1 or not 0 <= local_rank < local_size:
        raise ValueError(f"bad local rank {local_rank} of {local_size}")
    per = ncu // local_size
    lo = local_rank * per
    return f"{device}:{lo}-{lo + per - 1}"


def apply_cu_split(env: Optional[Mapping[str, str]] = None) -> Optional[str]:
    """Rehearsal helper (``MDT_CU_SPLIT=1``): several ranks sharing one GPU each
    get a disjoint share of its compute units through ``HSA_CU_MASK``, so one
    rank's collective jobs spinning on a peer's flags can never occupy the CUs
    that peer needs to produce them (on a real node every rank owns a GPU and
    this is off). Must run before the process initialises HIP; returns the
    mask set, or None."""
    e = _env(env)
    if e.get("MDT_CU_SPLIT", "0") != "1":
        return None
    size = local_size_from_env(e)
    if not size or size <= 1:
        return None
    mask = cu_split_mask(local_rank_from_env(e, init_comm_size_and_rank(e)[1], None), size)
    os.environ["HSA_CU_MASK"] = mask
    return mask
