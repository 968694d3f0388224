"""``mdtrun``: single-node launcher, one process per GPU.

    python -m multidisttorch_amd.launch -n 8 [--emulate {torchrun,slurm,ompi}] script.py args...

Sets the launcher environment the runtime discovers (SURVEY.md §2.2 env
contract): torchrun-style ``RANK/WORLD_SIZE/LOCAL_RANK`` by default, or the
variables SLURM (``SLURM_NPROCS/SLURM_PROCID/SLURM_LOCALID/SLURM_NODELIST``)
or Open MPI / jsrun (``OMPI_COMM_WORLD_SIZE/RANK/LOCAL_RANK``) would set —
the same emulation technique the survey used to exercise the reference's
code paths without a cluster. Always ``MASTER_ADDR=127.0.0.1``.

Failure handling: if any rank exits non-zero the others are terminated (their
process group only: each child runs in its own session) and the launcher
exits with that code; ``--timeout`` bounds the whole job.
"""

from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, emulate: str = "torchrun",
             base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "SLURM_NPROCS", "SLURM_PROCID", "SLURM_LOCALID",
              "SLURM_NODELIST", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_LOCAL_RANK",
              "LSB_HOSTS", "LSB_MCPU_HOSTS"):
        env.pop(k, None)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["MASTER_PORT"] = str(port)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # CPU ranks share the host: split the intra-op threads instead of oversubscribing
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // max(1, world))))
    if emulate == "torchrun":
        env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    elif emulate == "slurm":
        env.update(SLURM_NPROCS=str(world), SLURM_PROCID=str(rank), SLURM_LOCALID=str(rank),
                   SLURM_NODELIST="localhost")
    elif emulate == "ompi":
        env.update(OMPI_COMM_WORLD_SIZE=str(world), OMPI_COMM_WORLD_RANK=str(rank),
                   OMPI_COMM_WORLD_LOCAL_RANK=str(rank))
    else:
        raise ValueError(f"unknown launcher emulation {emulate!r}")
    return env


def launch(cmd: List[str], nproc: int, emulate: str = "torchrun", port: Optional[int] = None,
           timeout: Optional[float] = None, extra_env: Optional[Dict[str, str]] = None,
           capture: bool = False):
    """Run ``cmd`` on ``nproc`` local ranks. Returns (exit_code, outputs-or-None)."""
    port = port or free_port()
    procs = []
    for r in range(nproc):
        env = rank_env(r, nproc, port, emulate)
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True,
                                      stdout=subprocess.PIPE if capture else None,
                                      stderr=subprocess.STDOUT if capture else None,
                                      text=capture))
    t0 = time.time()
    rc = 0
    outs = [None] * nproc
    try:
        pending = set(range(nproc))
        while pending:
            for r in list(pending):
                p = procs[r]
                if capture:
                    try:
                        out, _ = p.communicate(timeout=0.05)
                        outs[r] = out
                    except subprocess.TimeoutExpired:
                        pass
                code = p.poll()
                if code is not None:
                    pending.discard(r)
                    if code != 0 and rc == 0:
                        rc = code
                        _kill(procs)
            if timeout is not None and time.time() - t0 > timeout:
                rc = rc or 124
                _kill(procs)
                break
            if not capture:
                time.sleep(0.05)
    finally:
        _kill(procs, only_alive=True)
    if capture:
        for r, p in enumerate(procs):
            if outs[r] is None:
                try:
                    outs[r], _ = p.communicate(timeout=5)
                except Exception:
                    outs[r] = ""
    return rc, outs if capture else None


def _kill(procs, only_alive=False):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + 5
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mdtrun")
    ap.add_argument("-n", "--nproc", type=int, default=1)
    ap.add_argument("--emulate", default="torchrun", choices=["torchrun", "slurm", "ompi"])
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = [sys.executable, a.script] + a.args
    rc, _ = launch(cmd, a.nproc, a.emulate, a.port, a.timeout)
    sys.exit(rc)


if __name__ == "__main__":
    main()
