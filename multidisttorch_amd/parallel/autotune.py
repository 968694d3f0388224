"""Measured bucket-size selection for intra-group gradient all-reduce over xGMI.

The reference uses torch DDP's fixed 25 MiB / 1 MiB-first buckets
(/root/reference/vae-hpo.py:130). On an 8x MI355X node a group of s GPUs
all-reduces over s-1 point-to-point xGMI links, and the best bucket size
depends on the group size, the model's gradient-ready profile and RCCL's
small-message latency. ``plan_buckets`` (ddp.py) gives the cost-model guess;
this module *measures*: every candidate layout is timed on a throw-away
trainer of the same configuration (so the real trial's state is untouched),
the per-rank times are max-reduced over the group so every member picks the
same layout, and the winner is cached per (model, group size, batch, arena).
``autotune_comm`` searches the reducer too: RCCL's ring (``rccl``) against the
one-shot hipIpc push over all s-1 xGMI links (``p2p1``), the same push fused
into the step's own launches (``xgmi``, csrc/kernels/comm_jobs.h) and, for
groups of 3+, the two-shot reduce-scatter + all-gather form (``p2p2``) and the
mixed one (``p2p``: two-shot for big buckets only), for every layout, when the
group is on GPUs of one node.
"""

from __future__ import annotations

import json
import os
import socket
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .ddp import make_arena_reducer

__all__ = ["autotune_buckets", "autotune_comm", "bucket_cache_path", "parse_bucket_mb", "comm_kinds"]


def bucket_cache_path() -> str:
    return os.getenv("MDT_BUCKET_CACHE",
                     os.path.join(os.path.expanduser("~"), ".cache", "multidisttorch_amd", "buckets.json"))


def parse_bucket_mb(v) -> Optional[object]:
    """'auto' | '' / None (default layout) | number (MiB cap, 0 = one bucket)."""
    if v is None or v == "":
        return None
    if isinstance(v, str) and v.lower() == "auto":
        return "auto"
    return float(v)


def _load_cache(path: str) -> Dict[str, dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _store_cache(path: str, key: str, entry: dict) -> None:
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        data = _load_cache(path)
        data[key] = entry
        tmp = path + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        os.replace(tmp, path)
    except OSError:
        pass


def comm_kinds(pg, device: torch.device) -> List[Optional[str]]:
    """Reducer kinds worth timing for this group: RCCL and the hipIpc p2p push
    (one-shot; two-shot too for groups of 3+, where it halves the bytes per
    link or better) when every member drives a GPU of the same node;
    otherwise the default."""
    if device.type != "cuda" or not dist.is_initialized() or dist.get_backend(pg) != "nccl":
        return [None]
    hosts = [None] * dist.get_world_size(pg)
    dist.all_gather_object(hosts, socket.gethostname(), group=pg)
    if len(set(hosts)) != 1:
        return ["rccl"]
    # groups of 3+: the mixed "p2p" kind (two-shot only for buckets >= MDT_P2P_TWO_SHOT_MB)
    # as well as all-one-shot and all-two-shot, and the fused jobs in both forms
    return ["rccl", "p2p1", "xgmi1"] + (["p2p", "p2p2", "xgmi2"] if len(hosts) >= 3 else [])


def autotune_buckets(make_trainer: Callable[[], object], pg, X: torch.Tensor, idx: torch.Tensor,
                     candidates: Sequence = (None, 0, 1, 2, 4, 8, 16), steps: int = 6, warmup: int = 2,
                     key: Optional[str] = None, cache: Optional[str] = None,
                     use_cache: bool = True) -> Tuple[List[int], Dict[str, float]]:
    """Time each candidate bucket layout with the default reducer; return
    (best bounds, {layout: seconds}). See ``autotune_comm``."""
    bounds, _, timings = autotune_comm(make_trainer, pg, X, idx, candidates, steps, warmup, key, cache,
                                       use_cache, kinds=[None])
    return bounds, timings


def autotune_comm(make_trainer: Callable[[], object], pg, X: torch.Tensor, idx: torch.Tensor,
                  candidates: Sequence = (None, 0, 1, 2, 4, 8, 16), steps: int = 6, warmup: int = 2,
                  key: Optional[str] = None, cache: Optional[str] = None, use_cache: bool = True,
                  kinds: Optional[Sequence[Optional[str]]] = None
                  ) -> Tuple[List[int], Optional[str], Dict[str, float]]:
    """Time every (reducer kind, bucket layout) pair; return (bounds, kind, timings).

    ``make_trainer()`` builds a fresh trainer with the real trial's config;
    candidate ``c`` becomes ``trainer.bucket_bounds(c)`` (duplicates collapse).
    ``kinds`` defaults to ``comm_kinds(pg, device)``; ``None`` = the default reducer.
    Collective: every member of ``pg`` must call with the same arguments.
    """
    tr = make_trainer()
    gsize = dist.get_world_size(pg) if dist.is_initialized() else 1
    cache = cache or bucket_cache_path()
    if kinds is None:
        kinds = comm_kinds(pg, tr.device)
    kinds = list(kinds)
    ckey = None if key is None else (key if kinds == [None] else f"{key}-{'+'.join(map(str, kinds))}")
    if ckey is not None and use_cache:
        hit = _load_cache(cache).get(ckey)
        if hit is not None and hit.get("group_size") == gsize:
            return list(hit["bounds"]), hit.get("kind"), dict(hit.get("timings", {}))
    layouts, seen = [], set()
    for c in candidates:
        b = tuple(int(x) for x in tr.bucket_bounds(c))
        if b not in seen:
            seen.add(b)
            layouts.append(list(b))
    B = tr.B
    nb = max(1, idx.numel() // B)
    tr.bind_train_data(X, idx)
    dev = tr.device
    on_gpu = dev.type == "cuda"
    t_dev = dev if (on_gpu and dist.is_initialized() and dist.get_backend(pg) == "nccl") else torch.device("cpu")
    timings: Dict[str, float] = {}
    best, best_kind, best_t = layouts[0], kinds[0], float("inf")
    for kind in kinds:
        for bounds in layouts:
            tr.set_cursor(0, nb)
            # the previous reducer is dropped here: every member finished its kernels
            # before the MAX all-reduce below, so no peer still writes into its region
            tr.attach_reducer(make_arena_reducer(pg, tr.grads, bounds, kind=kind))
            # graphs for this layout are captured here, outside the timer; a
            # replay that misses one raises instead of capturing while timed
            if hasattr(tr, "prepare"):
                tr.prepare([B])
                tr.strict_graphs = bool(getattr(tr, "use_graphs", False))
            tr.train_steps(warmup)
            if on_gpu:
                torch.cuda.synchronize(dev)
            if gsize > 1:
                dist.barrier(group=pg)
            t0 = time.perf_counter()
            tr.train_steps(steps)
            if on_gpu:
                torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            t = torch.tensor([dt], dtype=torch.float64 if t_dev.type == "cpu" else torch.float32, device=t_dev)
            if gsize > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
            dt = float(t.item()) / steps
            label = ",".join(map(str, bounds))
            timings[label if kind is None else f"{kind}:{label}"] = dt
            if dt < best_t:
                best, best_kind, best_t = bounds, kind, dt
    tr.attach_reducer(None)
    if ckey is not None and (not dist.is_initialized() or dist.get_rank(pg) == 0):
        _store_cache(cache, ckey, {"bounds": best, "kind": best_kind, "timings": timings, "group_size": gsize,
                                   "when": time.strftime("%Y-%m-%dT%H:%M:%S")})
    return best, best_kind, timings
