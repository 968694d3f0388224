"""Intra-group data parallelism over a flat gradient arena.

Reference: ``DistributedDataParallel(model, process_group=group)``
(/root/reference/vae-hpo.py:130) with torch's defaults — 25 MiB buckets, a
1 MiB first bucket, per-parameter copies into bucket storage and back into
``.grad`` after the all-reduce.

MI355X-first design:
  * gradients live in ONE contiguous arena; each ``param.grad`` is a view into
    it, so buckets are [begin, end) slices and RCCL reduces them in place;
  * bucket boundaries come from an xGMI cost model (``plan_buckets``): in a
    group of s GPUs on a fully connected 8-GPU xGMI mesh a ring uses ONE
    ~153 GB/s link per GPU, so per-bucket time is alpha + 2(s-1)/s * bytes/BW;
    buckets are sized so each one's transfer hides behind the backward compute
    that follows it, and tiny models get 1-2 buckets (latency-bound regime);
  * the collectives are issued natively: on GPU by ``RcclBucketReducer``
    (csrc/runtime/xgmi_comm.cpp) directly on the trial group's RCCL
    communicator (PreMulSum(1/s) averaging, high-priority comm stream, event
    fences, graph-capturable); on gloo (CPU tests) by the c10d-based
    ``BucketReducer`` (csrc/runtime/reducer.cpp).
"""

from __future__ import annotations

import math
import os
import sys
from typing import Dict, Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist
from torch import nn

from ..ops import native

__all__ = ["XgmiModel", "plan_buckets", "make_arena_reducer", "PyBucketReducer", "ArenaDDP",
           "broadcast_params", "rccl_comm_ptr", "reducer_kind", "make_p2p_reducer", "P2P_KINDS",
           "two_shot_min_bytes", "group_on_one_node", "overlap_pays", "graph_capturable",
           "XGMI_KINDS", "verify_group_agreement", "selftest_fused", "SELFTEST_LOG"]


class XgmiModel:
    """Cost model of a ring all-reduce inside a contiguous group on 8x MI355X."""

    def __init__(self, link_gbps: float = 153.0, alpha_us: float = 12.0, channels: int = 1):
        self.link = link_gbps * 1e9
        self.alpha = alpha_us * 1e-6
        self.channels = channels

    def allreduce_s(self, nbytes: int, group_size: int) -> float:
        if group_size <= 1:
            return 0.0
        s = group_size
        # RCCL on a full mesh can run several rings over distinct links; a
        # single ring is per-link bound. `channels` = usable disjoint rings.
        bw = self.link * max(1, min(self.channels, s - 1))
        return 2 * (s - 1) * self.alpha / max(1, s - 1) + 2 * (s - 1) / s * nbytes / bw


def plan_buckets(param_bytes: Sequence[int], group_size: int, bwd_compute_s: Optional[Sequence[float]] = None,
                 cap_bytes: int = 8 << 20, first_bytes: int = 1 << 20,
                 model: Optional[XgmiModel] = None) -> List[List[int]]:
    """Group parameter indices (in gradient-READY order) into buckets.

    Greedy: close a bucket when it reaches the cap, or when the remaining
    backward compute after this point can no longer hide a bigger transfer.
    Without compute estimates: torch-like first bucket, then `cap_bytes`.
    """
    model = model or XgmiModel()
    n = len(param_bytes)
    buckets, cur, cur_b = [], [], 0
    remaining = list(bwd_compute_s) if bwd_compute_s is not None else None
    for i, b in enumerate(param_bytes):
        cur.append(i)
        cur_b += b
        limit = first_bytes if not buckets else cap_bytes
        close = cur_b >= limit
        if remaining is not None and not close:
            rest = sum(remaining[i + 1:])
            # stop growing once this bucket's comm would exceed what is left to hide behind
            close = model.allreduce_s(cur_b, group_size) >= rest and cur_b >= (256 << 10)
        if close:
            buckets.append(cur)
            cur, cur_b = [], 0
    if cur:
        buckets.append(cur)
    return buckets


class PyBucketReducer:
    """Pure-Python reducer with the BucketReducer API (fallback when _C is absent)."""

    def __init__(self, pg, flat: torch.Tensor, bounds: Sequence[int], average: bool):
        self.pg, self.flat, self._bounds, self.average = pg, flat, list(bounds), average
        self.world = dist.get_world_size(pg)
        self.work = [None] * (len(self._bounds) - 1)
        self.param_bucket, self.need, self.have = [], [], []
        self._launched = 0
        self.use_avg = average and flat.is_cuda

    def num_buckets(self):
        return len(self._bounds) - 1

    def bounds(self):
        return list(self._bounds)

    def launch(self, b):
        if self.world == 1:
            return
        assert self.work[b] is None, f"bucket {b} launched twice"
        v = self.flat[self._bounds[b]:self._bounds[b + 1]]
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        self.work[b] = dist.all_reduce(v, op=op, group=self.pg, async_op=True)
        self._launched += 1

    def wait(self, b):
        w = self.work[b]
        if w is None:
            return
        w.wait()
        self.work[b] = None
        if self.average and not self.use_avg:
            self.flat[self._bounds[b]:self._bounds[b + 1]].div_(self.world)

    def launch_all(self):
        for b in range(self.num_buckets()):
            if self.work[b] is None:
                self.launch(b)

    def wait_all(self):
        for b in range(self.num_buckets()):
            self.wait(b)

    def set_param_map(self, pb):
        self.param_bucket = list(pb)
        self.need = [0] * self.num_buckets()
        for b in pb:
            self.need[b] += 1
        self.have = [0] * self.num_buckets()

    def mark_ready(self, p):
        b = self.param_bucket[p]
        self.have[b] += 1
        if self.have[b] == self.need[b]:
            self.launch(b)

    def reset_iteration(self):
        self.have = [0] * self.num_buckets()

    def pending(self):
        return sum(w is not None for w in self.work)

    def launched_count(self):
        return self._launched


COMM_WARMUPS = [0]  # lazy communicators forced into existence by rccl_comm_ptr (tests assert on it)


def rccl_comm_ptr(pg, device: torch.device) -> int:
    """ncclComm_t (as int) of a trial group's ProcessGroupNCCL on `device`.

    On a device-bound world (the default with one GPU per rank) the group's
    communicator was created eagerly by ``ncclCommSplit`` in ``new_group``
    and is used as is. A lazily created group (ranks sharing a GPU, or
    ``MDT_EAGER_COMM=0``) gets one tiny all-reduce that forces its
    communicator into existence. Either way the native reducer reuses torch's
    communicator: one communicator and one RCCL runtime per group."""
    backend = pg._get_backend(device)
    if not hasattr(backend, "_comm_ptr"):
        raise RuntimeError(f"process group backend {type(backend).__name__} is not RCCL")
    ptr = 0
    if getattr(pg, "bound_device_id", None) is not None:
        try:
            ptr = int(backend._comm_ptr())
        except RuntimeError:
            ptr = 0
    if not ptr:
        COMM_WARMUPS[0] += 1
        t = torch.zeros(1, device=device)
        dist.all_reduce(t, group=pg)
        torch.cuda.current_stream(device).synchronize()
        ptr = int(backend._comm_ptr())
    return ptr


def group_on_one_node(pg) -> bool:
    """True when every member of ``pg`` runs on this host (collective: all
    members call it). Such a group can map its peers' memory over xGMI."""
    import socket

    n = dist.get_world_size(pg)
    if n == 1:
        return True
    hosts = [None] * n
    dist.all_gather_object(hosts, socket.gethostname(), group=pg)
    return len(set(hosts)) == 1


def reducer_kind(pg, flat: torch.Tensor, comm_jobs: bool = True) -> str:
    """'xgmi' (hipIpc push over xGMI fused into the step's launches where the
    model supports it, a one-shot push kernel otherwise), 'rccl' (direct RCCL
    on torch's communicator), 'p2p' (one-shot, two-shot for big buckets of
    groups >= 3), 'p2p1' (one-shot only), 'p2p2' (two-shot only), 'c10d'
    (native reducer over the ProcessGroup) or 'python'. MDT_REDUCER overrides.

    Default on GPU, for a multi-rank group whose members share a node (every
    intra-node group on an 8x MI355X node): 'xgmi' when the trainer puts the
    all-reduce into its own launches (``comm_jobs``: ConvVaeTrainer; one-GPU
    structure cost 1.04x of the reducer-free 28x28 step against 1.12x for
    RCCL on the compute stream, profiles/r4_ddp_fused), 'rccl' when it does not
    (the MLP trainer: RCCL inline 1.16x against 1.39x for the standalone push
    kernel, profiles/r4_ddp_fused/ddp_structure_mlp.json). RCCL for a group
    that spans nodes. Collective (all members call it)."""
    forced = os.getenv("MDT_REDUCER", "")
    if forced:
        return forced
    if not native.available():
        return "python"
    if flat.is_cuda and dist.get_backend(pg) == "nccl":
        if comm_jobs and dist.get_world_size(pg) > 1 and group_on_one_node(pg):
            return "xgmi"
        return "rccl"
    return "c10d"


def make_arena_reducer(pg, flat: torch.Tensor, bounds: Sequence[int], average: bool = True,
                       prefer_native: bool = True, kind: Optional[str] = None, scale: float = 0.0,
                       comm_jobs: bool = True):
    """Bucket reducer over a flat gradient arena ([begin, end) buckets).

    On MI355X trial groups (RCCL) this is the direct-RCCL reducer of
    csrc/runtime/xgmi_comm.cpp: PreMulSum(1/s) averaging fused into the
    collective, a dedicated high-priority comm stream, event fences only.
    gloo groups (CPU tests, control plane) use the c10d-based native reducer.
    ``scale`` (RCCL only) replaces the 1/s pre-multiplier; any scale other
    than 1 issues the collective even on a one-rank group (tests use it to
    put real ``ncclAllReduce`` kernels into a one-GPU step graph).
    ``comm_jobs``: the trainer can host the fused all-reduce jobs (see
    ``reducer_kind``). A peer-to-peer kind whose hipIpc mapping fails on any
    member (e.g. GPU visibility restricted per rank) falls back, on every
    member together, to RCCL (nccl groups) or the c10d reducer.
    """
    if pg is None:
        pg = dist.distributed_c10d._get_default_group()
    kind = kind or (reducer_kind(pg, flat, comm_jobs) if prefer_native else "python")
    b = [int(x) for x in bounds]
    verify_group_agreement(pg, flat, b, kind)
    if kind in XGMI_KINDS or kind in P2P_KINDS:
        red = (make_p2p_reducer(pg, flat, b, average, two_shot=XGMI_KINDS[kind], fused=True, scale=scale)
               if kind in XGMI_KINDS else make_p2p_reducer(pg, flat, b, average, two_shot=P2P_KINDS[kind]))
        if red is not None:
            return red
        kind = "rccl" if dist.get_backend(pg) == "nccl" else "c10d"
        print(f"[mdt] peer mapping or data-plane self-test over xGMI failed in a group of {dist.get_world_size(pg)}: "
              f"falling back to the {kind} reducer", file=sys.stderr, flush=True)
    if kind == "rccl":
        size = dist.get_world_size(pg)
        return native.require().RcclBucketReducer(rccl_comm_ptr(pg, flat.device), size, flat, b, average, scale)
    if kind == "c10d" and native.available():
        return native.require().BucketReducer(pg, flat, b, average)
    if flat.is_cuda:
        native.require()  # on GPU the native reducer is mandatory: fail loudly
    return PyBucketReducer(pg, flat, bounds, average)


def graph_capturable(reducer) -> bool:
    """Whether a reducer's collectives can be captured into a replayed step
    graph: the RCCL and xGMI reducers issue device work only; the c10d/gloo
    reducers block on host-side work objects (a gloo world on GPU tensors,
    e.g. the IPC-failure fallback of a one-GPU rehearsal)."""
    return reducer is None or type(reducer).__name__ not in ("BucketReducer", "PyBucketReducer")


def overlap_pays(first_bucket_bytes: int, split_cost_us: float, link_gbps: float = 153.0) -> bool:
    """Whether issuing the first-ready bucket's all-reduce before the rest of
    the weight gradients (one extra launch boundary / stream hop) pays: only
    when that bucket's transfer over one xGMI link takes longer than the
    measured structure cost of the split (profiles/r4_ddp_fused: +6 us for the
    fused xGMI jobs, +31 us for RCCL on its own stream, per 28x28 step)."""
    return first_bucket_bytes / (link_gbps * 1e9) * 1e6 > split_cost_us


# reducer kind -> two-shot rule: "auto" (buckets >= MDT_P2P_TWO_SHOT_MB, default 4, in groups >= 3),
# "never" (one-shot), "always"
P2P_KINDS = {"p2p": "auto", "p2p1": "never", "p2p2": "always"}
# fused all-reduce jobs (comm_jobs.h): "xgmi" = one-shot (the
# two-shot form has only run with ranks sharing one GPU, so it stays opt-in
# until a multi-GPU record shows it correct and faster); "xgmi2" two-shot for
# every unit; "xgmia" two-shot in groups >= 3 with an arena of at least
# MDT_P2P_TWO_SHOT_MB (default 4: the 12-18 MB 128x128 model); "xgmi1" = "xgmi"
XGMI_KINDS = {"xgmi": "never", "xgmi1": "never", "xgmi2": "always", "xgmia": "auto"}

# construction-time self-test records of the fused data plane, newest last:
# {"result": "ok" | "fallback" | "skipped", "ms": float, "two_shot": bool, "status": [...]}
SELFTEST_LOG: List[dict] = []


def _desc_code(x) -> int:
    import zlib

    return zlib.crc32(repr(x).encode()) & 0x7FFFFFFF


def verify_group_agreement(pg, flat: torch.Tensor, bounds: Sequence[int], kind: str):
    """Every member of ``pg`` must build the same reducer before any gradient
    moves: arena numel and dtype, bucket bounds, reducer kind and its
    two-shot threshold. The fused xGMI jobs store into a peer's region by
    ARENA OFFSET, so a size or layout mismatch would be out-of-bounds remote
    writes on another GPU, and RCCL would hang on unequal counts; here it is a
    RuntimeError on EVERY member, naming the ranks that differ from group
    rank 0. Collective (all members call it).

    Reference counterpart: DDP's constructor verifies parameter shapes across
    the group and broadcasts their metadata before the first all-reduce
    (``_verify_param_shape_across_processes`` + metadata broadcast under
    /root/reference/vae-hpo.py:130)."""
    if pg is None or not dist.is_initialized():
        return
    s = dist.get_world_size(pg)
    if s == 1:
        return
    rule = XGMI_KINDS.get(kind, P2P_KINDS.get(kind, "never"))
    fields = ["numel", "dtype", "nbuckets", "bounds", "kind", "two_shot_min_bytes"]
    mine = [flat.numel(), _desc_code(str(flat.dtype)), len(bounds) - 1, _desc_code(tuple(int(x) for x in bounds)),
            _desc_code(kind), two_shot_min_bytes(rule, s)]
    on_dev = flat.is_cuda and dist.get_backend(pg) == "nccl"
    t = torch.tensor(mine, dtype=torch.int64, device=flat.device if on_dev else "cpu")
    got = [torch.empty_like(t) for _ in range(s)]
    dist.all_gather(got, t, group=pg)
    rows = [g.cpu().tolist() for g in got]
    bad = [(q, [f for f, a, b in zip(fields, rows[q], rows[0]) if a != b]) for q in range(1, s) if rows[q] != rows[0]]
    if bad:
        detail = "; ".join(f"group rank {q} differs in {', '.join(f)}" for q, f in bad)
        raise RuntimeError(f"intra-group reducer disagreement (this is group rank {dist.get_rank(pg)}): {detail} "
                           f"(group rank 0: numel {rows[0][0]}, {rows[0][2]} buckets, kind {kind!r} here)")


def _members_share_a_device(pg, dev: torch.device) -> bool:
    """True when two members of ``pg`` run on the same physical GPU (host +
    PCI location; one-GPU multi-rank rehearsals). Collective."""
    import socket
    import zlib

    p = torch.cuda.get_device_properties(dev)
    me = [zlib.crc32(socket.gethostname().encode()), p.pci_domain_id, p.pci_bus_id, p.pci_device_id]
    t = torch.tensor(me, dtype=torch.int64, device=dev if dist.get_backend(pg) == "nccl" else "cpu")
    got = [torch.empty_like(t) for _ in range(dist.get_world_size(pg))]
    dist.all_gather(got, t, group=pg)
    ids = [tuple(g.tolist()) for g in got]
    return len(set(ids)) < len(ids)


def selftest_fused(red, pg, flat: torch.Tensor, timeout_s: Optional[float] = None) -> bool:
    """Data-plane self-test of a connected fused xGMI reducer, before any real
    gradient moves: one push+reduce of a rank-coded pattern over the whole
    arena through the production jobs (``comm_unit_body`` in a
    ``jobs_multi_k`` launch, the production peer mappings, layout and 1/s
    scale), one-shot and -- when the reducer selected it -- two-shot, each with
    a ``timeout_s`` (default 2 s, ``MDT_XGMI_SELFTEST_TIMEOUT_S``) bound on
    every wait. The result must be BITWISE the rank-order sum x scale on every
    member (the pattern's values are exact in f32 at any group size), and
    the verdict is MIN-reduced over the group, so all members keep the fused
    reducer or all fall back together. On success the reducer's epochs are
    moved past the two used here. Collective."""
    C = native.require()
    s, r = dist.get_world_size(pg), dist.get_rank(pg)
    timeout_s = timeout_s or float(os.getenv("MDT_XGMI_SELFTEST_TIMEOUT_S", "2"))
    dev, n = flat.device, flat.numel()
    import time

    from ..runtime.faults import injected_rank

    t0 = time.perf_counter()
    marks = {}

    def mark(k):
        marks[k] = round((time.perf_counter() - t0) * 1e3, 2)

    # the rank-coded pattern (integers in [-2046, 2046] x 2^-6: any rank-order
    # sum of <= 8 is exact) and the bitwise check against sum x scale are
    # kernels of the extension (p2p_allreduce.hip: selftest_fill_k /
    # selftest_check_k) -- no framework kernel is loaded for the test
    G = torch.empty(n, dtype=torch.float32, device=dev)
    segs = C.make_grad_segs([[0, n, 0, 1, 0, 0, 0, 0, -1]], dev.index or 0)
    units = [[0, u, min(1024, n - u)] for u in range(0, n, 1024)]
    units_t = C.make_grad_units(units, dev.index or 0)
    state = C.TrialState(dev.index or 0)
    forms = [False] + ([True] if red.fused_two_shot() else [])
    on_dev = dist.get_backend(pg) == "nccl"
    # members on distinct devices (the production layout) run push+reduce in
    # ONE workgroup per unit, as the step's tail does; members that share a
    # device (one-GPU rehearsals) push, meet at a host barrier, then reduce --
    # a spinning reduce must not hold the CUs a co-located peer's push needs
    mark("setup")
    shared = _members_share_a_device(pg, dev)
    mark("identity")
    ok, statuses = True, []

    def run(mode, G, ctx):
        job = C.Job()
        C.comm_job(G, G, G, G, G, segs, units_t, len(units), state.train_state, state.hparams, False, ctx, mode, job)
        pack, grid = C.pack_jobs_multi([job])
        C.launch_jobs_multi(pack.to(dev), grid)

    for k, two in enumerate(forms):
        red.selftest_fill(G, r)
        state.set_step(False, k + 1)  # epoch k + 1 (ctx ep_base 0)
        ctx = red.selftest_ctx(timeout_s, two)
        if shared:
            run(1, G, ctx)
            torch.cuda.synchronize(dev)
            dist.barrier(group=pg)
            run(2, G, ctx)
        else:
            run(3, G, ctx)
        st = int(red.selftest_status(ctx))  # syncs the device
        statuses.append(st)
        ok = ok and st == 0 and int(red.selftest_check(G)) == 0
        mark(f"form{k}")
    if injected_rank("XGMI_SELFTEST_FAIL") == r:
        ok = False
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if on_dev else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=pg)
    agreed = int(flag.item()) == 1
    mark("verdict")
    if agreed:
        red.rebase_epochs(len(forms), 0)  # the trainer's first epoch lands past the self-test's
    ms = (time.perf_counter() - t0) * 1e3
    SELFTEST_LOG.append({"result": "ok" if agreed else "fallback", "ms": round(ms, 2), "two_shot": len(forms) > 1,
                         "status": statuses, "local_ok": ok, "group_size": s,
                         "form": "push|barrier|reduce" if shared else "push+reduce", "marks_ms": marks})
    if not agreed:
        print(f"[mdt] group rank {r}: xGMI data-plane self-test failed on "
              f"{'this rank' if not ok else 'a peer'} (status {statuses}, {ms:.1f} ms): falling back",
              file=sys.stderr, flush=True)
    return agreed


def two_shot_min_bytes(rule: str, group_size: int) -> int:
    """Smallest bucket (bytes) the p2p reducer runs two-shot; -1 = never.

    Per link, one-shot moves the whole bucket and two-shot 2/s of it for one
    extra hop: at s = 2 the bytes are equal, so "auto" keeps one-shot there."""
    if rule == "always":
        return 0
    if rule == "never" or group_size < 3:
        return -1
    return int(float(os.getenv("MDT_P2P_TWO_SHOT_MB", "4")) * (1 << 20))


def make_p2p_reducer(pg, flat: torch.Tensor, bounds: Sequence[int], average: bool = True,
                     max_blocks: Optional[int] = None, timeout_s: Optional[float] = None, two_shot: str = "auto",
                     fused: bool = False, scale: float = 0.0):
    """Peer-to-peer bucket all-reduce over xGMI (csrc/runtime/p2p_comm.cpp).

    Every group member allocates an uncached receive region, exports it with
    hipIpcGetMemHandle, and the 64-byte handles are all-gathered over the group
    itself; each rank then maps its peers' regions. A bucket is pushed to all
    s-1 peers at once (one xGMI hop, every link of the group busy) instead of
    RCCL's ring (2(s-1) hops over one link per step) -- the regime of the
    VAE models' 1-4 MB buckets. Big buckets run two-shot instead
    (reduce-scatter to chunk owners + all-gather, 2/s of the bucket per link;
    ``two_shot``: "auto" | "never" | "always", see ``two_shot_min_bytes``).
    Before that, every member checks collectively that all exported their
    region (nobody opens a zero handle), then that all mapped every peer;
    a fused reducer then passes ``selftest_fused`` (a real push+reduce over
    the mappings, bitwise-checked) before it is returned.
    All ranks of the group must share one node. Selected with
    ``MDT_REDUCER=p2p`` (or ``kind="p2p"/"p2p1"/"p2p2"``). Returns None on
    every member when any member could not map a peer's region (the caller
    falls back to another reducer).
    ``fused`` (kind "xgmi") also allocates the receive slots of the all-reduce
    JOBS (csrc/kernels/comm_jobs.h) that models with their own backward
    launches (ConvVaeTrainer) put into those launches: one stream, no events;
    ``scale`` replaces the 1/s pre-multiplier (tests).
    """
    if not flat.is_cuda:
        raise RuntimeError("the p2p reducer needs a GPU gradient arena")
    C = native.require()
    s, r = dist.get_world_size(pg), dist.get_rank(pg)
    max_blocks = max_blocks or int(os.getenv("MDT_P2P_BLOCKS", "64"))
    timeout_s = timeout_s or float(os.getenv("MDT_P2P_TIMEOUT_S", "60"))
    from ..runtime.faults import injected_rank

    red = C.XgmiP2PReducer(r, s, flat, [int(x) for x in bounds], average, float(scale), max_blocks, timeout_s,
                           two_shot_min_bytes(two_shot, s), fused)
    if s == 1:
        return red
    on_dev = dist.get_backend(pg) == "nccl"

    def agree(ok: int) -> bool:  # MIN over the group: every member takes the same branch
        flag = torch.tensor([ok], dtype=torch.int32, device=flat.device if on_dev else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=pg)
        return int(flag.item()) == 1

    ok = 1
    try:
        h = red.ipc_handle()
    except RuntimeError as e:
        ok, h = 0, torch.zeros(64, dtype=torch.uint8)
        print(f"[mdt] group rank {r}: cannot export the receive region: {e}", file=sys.stderr, flush=True)
    # a failed export anywhere: nobody opens a handle (an all-zero one included)
    if not agree(ok):
        return None
    if on_dev:
        h = h.to(flat.device)
    hs = [torch.empty_like(h) for _ in range(s)]
    dist.all_gather(hs, h, group=pg)
    # every peer zeroed its region (the ctor syncs the device) before publishing its handle
    try:
        if injected_rank("IPC_FAIL") == r:
            raise RuntimeError("injected hipIpcOpenMemHandle failure (MDT_TEST_IPC_FAIL_RANK)")
        red.connect([x.cpu() for x in hs])
    except RuntimeError as e:
        ok = 0
        print(f"[mdt] group rank {r}: cannot map a peer's memory: {e}", file=sys.stderr, flush=True)
    if not agree(ok):
        return None
    if fused and os.getenv("MDT_XGMI_SELFTEST", "1") != "0":
        if not selftest_fused(red, pg, flat):
            return None
    elif fused:
        SELFTEST_LOG.append({"result": "skipped", "ms": 0.0, "two_shot": bool(red.fused_two_shot()), "status": [],
                             "local_ok": True, "group_size": s})
    return red


@torch.no_grad()
def broadcast_params(tensors: Iterable[torch.Tensor], pg, src_group_rank: int = 0):
    """Sync replicas from group rank ``src`` (DDP's _sync_module_states)."""
    if pg is None or dist.get_world_size(pg) == 1:
        return
    src = dist.get_global_rank(pg, src_group_rank)
    for t in tensors:
        dist.broadcast(t, src=src, group=pg)


class ArenaDDP(nn.Module):
    """Data-parallel wrapper for generic modules with arena gradients.

    After construction every ``p.grad`` is a view into ``self.grad_arena``
    (laid out in reverse registration order = gradient-ready order, as torch
    DDP's rebuilt buckets). A post-accumulate hook per parameter marks it ready;
    a bucket's all-reduce launches the moment its last gradient lands, while
    autograd continues with earlier layers.
    """

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 8.0,
                 first_bucket_mb: float = 1.0, broadcast: bool = True, average: bool = True):
        super().__init__()
        self.module = module
        self.pg = process_group
        params = [p for p in module.parameters() if p.requires_grad]
        self._params = params
        order = list(reversed(range(len(params))))  # ready order
        dev = params[0].device
        dtype = params[0].dtype
        sizes = [params[i].numel() for i in order]
        offs, off = {}, 0
        for i, n in zip(order, sizes):
            offs[i] = off
            off += (n + 63) // 64 * 64
        self.grad_arena = torch.zeros(off, dtype=dtype, device=dev)
        for i, p in enumerate(params):
            p.grad = self.grad_arena[offs[i]:offs[i] + p.numel()].view_as(p)
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        buckets = plan_buckets([params[i].numel() * params[i].element_size() for i in order], self.world,
                               cap_bytes=int(bucket_cap_mb * (1 << 20)),
                               first_bytes=int(first_bucket_mb * (1 << 20)))
        bounds = [0]
        pb = [0] * len(params)
        for bi, bk in enumerate(buckets):
            for j in bk:
                pb[order[j]] = bi
            last = order[bk[-1]]
            bounds.append(offs[last] + (params[last].numel() + 63) // 64 * 64)
        bounds[-1] = off
        self.bucket_bounds = bounds
        self.param_bucket = pb
        self.reducer = None
        if self.world > 1:
            if broadcast:
                broadcast_params([p.data for p in params] + list(module.buffers()), process_group)
            self.reducer = make_arena_reducer(process_group, self.grad_arena, bounds, average, comm_jobs=False)
            self.reducer.set_param_map(pb)
            self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                           for i, p in enumerate(params)]

    def _make_hook(self, i):
        def hook(_p):
            self.reducer.mark_ready(i)
        return hook

    def forward(self, *a, **k):
        if self.reducer is not None:
            self.reducer.reset_iteration()
        return self.module(*a, **k)

    def finish_gradient_sync(self):
        """Launch any bucket whose params got no grad, then wait for all."""
        if self.reducer is not None:
            self.reducer.launch_all()
            self.reducer.wait_all()

    def zero_grad(self, set_to_none: bool = False):
        # grads must stay arena views: zero in place
        self.grad_arena.zero_()
