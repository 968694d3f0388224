"""One-shot peer-to-peer bucket all-reduce (csrc/kernels/p2p_allreduce.hip,
csrc/runtime/p2p_comm.cpp) vs a float64 torch reference of the mean.

A gpurun box has one MI355X, so the "peers" share it:
  * in-process: s reducers on one device, each with its own stream, mapped to
    each other's regions directly (connect_local);
  * multi-process: s processes on the same device exchange hipIpc handles over
    gloo (the production path, minus the xGMI hop).
Every wait in the kernel is time-bounded, so a missing peer shows up as a
status code, never as a hung GPU (test_missing_peer_times_out).
"""
import json
import sys
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def _pair(C, s, n, bounds, timeout=5.0, two_shot_min_bytes=-1):
    dev = torch.device("cuda", 0)
    flats = [torch.zeros(n, device=dev) for _ in range(s)]
    reds = [C.XgmiP2PReducer(r, s, flats[r], bounds, True, 0.0, 64, timeout, two_shot_min_bytes) for r in range(s)]
    bases = [r.local_base() for r in reds]
    for r in reds:
        r.connect_local(bases)
    return flats, reds


def _fill(flats, it):
    g = torch.Generator().manual_seed(it)
    vals = [torch.randn(f.numel(), generator=g) for f in flats]
    for f, v in zip(flats, vals):
        f.copy_(v.to(f.device))
    return sum(v.double() for v in vals) / len(vals)


def _same(flats):
    return all(torch.equal(flats[0], f) for f in flats[1:])


@pytest.mark.parametrize("s,two", [(2, -1), (2, 0), (2, 16384)])
def test_p2p_in_process_eager_and_graph(native_ext, s, two):
    """two = two_shot_min_bytes: -1 one-shot only, 0 two-shot for every bucket,
    16384 two-shot for the buckets of >= 4096 elements (mixed launch).

    The graph-replay form runs in a fresh process
    (test_p2p_in_process_graph_replay); the two-shot graph replays are covered
    by the multi-process test (one process per rank)."""
    C = native_ext
    n = 200_003  # odd size: vector body + scalar tail; tiny first bucket = one block
    bounds = [0, 100, 4096, 70_000, n]
    flats, reds = _pair(C, s, n, bounds, two_shot_min_bytes=two)
    assert reds[0].num_buckets() == 4 and reds[0].grids()[0] == 1 and reds[0].grids()[3] <= 64
    assert reds[0].two_shot() == [0 if two < 0 or 4 * w < two else 1 for w in (100, 3996, 65_904, 130_003)]
    ok = [0] * s
    for it in range(4):  # both epoch parities, twice
        ref = _fill(flats, it)
        torch.cuda.synchronize()
        for r in reds:
            r.launch_all()
        for r in reds:
            r.wait_all()
        torch.cuda.synchronize()
        assert [r.status() for r in reds] == ok
        assert _same(flats)  # rank-ordered sum: identical replicas
        torch.testing.assert_close(flats[0].cpu().double(), ref, rtol=0, atol=1e-6)
    # readiness counting launches a bucket when its last parameter is marked
    for r in reds:
        r.set_param_map([0, 1, 1, 2, 3])
    ref = _fill(flats, 10)
    torch.cuda.synchronize()
    for p in range(5):
        for r in reds:
            r.mark_ready(p)
    assert reds[0].pending() == 4
    for r in reds:
        r.wait_all()
        r.reset_iteration()
    torch.cuda.synchronize()
    torch.testing.assert_close(flats[1].cpu().double(), ref, rtol=0, atol=1e-6)


_GRAPH_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from multidisttorch_amd.ops import native
C = native.ensure_built()
dev = torch.device("cuda", 0)
n, bounds = 200_003, [0, 100, 4096, 70_000, 200_003]
# the graph streams first, before anything else in this process exists: the two
# in-process "ranks" progress only while their streams sit on different hardware
# queues (GPU_MAX_HW_QUEUES = 4 per process, assigned in creation order)
streams = [torch.cuda.Stream() for _ in range(2)]
flats = [torch.zeros(n, device=dev) for _ in range(2)]
reds = [C.XgmiP2PReducer(r, 2, flats[r], bounds, True, 0.0, 64, 5.0, -1) for r in range(2)]
bases = [r.local_base() for r in reds]
for r in reds:
    r.connect_local(bases)
graphs = []
for r, st in zip(reds, streams):
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        r.launch_all()
        r.wait_all()
    graphs.append(g)
torch.cuda.synchronize()
for it in range(20, 23):
    gen = torch.Generator().manual_seed(it)
    vals = [torch.randn(n, generator=gen) for _ in flats]
    for f, v in zip(flats, vals):
        f.copy_(v.to(dev))
    ref = sum(v.double() for v in vals) / 2
    torch.cuda.synchronize()
    for g, st in zip(graphs, streams):
        with torch.cuda.stream(st):
            g.replay()
    torch.cuda.synchronize()
    assert [r.status() for r in reds] == [0, 0], [r.status() for r in reds]
    assert torch.equal(flats[0], flats[1])
    torch.testing.assert_close(flats[0].cpu().double(), ref, rtol=0, atol=1e-6)
print("GRAPH_OK", flush=True)
"""


def test_p2p_in_process_graph_replay(native_ext):
    """hipGraph capture per in-process "rank", replays on separate streams, in
    a fresh process whose first two streams are the replay streams (the
    pytest process's stream history decides which hardware queue a new stream
    gets, and two ranks on one queue wait on each other until the kernel's
    timeout)."""
    import subprocess

    r = subprocess.run([sys.executable, "-c", _GRAPH_CHILD, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "GRAPH_OK" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])



def test_two_shot_is_bitwise_one_shot(native_ext):
    """Both forms sum the s contributions in rank order and scale once: the
    two-shot result has the same bits as the one-shot one (s = 2 here, one
    stream per "rank" within the hardware-queue budget; the multi-process test
    checks s = 3, 4)."""
    C = native_ext
    n, s = 1_000_001, 2
    outs = []
    for two in (-1, 0):
        flats, reds = _pair(C, s, n, [0, n], two_shot_min_bytes=two)
        for it in range(2):
            _fill(flats, 40 + it)
            torch.cuda.synchronize()
            for r in reds:
                r.launch_all()
            for r in reds:
                r.wait_all()
            torch.cuda.synchronize()
        assert [r.status() for r in reds] == [0] * s
        outs.append(flats[1].clone())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("two", [-1, 0])
def test_missing_peer_times_out(native_ext, two):
    """Rank 1 never launches: rank 0's blocks give up after the timeout and
    report the first bucket instead of spinning forever (one-shot, and the
    two-shot form's reduce-scatter wait)."""
    C = native_ext
    flats, reds = _pair(C, 2, 8192, [0, 4096, 8192], timeout=0.2, two_shot_min_bytes=two)
    reds[0].launch_all()
    reds[0].wait_all()
    torch.cuda.synchronize()
    assert reds[0].status() == 1


@pytest.mark.parametrize("s,kind", [(2, "p2p"), (4, "p2p"), (3, "p2p2"), (4, "p2p2")])
def test_p2p_multiprocess_ipc(s, kind):
    from multidisttorch_amd.launch import launch

    # several processes share the GPU: the fused 28x28 step keeps one workgroup
    # per sample (a paired sample whose partner is not resident falls back to
    # the solo form, whose f32 summation order differs at rounding level)
    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "MDT_F28_PAIR": "0"}
    rc, outs = launch([sys.executable, os.path.join(HERE, "p2p_worker.py"), kind], s, emulate="torchrun", timeout=100,
                      extra_env=env, capture=True)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    res = [json.loads(l[7:]) for l in text.splitlines() if l.startswith("RESULT ")]
    assert len(res) == s, text[-4000:]
    for r in res:
        assert r["two_shot"] == ([1, 1, 1] if kind == "p2p2" else [0, 0, 0]), r
        assert r["status"] == [0, 0, 0], r
        assert r["bitwise_one_shot"], r
        assert r["same"], r
        assert max(r["errs"] + r["gerrs"]) < 1e-5, r


def test_uncached_region_is_pooled_not_freed(native_ext):
    """A freed reducer's uncached region goes to the process pool (its
    address range is never handed to torch's caching allocator, see
    profiles/r4_determinism) and the next reducer of the same size gets it
    back with its flags / epochs zeroed, so it all-reduces correctly."""
    import gc

    C = native_ext
    dev = torch.device("cuda", 0)
    n, bounds = 5000, [0, 2000, 5000]
    f = torch.zeros(n, device=dev)
    red = C.XgmiP2PReducer(0, 1, f, bounds, True, 2.0, 64, 5.0, -1, True)
    base, nbytes = red.local_base(), red.region_bytes()
    f.fill_(1.0)
    red.launch_all()
    red.wait_all()
    torch.cuda.synchronize()
    assert torch.equal(f, torch.full_like(f, 2.0)) and int(red.status()) == 0
    del red
    gc.collect()
    # allocations after the free never land in the pooled region
    junk = [torch.empty(1 << 18, device=dev) for _ in range(64)]
    for t in junk:
        a = t.data_ptr()
        assert not (a < base + nbytes and a + t.numel() * 4 > base)
    red2 = C.XgmiP2PReducer(0, 1, f, bounds, True, 2.0, 64, 5.0, -1, True)
    assert red2.local_base() == base
    f.fill_(3.0)
    red2.launch_all()
    red2.wait_all()
    torch.cuda.synchronize()
    assert torch.equal(f, torch.full_like(f, 6.0)) and int(red2.status()) == 0
