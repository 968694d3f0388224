"""Diagnostic: the three-test sequence of test_fused_comm.py that makes the
third test's reducer-free solo eager reference non-reproducible
([True-True-False], [True-True-True], then [True-False-False]), replayed
outside pytest, then probed:
  a) three reference runs (8 steps back to back, as the test) -- equal?
  b) two reference trainers in lockstep with a device sync after every step,
     every per-step buffer compared -- the first buffer that differs.

    python scripts/diag/diag_repro.py [--skip1] [--skip2]
"""
import argparse
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip1", action="store_true")
    ap.add_argument("--skip2", action="store_true")
    ap.add_argument("--gc", action="store_true", help="gc.collect() after each replayed test")
    ap.add_argument("--parts", default="rfRF", help="r/f: test 1 reference / fused run, R/F: test 2's")
    ap.add_argument("--sync-steps", action="store_true", help="a): device sync after every step")
    a = ap.parse_args()
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    nb, steps = 4, 8

    def data():
        X = torch.rand(nb * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
        return X, torch.arange(nb * 128, device=dev, dtype=torch.int32)

    def trainer(graphs, pair=True, overlap=True):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=graphs, graph_steps=4)
        tr.f28_pair = pair
        tr.ddp_overlap = overlap
        return tr

    def run(tr, X, idx):
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        tr.train_steps(steps)
        torch.cuda.synchronize()
        return tr.params.clone(), tr.loss_history()[:steps].copy()

    def replay_test(graphs, pair, overlap, do_ref, do_fused):
        X, idx = data()
        if do_ref:
            run(trainer(graphs, pair, overlap), X, idx)
        if do_fused:
            tr = trainer(graphs, pair, overlap)
            red = tr.C.XgmiP2PReducer(0, 1, tr.grads, tr.default_bucket_bounds(), True, 0.0, 64, 20.0, -1, True)
            tr.attach_reducer(red)
            run(tr, X, idx)
        print(f"replayed test graphs={graphs} pair={pair} ref={do_ref} fused={do_fused}", flush=True)

    if not a.skip1:
        replay_test(False, True, True, "r" in a.parts, "f" in a.parts)
        if a.gc:
            gc.collect()
    if not a.skip2:
        replay_test(True, True, True, "R" in a.parts, "F" in a.parts)
        if a.gc:
            gc.collect()
    X, idx = data()

    def run_a():
        tr = trainer(False, False, True)
        if not a.sync_steps:
            return run(tr, X, idx)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        for _ in range(steps):
            tr.train_steps(1)
            torch.cuda.synchronize()
        return tr.params.clone(), tr.loss_history()[:steps].copy()

    res = [run_a() for _ in range(3)]
    eq = [bool(torch.equal(p, res[0][0])) for p, _ in res[1:]]
    print("a) reference re-runs equal to the first:", eq, flush=True)

    def bufs(tr):
        p = tr._plan28(128)
        b = {"xb": tr.xb, "mulv": tr.mulv, "eps": tr.eps, "z16": tr.z16, "dlog32": tr.dlog32}
        b.update({"act." + k: v for k, v in tr.acts.items()})
        b.update({"gact." + k: v for k, v in tr.gacts.items()})
        b.update({"dmulv": tr.dmulv, "f28_bias": tr.f28_bias, "f28_part": tr.f28_part})
        b.update({"slab." + k: t for k, (t, _) in p["slabs"].items() if k.endswith(".weight")})
        b.update({"params": tr.params, "exp_avg": tr.exp_avg, "exp_avg_sq": tr.exp_avg_sq, "w16": tr.w16,
                  "state": tr.state.train_state})
        return b

    A, B = trainer(False, False, True), trainer(False, False, True)
    for t in (A, B):
        t.bind_train_data(X, idx)
        t.set_cursor(0, nb)
    for s in range(steps):
        A.train_steps(1)
        torch.cuda.synchronize()
        B.train_steps(1)
        torch.cuda.synchronize()
        ba, bb = bufs(A), bufs(B)
        diff = [k for k in ba if not torch.equal(ba[k], bb[k])]
        if diff:
            print("b) step", s, json.dumps({k: int((ba[k] != bb[k]).sum()) for k in diff}), flush=True)
            break
    else:
        print("b) lockstep: no difference", flush=True)


if __name__ == "__main__":
    main()
