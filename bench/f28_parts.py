"""Time the launches of the fused 28x28 step separately on one MI355X.

Replays each launch (forward, backward, the multi-job weight-gradient launch,
each weight-gradient job alone, the finalize) N times between HIP events
after a few real steps, so the numbers are per launch in a warm state.

    python bench/f28_parts.py [--reps 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from multidisttorch_amd.data.datasets import synthetic_images
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    B = 128
    tr = ConvVaeTrainer(batch_size=B, image=28, device=dev, backend="hip", seed=0, use_graphs=False)
    X = synthetic_images(8 * B, device=dev)
    tr.bind_train_data(X, torch.arange(8 * B, device=dev, dtype=torch.int32))
    tr.set_cursor(0, 8)
    tr.train_steps(3)
    torch.cuda.synchronize()
    C, p, st = tr.C, tr._plan28(B), tr.state
    out = {}
    out["step_eager"] = timeit(lambda: tr._step28(B), a.reps)
    out["fwd"] = timeit(lambda: C.f28_forward(p["fwd"], B, B, 0, True), a.reps)
    out["bwd"] = timeit(lambda: C.f28_backward(p["bwd"], B), a.reps)
    out["wgrad_multi"] = timeit(lambda: C.launch_jobs_multi(p["jobs_pack"], p["jobs_grid"]), a.reps)
    L = {l.name: l for l in tr.spec}
    a1, a2, d0, d1 = tr.acts["enc1"], tr.acts["enc2"], tr.acts["dec_fc"], tr.acts["dec1"]
    gd1, gd0, ga2, ga1 = tr.gacts["dec1"], tr.gacts["dec_fc"], tr.gacts["enc2"], tr.gacts["enc1"]
    srcs = {"enc1": (ga1, tr.xb), "enc2": (ga2, a1), "enc_head": (tr.dmulv16, a2), "dec_fc": (gd0, tr.z16),
            "dec1": (d0, gd1), "dec2": (d1, tr.dlog32)}
    for name, (G, Xw) in srcs.items():
        d = tr._desc(L[name], B)
        slab = p["slabs"][name + ".weight"][0]
        plan = C.wgrad_plan(d)
        out[f"wgrad_{name}"] = {"us": timeit(lambda G=G, Xw=Xw, d=d, slab=slab: C.wgrad(G, Xw, d, slab), a.reps),
                                "plan": list(plan)}
    out["finalize"] = timeit(lambda: C.grad_finalize(tr.params, tr.grads, tr.exp_avg, tr.exp_avg_sq, tr.w16,
                                                     p["segs"], p["units"], p["nunits"], st.train_state,
                                                     st.hparams, False), a.reps)
    out["finalize_units"] = p["nunits"]
    out["slab_mb"] = {k: round(v[0].numel() * 4 / 2 ** 20, 3) for k, v in p["slabs"].items()}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
