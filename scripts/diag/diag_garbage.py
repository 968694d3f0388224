"""Diagnostic: does any launch of the fused 28x28 step read a device buffer
element that the step did not write first?

Fills one per-step scratch buffer at a time (weight-gradient partial slabs,
bias partial rows, loss partials, activations and their gradients) with NaN
before every step of an eager reducer-free trial; a buffer whose stale
contents leak into the result turns the parameters non-finite.

    python scripts/diag/diag_garbage.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    out = {}
    for pair in (True, False):
        def make():
            tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                                use_graphs=False)
            tr.f28_pair = pair
            tr.bind_train_data(X, idx)
            tr.set_cursor(0, 4)
            return tr

        ref = make()
        ref.train_steps(4)
        torch.cuda.synchronize()
        ref_p = ref.params.clone()
        tr = make()
        p = tr._plan28(128)
        bufs = {k: t for k, (t, _) in p["slabs"].items()}
        bufs.update({"f28_bias": tr.f28_bias, "f28_part": tr.f28_part, "dmulv": tr.dmulv, "dmulv16": tr.dmulv16,
                     "mulv": tr.mulv, "eps": tr.eps, "z16": tr.z16, "dlog32": tr.dlog32, "xb": tr.xb})
        bufs.update({"act." + k: v for k, v in tr.acts.items()})
        bufs.update({"gact." + k: v for k, v in tr.gacts.items()})
        res = {}
        for name in bufs:
            t2 = make()
            b2 = {k: t for k, (t, _) in t2._plan28(128)["slabs"].items()}
            b2.update({"f28_bias": t2.f28_bias, "f28_part": t2.f28_part, "dmulv": t2.dmulv, "dmulv16": t2.dmulv16,
                       "mulv": t2.mulv, "eps": t2.eps, "z16": t2.z16, "dlog32": t2.dlog32, "xb": t2.xb})
            b2.update({"act." + k: v for k, v in t2.acts.items()})
            b2.update({"gact." + k: v for k, v in t2.gacts.items()})
            for _ in range(4):
                b2[name].fill_(float("nan"))
                t2.train_steps(1)
            torch.cuda.synchronize()
            finite = bool(torch.isfinite(t2.params).all().item())
            same = bool(torch.equal(t2.params, ref_p))
            res[name] = {"finite": finite, "bitwise_as_clean": same}
            if not finite or not same:
                print(f"pair={pair} {name}: finite={finite} same={same}", flush=True)
        out[f"pair{int(pair)}"] = res
    print(json.dumps({k: [n for n, r in v.items() if not (r["finite"] and r["bitwise_as_clean"])]
                      for k, v in out.items()}))


if __name__ == "__main__":
    main()
