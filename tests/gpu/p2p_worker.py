"""Worker for tests/gpu/test_p2p_reducer.py: s processes share the box's single
MI355X, exchange hipIpc handles of their receive regions over gloo, and run the
p2p all-reduce kernel (eager and graph-replayed). argv: reducer kind (p2p |
p2p1 | p2p2). Prints RESULT json."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    dist.init_process_group("gloo")
    r, s = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    n = 300_001
    bounds = [0, 1000, 65_536, n]
    flat = torch.zeros(n, device=dev)
    os.environ["MDT_P2P_TIMEOUT_S"] = "10"
    kind = sys.argv[1] if len(sys.argv) > 1 else "p2p"
    red = make_arena_reducer(dist.group.WORLD, flat, bounds, kind=kind)
    gen = lambda rank, it: torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + rank))
    errs, iters = [], 5
    for it in range(iters):
        flat.copy_(gen(r, it).to(dev))
        torch.cuda.synchronize()
        red.launch_all()
        red.wait_all()
        torch.cuda.synchronize()
        ref = sum(gen(p, it).double() for p in range(s)) / s
        errs.append(float((flat.cpu().double() - ref).abs().max()))
    st = red.status()
    # bitwise identical on every replica
    out = [torch.empty(n) for _ in range(s)]
    dist.all_gather(out, flat.cpu())
    same = all(torch.equal(out[0], o) for o in out)
    # hipGraph: capture launch+wait once, replay with fresh inputs
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        red.launch_all()
        red.wait_all()
    torch.cuda.synchronize()
    dist.barrier()
    gerrs = []
    for it in range(iters, iters + 3):
        flat.copy_(gen(r, it).to(dev))
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        ref = sum(gen(p, it).double() for p in range(s)) / s
        gerrs.append(float((flat.cpu().double() - ref).abs().max()))
    st2 = red.status()
    red_two = red.two_shot()
    # the same inputs through the one-shot form: bitwise the same result
    flat.copy_(gen(r, 99).to(dev))
    torch.cuda.synchronize()
    red.launch_all()
    red.wait_all()
    torch.cuda.synchronize()
    got = flat.clone()
    one = make_arena_reducer(dist.group.WORLD, flat, bounds, kind="p2p1")
    flat.copy_(gen(r, 99).to(dev))
    torch.cuda.synchronize()
    one.launch_all()
    one.wait_all()
    torch.cuda.synchronize()
    bitwise = bool(torch.equal(got, flat))
    st3 = one.status()
    dist.barrier()  # peers stop touching our regions before they are freed
    del g, red, one
    torch.cuda.synchronize()
    dist.barrier()
    print("RESULT " + json.dumps({"rank": r, "errs": errs, "gerrs": gerrs, "status": [st, st2, st3], "same": same,
                                  "bitwise_one_shot": bitwise,
                                  "two_shot": list(red_two)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
