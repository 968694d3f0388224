"""Sub-group demo (drop-in for /root/reference/example-subgroup.py).

Every rank creates BOTH groups in the same order (torch names process groups
from a per-process counter, so creating only "your" group on each rank makes
the store keys collide — the anti-pattern commented at reference :10-17),
then each member all-gathers its rank inside its group. Unlike the reference
(CPU tensors: gloo only) the tensor lives on the bound device,
so the same script runs on RCCL over xGMI.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from utils import *  # noqa: F401,F403


def run(rank, world=8):
    device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    tensor = torch.tensor([rank], device=device)
    half = world // 2
    subgroup_ranks1 = list(range(0, half))
    subgroup_ranks2 = list(range(half, world))
    subgroup1 = dist.new_group(ranks=subgroup_ranks1)
    subgroup2 = dist.new_group(ranks=subgroup_ranks2)
    for ranks, pg in ((subgroup_ranks1, subgroup1), (subgroup_ranks2, subgroup2)):
        if rank in ranks:
            gather_list = [torch.zeros_like(tensor) for _ in ranks]
            dist.all_gather(gather_list, tensor, group=pg)
            print(rank, "gather_list:", [t.cpu() for t in gather_list])
            return [int(t.item()) for t in gather_list]


if __name__ == "__main__":
    comm_size, rank = setup_ddp()
    print("DDP setup:", comm_size, rank)
    want = int(os.getenv("MDT_EXAMPLE_WORLD", "8"))
    assert comm_size == want, f"This example is set to use {want} processes."
    run(rank, comm_size)
    # orderly teardown (every entry point does): no rank leaves while a peer's
    # gloo/RCCL threads still talk to it -- exiting straight after the gather
    # let the interpreter's teardown race a peer's exit (SIGABRT)
    from multidisttorch_amd.runtime.bootstrap import global_barrier, shutdown

    global_barrier()
    shutdown()
    print("Done.")
