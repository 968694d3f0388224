"""multidisttorch_amd — MI355X-native multi-group distributed training.

Same capabilities and public API as ORNL/MultiDistTorch (launcher-agnostic
bootstrap, K disjoint trial groups carved from one world, group-scoped logging,
concurrent VAE HPO trials), re-designed for MI355X: one process per GPU,
RCCL over xGMI, fused CDNA4 HIP kernels, native C++ runtime.
"""

__version__ = "0.1.0"

from .runtime import (setup_ddp, get_comm_size_and_rank, init_comm_size_and_rank, find_ifname,
                      parse_slurm_nodelist, control_group, global_barrier, bound_device)
from .parallel.groups import GroupPlan, setup_ddp_groups, print0, member_groups
