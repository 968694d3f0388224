from .env import (LaunchInfo, discover, init_comm_size_and_rank, local_rank_from_env,
                  parse_slurm_nodelist, find_ifname, discover_master)
from .bootstrap import (choose_backend, setup_ddp, get_comm_size_and_rank, control_group,
                        global_barrier, bound_device, shutdown)
