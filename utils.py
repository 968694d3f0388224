"""Compatibility module: the reference's ``utils`` API on the MI355X runtime.

Scripts written against ORNL/MultiDistTorch do ``from utils import *``
(/root/reference/vae-hpo.py:16, example-subgroup.py:4) and rely on the
star-import re-exporting ``os, socket, psutil, re, torch, dist``
(/root/reference/utils.py:1-7; vae-hpo.py calls ``os.makedirs`` without
importing ``os``). Every function keeps its reference signature, return value
and printed output; the implementations live in ``multidisttorch_amd``:

  init_comm_size_and_rank  utils.py:9-26    -> runtime.env (adds torchrun fallback)
  get_comm_size_and_rank   utils.py:28-38   -> runtime.bootstrap
  find_ifname              utils.py:40-56   -> runtime.env
  parse_slurm_nodelist     utils.py:59-90   -> runtime.env
  setup_ddp                utils.py:93-144  -> runtime.bootstrap (+ one-GPU-per-process binding)
  setup_ddp_groups         utils.py:146-163 -> parallel.groups
  print0                   utils.py:165-174 -> parallel.groups
"""

import os
import re
import socket

import psutil
import torch
import torch.distributed as dist

from multidisttorch_amd.parallel.groups import print0, setup_ddp_groups
from multidisttorch_amd.runtime.bootstrap import get_comm_size_and_rank, setup_ddp
from multidisttorch_amd.runtime.env import find_ifname, init_comm_size_and_rank, parse_slurm_nodelist

__all__ = [
    "os", "socket", "psutil", "re", "torch", "dist",
    "init_comm_size_and_rank", "get_comm_size_and_rank", "find_ifname", "parse_slurm_nodelist",
    "setup_ddp", "setup_ddp_groups", "print0",
]
