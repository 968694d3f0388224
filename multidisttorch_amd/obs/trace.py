"""Tracing: roctx ranges around driver phases + rocprofv3 recipes.

``range(name)`` pushes/pops a roctx range (torch.cuda.nvtx maps to roctx on
ROCm builds) when ``MDT_TRACE=1`` or ``enable()`` was called; otherwise it is
free. Ranges show up in ``rocprofv3 --marker-trace`` timelines next to the
kernel trace. ``ROCPROF_RECIPES`` lists the counter sets used to profile the
fused kernels (collect PMC in its own run, never combined with sys/runtime
tracing on the shared pool).
"""

from __future__ import annotations

import contextlib
import os

__all__ = ["enable", "enabled", "range", "ROCPROF_RECIPES"]

_ON = os.getenv("MDT_TRACE", "0") == "1"


def enable(on: bool = True):
    global _ON
    _ON = on


def enabled() -> bool:
    return _ON


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    if not _ON:
        yield
        return
    try:
        import torch

        torch.cuda.nvtx.range_push(name)
        pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            import torch

            torch.cuda.nvtx.range_pop()


ROCPROF_RECIPES = {
    "kernel_stats": "rocprofv3 --kernel-trace --stats --output-format csv -d {out} -- {cmd}",
    "occupancy": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d {out} -- {cmd}",
    "issue": "rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace --output-format csv -d {out} -- {cmd}",
    "cache": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d {out} -- {cmd}",
    "mfma": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d {out} -- {cmd}",
}
