"""HPO trial specifications.

The reference's only per-trial knob is the epoch count: trial g trains
``epochs + g`` epochs with lr fixed at 1e-3 and beta = 1
(/root/reference/vae-hpo.py:202, :131, :58). ``TrialSpec`` keeps that default
and adds the (lr, beta) sweep the north star asks for.
"""

from __future__ import annotations

import math
from dataclasses import asdict, dataclass
from typing import List, Optional, Sequence

__all__ = ["TrialSpec", "reference_schedule", "default_sweep", "parse_list", "build_specs"]


@dataclass(frozen=True)
class TrialSpec:
    group_id: int
    epochs: int
    lr: float = 1e-3
    beta: float = 1.0
    seed: int = 0

    def to_dict(self):
        return asdict(self)


def reference_schedule(num_groups: int, epochs: int, lr: float = 1e-3, beta: float = 1.0,
                       seed: int = 0) -> List[TrialSpec]:
    """Trial g: epochs + g epochs, same lr/beta (reference behaviour)."""
    return [TrialSpec(g, epochs + g, lr, beta, seed + g) for g in range(num_groups)]


def default_sweep(num_groups: int, epochs: int = 1, seed: int = 0) -> List[TrialSpec]:
    """A K-point (lr, beta) grid: lr log-spaced in [3e-4, 3e-3], beta in {0.5, 1, 2, 4}."""
    specs = []
    nb = 4 if num_groups >= 4 else max(1, num_groups)
    nl = math.ceil(num_groups / nb)
    for g in range(num_groups):
        li, bi = g // nb, g % nb
        lr = 3e-4 * (10 ** (li / max(1, nl - 1))) if nl > 1 else 1e-3
        beta = [1.0, 0.5, 2.0, 4.0][bi] if num_groups > 1 else 1.0
        specs.append(TrialSpec(g, epochs, float(lr), float(beta), seed + g))
    return specs


def parse_list(s: Optional[str], cast=float) -> Optional[List]:
    if s is None or s == "":
        return None
    return [cast(x) for x in str(s).split(",") if x.strip() != ""]


def build_specs(num_groups: int, epochs: int, lrs: Optional[Sequence[float]] = None,
                betas: Optional[Sequence[float]] = None, seed: int = 0,
                epoch_offset: bool = True) -> List[TrialSpec]:
    """Per-group specs. A single value broadcasts; a list is indexed by group (cycled)."""
    out = []
    for g in range(num_groups):
        lr = lrs[g % len(lrs)] if lrs else 1e-3
        b = betas[g % len(betas)] if betas else 1.0
        out.append(TrialSpec(g, epochs + (g if epoch_offset else 0), float(lr), float(b), seed + g))
    return out
