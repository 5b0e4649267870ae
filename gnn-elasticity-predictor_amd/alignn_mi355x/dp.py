"""Data parallelism for the training step: one process per GPU, each rank trains on
its own batch of graphs (weak scaling), and the ranks exchange ONE all_reduce of the flat gradient
buffer per step (RCCL over xGMI on MI355X; the 13.2 MB fp32 buffer is a single bucket) before the
reference's clip_grad_norm_(5.0) + AdamW, which then run identically on every rank.

The reference trains on one device (scripts/train.py:607-723); with the PyG lg_edge_index offset
rule a rank's batch is collated on its own, so DP parity means: every rank's
gradient equals the reference's on that rank's batch, and the update uses their mean.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist


def grad_allreduce_hook(world: Optional[int] = None, group=None) -> Callable[[torch.Tensor], None]:
    """Returns hook(grad): grad <- mean over ranks (all_reduce SUM, then 1/world), in place."""
    n = dist.get_world_size(group) if world is None else world
    inv = 1.0 / n

    def hook(grad: torch.Tensor) -> None:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
        grad.mul_(inv)

    return hook


def rank_graphs(per_rank: int, rank: int) -> range:
    """Global graph indices of a rank's batch (weak scaling: a fixed batch per rank)."""
    return range(rank * per_rank, (rank + 1) * per_rank)


def max_over_ranks(seconds: float, device) -> float:
    """The slowest rank's time (the step is only done when every rank is)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
