"""Data parallelism for the training step: one process per GPU, each rank trains on
its own batch of graphs (weak scaling), and the ranks exchange the flat gradient buffer per step
(RCCL over xGMI on MI355X, 13.2 MB fp32: one all_reduce, or two buckets with the first overlapped with
the backward's tail, GradBuckets) before the reference's clip_grad_norm_(5.0) + AdamW, which then run
identically on every rank.

The reference trains on one device (scripts/train.py:607-723); with the PyG lg_edge_index offset
rule a rank's batch is collated on its own, so DP parity means: every rank's
gradient equals the reference's on that rank's batch, and the update uses their mean.

Ensemble sharding: the reference trains its members one after the other
(scripts/train.py:2052-2093, member i has seed ``seed + 1007 i`` and fold ``i % num_folds``); here
member i lives on rank ``i % world`` with no per-step communication, and inference gathers every
member's [B, 2T] heads to rank 0 (one gather per batch) for the moment mix.
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


class GradBuckets:
    """The data-parallel gradient mean in two buckets, the first overlapped with the backward's tail.

    The flat layout (layout.flat_entries) puts the conv blocks' own parameters first: their
    gradients are final once the per-layer backward is done (engine.backward_layers; written on the
    main stream and the engine's side stream).  :meth:`start` — called between the per-layer backward
    and the tail — all_reduces that bucket (10.4 MB of the 13.2 MB at the reference's size) on the
    communication stream after both, while the tail (edge-projection chain rules, deferred angle-encoder
    backward, encoder MLPs) runs; :meth:`finish` — after the tail, every stream joined — reduces the
    rest, waits for both and scales by 1/world.  Sum then scale, as grad_allreduce_hook."""

    def __init__(self, grad: torch.Tensor, split: int, world: Optional[int] = None, group=None):
        if not 0 < split < grad.numel():
            raise ValueError(f"bucket split {split} outside the gradient (1..{grad.numel() - 1})")
        self.grad, self.group = grad, group
        self.first, self.rest = grad[:split], grad[split:]
        self.inv = 1.0 / (dist.get_world_size(group) if world is None else world)
        self.work = None

    def start(self, side: Optional[torch.cuda.Stream] = None) -> None:
        if self.grad.is_cuda:
            main = torch.cuda.current_stream(self.grad.device)
            s = side if side is not None else main
            if s is not main:
                s.wait_stream(main)
            with torch.cuda.stream(s):
                self.work = dist.all_reduce(self.first, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            self.work = dist.all_reduce(self.first, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self) -> None:
        dist.all_reduce(self.rest, op=dist.ReduceOp.SUM, group=self.group)
        if self.work is not None:
            self.work.wait()
            self.work = None
        self.grad.mul_(self.inv)


def rank_graphs(per_rank: int, rank: int) -> range:
    """Global graph indices of a rank's batch (weak scaling: a fixed batch per rank)."""
    return range(rank * per_rank, (rank + 1) * per_rank)


def max_over_ranks(seconds: float, device) -> float:
    """The slowest rank's time (the step is only done when every rank is)."""
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------------------------------------------
# Ensemble sharding: one (or more) members per rank
# ------------------------------------------------------------------------------------------------
def member_seed(base_seed: int, member: int) -> int:
    """Seed of ensemble member ``member`` (train.py:2053)."""
    return int(base_seed) + int(member) * 1007


def member_fold(member: int, num_folds: int) -> int:
    """Cross-validation fold member ``member`` trains against (train.py:2054)."""
    return int(member) % int(num_folds)


def members_of_rank(num_members: int, world: int, rank: int) -> List[int]:
    """Members placed on ``rank``: i % world == rank (5 members on 8 GPUs -> ranks 0-4 one each,
    ranks 5-7 none)."""
    if num_members < 1 or world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad placement: members={num_members} world={world} rank={rank}")
    return list(range(rank, num_members, world))


def gather_member_heads(local: torch.Tensor, num_members: int, dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Gathers every rank's member outputs ``local [m_rank, B, W]`` (its members in
    :func:`members_of_rank` order) to ``dst`` and returns them there as ``[num_members, B, W]`` in
    member order (``None`` on the other ranks).  Ranks pad to the same slot count so one fixed-size
    gather suffices (RCCL gather over xGMI; B x 2T x 4 bytes per member)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = members_of_rank(num_members, world, rank) if rank < num_members else []
    if local.size(0) != len(mine):
        raise ValueError(f"rank {rank} holds members {mine} but passed {local.size(0)} outputs")
    slots = -(-num_members // world)
    buf = local.new_zeros((slots,) + tuple(local.shape[1:]))
    if len(mine):
        buf[:len(mine)].copy_(local)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.stack([parts[i % world][i // world] for i in range(num_members)], 0)


def broadcast_(tensors: Sequence[torch.Tensor], src: int = 0, group=None) -> None:
    """Broadcast in place (e.g. the target normalizer stats, scaler_state, before training)."""
    for t in tensors:
        dist.broadcast(t, src=src, group=group)
