"""Data-parallel host logic (alignn_mi355x.dp) with world_size 2 over gloo on CPU: the gradient
all_reduce hook averages, the reference's clip_grad_norm_(5) + two-group AdamW then leave both
ranks with identical parameters equal to a single process stepping on the mean gradient, and the
step time is the max over ranks.  (The GPU run uses the same hook over RCCL.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from alignn_mi355x import dp

NPARAM, SIGMA_START = 1000, 900


def _grads(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(NPARAM, generator=g) * (3.0 + rank)   # large enough that clipping engages


def _step(flat, grad):
    p_base = torch.nn.Parameter(flat[:SIGMA_START].clone())
    p_sigma = torch.nn.Parameter(flat[SIGMA_START:].clone())
    p_base.grad, p_sigma.grad = grad[:SIGMA_START].clone(), grad[SIGMA_START:].clone()
    opt = torch.optim.AdamW([{"params": [p_base], "lr": 3e-4}, {"params": [p_sigma], "lr": 1e-4}], lr=3e-4,
                            weight_decay=1e-4)
    torch.nn.utils.clip_grad_norm_([p_base, p_sigma], max_norm=5.0)
    opt.step()
    return torch.cat([p_base.detach(), p_sigma.detach()])


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        flat = torch.randn(NPARAM, generator=torch.Generator().manual_seed(0))
        grad = _grads(rank)
        dp.grad_allreduce_hook(world)(grad)
        new = _step(flat, grad)
        t = dp.max_over_ranks(0.5 + rank, "cpu")
        torch.save({"grad": grad, "new": new, "t": t, "graphs": list(dp.rank_graphs(32, rank))},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(120)
def test_dp_allreduce_clip_adamw_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    mean = (_grads(0) + _grads(1)) / 2
    assert torch.allclose(r[0]["grad"], mean, rtol=1e-6, atol=1e-6)
    assert torch.equal(r[0]["grad"], r[1]["grad"])
    assert torch.equal(r[0]["new"], r[1]["new"])
    ref = _step(torch.randn(NPARAM, generator=torch.Generator().manual_seed(0)), mean)
    assert torch.allclose(r[0]["new"], ref, rtol=1e-6, atol=1e-7)
    assert r[0]["t"] == r[1]["t"] == 1.5
    assert r[0]["graphs"] == list(range(0, 32)) and r[1]["graphs"] == list(range(32, 64))
