"""Data-parallel host logic (alignn_mi355x.dp) with world_size 2 over gloo on CPU: the gradient
all_reduce hook averages, the reference's clip_grad_norm_(5) + two-group AdamW then leave both
ranks with identical parameters equal to a single process stepping on the mean gradient, and the
step time is the max over ranks.  (The GPU run uses the same hook over RCCL.)"""
import os
import socket
import weakref

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


# ------------------------------------------------------------------------------------------------
# Ensemble sharding: members placed i % world, heads gathered to rank 0 in member order
# ------------------------------------------------------------------------------------------------
def _member_heads(member, B=3, W=4):
    return torch.randn(B, W, generator=torch.Generator().manual_seed(500 + member))


def _ens_worker(rank, world, port, out_dir, num_members):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = dp.members_of_rank(num_members, world, rank)
        local = torch.stack([_member_heads(i) for i in mine], 0) if mine else torch.empty(0, 3, 4)
        got = dp.gather_member_heads(local, num_members)
        stats = torch.tensor([4.32, 3.56]) if rank == 0 else torch.zeros(2)
        dp.broadcast_([stats])
        torch.save({"got": got, "mine": mine, "stats": stats}, os.path.join(out_dir, f"e{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world,num_members", [(2, 5), (3, 2)])
def test_ensemble_member_gather(tmp_path, world, num_members):
    mp.spawn(_ens_worker, args=(world, _free_port(), str(tmp_path), num_members), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"e{i}.pt", weights_only=True) for i in range(world)]
    want = torch.stack([_member_heads(i) for i in range(num_members)], 0)
    assert torch.equal(r[0]["got"], want)
    assert all(x["got"] is None for x in r[1:])
    assert sorted(i for x in r for i in x["mine"]) == list(range(num_members))
    assert all(torch.equal(x["stats"], torch.tensor([4.32, 3.56])) for x in r)


def test_member_placement_and_seeds():
    # train.py:2053-2054: seed + 1007 i, fold i % num_folds; C4: 5 members over 8 ranks
    assert [dp.member_seed(42, i) for i in range(3)] == [42, 1049, 2056]
    assert [dp.member_fold(i, 5) for i in range(7)] == [0, 1, 2, 3, 4, 0, 1]
    assert [dp.members_of_rank(5, 8, r) for r in range(8)] == [[0], [1], [2], [3], [4], [], [], []]
    assert dp.members_of_rank(5, 2, 0) == [0, 2, 4] and dp.members_of_rank(5, 2, 1) == [1, 3]
    with pytest.raises(ValueError):
        dp.members_of_rank(5, 2, 2)


# ------------------------------------------------------------------------------------------------
# FusedTrainer.grad_hook between the two replayed launch plans (trainer._replay), world size 2
# ------------------------------------------------------------------------------------------------
class _Slot:
    """A captured batch stand-in (weak-referenceable, no tensors)."""


class _FakeLib:
    """Stands in for libalignn_hip's plan replay: plan 1 = forward/backward (writes this rank's
    gradient), plan 2 = clip + AdamW (the reference's two-group AdamW on CPU)."""

    def __init__(self, trainer, grad, log):
        self.tr, self.grad, self.log = trainer, grad, log

    def alignn_set_i64(self, ptr, value, stream):  # the per-step device seed (no GPU here)
        self.log.append("seed")
        return 0

    def alignn_plan_replay(self, plan, stream):
        if plan == 1:
            self.log.append("fb")
            self.tr.st.grad.copy_(self.grad)
        else:
            self.log.append("update")
            new = _step_flat(self.tr.st.flat, self.tr.st.grad, self.tr.st.P.sigma_start)
            self.tr.st.flat.copy_(new)
        return 0


def _step_flat(flat, grad, s0):
    p_base = torch.nn.Parameter(flat[:s0].clone())
    p_sigma = torch.nn.Parameter(flat[s0:].clone())
    p_base.grad, p_sigma.grad = grad[:s0].clone(), grad[s0:].clone()
    opt = torch.optim.AdamW([{"params": [p_base], "lr": 3e-4}, {"params": [p_sigma], "lr": 3e-4}], lr=3e-4,
                            weight_decay=1e-4)
    torch.nn.utils.clip_grad_norm_([p_base, p_sigma], max_norm=5.0)
    opt.step()
    return torch.cat([p_base.detach(), p_sigma.detach()])


def _trainer_worker(rank, world, port, out_dir):
    import alignn_mi355x as A
    from alignn_mi355x import _lib, ops, trainer as trainer_mod
    from alignn_mi355x.engine import batch_versions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)  # identical initial weights on both ranks
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(6, 8, 7, 289, 2, 32, 1, 1, 0.0), 2)
        tr = A.FusedTrainer(model, optimizer="torch")
        n = tr.st.flat.numel()
        grad = torch.randn(n, generator=torch.Generator().manual_seed(7 + rank)) * (2.0 + rank)
        log = []
        fake = _FakeLib(tr, grad, log)
        _lib.lib = lambda: fake            # the replay goes through the stub library
        ops.stream_ptr = lambda *a, **k: 0
        trainer_mod.check = lambda rc, what: None
        hook = dp.grad_allreduce_hook(world)

        def logged_hook(g):
            log.append("hook")
            hook(g)

        tr.grad_hook = logged_hook
        tr._seed_dev = torch.zeros(1, dtype=torch.int64)
        batch = _Slot()
        tr._graph = (None, None, batch, [1, 2])   # two captured plans, as capture(mode="plan") leaves them
        # ... holding this batch (the captured slot's contents)
        tr._bound, tr._bound_v = weakref.ref(batch), batch_versions(batch, trainer_mod.BATCH_FIELDS)
        tr._exchange = tr._exchange_mode()        # and the exchange they were captured for
        before = tr.st.flat.clone()
        tr.step(batch, seed=3)
        torch.save({"log": log, "before": before, "after": tr.st.flat.clone(), "grad": tr.st.grad.clone(),
                    "s0": tr.st.P.sigma_start, "steps": tr.step_count}, os.path.join(out_dir, f"t{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_fused_trainer_grad_hook_between_plan_phases_world2(tmp_path):
    """The replayed step runs plan 1 (forward/backward), then the DP hook (one gloo all_reduce of the
    flat gradient, mean over ranks), then plan 2 (clip + AdamW): afterwards both ranks hold the same
    parameters, equal to one process stepping on the mean gradient (trainer.py _replay)."""
    world = 2
    mp.spawn(_trainer_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"t{i}.pt", weights_only=True) for i in range(world)]
    for x in r:
        assert x["log"] == ["seed", "fb", "hook", "update"], x["log"]
        assert x["steps"] == 1
    n = r[0]["before"].numel()
    mean = sum(torch.randn(n, generator=torch.Generator().manual_seed(7 + i)) * (2.0 + i) for i in range(world)) / world
    assert torch.allclose(r[0]["grad"], mean, atol=1e-6) and torch.equal(r[0]["grad"], r[1]["grad"])
    want = _step_flat(r[0]["before"], mean, r[0]["s0"])
    assert torch.equal(r[0]["after"], r[1]["after"])
    assert torch.allclose(r[0]["after"], want, atol=1e-7)


# ------------------------------------------------------------------------------------------------
# Bucketed gradient exchange (dp.GradBuckets) between three replayed plans, world size 2
# ------------------------------------------------------------------------------------------------
class _FakeLib3(_FakeLib):
    """Plan 1 = forward + per-layer backward (writes the first bucket's gradient), plan 2 = the
    backward's tail (writes the rest), plan 3 = clip + AdamW."""

    def __init__(self, trainer, grad, log, split):
        super().__init__(trainer, grad, log)
        self.split = split

    def alignn_plan_replay(self, plan, stream):
        g = self.tr.st.grad
        if plan == 1:
            self.log.append("layers")
            g[:self.split].copy_(self.grad[:self.split])
            g[self.split:].fill_(float("nan"))     # not final yet: the tail writes it
        elif plan == 2:
            self.log.append("tail")
            g[self.split:].copy_(self.grad[self.split:])
        else:
            return super().alignn_plan_replay(2, stream)
        return 0


def _bucket_worker(rank, world, port, out_dir):
    import alignn_mi355x as A
    from alignn_mi355x import _lib, ops, trainer as trainer_mod
    from alignn_mi355x.engine import batch_versions
    from alignn_mi355x.layout import bucket_split
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(6, 8, 7, 289, 2, 32, 1, 1, 0.0), 2)
        tr = A.FusedTrainer(model, optimizer="torch")
        split = bucket_split(model.config, True)
        n = tr.st.flat.numel()
        grad = torch.randn(n, generator=torch.Generator().manual_seed(11 + rank)) * (1.0 + rank)
        log = []
        fake = _FakeLib3(tr, grad, log, split)
        _lib.lib = lambda: fake
        ops.stream_ptr = lambda *a, **k: 0
        trainer_mod.check = lambda rc, what: None
        buckets = dp.GradBuckets(tr.st.grad, split, world)
        orig_start, orig_finish = buckets.start, buckets.finish
        buckets.start = lambda side=None: (log.append("start"), orig_start(None))[1]
        buckets.finish = lambda: (log.append("finish"), orig_finish())[1]
        tr.grad_buckets = buckets
        tr._seed_dev = torch.zeros(1, dtype=torch.int64)
        tr.ctx.side = lambda dev: None
        batch = _Slot()
        tr._graph = (None, None, batch, [1, 2, 3])
        tr._bound, tr._bound_v = weakref.ref(batch), batch_versions(batch, trainer_mod.BATCH_FIELDS)
        tr._exchange = tr._exchange_mode()
        before = tr.st.flat.clone()
        tr.step(batch, seed=3)
        torch.save({"log": log, "before": before, "after": tr.st.flat.clone(), "grad": tr.st.grad.clone(),
                    "s0": tr.st.P.sigma_start, "split": split, "n": n}, os.path.join(out_dir, f"b{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_bucketed_gradient_exchange_world2(tmp_path):
    """Three replayed phases: per-layer backward, first bucket's all_reduce started, backward tail,
    second bucket reduced and both scaled, clip + AdamW — the same parameters on both ranks as one
    process stepping on the mean gradient; the flat layout puts the conv blocks first."""
    world = 2
    mp.spawn(_bucket_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"b{i}.pt", weights_only=True) for i in range(world)]
    for x in r:
        assert x["log"] == ["seed", "layers", "start", "tail", "finish", "update"], x["log"]
        assert 0 < x["split"] < x["n"]
    n = r[0]["n"]
    mean = sum(torch.randn(n, generator=torch.Generator().manual_seed(11 + i)) * (1.0 + i) for i in range(world)) / world
    assert torch.allclose(r[0]["grad"], mean, atol=1e-6) and torch.equal(r[0]["grad"], r[1]["grad"])
    assert torch.equal(r[0]["after"], r[1]["after"])
    assert torch.allclose(r[0]["after"], _step_flat(r[0]["before"], mean, r[0]["s0"]), atol=1e-7)


def test_layout_conv_blocks_first():
    """The first bucket is exactly the conv blocks' own parameters (no lin_edge / edge_proj, no
    encoder, readout or head), the second everything else."""
    from alignn_mi355x.layout import AlignnConfig, bucket_split, offsets
    cfg = AlignnConfig(206, 36, 11, 289, 2, 256, 4, 4)
    offs, total, s0 = offsets(cfg, True)
    split = bucket_split(cfg, True)
    first = {k for k, (o, _) in offs.items() if o < split}
    assert first and all((".edge_blocks." in k or ".node_blocks." in k) for k in first)
    assert not any("lin_edge" in k or "edge_proj" in k for k in first)
    assert all(o >= split for k, (o, _) in offs.items() if k not in first)
    assert s0 > split and total == 3307270 - 514
