"""Fused training step — the per-batch body of ``train_epoch_hetero`` (``scripts/train.py:639-699``).

Per step: feature jitter (train.py:641-646) -> forward (train.py:655) -> hetero NLL + log-sigma L2
(train.py:656-681) -> backward -> ``clip_grad_norm_(5.0)`` -> AdamW with the reference's two
parameter groups (train.py:1516-1542).  Forward, loss and backward run in libalignn_hip without
autograd; parameters and gradients live in one flat buffer each, so clip + AdamW touch two
contiguous segments (base + mean heads | logvar heads).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
from torch import nn

from . import ops, profiling
from .engine import MIN_LOGVAR_FLOOR, batch_cache, site_seed
from .model import HeteroAlignnRegressor
from .synthetic import TARGET_LOG_MEANS, TARGET_LOG_STDS


class FusedTrainer:
    def __init__(self, model: HeteroAlignnRegressor, lr: float = 3e-4, weight_decay: float = 1e-4,
                 sigma_lr: Optional[float] = 3e-4, max_norm: float = 5.0, log_sigma_l2: float = 0.1,
                 feature_jitter_std: float = 0.1, min_logvar_floor: float = MIN_LOGVAR_FLOOR,
                 target_log_means: Sequence[float] = TARGET_LOG_MEANS,
                 target_log_stds: Sequence[float] = TARGET_LOG_STDS, fused_adamw: bool = True,
                 optimizer: str = "hip", precision: Optional[str] = None):
        self.model = model
        if precision is not None:
            model.set_precision(precision)
        st = model._ensure_flat()
        self.st = st
        s0 = st.P.sigma_start
        # two contiguous segments == the reference's two param groups
        self.p_base = nn.Parameter(st.flat[:s0])
        self.p_sigma = nn.Parameter(st.flat[s0:])
        self.p_base.grad = st.grad[:s0]
        self.p_sigma.grad = st.grad[s0:]
        sigma_lr = lr if not sigma_lr else sigma_lr  # train.py:1521-1522 (0 disables the cap)
        kw = {"fused": True, "capturable": True} if (fused_adamw and st.flat.is_cuda) else {}
        self.opt = torch.optim.AdamW([{"params": [self.p_base], "lr": lr}, {"params": [self.p_sigma], "lr": sigma_lr}],
                                     lr=lr, weight_decay=weight_decay, **kw)
        # optimizer="hip": clip + AdamW in libalignn_hip over the flat buffers (alignn_adamw_f32), the
        # same update as torch's fused AdamW (betas (0.9, 0.999), eps 1e-8, decoupled decay)
        if optimizer not in ("torch", "hip"):
            raise ValueError("optimizer must be 'torch' or 'hip'")
        self.optimizer = optimizer
        self.lr, self.sigma_lr, self.weight_decay = lr, sigma_lr, weight_decay
        if optimizer == "hip":
            self.exp_avg = torch.zeros_like(st.flat)
            self.exp_avg_sq = torch.zeros_like(st.flat)
            self.hip_step = torch.zeros(1, device=st.flat.device)
            self.gnorm = torch.zeros(1, device=st.flat.device)
        self.max_norm = max_norm
        self.l2 = log_sigma_l2
        self.jitter = feature_jitter_std
        self.floor = min_logvar_floor
        dev = st.flat.device
        self.log_means = torch.tensor(list(target_log_means), dtype=torch.float32, device=dev)
        self.log_stds = torch.tensor(list(target_log_stds), dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, device=dev)
        self.step_count = 0
        self._graph = None
        self._seed_dev = None
        self.grad_hook = None  # called with the flat gradient between backward and clip (DP all_reduce)

    def set_lr(self, lr: float, sigma_lr: Optional[float] = None) -> None:
        self.opt.param_groups[0]["lr"] = lr
        self.opt.param_groups[1]["lr"] = lr if sigma_lr is None else sigma_lr
        self.lr, self.sigma_lr = lr, (lr if sigma_lr is None else sigma_lr)

    def forward_backward(self, batch, seed: int, training: bool = True,
                         sample_weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward + loss + backward into the flat gradient buffer; returns the loss (device).
        sample_weights: per-graph KNN weights [B] (train.py:660-674), or None."""
        model, st = self.model, self.st
        bc = batch_cache(batch)
        x, gx = batch.x, batch.global_x
        if training and self.jitter > 0.0:
            x = x.clone()
            gx = gx.clone()
            ops.add_noise(x, self.jitter, site_seed(seed, 1 << 20))
            ops.add_noise(gx, self.jitter, site_seed(seed, (1 << 20) + 1))
        out, ctx = model._engine.forward(st.P, batch, bc, training, seed, x, gx, "hetero")
        dout = torch.empty_like(out)
        ops.hetero_nll(out, batch.y.contiguous().float(), self.log_means, self.log_stds, self.floor, self.l2,
                       self.loss, dout, weights=sample_weights)
        model._engine.backward(st.P, st.G, ctx, dout)
        return self.loss

    def step(self, batch, seed: Optional[int] = None, sample_weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        if seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        if self._graph is not None and self._graph[2] is batch and sample_weights is None:
            return self._replay(seed)
        loss = self.forward_backward(batch, seed, sample_weights=sample_weights)
        if self.grad_hook is not None:
            self.grad_hook(self.st.grad)
        self._clip_and_update()
        self.step_count += 1
        return loss

    def _clip_and_update(self) -> None:
        if self.optimizer == "hip":
            st = self.st
            ops.grad_norm(st.grad, self.gnorm)
            ops.adamw_step(st.flat, st.grad, self.exp_avg, self.exp_avg_sq, st.P.sigma_start, self.lr, self.sigma_lr,
                           self.weight_decay, norm=self.gnorm, max_norm=self.max_norm, step=self.hip_step)
            return
        torch.nn.utils.clip_grad_norm_([self.p_base, self.p_sigma], max_norm=self.max_norm)
        self.opt.step()

    # --------------------------------------------------------------------------------------------
    # HIP-graph mode: the step (jitter, forward, loss, backward | clip, AdamW: ~300 kernels) is
    # captured once for a fixed batch as two graphs and replayed — no per-kernel host work and no
    # launch gaps.  ``grad_hook`` (e.g. the data-parallel all_reduce) runs eagerly between the two.
    # Randomness stays per step: the kernels read a device step seed (ops.set_step_seed) that
    # step() updates before each replay.  The learning rate is baked in at capture.
    # --------------------------------------------------------------------------------------------
    def capture(self, batch) -> None:
        """Capture the training step on ``batch`` (which must stay alive with unchanged shapes; its
        tensors may be refilled in place).  Model and optimizer state are left as they were."""
        dev = self.st.flat.device
        if self._seed_dev is None:
            self._seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        ops.set_step_seed(self._seed_dev)
        batch_cache(batch)
        # warm-up (allocations, optimizer state) on a side stream, then restore the state
        snap = self._snapshot()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                self.forward_backward(batch, 0)
                self._clip_and_update()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        profiling.clear()  # roofline probes (bench.py): keep only the launches captured below
        g_fb, g_up = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            self.forward_backward(batch, 0)
        with torch.cuda.graph(g_up, pool=g_fb.pool()):
            self._clip_and_update()
        torch.cuda.synchronize(dev)
        self._restore(snap)
        self._graph = (g_fb, g_up, batch)

    def _replay(self, seed: int) -> torch.Tensor:
        self._seed_dev.fill_(int(seed) & (2**63 - 1))
        self._graph[0].replay()
        if self.grad_hook is not None:
            self.grad_hook(self.st.grad)
        self._graph[1].replay()
        self.step_count += 1
        return self.loss

    def _snapshot(self):
        opt_state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                     for p, st in self.opt.state.items()}
        hip = None
        if self.optimizer == "hip":
            hip = (self.exp_avg.clone(), self.exp_avg_sq.clone(), self.hip_step.clone())
        return self.st.flat.clone(), opt_state, hip

    def _restore(self, snap) -> None:
        flat, opt_state, hip = snap
        self.st.flat.copy_(flat)
        if hip is not None:
            self.exp_avg.copy_(hip[0])
            self.exp_avg_sq.copy_(hip[1])
            self.hip_step.copy_(hip[2])
        for p, st in self.opt.state.items():
            saved = opt_state.get(id(p))
            for k, v in st.items():
                if torch.is_tensor(v):
                    if saved is not None and k in saved:
                        v.copy_(saved[k])
                    else:
                        v.zero_()
