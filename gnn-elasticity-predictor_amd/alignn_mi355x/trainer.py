"""Fused training step — the per-batch body of ``train_epoch_hetero`` (``scripts/train.py:639-699``).

Per step: feature jitter (train.py:641-646) -> forward (train.py:655) -> hetero NLL + log-sigma L2
(train.py:656-681) -> backward -> ``clip_grad_norm_(5.0)`` -> AdamW with the reference's two
parameter groups (train.py:1516-1542).  Forward, loss and backward run in libalignn_hip without
autograd; parameters and gradients live in one flat buffer each, so clip + AdamW touch two
contiguous segments (base + mean heads | logvar heads).
"""
from __future__ import annotations

import ctypes
import warnings
import weakref
from typing import Optional, Sequence

import torch
from torch import nn

from . import _lib, ops, profiling
from ._lib import check
from .engine import MIN_LOGVAR_FLOOR, adopt, batch_cache, batch_versions, clone_batch, site_seed

# batch fields a recorded step reads (train.py:547-573, :648-650); a re-bound batch is copied into
# the captured batch's buffers field by field
BATCH_FIELDS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y",
                "batch", "ptr")
from .model import HeteroAlignnRegressor
from .synthetic import TARGET_LOG_MEANS, TARGET_LOG_STDS


class FusedTrainer:
    def __init__(self, model: HeteroAlignnRegressor, lr: float = 3e-4, weight_decay: float = 1e-4,
                 sigma_lr: Optional[float] = 3e-4, max_norm: float = 5.0, log_sigma_l2: float = 0.1,
                 feature_jitter_std: float = 0.1, min_logvar_floor: float = MIN_LOGVAR_FLOOR,
                 target_log_means: Sequence[float] = TARGET_LOG_MEANS,
                 target_log_stds: Sequence[float] = TARGET_LOG_STDS, fused_adamw: bool = True,
                 optimizer: str = "hip", precision: Optional[str] = None, grad_scaler: Optional[bool] = None,
                 init_scale: float = 65536.0, growth_interval: int = 2000, amp_loss: Optional[bool] = None):
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
        # update of the reference's CPU AdamW (betas (0.9, 0.999), eps 1e-8, decoupled decay)
        if optimizer not in ("torch", "hip"):
            raise ValueError("optimizer must be 'torch' or 'hip'")
        self.optimizer = optimizer
        self.lr, self.sigma_lr, self.weight_decay = lr, sigma_lr, weight_decay
        if optimizer == "hip":
            self.exp_avg = torch.zeros_like(st.flat)
            self.exp_avg_sq = torch.zeros_like(st.flat)
            self.hip_step = torch.zeros(1, device=st.flat.device)
            self.gnorm = torch.zeros(1, device=st.flat.device)
        # GradScaler (train.py:690-695, built at :1475-1476 whenever the reference runs on the GPU,
        # i.e. with autocast: our bf16 precision): a step with non-finite (scaled) gradients is skipped
        # and the scale halves; device state [scale, growth_tracker, found_inf, skipped steps]
        # (default on for bf16 with the HIP optimizer; torch's optimizer runs without one)
        if grad_scaler is None:
            grad_scaler = model._engine.precision == "bf16" and optimizer == "hip"
            if model._engine.precision == "bf16" and optimizer == "torch":
                # the reference builds a GradScaler whenever it runs autocast on the GPU (train.py:1475-1476,
                # :690-695); torch's optimizer here has none: a non-finite step is applied, not skipped
                warnings.warn("FusedTrainer(precision='bf16', optimizer='torch') runs without a GradScaler: a step "
                              "with non-finite gradients is applied instead of skipped (optimizer='hip' skips it)",
                              stacklevel=2)
        if grad_scaler and optimizer != "hip":
            raise ValueError("grad_scaler needs optimizer='hip'")
        self.growth_interval = int(growth_interval)
        self.scaler = (torch.tensor([float(init_scale), 0.0, 0.0, 0.0], device=st.flat.device) if grad_scaler
                       else None)
        # bf16: the loss on the heads as autocast returns them (bf16) with autocast's dtypes and
        # autograd's gradient roundings (train.py:653-681; ops.hetero_nll amp) — the step the module
        # API runs under the reference's own autocast + GradScaler loop, bit for bit
        self.amp_loss = (model._engine.precision == "bf16") if amp_loss is None else bool(amp_loss)
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
        self._bound, self._bound_v = (lambda: None), ()   # the batch the captured slot holds
        self._seed_dev = None
        # the engine's execution context (workspaces, side stream, device step seed): every launch of
        # this trainer's step runs in it, and a recorded plan owns it (its buffers never move)
        self.ctx = model._engine.ctx
        self.grad_hook = None  # called with the flat gradient between backward and clip (DP all_reduce)
        # data-parallel gradient mean in two buckets (dp.GradBuckets): the first reduced while the
        # backward's tail runs; takes the place of grad_hook when set
        self.grad_buckets = None
        # re-binding (step() on a batch other than the captured one): copy it into the captured
        # batch's buffers and replay when its signature matches (BatchCache.signature), else eager
        self.rebind = True
        # check mode of the filtered re-binding copy: copy every buffer of the batch and its cache, not
        # only those alignn_plan_refs finds among the recorded arguments (a test replays both ways and
        # compares: a recorded kernel reaching batch memory some other way would show up there)
        self.rebind_copy_all = False
        self.rebinds = 0
        self.rebind_misses = 0
        # roofline probes (bench.py): replay the plans serialised on one stream (each kernel alone on
        # the device; alignn_plan_replay_serial) instead of on their recorded streams
        self.serial_replay = False
        self.replays = 0
        self.lr_dev = None
        self._wbuf = None      # a weighted capture's per-graph weights (device [real graphs])
        self._exchange = ("none", None)   # the gradient exchange the captured phases were cut for

    def use_step_seed(self, t: Optional[torch.Tensor]) -> None:
        """Device int64[1] step seed the dropout/jitter kernels of this trainer mix in (None: host
        seeds only).  capture() installs its own; tests share one between two trainers."""
        if t is not None and (t.dtype != torch.int64 or t.numel() != 1 or not t.is_cuda):
            raise ValueError("step seed must be a device int64 tensor with one element")
        self.ctx.step_seed = t

    def set_lr(self, lr: float, sigma_lr: Optional[float] = None) -> None:
        """The reference's per-epoch learning rate (train.py:1641-1652; cosine schedule :1215-1232).
        The HIP optimizer reads the rates from a device scalar pair, so captured plans follow."""
        self.opt.param_groups[0]["lr"] = lr
        self.opt.param_groups[1]["lr"] = lr if sigma_lr is None else sigma_lr
        self.lr, self.sigma_lr = lr, (lr if sigma_lr is None else sigma_lr)
        if self.lr_dev is not None:
            # stream-ordered: steps already queued keep the old rates, later ones get the new
            self.lr_dev.copy_(torch.tensor([float(self.lr), float(self.sigma_lr)], dtype=torch.float64),
                              non_blocking=False)

    def forward_backward(self, batch, seed: int, training: bool = True,
                         sample_weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward + loss + backward into the flat gradient buffer; returns the loss (device).
        sample_weights: per-graph KNN weights [B] (train.py:660-674), or None.  With grad_buckets the
        first bucket's reduction is started between the per-layer backward and the tail (it is
        finished by step())."""
        t = self._fb_layers(batch, seed, training, sample_weights)
        if self.grad_buckets is not None:
            self.grad_buckets.start(self.ctx.side(self.st.flat.device))
        self._fb_tail(t)
        return self.loss

    def _fb_layers(self, batch, seed: int, training: bool = True, sample_weights: Optional[torch.Tensor] = None):
        """Forward, loss and the per-layer backward (the first phase of a captured step)."""
        adopt(batch)
        with ops.using(self.ctx):
            return self._forward_backward(batch, seed, training, sample_weights)

    def _fb_tail(self, t) -> None:
        """The backward's tail (the second phase)."""
        with ops.using(self.ctx):
            self.model._engine.backward_tail(t)

    def _forward_backward(self, batch, seed: int, training: bool, sample_weights: Optional[torch.Tensor]):
        model, st = self.model, self.st
        bc = batch_cache(batch)
        x, gx = batch.x, batch.global_x
        if training and self.jitter > 0.0:
            # jittered copies of the node and global features (train.py:641-646), one launch
            x, gx = ops.noisy_copies(x, site_seed(seed, 1 << 20), gx, site_seed(seed, (1 << 20) + 1), self.jitter)
        out, ctx = model._engine.forward(st.P, batch, bc, training, seed, x, gx, "hetero")
        dout = torch.empty_like(out)
        # a batch padded to a capacity (store.BatchCapacity): the loss is the real graphs' mean and the
        # ghost graph's heads get a zero gradient
        nr = out.size(0) if bc.real_graphs is None else bc.real_graphs
        y = batch.y.contiguous().float()
        ops.hetero_nll(out[:nr], y[:nr * (out.size(1) // 2)], self.log_means, self.log_stds, self.floor, self.l2,
                       self.loss, dout[:nr], weights=sample_weights, amp=self.amp_loss)
        if nr < out.size(0):
            ops.zero_(dout[nr:])
        return model._engine.backward_layers(st.P, st.G, ctx, dout)

    def step(self, batch, seed: Optional[int] = None, sample_weights: Optional[torch.Tensor] = None) -> torch.Tensor:
        if seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        adopt(batch)   # a loader-prepared batch: wait for it and mark its buffers as used here (any path)
        if self._graph is not None and self._weights_match(sample_weights):
            # a weighted capture (KNN weights, train.py:660-674) reads the per-graph weights from its
            # own device buffer: the step's weights are copied there in the re-binding launch
            extra = [] if sample_weights is None else [(self._wbuf, sample_weights)]
            if self._bound() is batch and batch_versions(batch, BATCH_FIELDS) == self._bound_v:
                # the slot holds this batch already (the captured batch, or the last one re-bound)
                if extra:
                    with ops.using(self.ctx):
                        ops.copy_many(extra)
                return self._replay(seed)
            if self.rebind and self._rebind(batch, extra):
                return self._replay(seed)
        loss = self.forward_backward(batch, seed, sample_weights=sample_weights)
        if self.grad_buckets is not None:
            self.grad_buckets.finish()
        elif self.grad_hook is not None:
            self.grad_hook(self.st.grad)
        self._clip_and_update()
        self.step_count += 1
        return loss

    def _weights_match(self, w: Optional[torch.Tensor]) -> bool:
        """The step's sample weights fit the captured step: none for an unweighted capture; for a
        weighted one, a float32 device tensor of the captured batch's real-graph count."""
        if (w is None) != (self._wbuf is None):
            return False
        return w is None or (w.dtype == torch.float32 and w.is_cuda and w.shape == self._wbuf.shape
                             and w.device == self._wbuf.device)

    def _rebind(self, batch, extra=()) -> bool:
        """Copies ``batch`` into the captured batch's buffers (fields and device cache) when every
        size the recorded launches depend on matches; False (nothing copied) otherwise.  A batch
        prepared on another stream (engine.prepare_batch) was adopted by step() (engine.adopt)."""
        slot = self._graph[2]
        v = batch_versions(batch, BATCH_FIELDS)
        for k in BATCH_FIELDS:
            a, b = getattr(batch, k, None), getattr(slot, k, None)
            if (a is None) != (b is None):
                self.rebind_misses += 1
                return False
            if a is not None and (a.shape != b.shape or a.dtype != b.dtype or a.device != b.device):
                self.rebind_misses += 1
                return False
        with ops.using(self.ctx):   # a cache built here uses the engine's workspaces, not the shared ones
            bc_new, bc_slot = batch_cache(batch), batch_cache(slot)
            if bc_new.signature() != bc_slot.signature():
                self.rebind_misses += 1
                return False
            pairs = [(getattr(slot, k), getattr(batch, k)) for k in BATCH_FIELDS
                     if getattr(batch, k, None) is not None and getattr(batch, k).numel()]
            pairs += bc_new.copy_pairs(bc_slot)
            used = self._graph[5]   # data_ptr of every captured buffer the plans touch (None: all)
            if used is not None and not self.rebind_copy_all:
                pairs = [(d, s) for d, s in pairs if d.data_ptr() in used]
            ops.copy_many(pairs + list(extra))   # one launch for the batch, its cache and the weights
        self._bound, self._bound_v = weakref.ref(batch), v
        self.rebinds += 1
        return True

    def _clip_and_update(self) -> None:
        if self.optimizer == "hip":
            st = self.st
            if self.lr_dev is None:
                self.lr_dev = torch.tensor([float(self.lr), float(self.sigma_lr)], dtype=torch.float64,
                                           device=st.flat.device)
            with ops.using(self.ctx):
                if self.scaler is not None:
                    ops.grad_norm_amp(st.grad, self.gnorm, self.scaler)
                else:
                    ops.grad_norm(st.grad, self.gnorm)
                ops.adamw_step(st.flat, st.grad, self.exp_avg, self.exp_avg_sq, st.P.sigma_start, self.lr,
                               self.sigma_lr, self.weight_decay, norm=self.gnorm, max_norm=self.max_norm,
                               step=self.hip_step, lr_dev=self.lr_dev, scaler=self.scaler,
                               growth_interval=self.growth_interval)
            return
        torch.nn.utils.clip_grad_norm_([self.p_base, self.p_sigma], max_norm=self.max_norm)
        self.opt.step()

    # --------------------------------------------------------------------------------------------
    # Captured step (fixed batch).  The step (jitter, forward, loss, backward | clip, AdamW: ~300
    # kernels on two streams) is recorded once and re-issued without per-kernel Python work.
    #   mode "plan" (default): two native launch plans (plan.hip) — every library launch and every
    #     cross-stream edge of the step, replayed from C++ onto the same two streams.  Recorded
    #     inside a torch graph capture, whose private memory pool keeps every buffer of the step at
    #     its address; the captured graph's node census must match the plan (nothing foreign), and
    #     every device pointer the plan holds must lie in a buffer the trainer owns (its state, the
    #     batch and its CSR cache, its engine's workspaces — sized by the warm-up steps and frozen
    #     during the recording — or the capture's pool): alignn_plan_check_ptrs.
    #   mode "graph": ROCm HIP graphs of the same capture (measured slower on MI355X: 5.5 vs 5.2 ms
    #     eager, the two streams' branches lose concurrency).
    # ``grad_hook`` (e.g. the data-parallel all_reduce) runs eagerly between the two phases.
    # Randomness stays per step: the kernels read a device step seed (ops.set_step_seed) that
    # step() updates before each replay.  The learning rates are a device pair (set_lr).
    # A new batch of the same signature is copied into the captured batch (``_rebind``), so the
    # reference's loop over fresh batches (train.py:639-711) replays the plan every step.
    # --------------------------------------------------------------------------------------------
    def capture(self, batch, mode: str = "plan", weighted: bool = False) -> None:
        """Capture the training step on ``batch``.  The plans read a private copy of it (the slot): a
        step on another batch of the same signature copies that batch into the slot (re-binding), and a
        step on the batch the slot holds — unmodified since (torch's in-place version counters) —
        replays directly; the caller's tensors are never written.  Model and optimizer state are left
        as they were.
        weighted: the step of the reference's KNN-weighted epochs (train.py:660-674) — the loss reads
        per-graph weights from a device buffer of this trainer that step(sample_weights=w) fills."""
        if mode not in ("plan", "graph"):
            raise ValueError("capture mode must be 'plan' or 'graph'")
        if mode == "plan" and self.optimizer != "hip":
            raise ValueError("plan capture needs optimizer='hip' (torch's AdamW launches outside the library)")
        dev = self.st.flat.device
        self.release_capture()
        adopt(batch)
        self._bound, self._bound_v = weakref.ref(batch), batch_versions(batch, BATCH_FIELDS)
        batch = clone_batch(batch)
        if self._seed_dev is None:
            self._seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.use_step_seed(self._seed_dev)
        with ops.using(self.ctx):
            bc = batch_cache(batch)
        self._wbuf = None
        if weighted:
            nr = bc.real_graphs if bc.real_graphs is not None else bc.B
            self._wbuf = torch.ones(nr, device=dev)
        w = self._wbuf
        # warm-up (allocations, optimizer state, every workspace at this batch's sizes) on a side
        # stream, then restore the state
        snap = self._snapshot()
        s = ops.warmup_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fb_tail(self._fb_layers(batch, 0, sample_weights=w))   # (no gradient exchange here)
                self._clip_and_update()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        profiling.clear()  # roofline probes (bench.py): keep only the launches captured below
        keep = mode == "plan"
        # phases: forward/backward | clip/AdamW; with grad_buckets the backward splits at the end of
        # the per-layer part, where the first bucket's all_reduce is issued between the two phases
        state = {}
        if self.grad_buckets is None:
            phases = [("forward/backward", lambda: self._fb_tail(self._fb_layers(batch, 0, sample_weights=w)))]
        else:
            def layers_phase():
                state["t"] = self._fb_layers(batch, 0, sample_weights=w)
                join_forks()
            phases = [("forward/backward layers", layers_phase),
                      ("backward tail", lambda: self._fb_tail(state["t"]))]
        phases.append(("clip/AdamW", self._clip_and_update))
        # the per-layer phase leaves weight-gradient work queued on the engine's side stream; a graph
        # capture must end with every forked stream joined, and the join is part of the recorded plan
        # too: the next phase's allocations may reuse memory that this work still reads (the capture's
        # allocator releases cross-stream blocks at the end of each captured phase), so a replay
        # without the join let the tail overwrite the last blocks' weight-gradient inputs
        # (test_bucketed_dp_plan_replay_bitwise, intermittent).  The first bucket's exchange, issued
        # after the phase, still overlaps the tail.
        engine_ctx = self.model._engine.ctx

        def join_forks():
            cur = torch.cuda.current_stream(dev)
            for st in list(engine_ctx._side.values()) + list(engine_ctx._aux.values()):
                ops.stream_wait(cur, st)   # a torch wait, noted in the plan being recorded
        graphs = [torch.cuda.CUDAGraph(keep_graph=keep) for _ in phases]
        plans = []
        try:
            with ops.recording():
                for i, (g, (_, fn)) in enumerate(zip(graphs, phases)):
                    with torch.cuda.graph(g, pool=(graphs[0].pool() if i else None)):
                        if keep:
                            plans.append(_record_plan(fn))
                        else:
                            fn()
            state.clear()
            torch.cuda.synchronize(dev)
            self._restore(snap)
            if keep:
                ranges = self._held_ranges(batch, graphs[0].pool())
                for g, pl, (what, _) in zip(graphs, plans, phases):
                    _check_census(g, pl, what)
                    _check_deps(g, pl, what)
                    _check_ownership(pl, ranges, what)
        except Exception:
            for pl in plans:
                _lib.lib().alignn_plan_destroy(pl)
            self._wbuf = None
            raise
        self._graph = (graphs[0], graphs[-1], batch, plans if keep else None, graphs,
                       _plan_refs(plans, self._rebind_targets(batch)) if keep else None)
        # the gradient exchange the phases were cut for (the bucketed exchange needs three phases, a
        # hook or none two): a replay checks that it is still the one in place
        self._exchange = self._exchange_mode()
        self.ctx.freeze()   # the plans hold the workspaces' addresses: eager steps may not replace them

    def _exchange_mode(self):
        if self.grad_buckets is not None:
            return ("buckets", self.grad_buckets)
        return ("hook", self.grad_hook) if self.grad_hook is not None else ("none", None)

    @staticmethod
    def _rebind_targets(batch):
        """The captured batch's buffers a re-binding copy may write: its fields and its device cache."""
        ts = [getattr(batch, k) for k in BATCH_FIELDS if getattr(batch, k, None) is not None]
        ts += [t for t in batch_cache(batch).device_tensors() if t is not None]
        return [t for t in ts if t.numel()]

    def _held_ranges(self, batch, pool_id):
        """[lo, hi) device byte ranges this trainer holds for as long as a captured plan lives: its own
        state, the model's buffers, the batch and its device caches, the engine's workspaces, and the
        segments of the capture's private memory pool (kept by the captured graph)."""
        ranges = []
        for t in _cuda_tensors((self.st.flat, self.st.grad, getattr(self, "exp_avg", None),
                                getattr(self, "exp_avg_sq", None), getattr(self, "hip_step", None),
                                getattr(self, "gnorm", None), self.scaler, self.lr_dev, self.loss, self.log_means, self.log_stds,
                                self._seed_dev, self._wbuf, self.ctx.tensors(), batch, list(self.model.buffers()))):
            s = t.untyped_storage()
            ranges.append((s.data_ptr(), s.data_ptr() + s.nbytes()))
        pool = tuple(pool_id)
        for seg in torch.cuda.memory_snapshot():
            if tuple(seg.get("segment_pool_id", ())) == pool:
                ranges.append((seg["address"], seg["address"] + seg["total_size"]))
        return ranges

    def release_capture(self) -> None:
        self._wbuf = None
        if self._graph is not None:
            if self._graph[3]:
                for pl in self._graph[3]:
                    _lib.lib().alignn_plan_destroy(pl)
            self.ctx.thaw()
        self._graph = None

    def __del__(self):
        try:
            self.release_capture()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _replay(self, seed: int) -> torch.Tensor:
        mode = self._exchange_mode()
        if mode[0] != self._exchange[0] or mode[1] is not self._exchange[1]:
            raise RuntimeError(f"gradient exchange changed after capture (captured: {self._exchange[0]}, now: "
                               f"{mode[0]}): set grad_buckets / grad_hook before capture(), or capture again")
        check(_lib.lib().alignn_set_i64(self._seed_dev.data_ptr(), int(seed) & (2**63 - 1), ops.stream_ptr()),
              "alignn_set_i64")
        plans = self._graph[3]
        graphs = self._graph[4] if len(self._graph) > 4 else [self._graph[0], self._graph[1]]
        n = len(plans) if plans else len(graphs)

        def run(i):
            if plans and self.serial_replay:
                check(_lib.lib().alignn_plan_replay_serial(plans[i], ops.stream_ptr()), "alignn_plan_replay_serial")
            elif plans:
                check(_lib.lib().alignn_plan_replay(plans[i], ops.stream_ptr()), "alignn_plan_replay")
            else:
                graphs[i].replay()

        run(0)
        if n == 3:   # bucketed: first bucket beside the backward's tail, the rest after it
            self.grad_buckets.start(self.ctx.side(self.st.flat.device))
            run(1)
            self.grad_buckets.finish()
        elif self.grad_hook is not None:
            self.grad_hook(self.st.grad)
        run(n - 1)
        self.step_count += 1
        self.replays += 1
        return self.loss

    def _snapshot(self):
        opt_state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                     for p, st in self.opt.state.items()}
        hip = None
        if self.optimizer == "hip":
            hip = (self.exp_avg.clone(), self.exp_avg_sq.clone(), self.hip_step.clone(),
                   None if self.scaler is None else self.scaler.clone())
        return self.st.flat.clone(), opt_state, hip

    def _restore(self, snap) -> None:
        flat, opt_state, hip = snap
        self.st.flat.copy_(flat)
        if hip is not None:
            self.exp_avg.copy_(hip[0])
            self.exp_avg_sq.copy_(hip[1])
            self.hip_step.copy_(hip[2])
            if hip[3] is not None:
                self.scaler.copy_(hip[3])
        for p, st in self.opt.state.items():
            saved = opt_state.get(id(p))
            for k, v in st.items():
                if torch.is_tensor(v):
                    if saved is not None and k in saved:
                        v.copy_(saved[k])
                    else:
                        v.zero_()


def _record_plan(fn) -> int:
    """Runs fn (inside the caller's capture) while the library records a launch plan."""
    lib = _lib.lib()
    check(lib.alignn_plan_begin(ops.stream_ptr()), "alignn_plan_begin")
    profiling.plan_recording(True)
    try:
        fn()
    except BaseException:
        lib.alignn_plan_abort()
        raise
    finally:
        profiling.plan_recording(False)
    plan = lib.alignn_plan_end()
    if not plan:
        check(-1, "alignn_plan_end")
    profiling.bind_plan(plan)
    return plan


def _plan_refs(plans, tensors) -> set:
    """data_ptr of each tensor some recorded plan points into (alignn_plan_refs over all phases):
    a re-bound batch is copied into these buffers only — the raw line-graph index and angle
    features, for instance, are read when the batch's cache is built, never by the step."""
    arr = (ctypes.c_uint64 * (2 * len(tensors)))(*[v for t in tensors
                                                    for v in (t.data_ptr(), t.data_ptr() + t.numel() * t.element_size())])
    used = set()
    for pl in plans:
        hit = (ctypes.c_int32 * len(tensors))()
        check(_lib.lib().alignn_plan_refs(pl, arr, len(tensors), hit), "alignn_plan_refs")
        used.update(t.data_ptr() for t, h in zip(tensors, hit) if h)
    return used


def plan_info(plan) -> dict:
    v = [ctypes.c_int64() for _ in range(4)]
    check(_lib.lib().alignn_plan_info(plan, *[ctypes.byref(x) for x in v]), "alignn_plan_info")
    return dict(zip(("launches", "edges", "streams", "arg_bytes"), (x.value for x in v)))


def _cuda_tensors(root, depth: int = 6):
    """Every device tensor reachable from ``root`` through containers and object attributes."""
    out, seen = [], set()

    def walk(o, d):
        if o is None or id(o) in seen or d < 0:
            return
        seen.add(id(o))
        if torch.is_tensor(o):
            if o.is_cuda and o.numel():
                out.append(o)
            return
        if isinstance(o, (list, tuple, set)):
            for v in o:
                walk(v, d - 1)
        elif isinstance(o, dict):
            for v in o.values():
                walk(v, d - 1)
        elif not isinstance(o, (int, float, str, bytes, bool, torch.nn.Module)) and not callable(o):
            for v in getattr(o, "__dict__", {}).values():
                walk(v, d - 1)
            for k in getattr(type(o), "__slots__", ()):
                walk(getattr(o, k, None), d - 1)

    walk(root, depth)
    return out


def _check_ownership(plan, ranges, what: str) -> None:
    """Every device pointer the recorded plan holds lies in a buffer the trainer holds (host check)."""
    arr = (ctypes.c_uint64 * (2 * len(ranges)))(*[v for r in ranges for v in r])
    bad, idx, n = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int64()
    rc = _lib.lib().alignn_plan_check_ptrs(plan, arr, len(ranges), ctypes.byref(bad), ctypes.byref(idx),
                                           ctypes.byref(n))
    if rc != 0:
        msg = _lib.lib().alignn_last_error()
        raise RuntimeError(f"launch plan of the {what} phase references memory the trainer does not hold "
                           f"(launch {idx.value}, 0x{bad.value:x}): {msg.decode() if msg else ''}")


def _check_deps(graph: torch.cuda.CUDAGraph, plan, what: str) -> int:
    """Every ordering the captured graph has between two kernels must be one the plan replays (its
    slot order + the waits noted by ops.stream_wait), and the plan must end with every stream joined
    (alignn_plan_check_deps).  A torch-level wait that bypassed ops.stream_wait fails the capture here
    instead of racing on replay.  Returns the number of kernel dependencies checked."""
    a, b, e = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = _lib.lib().alignn_plan_check_deps(plan, ctypes.c_void_p(graph.raw_cuda_graph()), ctypes.byref(a),
                                           ctypes.byref(b), ctypes.byref(e))
    if rc != 0:
        msg = _lib.lib().alignn_last_error()
        raise RuntimeError(f"launch plan of the {what} phase misses a stream dependency of its capture "
                           f"(launches {a.value} -> {b.value}): {msg.decode() if msg else ''}")
    return e.value


def _check_census(graph: torch.cuda.CUDAGraph, plan, what: str) -> None:
    """Every kernel node of the captured graph must be a recorded launch and nothing else may be
    in it (a torch op inside the step would run in the graph but not in the plan)."""
    k, o = ctypes.c_int64(), ctypes.c_int64()
    check(_lib.lib().alignn_graph_census(ctypes.c_void_p(graph.raw_cuda_graph()), ctypes.byref(k), ctypes.byref(o)),
          "alignn_graph_census")
    info = plan_info(plan)
    if k.value != info["launches"] or o.value != 0:
        raise RuntimeError(f"launch plan of the {what} phase is incomplete: the captured graph holds {k.value} "
                           f"kernel and {o.value} other nodes, the plan {info['launches']} launches")
