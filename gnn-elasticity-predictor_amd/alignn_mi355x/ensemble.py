"""Deep-ensemble inference on the MI355X engine.

Reference: ``ensemble_collect`` / ``ensemble_collect_embeddings`` (scripts/train.py:849-927),
``_fit_affine_debias`` / ``conformal_calibration`` / ``apply_conformal_intervals``
(train.py:1013-1076) and ``predict.ensemble_predict`` (scripts/predict.py:582-653).

MI355X design: the M members share one batch preparation (CSR lists, line-graph compaction); their
forwards (eval mode, no autograd) run concurrently, one HIP stream per member — the attention
kernels are latency-bound, so members overlap on the CUs — and one kernel
(``alignn_ensemble_moments``) does the moment mix and the log-normal conversion.  Calibration
(affine debias, conformal quantile) runs on the host over the collected [n, T] predictions, as in
the reference.  Members on different GPUs: run one ``EnsemblePredictor`` of one member per rank and
gather the [B, 2T] heads to one rank (:class:`ShardedEnsemble`).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib, infer
from .engine import MIN_LOGVAR_FLOOR, batch_cache
from .ops import stream_ptr
from .synthetic import TARGET_LOG_MEANS, TARGET_LOG_STDS

Z_SCORE_90 = 1.6448536269514722  # predict.py:63


class EnsemblePredictor:
    def __init__(self, models: Sequence, min_logvar_floor: float = MIN_LOGVAR_FLOOR,
                 target_log_means: Sequence[float] = TARGET_LOG_MEANS,
                 target_log_stds: Sequence[float] = TARGET_LOG_STDS, concurrent: bool = True):
        if not models:
            raise ValueError("EnsemblePredictor needs at least one member")
        self.models = list(models)
        self.floor = float(min_logvar_floor)
        self.concurrent = concurrent
        self._streams: List[torch.cuda.Stream] = []
        self._log_means = list(target_log_means)
        self._log_stds = list(target_log_stds)
        self._lm = self._ls = None

    def _member_streams(self, dev) -> List[Optional[torch.cuda.Stream]]:
        if not self.concurrent:
            return [None] * len(self.models)
        while len(self._streams) < len(self.models):
            self._streams.append(torch.cuda.Stream(device=dev))
        return self._streams[:len(self.models)]

    def member_outputs(self, batch, mode: str = "hetero") -> torch.Tensor:
        """[M, B, 2T] heads (hetero) or [M, B, D] embeddings, members in eval mode (dropout off)."""
        batch_cache(batch)   # the batch's cache built once, on the caller's stream
        dev = batch.x.device
        main = torch.cuda.current_stream(dev)
        outs = []
        for m, s in zip(self.models, self._member_streams(dev)):
            # each member's forward as a replayed launch plan once the batch signature repeats
            # (infer.forward; its output lives in the plan until the stack below copies it)
            if s is None:
                out = infer.forward(m, batch, mode)
            else:
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    out = infer.forward(m, batch, mode)
                out.record_stream(main)
            outs.append(out)
        for s in self._member_streams(dev):
            if s is not None:
                main.wait_stream(s)
        return torch.stack(outs, 0)

    def _stats(self, dev):
        if self._lm is None or self._lm.device != dev:
            self._lm = torch.tensor(self._log_means, dtype=torch.float32, device=dev)
            self._ls = torch.tensor(self._log_stds, dtype=torch.float32, device=dev)
        return self._lm, self._ls

    def _moments(self, heads: torch.Tensor, convert: bool) -> Dict[str, torch.Tensor]:
        lm, ls = self._stats(heads.device)
        return ensemble_moments(heads, self.floor, lm if convert else None, ls if convert else None)

    def predict_batch(self, batch) -> Dict[str, torch.Tensor]:
        """predict.ensemble_predict for one batch (device tensors, [B, T] each): mean_z, std_z
        (standardized log space), mean_orig (= mu), std_lin (= sigma), lo90/hi90 (ci90)."""
        return self._moments(self.member_outputs(batch), convert=True)

    def collect(self, batches) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """ensemble_collect (hetero): (mean_z [n,T], targets [n,T], std_z [n,T]) on the host."""
        means, stds, ys = [], [], []
        for b in batches:
            r = self._moments(self.member_outputs(b), convert=False)
            means.append(r["mean_z"].cpu())
            stds.append(r["std_z"].cpu())
            ys.append(b.y.view(b.num_graphs, -1).float().cpu())
        if not means:
            raise ValueError("No batches produced predictions.")
        return torch.cat(means), torch.cat(ys), torch.cat(stds)

    def embed(self, batches) -> torch.Tensor:
        """ensemble_collect_embeddings: member-mean of embed() per graph, host [n, D]."""
        out = []
        for b in batches:
            out.append(member_mean(self.member_outputs(b, mode="embed")).cpu())
        if not out:
            raise ValueError("No batches produced embeddings.")
        return torch.cat(out)


def ensemble_moments(heads: torch.Tensor, floor: float, log_means: Optional[torch.Tensor] = None,
                     log_stds: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """One kernel over member heads ``[M, B, 2T]`` (mean | logvar): mean_z, std_z
    (train.py:875-902); with the target stats on the device also mean_orig, std_lin, lo90, hi90
    (predict.py:616-640)."""
    M, B, W = heads.shape
    T = W // 2
    dev = heads.device
    convert = log_means is not None
    names = ("mean_z", "std_z") + (("mean_orig", "std_lin", "lo90", "hi90") if convert else ())
    res = {k: torch.empty(B, T, device=dev) for k in names}
    ptr = lambda k: res[k].data_ptr() if k in res else None  # noqa: E731
    h = heads.contiguous()
    _lib.check(_lib.lib().alignn_ensemble_moments(
        M, B, T, h.data_ptr(), h.stride(0), h.stride(1), float(floor),
        log_means.data_ptr() if convert else None, log_stds.data_ptr() if convert else None,
        ptr("mean_z"), ptr("std_z"), ptr("mean_orig"), ptr("std_lin"), ptr("lo90"), ptr("hi90"),
        stream_ptr()), "alignn_ensemble_moments")
    return res


def member_mean(outs: torch.Tensor) -> torch.Tensor:
    """Mean over members of ``[M, B, D]`` (ensemble_collect_embeddings, train.py:907-927)."""
    e = outs.contiguous()
    mean = torch.empty(e.shape[1:], device=e.device)
    _lib.check(_lib.lib().alignn_member_mean_f32(e.size(0), mean.numel(), e.data_ptr(), e.stride(0),
                                                 mean.data_ptr(), stream_ptr()), "alignn_member_mean_f32")
    return mean


class ShardedEnsemble:
    """Members spread over the ranks of a process group (one member per GPU).

    Rank r runs the members ``dp.members_of_rank(num_members, world, r)`` (``local_models``, in that
    order; an empty list on ranks without members) concurrently on its GPU; every batch ends with one
    gather of the [m_r, B, W] outputs to ``dst``, which does the moment mix.  Same results as an
    :class:`EnsemblePredictor` holding all members on one device; the methods return ``None`` on
    ranks other than ``dst``.  Every rank must call them with the same batches (same graph counts)."""

    def __init__(self, local_models: Sequence, num_members: int, target_dim: int = 2, hidden: int = 256,
                 dst: int = 0, group=None, min_logvar_floor: float = MIN_LOGVAR_FLOOR,
                 target_log_means: Sequence[float] = TARGET_LOG_MEANS,
                 target_log_stds: Sequence[float] = TARGET_LOG_STDS, concurrent: bool = True):
        from . import dp
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        mine = dp.members_of_rank(num_members, self.world, self.rank)
        if len(local_models) != len(mine):
            raise ValueError(f"rank {self.rank} must hold members {mine}, got {len(local_models)} models")
        self.num_members, self.dst, self.group = int(num_members), int(dst), group
        self.widths = {"hetero": 2 * int(target_dim), "embed": int(hidden)}
        self.local = (EnsemblePredictor(local_models, min_logvar_floor, target_log_means, target_log_stds, concurrent)
                      if local_models else None)
        self.floor = float(min_logvar_floor)
        self._log_means, self._log_stds = list(target_log_means), list(target_log_stds)

    def _gathered(self, batch, mode: str) -> Optional[torch.Tensor]:
        from . import dp
        if self.local is not None:
            out = self.local.member_outputs(batch, mode)
        else:
            out = torch.empty(0, int(batch.num_graphs), self.widths[mode], device=batch.x.device)
        return dp.gather_member_heads(out, self.num_members, dst=self.dst, group=self.group)

    def _mix(self, heads: torch.Tensor, convert: bool) -> Dict[str, torch.Tensor]:
        if not convert:
            return ensemble_moments(heads, self.floor)
        dev = heads.device
        lm = torch.tensor(self._log_means, dtype=torch.float32, device=dev)
        ls = torch.tensor(self._log_stds, dtype=torch.float32, device=dev)
        return ensemble_moments(heads, self.floor, lm, ls)

    def predict_batch(self, batch) -> Optional[Dict[str, torch.Tensor]]:
        heads = self._gathered(batch, "hetero")
        return None if heads is None else self._mix(heads, convert=True)

    def collect(self, batches) -> Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        means, stds, ys = [], [], []
        for b in batches:
            heads = self._gathered(b, "hetero")
            if heads is None:
                continue
            r = self._mix(heads, convert=False)
            means.append(r["mean_z"].cpu())
            stds.append(r["std_z"].cpu())
            ys.append(b.y.view(b.num_graphs, -1).float().cpu())
        if self.rank != self.dst:
            return None
        if not means:
            raise ValueError("No batches produced predictions.")
        return torch.cat(means), torch.cat(ys), torch.cat(stds)

    def embed(self, batches) -> Optional[torch.Tensor]:
        out = []
        for b in batches:
            e = self._gathered(b, "embed")
            if e is not None:
                out.append(member_mean(e).cpu())
        if self.rank != self.dst:
            return None
        if not out:
            raise ValueError("No batches produced embeddings.")
        return torch.cat(out)


class EnsembleTrainer:
    """Ensemble training sharded member-per-rank.

    The reference trains its members one after the other on one device (train.py:2052-2095):
    member i is seeded ``seed + 1007 i`` (train.py:2053, before the model is built) and trains against
    fold ``i % num_folds`` (:2054).  Here member i lives on rank ``i % world`` (dp.members_of_rank);
    a rank's members each get their own :class:`FusedTrainer` (own execution context, workspaces and
    device step seed), captured as a native launch plan on its own batch, and :meth:`step` issues
    every local member's step at once, one HIP stream per member, so their latency-bound attention
    kernels share the CUs.  Members never communicate while training.

    ``build_model()`` is called right after ``torch.manual_seed(member_seed(seed, i))`` and must return
    the member's model on the device; ``batch_for(i, fold)`` returns member i's (resident) batch."""

    def __init__(self, num_members: int, build_model, batch_for, world: int = 1, rank: int = 0, seed: int = 42,
                 num_folds: int = 5, precision: Optional[str] = None, capture: bool = True, concurrent: bool = True,
                 trainer_kw: Optional[Dict] = None, members: Optional[Sequence[int]] = None):
        from . import dp
        from .trainer import FusedTrainer
        self.num_members, self.seed = int(num_members), int(seed)
        self.ids = list(members) if members is not None else dp.members_of_rank(num_members, world, rank)
        self.members = []
        for i in self.ids:
            torch.manual_seed(dp.member_seed(seed, i))
            model = build_model()
            tr = FusedTrainer(model, precision=precision, **(trainer_kw or {}))
            batch = batch_for(i, dp.member_fold(i, num_folds))
            if capture:
                tr.capture(batch)
            self.members.append((i, model, tr, batch))
        dev = self.members[0][1]._ensure_flat().flat.device if self.members else None
        self.streams = [torch.cuda.Stream(device=dev) if concurrent else None for _ in self.members]

    def step_seed(self, i: int, k: int) -> int:
        """Host seed of member i's k-th step (a function of the member, not of its placement)."""
        from . import dp
        return dp.member_seed(self.seed, i) * 1000003 + int(k)

    def step(self, k: int) -> None:
        """Step k of every local member (concurrently: one stream each, joined at the end)."""
        if not self.members:
            return
        dev = self.members[0][3].x.device
        main = torch.cuda.current_stream(dev)
        for (i, _, tr, batch), s in zip(self.members, self.streams):
            if s is None:
                tr.step(batch, seed=self.step_seed(i, k))
                continue
            s.wait_stream(main)
            with torch.cuda.stream(s):
                tr.step(batch, seed=self.step_seed(i, k))
        for s in self.streams:
            if s is not None:
                main.wait_stream(s)

    def models(self) -> List:
        return [m for _, m, _, _ in self.members]

    def release(self) -> None:
        for _, _, tr, _ in self.members:
            tr.release_capture()


# ------------------------------------------------------------------------------------------------
# Calibration on the collected predictions (host, as in the reference)
# ------------------------------------------------------------------------------------------------
def fit_affine_debias(pred_z: torch.Tensor, target_z: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """train.py:1013-1026: per-target least squares target_z ~ a * pred_z + b (float64 solve)."""
    p = pred_z.detach().float().cpu().numpy()
    t = target_z.detach().float().cpu().numpy()
    a = np.zeros(p.shape[1])
    b = np.zeros(p.shape[1])
    for k in range(p.shape[1]):
        X = np.stack([p[:, k], np.ones_like(p[:, k])], axis=1)
        sol = np.linalg.lstsq(X, t[:, k], rcond=None)[0]
        a[k], b[k] = sol[0], sol[1]
    return (torch.from_numpy(a).to(pred_z.device, pred_z.dtype), torch.from_numpy(b).to(pred_z.device, pred_z.dtype))


def _to_z(targets: torch.Tensor, log_means, log_stds) -> torch.Tensor:
    m = torch.as_tensor(log_means, dtype=targets.dtype).view(1, -1)
    s = torch.as_tensor(log_stds, dtype=targets.dtype).view(1, -1)
    return (torch.log(torch.clamp(targets, min=1e-12)) - m) / s


def conformal_calibration(mean_z, std_z, targets, alpha: float, method: str,
                          log_means=TARGET_LOG_MEANS, log_stds=TARGET_LOG_STDS) -> Dict:
    """train.py:1029-1051: split-conformal quantile of |target_z - mean_z| (/ std_z if 'scaled')."""
    tz = _to_z(targets, log_means, log_stds) if log_means is not None else targets
    if method == "scaled" and std_z is not None:
        s = (tz - mean_z).abs() / torch.clamp(std_z, min=1e-12)
    else:
        s = (tz - mean_z).abs()
        method = "absolute"
    n = s.size(0)
    q_level = min(max(math.ceil((n + 1) * (1 - alpha)) / n, 0.0), 1.0)
    return {"q": torch.quantile(s, q_level, dim=0), "method": method, "alpha": alpha}


def apply_conformal_intervals(mean_z, std_z, conf: Dict, log_means=TARGET_LOG_MEANS, log_stds=TARGET_LOG_STDS):
    """train.py:1054-1076: (mean, lower, upper) on the target scale."""
    q = conf["q"].to(mean_z)
    if conf.get("method") == "scaled" and std_z is not None:
        lo, hi = mean_z - q * std_z.to(mean_z), mean_z + q * std_z.to(mean_z)
    else:
        lo, hi = mean_z - q, mean_z + q
    if log_means is None:
        return mean_z, lo, hi
    m = torch.as_tensor(log_means, dtype=mean_z.dtype, device=mean_z.device).view(1, -1)
    s = torch.as_tensor(log_stds, dtype=mean_z.dtype, device=mean_z.device).view(1, -1)
    inv = lambda z: torch.exp(z * s + m)  # noqa: E731  (LogTransformer.inverse_transform_tensor)
    return inv(mean_z), inv(lo), inv(hi)
