"""Drop-in ``torch.nn.Module`` API of the reference's ALIGNN model (``scripts/train.py:303-401``,
``:528-586``) backed by the MI355X engine.

Constructor signatures, forward signatures, ``ValueError`` checks and state-dict keys match the
reference, so reference checkpoints load unchanged (``predict.py:328``,
``evaluate.py:454``) and callers (``train_epoch_hetero``, ``ensemble_collect``, ...) work as is.
Forward/backward run through ``libalignn_hip.so``; a model on the CPU raises (no CPU path).

* ``TransformerConv`` — parameter holder with PyG 2.7.0's names (lin_key, lin_query, lin_value,
  lin_edge, lin_skip, lin_beta); it executes fused inside the blocks.
* ``EdgeUpdateBlock`` / ``NodeUpdateBlock`` — standalone forward through one fused block.
* ``AlignnRegressor`` / ``HeteroAlignnRegressor`` — whole-model forward through one engine call
  (one autograd node); parameters are re-pointed into one flat fp32 buffer (:mod:`layout`).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F  # noqa: F401
from torch import nn

from . import infer, ops
from .engine import (AlignnEngine, BatchCache, FlatViews, _Conv, batch_cache, block_backward, block_forward,
                     proj_grads, proj_weights, site_seed)
from .layout import AlignnConfig, offsets


def _next_seed() -> int:
    # dropout masks are driven by torch's default CPU generator, so torch.manual_seed controls them
    return int(torch.randint(0, 2**62, (1,)).item())


def _require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X engine runs on the HIP device only (move model and data "
                           f"with .to('cuda')); there is no CPU fallback")


class TransformerConv(nn.Module):
    """PyG 2.7.0 ``TransformerConv`` parameter layout (the configuration the reference builds at
    train.py:308/:326: concat=True, beta=True, root_weight=True, bias=True, edge_dim set)."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True, beta: bool = False,
                 dropout: float = 0.0, edge_dim: Optional[int] = None, bias: bool = True, root_weight: bool = True,
                 **kwargs):
        super().__init__()
        if not (concat and beta and root_weight and bias and edge_dim is not None):
            raise NotImplementedError("the engine implements TransformerConv(concat=True, beta=True, root_weight=True, "
                                      "bias=True, edge_dim=...) — the configuration of train.py:308/:326")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.beta, self.dropout, self.edge_dim, self.root_weight = concat, beta, dropout, edge_dim, root_weight
        HC = heads * out_channels
        self.lin_key = nn.Linear(in_channels, HC)
        self.lin_query = nn.Linear(in_channels, HC)
        self.lin_value = nn.Linear(in_channels, HC)
        self.lin_edge = nn.Linear(edge_dim, HC, bias=False)
        self.lin_skip = nn.Linear(in_channels, HC, bias=bias)
        self.lin_beta = nn.Linear(3 * HC, 1, bias=False)

    def forward(self, *args, **kwargs):
        raise NotImplementedError("TransformerConv executes fused inside EdgeUpdateBlock/NodeUpdateBlock "
                                  "(gate + LayerNorm + ReLU + residual in one kernel)")


# ------------------------------------------------------------------------------------------------
# Standalone blocks
# ------------------------------------------------------------------------------------------------
def _csr_for(edge_index: torch.Tensor, n: int) -> ops.GraphCSR:
    key = (n, edge_index.data_ptr(), edge_index.size(1))
    cached = getattr(edge_index, "_alignn_csr", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    g = ops.GraphCSR(edge_index, n)
    g.check_indices("edge_index")
    try:
        edge_index._alignn_csr = (key, g)
    except (AttributeError, RuntimeError):
        pass
    return g


def _conv_params(conv: TransformerConv, norm: nn.LayerNorm, proj: Optional[nn.Linear]) -> List[torch.Tensor]:
    ps = [conv.lin_query.weight, conv.lin_key.weight, conv.lin_value.weight, conv.lin_skip.weight,
          conv.lin_query.bias, conv.lin_key.bias, conv.lin_value.bias, conv.lin_skip.bias,
          conv.lin_edge.weight, conv.lin_beta.weight, norm.weight, norm.bias]
    if proj is not None:
        ps += [proj.weight, proj.bias]
    return ps


def _conv_struct(ps: List[torch.Tensor]) -> _Conv:
    cv = _Conv()
    cv.Wqkvr = torch.cat([p.reshape(-1) for p in ps[0:4]]).view(-1, ps[0].size(1))
    cv.bqkvr = torch.cat([p.reshape(-1) for p in ps[4:8]])
    cv.We = ps[8].contiguous()
    cv.wbeta = ps[9].reshape(-1).contiguous()
    cv.lnw, cv.lnb = ps[10].contiguous(), ps[11].contiguous()
    cv.Wp = ps[12].contiguous() if len(ps) > 12 else None
    cv.bp = ps[13].contiguous() if len(ps) > 12 else None
    return cv


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, X, Fe, *ps):
        edge_index, heads, p_drop, seed = meta
        # under the reference's CUDA autocast the block's Linears take bf16 inputs (fp32 accumulation);
        # LayerNorm runs in fp32, so the block's output stays fp32 as autocast's layer_norm returns it
        ctx.precision = "bf16" if _autocast_dtype() is not None else "fp32"
        with torch.autocast("cuda", enabled=False), ops.gemm_precision(ctx.precision):
            return _BlockFn._fwd(ctx, meta, X, Fe, *ps)

    @staticmethod
    def _fwd(ctx, meta, X, Fe, *ps):
        edge_index, heads, p_drop, seed = meta
        X = X.contiguous().float()
        Fe = Fe.contiguous().float()
        n = X.size(0)
        g = _csr_for(edge_index, n)
        cv = _conv_struct([p.detach() for p in ps])
        if len(ps) > 12:
            M, wbar = proj_weights(cv.We, cv.Wp, cv.bp)
        else:
            M, wbar = cv.We, None
        Xn, c = block_forward(cv, X, g, Fe, g.perm_dst, M, wbar, heads, p_drop, site_seed(seed, 0),
                              site_seed(seed, 1))
        ctx.meta, ctx.g, ctx.cv, ctx.c, ctx.nps = meta, g, cv, c, len(ps)
        ctx.F_shape = Fe.shape
        return Xn

    @staticmethod
    def backward(ctx, dXn):
        with ops.gemm_precision(ctx.precision):
            return _BlockFn._bwd(ctx, dXn)

    @staticmethod
    def _bwd(ctx, dXn):
        cv, c, g = ctx.cv, ctx.c, ctx.g
        D = cv.We.size(0)
        dev = dXn.device
        dX = dXn.float().contiguous().clone()
        dF = torch.empty(ctx.F_shape, device=dev)
        gv = _Conv()
        gv.Wqkvr = torch.zeros(4 * D, D, device=dev)
        gv.bqkvr = torch.zeros(4 * D, device=dev)
        gv.We = torch.zeros_like(cv.We)
        gv.wbeta = torch.zeros_like(cv.wbeta)
        gv.lnw, gv.lnb = torch.zeros_like(cv.lnw), torch.zeros_like(cv.lnb)
        if ctx.nps > 12:
            gv.Wp, gv.bp = torch.zeros_like(cv.Wp), torch.zeros_like(cv.bp)
            dM, dwbar = torch.empty(D, D, device=dev), torch.empty(D, device=dev)
            block_backward(cv, gv, c, g, dX, dF, False, dM, dwbar)
            proj_grads(cv.We, cv.Wp, cv.bp, dM, dwbar, gv.We, gv.Wp, gv.bp)
        else:
            block_backward(cv, gv, c, g, dX, dF, False)
        grads = list(gv.Wqkvr.view(4, D, D).unbind(0)) + list(gv.bqkvr.view(4, D).unbind(0))
        grads += [gv.We, gv.wbeta.view(1, -1), gv.lnw, gv.lnb]
        if ctx.nps > 12:
            grads += [gv.Wp, gv.bp]
        return (None, dX, dF, *grads)


class EdgeUpdateBlock(nn.Module):
    """train.py:303-317 — ``e + Dropout(ReLU(LayerNorm(TransformerConv(e, lg_edge_index, angle_emb))))``."""

    def __init__(self, hidden: int, heads: int, dropout: float):
        super().__init__()
        if hidden % heads != 0:
            raise ValueError("hidden size must be divisible by number of heads")
        self.conv = TransformerConv(hidden, hidden // heads, heads=heads, edge_dim=hidden, dropout=dropout, beta=True)
        self.norm = nn.LayerNorm(hidden)
        self.dropout = nn.Dropout(dropout)

    def forward(self, edge_state: torch.Tensor, lg_edge_index: torch.Tensor, angle_emb: torch.Tensor) -> torch.Tensor:
        if edge_state.numel() == 0 or angle_emb.numel() == 0 or lg_edge_index.numel() == 0:
            return edge_state
        _require_device(edge_state, "EdgeUpdateBlock")
        p = self.dropout.p if self.training else 0.0
        meta = (lg_edge_index, self.conv.heads, p, _next_seed())
        return _BlockFn.apply(meta, edge_state, angle_emb, *_conv_params(self.conv, self.norm, None))


class NodeUpdateBlock(nn.Module):
    """train.py:320-336 — ``h + Dropout(ReLU(LayerNorm(TransformerConv(h, edge_index, edge_proj(e)))))``."""

    def __init__(self, hidden_node: int, hidden_edge: int, heads: int, dropout: float):
        super().__init__()
        if hidden_node % heads != 0:
            raise ValueError("hidden size must be divisible by number of heads")
        self.edge_proj = nn.Linear(hidden_edge, hidden_edge)
        self.conv = TransformerConv(hidden_node, hidden_node // heads, heads=heads, edge_dim=hidden_edge,
                                    dropout=dropout, beta=True)
        self.norm = nn.LayerNorm(hidden_node)
        self.dropout = nn.Dropout(dropout)

    def forward(self, node_state: torch.Tensor, edge_index: torch.Tensor, edge_state: torch.Tensor) -> torch.Tensor:
        if edge_state.numel() == 0 or edge_index.numel() == 0:
            return node_state
        _require_device(node_state, "NodeUpdateBlock")
        if self.edge_proj.weight.size(0) != node_state.size(1):
            raise NotImplementedError("the fused node block needs hidden_edge == hidden_node")
        p = self.dropout.p if self.training else 0.0
        meta = (edge_index, self.conv.heads, p, _next_seed())
        return _BlockFn.apply(meta, node_state, edge_state, *_conv_params(self.conv, self.norm, self.edge_proj))


# ------------------------------------------------------------------------------------------------
# Whole-model engine call
# ------------------------------------------------------------------------------------------------
class FlatState:
    """One flat parameter buffer + one flat gradient buffer and their views."""

    def __init__(self, flat: torch.Tensor, cfg: AlignnConfig, hetero: bool):
        self.flat = flat
        self.grad = torch.zeros_like(flat)
        self.P = FlatViews(flat, cfg, hetero)
        self.G = FlatViews(self.grad, cfg, hetero)
        self.names = list(self.P.named.keys())


def _autocast_dtype() -> Optional[torch.dtype]:
    """The reference's CUDA step calls ``model(batch)`` inside ``autocast(device_type="cuda",
    dtype=bfloat16)`` (train.py:632-636, :653-655).  Under an enabled CUDA autocast the engine runs that
    call at bf16 precision (bf16 matrix-core inputs, fp32 accumulation; the C3 path) and the outputs
    come back in the autocast dtype, as autocast's Linear heads return them.  None: no autocast."""
    if not torch.is_autocast_enabled("cuda"):
        return None
    dt = torch.get_autocast_dtype("cuda")
    if dt != torch.bfloat16:
        # the reference picks float16 only on GPUs without bf16 (train.py:634-635); MI355X has bf16
        raise NotImplementedError(f"autocast dtype {dt}: the engine implements the reference's bfloat16 autocast")
    return dt


class _ModelFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, holder, x, global_x, *params):
        model, batch, bc, mode, seed, precision = holder
        st = model._flat_state
        with torch.autocast("cuda", enabled=False), model._engine.using_precision(precision):
            out, ectx = model._engine.forward(st.P, batch, bc, model.training, seed, x, global_x, mode)
        ctx.model, ctx.ectx, ctx.precision = model, ectx, precision
        return out

    @staticmethod
    def backward(ctx, dout):
        st = ctx.model._flat_state
        with ctx.model._engine.using_precision(ctx.precision):
            ctx.model._engine.backward(st.P, st.G, ctx.ectx, dout.float())
        return (None, None, None, *[st.G.named[n] for n in st.names])


class _EngineModelMixin:
    _hetero: bool = True

    def set_precision(self, precision: str):
        """GEMM arithmetic of this model's forward/backward: "fp32" (default; the reference's CPU
        path) or "bf16" (bf16 matrix-core inputs, fp32 accumulation and storage — the reference's
        CUDA autocast GEMMs, train.py:632-636).  Returns self."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        self._engine.precision = precision
        return self

    def _flat_params(self) -> Dict[str, nn.Parameter]:
        named = dict(self.named_parameters())
        _, total, _ = offsets(self.config, self._hetero)
        return named

    def _ensure_flat(self) -> FlatState:
        st = getattr(self, "_flat_state", None)
        slots = getattr(self, "_flat_slots", None)
        if st is not None and slots is not None:
            # fast check (every call of the module API: ~20 us instead of ~170): each parameter is still
            # the object placed in the flat buffer, at its offset (a replaced Parameter or a new .data
            # fails it and the flat buffer is rebuilt below)
            if all(d.get(n) is p and p.data_ptr() == ptr for d, n, p, ptr in slots):
                return st
        cfg = self.config
        offs, total, _ = offsets(cfg, self._hetero)
        named = dict(self.named_parameters())
        first = named[next(iter(offs))]
        if st is not None and st.flat.device == first.device:
            base = st.flat.data_ptr()
            if all(named[k].data_ptr() == base + 4 * o for k, (o, _) in offs.items()):
                self._set_flat_slots(offs, st)
                return st
        flat = torch.empty(total, device=first.device, dtype=torch.float32)
        with torch.no_grad():
            for k, (o, shape) in offs.items():
                p = named[k]
                nel = p.numel()
                flat[o:o + nel].copy_(p.detach().reshape(-1))
                p.data = flat[o:o + nel].view(shape)
        st = FlatState(flat, cfg, self._hetero)
        object.__setattr__(self, "_flat_state", st)
        self._set_flat_slots(offs, st)
        return st

    def _set_flat_slots(self, offs, st: FlatState) -> None:
        """(owning module's parameter dict, name, parameter, its address in the flat buffer) per
        parameter, for _ensure_flat's fast check."""
        base = st.flat.data_ptr()
        slots = []
        for k, (o, _) in offs.items():
            mod_name, _, pname = k.rpartition(".")
            mod = self.get_submodule(mod_name) if mod_name else self
            slots.append((mod._parameters, pname, mod._parameters[pname], base + 4 * o))
        object.__setattr__(self, "_flat_slots", tuple(slots))

    def _run(self, data, mode: str):
        _require_device(data.x, type(self).__name__)
        st = self._ensure_flat()
        _require_device(st.flat, type(self).__name__)
        amp = _autocast_dtype()
        precision = "bf16" if amp is not None else self._engine.precision
        seed = _next_seed()
        if not self.training and not torch.is_grad_enabled():
            # inference (eval_epoch_hetero, ensemble_collect, predict: no_grad + eval): the forward as a
            # replayed launch plan once its batch signature repeats (infer.py), bitwise the eager one
            out = infer.forward(self, data, mode, precision)
            return out.clone() if amp is None else out.to(amp)
        bc = batch_cache(data)
        params = [dict(self.named_parameters())[n] for n in st.names]
        holder = (self, data, bc, mode, seed, precision)
        out = _ModelFn.apply(holder, data.x.contiguous().float(), data.global_x.contiguous().float(), *params)
        # autocast's Linear outputs (heads / feat_proj) are bf16: the fp32-accumulated outputs rounded
        # once, their gradient handed back to the engine in fp32
        return out if amp is None else out.to(amp)


class AlignnRegressor(_EngineModelMixin, nn.Module):
    """train.py:339-401 (base regressor; ``forward`` uses ``output_heads``)."""

    _hetero = False

    def __init__(self, node_dim: int, edge_dim: int, angle_dim: int, global_dim: int, target_dim: int, hidden: int,
                 layers: int, heads: int, dropout: float):
        super().__init__()
        if heads <= 0:
            raise ValueError("heads must be positive")
        if target_dim <= 0:
            raise ValueError("target_dim must be positive")
        if hidden % heads != 0:
            raise ValueError("hidden size must be divisible by number of heads")
        self.hidden = hidden
        self.heads = heads
        self.config = AlignnConfig(node_dim, edge_dim, angle_dim, global_dim, target_dim, hidden, layers, heads, dropout)
        self.node_encoder = nn.Sequential(nn.Linear(node_dim, hidden), nn.ReLU(), nn.Linear(hidden, hidden))
        self.edge_encoder = nn.Sequential(nn.Linear(edge_dim, hidden), nn.ReLU(), nn.Linear(hidden, hidden))
        self.angle_encoder = nn.Sequential(nn.Linear(angle_dim, hidden), nn.ReLU(),
                                           nn.Linear(hidden, hidden)) if angle_dim > 0 else None
        self.edge_blocks = nn.ModuleList([EdgeUpdateBlock(hidden, heads, dropout) for _ in range(layers)])
        self.node_blocks = nn.ModuleList([NodeUpdateBlock(hidden, hidden, heads, dropout) for _ in range(layers)])
        self.dropout = nn.Dropout(dropout)
        self.feat_proj = nn.Sequential(nn.Linear(hidden + global_dim, hidden), nn.ReLU(), nn.Dropout(dropout))
        self.output_heads = nn.ModuleList([nn.Linear(hidden, 1) for _ in range(target_dim)])
        self._engine = AlignnEngine(self.config)

    def forward(self, data):
        return self._run(data, "base")


class HeteroAlignnRegressor(_EngineModelMixin, nn.Module):
    """train.py:528-586: per-target mean and log-variance heads on the shared readout."""

    _hetero = True

    def __init__(self, base: AlignnRegressor, target_dim: int):
        super().__init__()
        self.base = base
        self.config = AlignnConfig(**{**base.config.__dict__, "target_dim": target_dim})
        self.mean_heads = nn.ModuleList([nn.Linear(base.feat_proj[0].out_features, 1) for _ in range(target_dim)])
        self.logvar_heads = nn.ModuleList([nn.Linear(base.feat_proj[0].out_features, 1) for _ in range(target_dim)])
        self._engine = AlignnEngine(self.config)

    def embed(self, data) -> torch.Tensor:
        return self._run(data, "embed")

    def forward(self, data):
        out = self._run(data, "hetero")
        T = self.config.target_dim
        return out[:, :T], out[:, T:]
